cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
for v in 1 0 1 0; do
  echo "== TORCH_BLAS_PREFER_HIPBLASLT=$v"
  TORCH_BLAS_PREFER_HIPBLASLT=$v timeout -k 10 240 python bench.py --learn-only --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/ab/learn_$v.json 2> gpurun_out/ab/learn_$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab/learn_$v.json'));print(json.dumps(d.get('learn',d))[:400])"
done
