# round-4 evidence, part 1: the whole GPU suite, smoke, the default bench line
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_all.log 2>&1
echo "pytest rc=$?"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?"
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r04.json 2> gpurun_out/bench_r04.err
echo "bench rc=$?"
