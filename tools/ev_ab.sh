cd $GRAFT_REPO_ROOT
for e in 1 4 1000; do
  timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --no-cpu-baseline --no-rollout --event-every $e | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('every $e', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))"
done
