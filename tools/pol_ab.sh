cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_rollout.py -m gpu -q -x > gpurun_out/pt.log 2>&1; tail -1 gpurun_out/pt.log
for v in 16 8; do
  if [ $v = 8 ]; then export GO1_ROLLOUT_LIB_OVERRIDE=$PWD/legged_tracking_amd/_build/libgo1_rollout_w8.so; fi
  timeout -k 10 200 python bench.py --rollout-only --steps 240 --warmup 24 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('waves $v', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4))"
done
