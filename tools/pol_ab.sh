#!/bin/bash
# A/B of policy-kernel variants in the rollout loop: bash tools/pol_ab.sh NAME [NAME ...]
# (NAME = suffix of legged_tracking_amd/_build/libgo1_rollout_NAME.so, or "current")
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = current ]; then unset GO1_ROLLOUT_LIB_OVERRIDE; else export GO1_ROLLOUT_LIB_OVERRIDE=$PWD/legged_tracking_amd/_build/libgo1_rollout_$v.so; fi
  timeout -k 10 300 python -m pytest tests/test_rollout.py -m gpu -q -x > gpurun_out/pt_$v.log 2>&1 || { echo "$v tests failed"; tail -5 gpurun_out/pt_$v.log; exit 1; }
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --rollout-only --steps 240 --warmup 24 > gpurun_out/pol_$v.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/pol_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4))"
  done
done
