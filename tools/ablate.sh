#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
export GO1_BENCH_ALLOW_NONFINITE=1
for v in full NO_MLP NO_PHYS NO_CONTACT; do
  if [ $v = full ]; then unset GO1_LIB_OVERRIDE; else export GO1_LIB_OVERRIDE=$PWD/legged_tracking_amd/_build/libgo1_abl_$v.so; fi
  echo "== $v"
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/abl_$v.log 2>&1 || { echo "fail rc=$?"; tail -5 gpurun_out/abl_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), 'ms/step kernel', round(d['roofline']['kernel_ms'],4), 'value', round(d['value']/1e6,2),'M')"
done
