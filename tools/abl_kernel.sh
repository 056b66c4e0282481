#!/bin/bash
# In-situ cost by ablation: the fused kernel alone (bench.py --kernel-only) on the product
# library and on ablation builds (legged_tracking_amd/_build/libgo1_abl_*.so, built locally with
# -DGO1_ABL_<NAME>).  Usage (gpurun): bash tools/abl_kernel.sh NO_MLP NO_PHYS ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export GO1_BENCH_ALLOW_NONFINITE=1
for v in full "$@"; do
  if [ "$v" = full ]; then unset GO1_LIB_OVERRIDE; else export GO1_LIB_OVERRIDE=$PWD/legged_tracking_amd/_build/libgo1_abl_$v.so; fi
  timeout -k 10 120 python bench.py --kernel-only --steps 300 --warmup 30 > gpurun_out/ablk_$v.log 2>&1 || { echo "$v rc=$?"; tail -3 gpurun_out/ablk_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ablk_$v.log)"
done
