#!/bin/bash
# A/B timing of compile-time variants of the step kernel.
#   local:  bash tools/variants.sh build NAME "-DFLAG=1 ..." [NAME "FLAGS" ...]
#   gpurun: bash tools/variants.sh run NAME [NAME ...]
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
B="$ROOT/legged_tracking_amd/_build"
BASEFLAGS=${BASEFLAGS--fno-slp-vectorize}
if [ "$1" = build ]; then
  shift
  while [ $# -gt 1 ]; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off $BASEFLAGS $2 \
      -o "$B/libgo1_var_$1.so" "$ROOT/legged_tracking_amd/csrc/go1_step.hip" "$ROOT/legged_tracking_amd/csrc/go1_terrain.hip" || exit 1
    echo "built $1: $2"; shift 2
  done
  exit 0
fi
shift
cd "$ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = current ]; then unset GO1_LIB_OVERRIDE; else export GO1_LIB_OVERRIDE="$B/libgo1_var_$v.so"; fi
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-rollout > gpurun_out/var_$v.log 2>&1 || { echo "$v failed rc=$?"; tail -3 gpurun_out/var_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/var_$v.log').read().strip().splitlines()[-1]); print('$v', 'kernel_ms', round(d['roofline']['kernel_ms'],4), 'ms/step', round(d['ms_per_step'],4))"
  done
done
