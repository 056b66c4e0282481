#!/bin/bash
# PMC passes of the velocity step (bench.py --velocity-only), one rocprofv3 run per counter set, and the curriculum
# launch's stamps: bash tools/profile_vel.sh TAG, then
#   python tools/prof_summary.py gpurun_out/prof_vel_TAG OUTDIR vel go1_vel_step_kernel
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-vel}
OUT="$ROOT/gpurun_out/prof_vel_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --velocity-only --steps 60 --warmup 10 --no-cpu-baseline"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o p$i -- python3 $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -3 "$OUT/p$i.log"; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $B > "$OUT/trace.log" 2>&1 || exit 1
echo ok
