#!/bin/bash
# Kernel trace + SQ instruction-mix counters of the step kernel (one pass each, no tracing combined
# with counters); summary via tools/prof_summary.py.  Usage: bash tools/gpu_prof_step.sh TAG
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-step}
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rollout"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $B > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$OUT/trace.log"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sq" -o sq -- python3 $B > "$OUT/sq.log" 2>&1 || { echo "sq rc=$?"; tail -5 "$OUT/sq.log"; exit 1; }
if [ "$2" = "full" ]; then
  timeout -k 10 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/sq2" -o sq2 -- python3 $B > "$OUT/sq2.log" 2>&1 || { echo "sq2 rc=$?"; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 $B > "$OUT/fetch.log" 2>&1 || { echo "fetch rc=$?"; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 $B > "$OUT/write.log" 2>&1 || { echo "write rc=$?"; exit 1; }
fi
tail -1 "$OUT/trace.log" | cut -c1-300
echo ok
