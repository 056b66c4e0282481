#!/bin/bash
# rocprofv3 passes for the bench (run under gpurun).  Counters are collected in
# their own passes (never combined with tracing), per the pool's rules.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rollout"
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $B > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 $B > "$OUT/fetch.log" 2>&1 || { echo "fetch rc=$?"; exit 1; }
echo fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 $B > "$OUT/write.log" 2>&1 || { echo "write rc=$?"; exit 1; }
echo write ok
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sq" -o sq -- python3 $B > "$OUT/sq.log" 2>&1 || { echo "sq rc=$?"; tail -20 "$OUT/sq.log"; }
echo sq done
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/sq2" -o sq2 -- python3 $B > "$OUT/sq2.log" 2>&1 || { echo "sq2 rc=$?"; tail -20 "$OUT/sq2.log"; }
echo sq2 done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --output-format csv -d "$OUT/lds" -o lds -- python3 $B > "$OUT/lds.log" 2>&1 || { echo "lds rc=$?"; tail -20 "$OUT/lds.log"; }
echo lds done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 --output-format csv -d "$OUT/flop" -o flop -- python3 $B > "$OUT/flop.log" 2>&1 || { echo "flop rc=$?"; tail -20 "$OUT/flop.log"; }
echo flop done
# the rollout's stores (Runner.learn: no contact forces, no aux block): the kernel alone, HBM passes only
if [ "${ROLLOUT_PASS:-1}" = 1 ]; then
  R="$ROOT/gpurun_out/prof_${TAG}_rollout"; mkdir -p "$R"
  K="$ROOT/bench.py --kernel-only --rollout-outputs --steps 300 --warmup 20"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/fetch" -o fetch -- python3 $K > "$R/fetch.log" 2>&1 || { echo "rollout fetch rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/write" -o write -- python3 $K > "$R/write.log" 2>&1 || { echo "rollout write rc=$?"; exit 1; }
  echo rollout passes ok
fi
find "$OUT" -name "*.csv" | head -20
