#!/bin/bash
# Extra SQ counter passes for the step kernel (run under gpurun): instruction fetch,
# wait / active cycles, LDS and transcendental mix.  One counter set per pass.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sq2}
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout"
i=0
for set in "SQ_WAVES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY" \
           "SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32" \
           "SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES" \
           "SQ_WAVES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o p$i -- python3 $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
