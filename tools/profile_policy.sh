#!/bin/bash
# PMC passes of the rollout loop (policy_kernel_split beside the step kernel), one rocprofv3 run per counter set,
# into gpurun_out/prof_policy/pol_pN (the pol_ prefix is what tools/prof_summary.py selects for a policy kernel):
#   bash tools/profile_policy.sh && python tools/prof_summary.py gpurun_out/prof_policy OUTDIR policy policy_kernel_split
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/prof_policy"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --rollout-only --steps 48 --warmup 8"
i=0
for set in "SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "FETCH_SIZE" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/pol_p$i" -o p$i -- python3 $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -3 "$OUT/p$i.log"; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $B > "$OUT/trace.log" 2>&1 || exit 1
echo ok
