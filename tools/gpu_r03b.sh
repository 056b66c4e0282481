#!/bin/bash
# Round-3 measurement batch: velocity env (tests, host profile, side-stream A/B), policy kernel
# (phase stamps, PMC passes under the rollout loop).  Every GPU step under its own timeout; stop at
# the first failure.
set -e
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/r03b"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_velocity.py -x -v --timeout 250 --timeout-method thread > "$OUT/pytest_vel.log" 2>&1
timeout -k 10 200 python -u tools/env_host_prof.py 512 --velocity > "$OUT/vel_host_prof.txt" 2>&1
timeout -k 10 200 python bench.py --velocity-only --steps 500 --warmup 50 > "$OUT/vel_bench_side.json" 2>&1
GO1_VEL_SHIFT_SIDE=0 timeout -k 10 200 python bench.py --velocity-only --steps 500 --warmup 50 > "$OUT/vel_bench_noside.json" 2>&1
timeout -k 10 200 python -u tools/policy_stamps.py > "$OUT/policy_stamps.txt" 2>&1
B="$ROOT/bench.py --rollout-only --steps 48 --warmup 8"
i=0
for set in "SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/pol_p$i" -o p$i -- python3 $B > "$OUT/pol_p$i.log" 2>&1
done
echo ok > "$OUT/done"
