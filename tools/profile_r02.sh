#!/bin/bash
# Round-2 profile set (gpurun): kernel trace + PMC passes of the step kernel under the bench
# loop, the L2 hit rate, the rollout loop's kernel trace, and the env-count sweep.  One counter
# set per pass, never combined with tracing.  Output: gpurun_out/prof_r02/.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/prof_r02"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rollout"
pass() {  # name, rocprofv3 args...
  local n=$1; shift
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d "$OUT/$n" -o "$n" -- python3 $B > "$OUT/$n.log" 2>&1 || { echo "$n rc=$?"; tail -5 "$OUT/$n.log"; exit 1; }
  echo "$n ok"
}
pass trace --kernel-trace --stats
pass fetch --pmc FETCH_SIZE
pass write --pmc WRITE_SIZE
pass sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY
pass sq2 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY
pass tcc --pmc TCC_HIT_sum TCC_MISS_sum
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rollout" -o rollout -- python3 "$ROOT/bench.py" --rollout-only --steps 120 --warmup 24 > "$OUT/rollout.log" 2>&1 || { echo "rollout rc=$?"; tail -5 "$OUT/rollout.log"; exit 1; }
echo rollout ok
cd "$ROOT" && timeout -k 10 400 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-rollout --sweep 16384,65536,262144 > "$OUT/sweep.log" 2>&1 || { echo "sweep rc=$?"; tail -5 "$OUT/sweep.log"; exit 1; }
echo sweep ok
