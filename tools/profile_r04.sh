#!/bin/bash
# Round-4 profile set (gpurun): available counters, the FLOP-counter calibration probe, kernel trace
# + PMC passes of the step kernel under the bench loop, and the kernel traces of the rollout loop
# and of whole Runner iterations (learn).  One counter set per pass, never combined with tracing.
# Output: gpurun_out/prof_r04/.  Argument 1 / 2: the step-kernel passes / the rest (one gpurun call each).  A pass that fails fast (rc 1/2: e.g. a counter name the pool's
# rocprofv3 does not know) is reported and skipped; a timeout / signal ends the script.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/prof_r04"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-rollout --no-learn"
run() {  # name, timeout, rocprofv3 args... -- program...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" rocprofv3 "$@" > "$OUT/$n.log" 2>&1
  local rc=$?
  if [ $rc -eq 0 ]; then echo "$n ok"; return 0; fi
  echo "$n rc=$rc"; tail -3 "$OUT/$n.log"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
PART="${1:-all}"
if [ "$PART" != 2 ]; then
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/list_avail.txt" 2>&1; echo "list rc=$?"
FL="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MFMA_MOPS_F32"
run probe_flops 60 --pmc $FL --output-format csv -d "$OUT/probe_flops" -o probe -- "$ROOT/tools/probes/flop_count"
run probe_valu 60 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$OUT/probe_valu" -o probe -- "$ROOT/tools/probes/flop_count"
run trace 240 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $B
run fetch 240 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 $B
run write 240 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 $B
run sq 240 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sq" -o sq -- python3 $B
run sq2 240 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/sq2" -o sq2 -- python3 $B
run flops 240 --pmc $FL --output-format csv -d "$OUT/flops" -o flops -- python3 $B
run tcc 240 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/tcc" -o tcc -- python3 $B
fi
if [ "$PART" != 1 ]; then
run engine 240 --kernel-trace --stats --output-format csv -d "$OUT/engine" -o engine -- python3 "$ROOT/tools/prof_engine.py"
run lds 240 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/lds" -o lds -- python3 $B
run rollout 240 --kernel-trace --stats --output-format csv -d "$OUT/rollout" -o rollout -- python3 "$ROOT/bench.py" --rollout-only --steps 120 --warmup 24
run learn 300 --kernel-trace --stats --output-format csv -d "$OUT/learn" -o learn -- python3 "$ROOT/bench.py" --learn-only
# the velocity env (configs[1]): VecEnv.step loop and whole Runner iterations
run vel 240 --kernel-trace --stats --output-format csv -d "$OUT/vel" -o vel -- python3 "$ROOT/bench.py" --velocity-only --steps 300 --warmup 30
run vel_learn 400 --kernel-trace --stats --output-format csv -d "$OUT/vel_learn" -o vel_learn -- python3 "$ROOT/bench.py" --velocity-learn
# the policy kernel under the rollout loop
R="$ROOT/bench.py --rollout-only --steps 48 --warmup 8"
run pol_sq 240 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d "$OUT/pol_sq" -o p -- python3 $R
run pol_sq2 240 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d "$OUT/pol_sq2" -o p -- python3 $R
run pol_tcp 240 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d "$OUT/pol_tcp" -o p -- python3 $R
run pol_fetch 240 --pmc FETCH_SIZE --output-format csv -d "$OUT/pol_fetch" -o p -- python3 $R
cd "$ROOT" && timeout -k 10 600 python bench.py --steps 500 --warmup 50 > "$OUT/bench_full.log" 2>&1; echo "bench rc=$?"
# whole-loop traces are tens of MB: keep their stats only (gpurun copies back at most 64 MiB)
rm -f "$OUT"/learn/*_kernel_trace.csv "$OUT"/vel_learn/*_kernel_trace.csv
fi
