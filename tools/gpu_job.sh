#!/bin/bash
# The GPU job of a measurement session (run under gpurun): bash tools/gpu_job.sh TAG
# Steps, each under its own time limit, chained so that a failure ends the job:
#   SUITE=1  pytest -m gpu (TESTS=... narrows it) and smoke()
#   BENCH=1  the driver-shaped bench line (--steps 20 --warmup 5) and, with SWEEP=list, the envs/GPU sweep
#   LEGS=1   rocprof kernel stats of the step (kernel-only), velocity, rollout and learn legs
#   PMC=1    the step kernel's counter passes (tools/profile.sh: trace, FETCH, WRITE, SQ mix, waits, LDS)
#   STAMPS=1 the section stamps of a -DGO1_STAMPS build (built beforehand: bash tools/variants.sh build stamps -DGO1_STAMPS)
# ISA_MIX=profiles/rNN/step_isa_mix.json gives the FLOP count its packed shares.
# Output: gpurun_out/TAG/ (summarise into profiles/ with tools/prof_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=${1:-job}
O=gpurun_out/$TAG
mkdir -p "$O"
R=$PWD
if [ "${SUITE:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest ${PYX--x} -v --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; exit 1; }
  echo "pytest ok: $(tail -1 $O/pytest_gpu.log)"
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  tail -c 1500 $O/bench.json
  if [ -n "$SWEEP" ]; then
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-rollout --no-cpu-baseline --sweep "$SWEEP" > $O/bench_sweep.json 2> $O/bench_sweep.err || { echo "sweep failed"; tail -20 $O/bench_sweep.err; exit 1; }
    echo "sweep ok"
  fi
fi
export TMPDIR=/tmp
if [ "${LEGS:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/step -o step -- python3 -u $R/bench.py --kernel-only --steps 2000 --warmup 100 --no-cpu-baseline > $O/step.log 2>&1 || { echo "step prof rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/vel -o vel -- python3 -u $R/bench.py --velocity-only --steps 600 --warmup 50 --no-cpu-baseline > $O/vel.log 2>&1 || { echo "vel prof rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/roll -o roll -- python3 -u $R/bench.py --rollout-only --steps 240 --warmup 24 --no-cpu-baseline > $O/roll.log 2>&1 || { echo "roll prof rc=$?"; exit 1; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/learn -o learn -- python3 -u $R/bench.py --learn-only --no-cpu-baseline > $O/learn.log 2>&1 || { echo "learn prof rc=$?"; exit 1; }
  find $O/step $O/vel $O/roll $O/learn -type f ! -name "*kernel_stats.csv" -delete  # (gpurun copies back <= 64 MiB)
  echo "leg profiles ok"
fi
if [ "${PMC:-0}" = 1 ]; then
  timeout -k 10 1200 bash tools/profile.sh $TAG > $O/profile_sh.log 2>&1 || { echo "profile.sh failed"; tail -5 $O/profile_sh.log; exit 1; }
  [ -f "$ISA_MIX" ] && cp "$ISA_MIX" $O/step_isa_mix.json  # packed shares for the FLOP count (tools/isa_sections.py)
  python tools/prof_summary.py gpurun_out/prof_$TAG $O step go1_step_kernel > $O/prof_summary.log 2>&1 || { echo "summary failed"; tail -5 $O/prof_summary.log; exit 1; }
  if [ -d gpurun_out/prof_${TAG}_rollout ]; then
    python tools/prof_summary.py gpurun_out/prof_${TAG}_rollout $O step_rollout go1_step_kernel >> $O/prof_summary.log 2>&1 || { echo "rollout summary failed"; exit 1; }
  fi
  rm -rf gpurun_out/prof_$TAG gpurun_out/prof_${TAG}_rollout  # raw counter CSVs of whole bench runs: far above what gpurun copies back
  echo "pmc ok"; tail -8 $O/prof_summary.log
fi
if [ "${STAMPS:-0}" = 1 ]; then
  cd $R && timeout -k 10 300 python -u tools/stamps.py > $O/step_stamps.txt 2>&1 || { echo "stamps failed"; tail -5 $O/step_stamps.txt; exit 1; }
  head -5 $O/step_stamps.txt
fi
exit 0
