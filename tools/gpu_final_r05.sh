# round-5 evidence: the whole GPU suite, smoke, the bench line (--steps 20 --warmup 5, as the driver runs it),
# rocprof kernel stats of the step / rollout / velocity / learn legs, the step kernel's PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final_r05
mkdir -p $O
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
  echo "pytest ok: $(tail -1 $O/pytest_gpu.log)"
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_final.json 2> $O/bench_final.err || { echo "bench failed"; tail -20 $O/bench_final.err; exit 1; }
echo "bench ok"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vel -o vel -- python -u bench.py --velocity-only --steps 600 --warmup 50 --no-cpu-baseline > $O/vel.log 2>&1 || { echo "vel prof rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/roll -o roll -- python -u bench.py --rollout-only --steps 240 --warmup 24 --no-cpu-baseline > $O/roll.log 2>&1 || { echo "roll prof rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/learn -o learn -- python -u bench.py --learn-only --no-cpu-baseline > $O/learn.log 2>&1 || { echo "learn prof rc=$?"; exit 1; }
echo "leg profiles ok"
timeout -k 10 900 bash tools/profile.sh final_r05 > $O/profile_sh.log 2>&1 || { echo "profile.sh failed"; tail -5 $O/profile_sh.log; exit 1; }
echo "pmc ok"
