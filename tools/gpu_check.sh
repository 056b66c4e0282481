#!/bin/bash
# GPU validation pass (run under gpurun).  Every GPU step has its own time limit;
# a crash / fault / timeout (exit >= 2 other than pytest's "tests failed" = 1) ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -5 "gpurun_out/$name.log"
  return $rc
}
MODE=${1:-all}
run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ "$MODE" = "tests" ] && exit $rc
run bench 600 python bench.py --steps 500 --warmup 50 || exit $?
cd /tmp && run_prof() { timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o r1 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1; }
echo "== rocprof"; run_prof; echo "rc=$?"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
