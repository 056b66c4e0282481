# round-5 GPU job: suite (or TESTS=...) + driver-shaped bench + rocprof stats of the step kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05}
mkdir -p $O
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu > $O/gpu_all.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/gpu_all.log | head -30; exit 1; }
  echo "pytest ok"; tail -2 $O/gpu_all.log
fi
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --kernel-only --steps 2000 --warmup 100 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -8 {} \;
