cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out/pv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv/vel -o vel -- python -u bench.py --velocity-only --steps 600 --warmup 50 --no-cpu-baseline > gpurun_out/pv/vel.log 2>&1 || { echo "vel prof rc=$?"; tail -5 gpurun_out/pv/vel.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv/roll -o roll -- python -u bench.py --rollout-only --steps 240 --warmup 24 --no-cpu-baseline > gpurun_out/pv/roll.log 2>&1 || { echo "roll prof rc=$?"; tail -5 gpurun_out/pv/roll.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pv/bench.json 2> gpurun_out/pv/bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/pv/bench.err; exit 1; }
find gpurun_out/pv -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -8 "$f" | cut -c1-200; done
tail -c 1500 gpurun_out/pv/bench.json
