cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out/vj
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_velocity.py -m gpu > gpurun_out/vj/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/vj/tests.log | head -20; exit 1; }
tail -1 gpurun_out/vj/tests.log
timeout -k 10 200 python tools/vel_stamps.py > gpurun_out/vj/vst.txt 2>&1 || { echo "stamps failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vj/vel -o vel -- python -u bench.py --velocity-only --steps 600 --warmup 50 --no-cpu-baseline > gpurun_out/vj/vel.log 2>&1 || { echo "vel prof rc=$?"; exit 1; }
grep -h "curriculum\|vel_step" gpurun_out/vj/vel/vel_kernel_stats.csv | cut -d, -f1-8
tail -c 400 gpurun_out/vj/vel.log
