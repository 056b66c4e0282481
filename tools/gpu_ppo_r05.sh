# PPO engine job: its GPU tests, then the learn leg under rocprof (kernel stats)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out/pj
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ppo_engine.py -m gpu > gpurun_out/pj/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pj/tests.log | head -20; exit 1; }
tail -1 gpurun_out/pj/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pj/learn -o learn -- python -u bench.py --learn-only --no-cpu-baseline > gpurun_out/pj/learn.log 2>&1 || { echo "learn prof rc=$?"; exit 1; }
tail -c 300 gpurun_out/pj/learn.log
