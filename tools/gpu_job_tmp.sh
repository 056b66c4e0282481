set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python -u tools/ppo_gemm_bench.py legged_tracking_amd/_build/variants/ppo_v1.so legged_tracking_amd/_build/variants/ppo_v2.so > gpurun_out/gb5.log 2>&1
timeout -k 10 300 python -u tools/vel_stamps.py > gpurun_out/vstamps2.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_velocity.py tests/test_ppo_engine.py -m gpu > gpurun_out/t9.log 2>&1
timeout -k 10 120 python -u tools/xw_stamps.py legged_tracking_amd/_build/variants/ppo_stamps.so > gpurun_out/st4.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/velprof3 -o run -- python3 $R/bench.py --velocity-only --steps 600 > $R/gpurun_out/velprof3.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/eprof2 -o run -- python3 $R/tools/prof_engine.py > $R/gpurun_out/eprof2.log 2>&1
cd $R
timeout -k 10 200 python -u tools/physics_ab.py > gpurun_out/pab7.log 2>&1
