set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_self_collision.py tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_velocity.py -m gpu > gpurun_out/t10.log 2>&1
timeout -k 10 200 python -u tools/physics_ab.py > gpurun_out/pab8.log 2>&1
timeout -k 10 400 python -u bench.py --no-learn --no-rollout > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err
