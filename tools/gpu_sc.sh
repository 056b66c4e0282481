# self-collision round-5 job: the GPU tests the change touches, then the step kernel A/B against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sc
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_self_collision.py tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_hip_capsule.py tests/test_physics_invariants.py tests/test_gpu_velocity.py tests/test_gpu_shard8.py -m gpu > gpurun_out/sc/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/sc/tests.log | head -30; exit 1; }
echo "tests ok"; grep -E "passed|self-contact|pair classes" gpurun_out/sc/tests.log | tail -5
ROUNDS=${ROUNDS:-2} bash tools/ab_kernel.sh ${AB:-old direct3 nself}
