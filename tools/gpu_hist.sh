#!/bin/bash
# Sliding-window velocity history: its GPU tests, the rollout tests, and the velocity legs of the bench.
set -e
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/hist"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_velocity.py tests/test_rollout.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 300 python bench.py --velocity-only --steps 300 --warmup 30 > "$OUT/vel.json" 2> "$OUT/vel.err"
timeout -k 10 400 python bench.py --velocity-learn > "$OUT/vel_learn.json" 2> "$OUT/vel_learn.err"
echo ok > "$OUT/done"
