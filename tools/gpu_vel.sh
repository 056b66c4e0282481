#!/bin/bash
# Velocity step: GPU parity tests, curriculum-launch stamps, bench line, kernel trace.
set -e
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/vel"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_velocity.py -x -v --timeout 250 --timeout-method thread > "$OUT/pytest_vel.log" 2>&1
timeout -k 10 200 python -u tools/vel_stamps.py > "$OUT/vel_stamps.txt" 2>&1
timeout -k 10 200 python bench.py --velocity-only --steps 500 --warmup 50 > "$OUT/vel_bench.json" 2>&1
timeout -k 10 200 python -u tools/env_host_prof.py 512 --velocity > "$OUT/vel_host_prof.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o vel -- python3 bench.py --velocity-only --steps 300 --warmup 30 > "$OUT/prof.log" 2>&1
echo ok > "$OUT/done"
