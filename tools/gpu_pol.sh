#!/bin/bash
# Policy kernel: GPU rollout tests, A/B against libgo1_rollout_<name>.so builds (POLICY_AB="current name"), phase stamps.
set -e
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/pol"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_rollout.py -m gpu -x -v --timeout 250 --timeout-method thread > "$OUT/pytest_rollout.log" 2>&1
timeout -k 10 300 python -u tools/policy_bench.py ${POLICY_AB:-current} > "$OUT/policy_ab.txt" 2>&1
timeout -k 10 200 python -u tools/policy_stamps.py > "$OUT/policy_stamps.txt" 2>&1
timeout -k 10 200 python bench.py --rollout-only --steps 240 --warmup 24 > "$OUT/rollout.json" 2>&1
echo ok > "$OUT/done"
