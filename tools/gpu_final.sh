#!/bin/bash
# Round-end check: the whole GPU test suite, smoke(), then the default bench line (N=1).
set -e
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/final"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo ok > "$OUT/done"
