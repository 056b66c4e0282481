#!/bin/bash
# Kernel trace of whole Runner iterations (trajectory task), stats only.
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/prof_learn"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/learn" -o learn -- python3 "$ROOT/bench.py" --learn-only > "$OUT/learn.log" 2>&1
rc=$?
rm -f "$OUT"/learn/*_kernel_trace.csv
exit $rc
