#!/bin/bash
# GPU tests (verbose, with the invariant measurements printed) + integrator error statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; grep -E "^hip:|oracle:" gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/integrator_stats.py 4096 single_path > gpurun_out/integrator_stats.json 2>&1 || exit $?
timeout -k 10 300 python tools/integrator_stats.py 4096 plane > gpurun_out/integrator_stats_plane.json 2>&1 || exit $?
echo done
