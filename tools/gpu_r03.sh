#!/bin/bash
# Round-3 GPU iteration: verbose GPU suite, integrator error statistics, quick bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/integrator_stats.py 4096 single_path > gpurun_out/integrator_stats.json 2>&1 || exit $?
timeout -k 10 300 python tools/integrator_stats.py 4096 plane > gpurun_out/integrator_stats_plane.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline $BENCH_EXTRA > gpurun_out/bench_quick.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_quick.log').read().strip().splitlines()[-1]); print('value', round(d['value']/1e6,2), 'M env-steps/s; ms/step', round(d['ms_per_step'],4), 'kernel ms', round(d['roofline']['kernel_ms'],4), 'rollout', round(d['rollout']['value']/1e6, 2))"
exit $rc
