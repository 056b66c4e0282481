#!/bin/bash
# A/B of a locally built velocity library variant (legged_tracking_amd/_build/libgo1_velocity_$1.so) against the
# product one: bench.py --velocity-only on each (the variant copied over the product library in this scratch copy).
set -e
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
mkdir -p gpurun_out/velab
B=legged_tracking_amd/_build
timeout -k 10 200 python bench.py --velocity-only --steps 300 --warmup 30 > gpurun_out/velab/base.json 2>/dev/null
cp $B/libgo1_velocity.so $B/libgo1_velocity_base.so
cp $B/libgo1_velocity_$1.so $B/libgo1_velocity.so
timeout -k 10 200 python bench.py --velocity-only --steps 300 --warmup 30 > gpurun_out/velab/$1.json 2>/dev/null
cp $B/libgo1_velocity_base.so $B/libgo1_velocity.so
timeout -k 10 200 python bench.py --velocity-only --steps 300 --warmup 30 > gpurun_out/velab/base2.json 2>/dev/null
for f in base $1 base2; do python -c "import json;d=json.load(open('gpurun_out/velab/$f.json'));print('$f',d['value'],d['kernel_ms'])"; done
