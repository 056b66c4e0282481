#!/bin/bash
# SQ counters of the step kernel for the product library and ablation builds (one --pmc pass
# per counter set, kernel-only bench).  Usage (gpurun): bash tools/pmc_variant.sh full NO_PM ...
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
export GO1_BENCH_ALLOW_NONFINITE=1
B="$ROOT/bench.py --kernel-only --steps 60 --warmup 10"
for v in "$@"; do
  if [ "$v" = full ]; then unset GO1_LIB_OVERRIDE; else export GO1_LIB_OVERRIDE=$ROOT/legged_tracking_amd/_build/libgo1_${PREFIX:-abl}_$v.so; fi
  O="$ROOT/gpurun_out/pmc_$v"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH --output-format csv -d "$O/a" -o a -- python3 $B > "$O.a.log" 2>&1 || { echo "$v a rc=$?"; tail -3 "$O.a.log"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d "$O/b" -o b -- python3 $B > "$O.b.log" 2>&1 || { echo "$v b rc=$?"; tail -3 "$O.b.log"; exit 1; }
  python3 - "$O" "$v" <<'PY'
import csv, glob, sys, collections
O, v = sys.argv[1], sys.argv[2]
d = collections.defaultdict(list)
for f in glob.glob(O + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "go1_step_kernel<false" in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = sum(d["SQ_WAVES"]) / len(d["SQ_WAVES"])
print(v, {k: round(sum(x) / len(x) / w, 1) for k, x in sorted(d.items())})
PY
done
