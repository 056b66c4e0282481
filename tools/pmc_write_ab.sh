# WRITE_SIZE / FETCH_SIZE per step-kernel dispatch of variant builds (libgo1_var_NAME.so): bash tools/pmc_write_ab.sh NAME ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp GO1_BENCH_ALLOW_NONFINITE=1
mkdir -p gpurun_out/pmcab
for v in "$@"; do
  export GO1_LIB_OVERRIDE=$PWD/legged_tracking_amd/_build/libgo1_var_$v.so
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcab/${v}_$c -o p -- python -u bench.py --kernel-only --steps 200 --warmup 20 > gpurun_out/pmcab/${v}_$c.log 2>&1 || { echo "$v $c rc=$?"; exit 1; }
    python - "$v" "$c" <<'PY'
import csv, glob, sys
v, c = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/pmcab/{v}_{c}/**/*counter_collection.csv", recursive=True)[0]
vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "go1_step_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c]
print(v, c, "KiB/dispatch mean %.1f  (%d dispatches) -> B/env %.0f" % (sum(vals) / len(vals), len(vals), sum(vals) / len(vals) * 1024 / 4096))
PY
  done
done
