# record kernel (tools/experiments/record_flat.patch built as libgo1_rollout_flat.so): parity + A/B in the rollout loop
R=$GRAFT_REPO_ROOT
cd $R
export GO1_ROLLOUT_LIB_OVERRIDE=$R/legged_tracking_amd/_build/libgo1_rollout_flat.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rollout.py tests/test_gpu_full_size.py tests/test_gpu_velocity.py -m gpu > gpurun_out/t18.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in 1 0 1 0; do
  GO1_RECORD_FLAT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/recf_$v -o p -- python3 $R/bench.py --rollout-only --steps 120 --warmup 24 > $R/gpurun_out/recf_$v.log 2>&1 || exit 1
  python3 - $R $v >> $R/gpurun_out/recf_summary.txt <<'PY'
import csv, json, sys
R, v = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"{R}/gpurun_out/recf_{v}/p_kernel_stats.csv")):
    if "record" in r["Name"]:
        print(v, r["Name"][:40], r["Calls"], r["AverageNs"])
l = [x for x in open(f"{R}/gpurun_out/recf_{v}.log") if x.startswith("{")]
print(v, "rollout", json.loads(l[-1])["value"] if l else None)
PY
done
