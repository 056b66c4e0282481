#!/bin/bash
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/prof_rollout"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o ro -- python3 "$ROOT/bench.py" --rollout-only --steps 96 --warmup 24 > "$OUT/ro.log" 2>&1 || { echo "rc=$?"; tail -5 "$OUT/ro.log"; exit 1; }
tail -1 "$OUT/ro.log"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:110]}')
PY
# idle gaps between consecutive kernels on the GPU timeline of the timed rollout steps
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
pol = [i for i, r in enumerate(rows) if "policy_kernel" in r["Kernel_Name"]]
rows = rows[pol[-60]:pol[-1]]  # the last 60 rollout steps
gap = collections.defaultdict(float)
busy = collections.defaultdict(float)
for a, b in zip(rows, rows[1:]):
    g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
    gap[(a["Kernel_Name"][:40], b["Kernel_Name"][:40])] += max(g, 0) / 59e3
for r in rows:
    busy[r["Kernel_Name"][:60]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 59e3
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 59e3
print(f"per rollout step: span {span:.1f} us, busy {sum(busy.values()):.1f} us, idle {sum(gap.values()):.1f} us")
for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:8]:
    print(f"  busy {v:7.2f} us  {k}")
for k, v in sorted(gap.items(), key=lambda kv: -kv[1])[:8]:
    print(f"  gap  {v:7.2f} us  {k[0]} -> {k[1]}")
PY
