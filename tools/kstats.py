"""Per-launch-shape kernel time summary of a rocprofv3 --kernel-trace CSV (name, grid, LDS, VGPRs):
python tools/kstats.py gpurun_out/<dir>/run_kernel_trace.csv [divisor]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
d = collections.defaultdict(list)
for r in rows:
    nm = r["Kernel_Name"]
    short = nm.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[-40:]
    key = (short, r["Grid_Size_X"], r["Workgroup_Size_X"], r["LDS_Block_Size"], r["VGPR_Count"])
    d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:30]:
    print(f"{sum(v) / 1e3 / div:9.1f}us/div {100 * sum(v) / tot:5.1f}%  n={len(v):4d} avg={sum(v) / len(v) / 1e3:8.1f}us  {k}")
print(f"total {tot / 1e3 / div:.1f} us/div")
