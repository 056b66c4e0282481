"""Per-mini-batch kernel time of the PPO update engine from a rocprofv3 kernel trace of tools/prof_engine.py:
python tools/minibatch_summary.py TRACE.csv N_MINIBATCHES  (lines: us per mini-batch, share, calls, average,
(kernel, grid, workgroup, LDS bytes, VGPRs))."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
div = int(sys.argv[2])
tot = collections.Counter()
cnt = collections.Counter()
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    n = (n[5:] if n.startswith("void ") else n).split("(")[0][-40:]
    key = (n, r["Grid_Size_X"], r["Workgroup_Size_X"], r["LDS_Block_Size"], r["VGPR_Count"])
    tot[key] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    cnt[key] += 1
S = sum(tot.values())
print(f"total {S / 1e3 / div:.1f} us per mini-batch over {div} mini-batches")
for k, v in tot.most_common(30):
    print(f"{v / 1e3 / div:9.1f}us/div {100 * v / S:5.1f}%  n={cnt[k]:4d} avg={v / 1e3 / cnt[k]:9.1f}us  {k}")
