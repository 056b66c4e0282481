"""Condense gpurun_out/prof_r03 (tools/profile_r03.sh) into the files committed under profiles/r03.

  python tools/collect_r03.py [src=gpurun_out/prof_r03] [dst=profiles/r03]

step_kernel_stats.csv / step_counters.json (tools/prof_summary.py, FLOPs with the packed shares of
step_isa_mix.json), rollout_kernel_stats.csv (rollout loop), learn_kernel_stats.csv (whole Runner
iterations: every kernel, incl. torch / hipBLASLt), flop_probe.json (counter calibration) and
bench_full.json (the bench line of the same session)."""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stats(src, name, dst, out, keep_all=False):
    f = glob.glob(os.path.join(src, name, "*kernel_stats.csv"))
    if not f:
        return
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    with open(os.path.join(dst, out), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows if keep_all else rows[:40])


def probe(src, dst):
    res = {}
    for d in ("probe_flops", "probe_valu"):
        f = glob.glob(os.path.join(src, d, "*counter_collection.csv"))
        if not f:
            continue
        acc = defaultdict(float)
        for r in csv.DictReader(open(f[0])):
            acc[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (di, n), v in acc.items():
            res.setdefault(di, {})[n] = v
    names = ["v_fma_f32", "v_pk_fma_f32", "v_add_f32", "v_pk_add_f32", "v_mul_f32", "v_pk_mul_f32",
             "v_mfma_f32_16x16x4_f32", "v_rcp_f32"]
    out = {"what": "tools/probes/flop_count.hip: one wave, 8000 instructions of each kind; per-dispatch counters",
           "dispatches": {names[di - 1] if 0 < di <= len(names) else str(di): v for di, v in sorted(res.items())}}
    json.dump(out, open(os.path.join(dst, "flop_probe.json"), "w"), indent=1)


def policy_counters(src, dst):
    """Per-launch means of the policy kernel's PMC passes (rollout loop)."""
    acc = defaultdict(list)
    for d in ("pol_sq", "pol_sq2", "pol_tcp", "pol_fetch"):
        for f in glob.glob(os.path.join(src, d, "*counter_collection.csv")):
            per = defaultdict(float)
            for r in csv.DictReader(open(f)):
                if "policy_kernel" in r["Kernel_Name"]:
                    per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
            for (_, n), v in per.items():
                acc[n].append(v)
    if not acc:
        return
    mean = {n: sum(v) / len(v) for n, v in acc.items()}
    out = {"kernel": "policy_kernel_split (rollout loop, 4096 envs)", "per_launch_mean": mean,
           "launches_per_counter": {n: len(v) for n, v in acc.items()}}
    if "TCP_TCC_READ_REQ_sum" in mean:
        out["l2_to_cu_bytes_per_launch_128B_requests"] = mean["TCP_TCC_READ_REQ_sum"] * 128
    json.dump(out, open(os.path.join(dst, "policy_counters.json"), "w"), indent=1)


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "prof_r03")
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "r03")
    os.makedirs(dst, exist_ok=True)
    mix = subprocess.run([sys.executable, os.path.join(REPO, "tools", "isa_sections.py")], capture_output=True,
                         text=True, check=True).stdout.strip().splitlines()[-1]
    open(os.path.join(dst, "step_isa_mix.json"), "w").write(mix + "\n")
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_summary.py"), src, dst, "step",
                    "go1_step_kernel"], check=True, capture_output=True)
    stats(src, "rollout", dst, "rollout_kernel_stats.csv")
    stats(src, "learn", dst, "learn_kernel_stats.csv", keep_all=True)
    stats(src, "vel", dst, "vel_kernel_stats.csv")
    stats(src, "vel_learn", dst, "vel_learn_kernel_stats.csv", keep_all=True)
    policy_counters(src, dst)
    probe(src, dst)
    b = os.path.join(src, "bench_full.log")
    if os.path.exists(b):
        line = [l for l in open(b).read().splitlines() if l.startswith("{")]
        if line:
            json.dump(json.loads(line[-1]), open(os.path.join(dst, "bench_full.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
