"""Condense a tools/profile.sh output directory into the files committed under profiles/.

  python tools/prof_summary.py gpurun_out/prof_r01 profiles/r01 [tag]

Writes <tag>_kernel_stats.csv (the rocprofv3 --stats rows of this repo's kernels)
and <tag>_counters.json (per-dispatch means of every PMC counter collected, for
the fused step kernel, plus the HBM traffic per launch derived from them).

Counter units / corrections (MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and
WRITE_SIZE are in KiB per dispatch.  FETCH_SIZE reads exactly half of the bytes
of wide (16 B/lane) coalesced loads; the step kernel's loads are 4 B/lane SoA
rows, an uncalibrated width, so the raw value is reported and the doubled value
is given as the upper bound.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

OURS = ("go1_", "mlp", "gae", "ppo", "rollout")


def kernel_stats(src):
    rows = []
    for f in glob.glob(os.path.join(src, "trace", "*kernel_stats.csv")):
        with open(f) as fh:
            r = csv.DictReader(fh)
            for row in r:
                if any(k in row["Name"] for k in OURS):
                    rows.append(row)
    return rows


def counters(src, match="go1_step_kernel"):
    """Per-dispatch means of every counter: instances (XCD / SE) of one dispatch are
    summed, then averaged over dispatches; a counter collected in several passes is
    averaged over the passes."""
    per = defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(src, "*", "*counter_collection.csv"))):
        # the pol_* passes profile the rollout loop (whose step kernel runs beside the policy kernel)
        if os.path.basename(os.path.dirname(f)).startswith("pol_") != match.startswith("policy"):
            continue
        acc = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if match in row["Kernel_Name"]:
                    acc[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
                    if not meta:
                        meta = {k: row[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
                                                    "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
        by_name = defaultdict(list)
        for (disp, name), v in acc.items():
            by_name[name].append(v)
        for name, vals in by_name.items():
            per[name].append(sum(vals) / len(vals))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}, meta


def main():
    src, dst = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else "step"
    os.makedirs(dst, exist_ok=True)
    rows = kernel_stats(src)
    if rows:
        with open(os.path.join(dst, f"{tag}_kernel_stats.csv"), "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    match = sys.argv[4] if len(sys.argv) > 4 else "go1_step_kernel"
    means, counts, meta = counters(src, match)
    out = {"kernel": match, "passes_per_counter": counts, "per_dispatch_mean": means,
           "resources": meta}
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        fetch = means["FETCH_SIZE"] * 1024
        write = means["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = {"fetch": fetch, "write": write, "traffic": fetch + write,
                                       "traffic_upper_fetch_doubled": 2 * fetch + write}
    # FP32 FLOPs per launch from the VALU / MFMA FLOP counters.  SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F32
    # count instructions per wave, a packed v_pk_* instruction once (tools/probes/flop_count.hip,
    # profiles/r03/flop_probe.json); SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 = MFMA FLOPs.  The packed share
    # of each class comes from the kernel's trip-count-weighted static ISA (tools/isa_sections.py ->
    # <dst>/<tag>_isa_mix.json); without it the count is the lower bound (packed counted once).
    if all(k in means for k in ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
                                "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_MFMA_MOPS_F32")):
        pk = {"fma": 0.0, "add": 0.0, "mul": 0.0}
        mix_path = os.path.join(dst, f"{tag}_isa_mix.json")
        if os.path.exists(mix_path):
            mix = json.load(open(mix_path))["weighted_static_f32_mix"]
            pk = {k: mix[k]["packed_share"] for k in pk}
        lanes = 64

        def flops(p):
            return lanes * (2 * means["SQ_INSTS_VALU_FMA_F32"] * (1 + p["fma"]) +
                            means["SQ_INSTS_VALU_ADD_F32"] * (1 + p["add"]) +
                            means["SQ_INSTS_VALU_MUL_F32"] * (1 + p["mul"]) +
                            means["SQ_INSTS_VALU_TRANS_F32"]) + 512 * means["SQ_INSTS_VALU_MFMA_MOPS_F32"]
        out["flops_per_launch"] = flops(pk)
        out["flops_per_launch_lower_bound"] = flops({"fma": 0.0, "add": 0.0, "mul": 0.0})
        out["flops_packed_share"] = pk
    if "SQ_WAVES" in means and means["SQ_WAVES"]:
        w = means["SQ_WAVES"]
        out["per_wave"] = {k: means[k] / w for k in means if k.startswith("SQ_") and k != "SQ_WAVES"}
    with open(os.path.join(dst, f"{tag}_counters.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for r in rows:
        print(r["Name"][:60], r["Calls"], r["AverageNs"])
    print(json.dumps(out.get("hbm_bytes_per_launch"), indent=1))


if __name__ == "__main__":
    main()
