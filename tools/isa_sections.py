"""Static instruction counts between MARK() section markers of the step kernel.

  python tools/isa_sections.py   (compiles go1_step.hip with -DGO1_ISA_MARKS into /tmp; counts the specialised product kernel)

Straight-line sections inside the sub-step loop run decimation x n_internal
times per step, so static counts x trip counts ~ the dynamic SQ_INSTS_VALU."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = "/tmp/go1_isa"
sys.path.insert(0, REPO)
from legged_tracking_amd.build import STEP_FLAGS as PKFLAGS  # noqa: E402


def main():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(REPO, "legged_tracking_amd", "csrc", "go1_step.hip")
    extra = sys.argv[1:]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", *PKFLAGS,
                    "-DGO1_ISA_MARKS", *extra, "-c", "--save-temps", "-o", os.path.join(OUT, "k.o"), src],
                   cwd=OUT, check=True)
    s = open(os.path.join(OUT, "go1_step-hip-amdgcn-amd-amdhsa-gfx950.s")).read().splitlines()
    start = next(i for i, l in enumerate(s) if l.startswith("_Z15go1_step_kernelILb0ELi7ELb1EE"))
    end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
    cur, counts = "prologue", {}
    for l in s[start:end]:
        m = re.search(r"; MARK (\w+)", l)
        if m:
            cur = m.group(1)
            continue
        t = l.strip()
        c = counts.setdefault(cur, [0, 0, 0, 0, 0, 0])
        if t.startswith("scratch_") or (t.startswith("buffer_") and "off, s[0:3]" in t):
            c[5] += 1  # register spill traffic
        if t.startswith("v_"):
            c[0] += 1
            if "mfma" in t:
                c[1] += 1
        elif t.startswith(("global_", "buffer_")):
            c[2] += 1
        elif t.startswith("ds_"):
            c[3] += 1
        elif t.startswith("s_"):
            c[4] += 1
    print(f"{'section (code after marker)':32s} {'VALU':>6s} {'MFMA':>5s} {'VMEM':>5s} {'LDS':>5s} {'SALU':>5s} {'SPILL':>5s}")
    for k, (v, mf, vm, ld, sa, sp) in counts.items():
        print(f"{k:32s} {v:6d} {mf:5d} {vm:5d} {ld:5d} {sa:5d} {sp:5d}")
    # f32 arithmetic by class, scalar vs packed (the SQ_INSTS_VALU_{FMA,ADD,MUL}_F32 counters count a
    # v_pk_* instruction once, tools/probes/flop_count.hip): the packed share of each class, for the
    # FP32-roofline FLOP count (profiles/r03/step_counters.json "flops_per_launch")
    cls = {"fma": (r"^v_(fma|fmac|fmaak|fmamk|mad|mac)_f32", r"^v_pk_fma_f32"),
           "add": (r"^v_(add|sub|subrev)_f32", r"^v_pk_add_f32"),
           "mul": (r"^v_mul_f32", r"^v_pk_mul_f32")}
    tally = {c: [0, 0] for c in cls}
    loop = {"mlp_done", "leg_kin_contacts_done", "integrate_done", "leg_kin_done", "backward_done", "base_solve_done",
            "forward_done", "phys_begin"}
    cur = "prologue"
    for l in s[start:end]:
        m = re.search(r"; MARK (\w+)", l)
        if m:
            cur = m.group(1)
            continue
        t = l.strip()
        w = 4 if cur in loop else 1  # decimation 4 x n_internal 1
        for c, (sc, pk) in cls.items():
            if re.match(pk, t):
                tally[c][1] += w
            elif re.match(sc, t):
                tally[c][0] += w
    out = {c: {"scalar": a, "packed": b, "packed_share": b / max(a + b, 1)} for c, (a, b) in tally.items()}
    import json
    print(json.dumps({"weighted_static_f32_mix": out}))


if __name__ == "__main__":
    main()
