"""Static instruction mix of the step kernel per loop (the sub-step loop body runs decimation times per step).

  python tools/isa_loops.py [extra hipcc flags]   (compiles go1_step.hip into /tmp/go1_isa_loops)"""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = "/tmp/go1_isa_loops"
sys.path.insert(0, REPO)
from legged_tracking_amd.build import STEP_FLAGS  # noqa: E402


def main():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(REPO, "legged_tracking_amd", "csrc", "go1_step.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", *STEP_FLAGS,
                    *sys.argv[1:], "-c", "--save-temps", "-o", os.path.join(OUT, "k.o"), src], cwd=OUT, check=True,
                   stderr=subprocess.DEVNULL)
    s = open(os.path.join(OUT, "go1_step-hip-amdgcn-amd-amdhsa-gfx950.s")).read().splitlines()
    start = next(i for i, l in enumerate(s) if l.startswith("_Z15go1_step_kernelILb0ELi7ELb1EE"))
    end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
    loop = "top"
    per = collections.defaultdict(collections.Counter)
    for l in s[start:end]:
        if re.match(r"^\.?\w+:", l):
            m = re.search(r"Loop: Header=(\w+) Depth=(\d+)", l)
            h = re.search(r"Loop Header: Depth=(\d+)", l)
            if m:
                loop = f"{m.group(1)}@{m.group(2)}"
            elif h:
                loop = f"{l.split(':')[0].lstrip('.L')}@{h.group(1)}"
            else:
                loop = "top"
            continue
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")):
            continue
        per[loop][t[0]] += 1
    for lp, c in per.items():
        v = sum(n for k, n in c.items() if k.startswith("v_"))
        print(f"== {lp}: {v} VALU-class, {sum(c.values())} total")
        for k, n in c.most_common(int(os.environ.get("TOP", "25"))):
            print(f"   {n:5d} {k}")


if __name__ == "__main__":
    main()
