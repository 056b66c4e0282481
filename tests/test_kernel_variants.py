"""Every diagnostic build of the step kernels still compiles (no GPU needed).

go1_step.hip (with the device code it shares with the velocity step, go1_device.h) keeps two kinds of compile-time switches, both measurement instrumentation, never
shipped: the ablation builds of tools/abl_kernel.sh (GO1_ABL_*: a section of the kernel compiled
out, to price it in situ) and the timing / accounting builds (GO1_STAMPS: s_memtime stamps for
tools/stamps.py; GO1_ISA_MARKS: section markers for tools/isa_sections.py).  Variants that were
measured and rejected are deleted from the source, not kept behind switches.  A front-end pass
(hipcc -fsyntax-only, host and gfx950 device) per variant keeps them from rotting.  go1_velocity.hip
has the curriculum launch's stamps (GO1_VEL_STAMPS, tools/vel_stamps.py)."""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "legged_tracking_amd", "csrc")
SRC = os.path.join(CSRC, "go1_step.hip")
SCANNED = [SRC, os.path.join(CSRC, "go1_device.h")]
VEL_SRC = os.path.join(CSRC, "go1_velocity.hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _switches():
    src = "".join(open(f).read() for f in SCANNED)
    return sorted(set(re.findall(r"#\s*if(?:n?def)?\s+(?:defined\()?(GO1_(?:ABL_\w+|STAMPS|ISA_MARKS))", src)))


def test_only_diagnostic_switches_remain():
    src = "".join(open(f).read() for f in SCANNED + [VEL_SRC])
    conds = set(re.findall(r"#\s*(?:if|ifdef|ifndef|elif)\s+(?:defined\()?(\w+)", src))
    allowed = {"GO1_STAMPS", "GO1_ISA_MARKS", "GO1_VEL_STAMPS", "GO1_DEVICE_H"}
    stray = {c for c in conds if c.startswith("GO1_") and c not in allowed and not c.startswith("GO1_ABL_")}
    assert not stray, f"variant switches outside the diagnostic set: {sorted(stray)}"


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
def test_diagnostic_builds_compile():
    variants = [([], SRC)] + [([f"-D{s}"], SRC) for s in _switches()] + [(["-DGO1_VEL_STAMPS"], VEL_SRC)]
    assert len(variants) >= 10  # 8 ablations + stamps / ISA marks + the velocity stamps

    def one(v):
        flags, src = v
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-ffp-contract=off",
                            *flags, src], capture_output=True, text=True, cwd="/tmp")
        errs = [l for l in r.stderr.splitlines() if "error" in l]
        return flags, r.returncode, errs[:5]

    with ThreadPoolExecutor(4) as ex:
        for flags, rc, errs in ex.map(one, variants):
            assert rc == 0, (flags, errs)
