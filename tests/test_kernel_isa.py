"""Machine-code guards on the built step libraries (no GPU needed: the gfx950 code object inside the in-tree .so).

The step kernels run one wave per SIMD, so every exposed latency is launch time.  Two regressions this guards,
both found by reading the ISA: LDS values re-read through an opaque *pointer* compile to flat loads
(an address-space-agnostic access with a longer latency than ds_read; 68 per step before round 6's fix), and a
register-pressure spill puts scratch traffic into the sub-step loop.  Checked on the specialised README-config
step kernel (go1_step_kernel<false, 7, true>) and the velocity step kernel."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "legged_tracking_amd", "_build")
LLVM = "/opt/rocm/lib/llvm/bin"
KERNELS = {"libgo1_mi355x.so": "_Z15go1_step_kernelILb0ELi7ELb1EEvPK10go1_config",
           "libgo1_velocity.so": "_Z19go1_vel_step_kernelILb0E"}


def _disasm(lib):
    with tempfile.TemporaryDirectory() as t:
        fb, dev = os.path.join(t, "fb.bin"), os.path.join(t, "dev.o")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fb, lib], check=True,
                       capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fb,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + dev], check=True,
                       capture_output=True)
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", dev], check=True, capture_output=True,
                              text=True).stdout


def _kernel_body(text, name):
    """instruction mnemonics of the first function whose symbol starts with `name`"""
    out, on = [], False
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            if on:
                break
            on = m.group(1).startswith(name)
            continue
        if on:
            parts = line.strip().split()
            if parts and re.match(r"^[a-z_]", parts[0]):
                out.append(parts[0])
    return out


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")), reason="ROCm LLVM tools not available")
@pytest.mark.parametrize("lib", sorted(KERNELS))
def test_step_kernel_has_no_flat_or_scratch_access(lib):
    path = os.path.join(BUILD, lib)
    if not os.path.exists(path):
        pytest.skip(f"{lib} not built (python -c 'import __graft_entry__ as g; g.build()')")
    ins = _kernel_body(_disasm(path), KERNELS[lib])
    assert len(ins) > 1000, f"kernel {KERNELS[lib]} not found in {lib}"
    flat = [i for i in ins if i.startswith("flat_")]
    scratch = [i for i in ins if i.startswith("scratch_")]
    assert not flat, f"{len(flat)} flat memory instructions (an LDS or global access lost its address space)"
    assert not scratch, f"{len(scratch)} scratch instructions (register spills)"
    assert sum(i.startswith("v_mfma") for i in ins) >= 60  # the actuator net on the matrix cores
