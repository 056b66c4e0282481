"""Section timing of the velocity curriculum launch's block 0 (diagnostic build with -DGO1_VEL_STAMPS).

  local:  hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-slp-vectorize \\
              -mllvm -amdgpu-kernarg-preload-count=16 -DGO1_VEL_STAMPS -o legged_tracking_amd/_build/libgo1_velocity_stamps.so \\
              legged_tracking_amd/csrc/go1_velocity.hip
  gpurun: python tools/vel_stamps.py

Runs the bench's velocity loop (4096 envs, N(0,1) actions) and prints, per resample phase (B: the envs the
step reset, A: the next step's interval envs), the mean s_memtime cycles of each section over the phases
that had selected envs (scan over all phases)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GO1_VEL_LIB_OVERRIDE"] = os.environ.get("VEL_STAMPS_LIB") or os.path.join(ROOT, "legged_tracking_amd", "_build", "libgo1_velocity_stamps.so")
NAMES = {0: "scan (all phases)", 15: "count>0 entry", 1: "success hist", 2: "weights update", 3: "cdf",
         4: "sampling (clear + barrier)", 5: "sampling: records, loads, draws", 6: "sampling: cdf search + shfl",
         7: "sampling: centre, commands, stores", 14: "cdf recomputes (count)", 10: "prologue (phase B row: every launch)",
         11: "commit (phase B row, launches that commit)"}


def main():
    import torch
    from legged_tracking_amd import env as E, velocity as VEL
    n, steps = 4096, 300
    dev = torch.device("cuda", 0)
    env = E.HistoryWrapper(VEL.VelocityTrackingEasyEnv(sim_device=str(dev), num_envs=n, seed=11))
    env.reset()
    ring = torch.randn((64, n, 12), device=dev, generator=torch.Generator(device=dev).manual_seed(7))
    for k in range(30):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    lib = VEL.lib()
    lib.go1_vel_stamps.argtypes = [C.c_void_p, C.c_int]
    assert lib.go1_vel_stamps(None, 1) == 0
    calls = 0
    for k in range(steps):
        env.step(ring[k % 64])
        calls += 1
    torch.cuda.synchronize()
    buf = np.zeros((2, 16), np.uint64)
    assert lib.go1_vel_stamps(buf.ctypes.data, 0) == 0
    for ph, name in ((0, "B (reset envs)"), (1, "A (next interval envs)")):
        ran = max(int(buf[ph, 15] > 0), 1)
        print(f"phase {name}: {calls} launches")
        for k in (10, 11, 0, 15, 1, 2, 3, 5, 6, 7, 4, 14):
            print(f"  {NAMES[k]:<26} {int(buf[ph, k]):>14}  per launch {buf[ph, k] / calls:10.0f}")
    env.env.close()


if __name__ == "__main__":
    main()
