"""Dump the bench workload's state after its warm-up (gpurun): the step kernel's inputs at steady state, for CPU
studies of the narrow phase's candidate pairs (tools/narrow_stats.py).
  python tools/dump_states.py [steps]         -> gpurun_out/bench_states.npz (the VecEnv loop after its warm-up)
  python tools/dump_states.py kernel [steps]  -> gpurun_out/kernel_states.npz (bench.py --kernel-only's loop)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    kernel = len(sys.argv) > 1 and sys.argv[1] == "kernel"
    args = sys.argv[2:] if kernel else sys.argv[1:]
    steps = int(args[0]) if args else 3000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = bench.make_env(4096, 0, 1, dev)
    env.reset()
    ring = torch.randn((64, 4096, 12), device=dev, generator=torch.Generator(device=dev).manual_seed(100))
    out = {}
    if kernel:  # bench.kernel_loop's workload: the fused kernel alone from the reset
        for half in (steps // 2, steps - steps // 2):
            bench.kernel_loop(env, ring, half, 0, every=1)
            torch.cuda.synchronize()
            st = env.env._sim.state
            k = steps // 2 if half == steps // 2 and "root_%d" % (steps // 2) not in out else steps
            out[f"root_{k}"] = st["root"].cpu().numpy()
            out[f"dof_pos_{k}"] = st["dof_pos"].cpu().numpy()
            print("dumped", k, flush=True)
        np.savez(os.path.join(ROOT, "gpurun_out", "kernel_states.npz"), **out)
        return
    for k in range(steps):
        env.step(ring[k % 64])
        if k + 1 in (steps // 2, steps):
            torch.cuda.synchronize()
            st = env.env._sim.state
            out[f"root_{k + 1}"] = st["root"].cpu().numpy()
            out[f"dof_pos_{k + 1}"] = st["dof_pos"].cpu().numpy()
            print("dumped", k + 1, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "bench_states.npz"), **out)


if __name__ == "__main__":
    main()
