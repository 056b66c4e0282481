"""A/B cost of self-collision on the velocity step kernel (bench.velocity_rate's workload: 4096 envs, plane,
scripts/train_velocity_tracking.py config, N(0, 1) actions): python tools/physics_ab_vel.py [steps]

Arms: asset.self_collisions = 0 (the reference scene) / 1, alternated twice; kernel time per step from HIP events
on the step kernel's dispatch (every 4th step)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from legged_tracking_amd import env as E, velocity as VEL, velocity_config as V  # noqa: E402


def run(self_on, steps, warmup=30, n=4096):
    cfg = V.train_velocity_config(n_envs=n)
    cfg.asset.self_collisions = 0 if self_on else 1
    dev = torch.device("cuda", 0)
    env = E.HistoryWrapper(VEL.VelocityTrackingEasyEnv(sim_device=str(dev), num_envs=n, seed=11, cfg=cfg))
    env.reset()
    env.get_observations()
    ring = torch.randn((64, n, 12), device=dev, generator=torch.Generator(device=dev).manual_seed(7))
    for k in range(warmup):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    every = 4
    ev = bench.EventPairs((steps + every - 1) // every)
    env.env.kernel_events.extend(ev.pair(k // every) if k % every == 0 else None for k in range(steps))
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    env.env.kernel_events.clear()
    kms = float(np.mean([ev.ms(i) for i in range((steps + every - 1) // every)]))
    ev.close()
    env.env.close()
    return kms * 1e3, dt / steps * 1e6


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    res = {"self on": [], "self off": []}
    for rep in range(2):
        for name, on in (("self on", True), ("self off", False)):
            res[name].append(run(on, steps))
    for name, v in res.items():
        print(f"{name:9s} kernel {np.mean([a for a, _ in v]):7.2f} us, step {np.mean([b for _, b in v]):7.2f} us  "
              f"({', '.join(f'{a:.2f}' for a, _ in v)})", flush=True)


if __name__ == "__main__":
    main()
