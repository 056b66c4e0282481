"""How often the hip capsules touch in the bench workload (bench.py make_env: README single_path config,
4096 envs, N(0, 1) actions): the fraction of envs with a hip contact force, and of 4-env waves in which
the step kernel's hip-contact branch runs (csrc/go1_device.h hip_contact).  GPU diagnostic:
  python tools/hip_contact_stats.py [steps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda", 0)
    env = bench.make_env(4096, 0, 1, dev)
    env.reset()
    ring = torch.randn((64, 4096, 12), device=dev)
    hip_env, hip_wave, thigh_env, base_env = [], [], [], []
    for k in range(steps):
        env.step(ring[k % 64])
        cf = env.env.contact_forces.reshape(4096, 17, 3)
        hip = cf[:, 1::4].abs().amax(dim=(1, 2)) > 0
        hip_env.append(hip.float().mean().item())
        hip_wave.append(hip.reshape(-1, 4).any(dim=1).float().mean().item())
        thigh_env.append((cf[:, 2::4].abs().amax(dim=(1, 2)) > 0.1).float().mean().item())
        base_env.append((cf[:, 0].abs().amax(dim=1) > 0).float().mean().item())
    tail = slice(steps // 3, None)
    print(json.dumps({"steps": steps, "hip_env_frac": float(np.mean(hip_env[tail])),
                      "hip_wave_frac": float(np.mean(hip_wave[tail])),
                      "thigh_env_frac": float(np.mean(thigh_env[tail])),
                      "base_env_frac": float(np.mean(base_env[tail]))}))


if __name__ == "__main__":
    main()
