"""Time the fused policy kernel alone (PPO.act path, 4096 envs): mean over 200 launches.
  python tools/policy_bench.py [lib-suffix ...]   (libgo1_rollout_<suffix>.so, or "current")"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, time
sys.path.insert(0, %r)
import torch
from legged_tracking_amd import rollout as R
n = 4096
dev = torch.device("cuda", 0)
ac = R.ActorCritic(261, 2, 261, 12).to(dev)
alg = R.PPO(ac, device=dev)
alg.init_storage(n, 24, [261], [2], [261], [12])
obs = torch.randn(n, 261, device=dev); priv = torch.randn(n, 2, device=dev)
with torch.inference_mode():
    for _ in range(20):
        alg.fused.forward(obs, priv, sample=(1, 1, 0))
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for k in range(200):
        alg.fused.forward(obs, priv, sample=(1, k, 0))
    e.record(); torch.cuda.synchronize()
print("%%.2f" %% (s.elapsed_time(e) / 200 * 1000))
''' % ROOT


def main():
    for v in sys.argv[1:] or ["current"]:
        env = dict(os.environ)
        if v != "current":
            env["GO1_ROLLOUT_LIB_OVERRIDE"] = os.path.join(ROOT, "legged_tracking_amd", "_build", f"libgo1_rollout_{v}.so")
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        print(v, "policy forward us:", r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-500:])


if __name__ == "__main__":
    main()
