"""Host-side time of each rollout-loop iteration (bench.py rollout_rate's loop, no per-step sync):
iterations that block the host (a hidden synchronisation, a large host copy) show up as outliers.

  gpurun: python tools/rollout_jitter.py [n_envs] [steps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from legged_tracking_amd import rollout as R
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    dev = torch.device("cuda", 0)
    from legged_tracking_amd import env as E
    prof = {}

    def timed(cls, name):
        f = getattr(cls, name)

        def w(self, *a, **k):
            t = time.perf_counter()
            r = f(self, *a, **k)
            prof.setdefault(name, []).append((time.perf_counter() - t) * 1e6)
            return r
        setattr(cls, name, w)
    for nm in ("advance", "_drain_inflight", "_half_rows", "_defer", "_process_rows", "next_slot"):
        timed(E.EpisodeLogRing, nm)
    env = bench.make_env(n, 0, 1, dev)
    ac = R.ActorCritic(env.num_obs, env.num_privileged_obs, env.num_obs_history, env.num_actions).to(dev)
    alg = R.PPO(ac, device=dev)
    T = 24
    alg.init_storage(n, T, [env.num_obs], [env.num_privileged_obs], [env.num_obs_history], [env.num_actions])
    env.reset()
    od = env.get_observations()
    obs, priv, hist = od["obs"], od["privileged_obs"], od["obs_history"]
    host = np.zeros((steps, 4))
    with torch.inference_mode():
        for t in range(steps):
            t0 = time.perf_counter()
            if alg.storage.step == T:
                alg.storage.clear()
            a = alg.act(obs, priv, hist)
            t1 = time.perf_counter()
            od, rew, done, info = env.step(a)
            t2 = time.perf_counter()
            obs, priv, hist = od["obs"], od["privileged_obs"], od["obs_history"]
            alg.process_env_step(rew, done, info)
            t3 = time.perf_counter()
            host[t] = (t1 - t0, t2 - t1, t3 - t2, t3 - t0)
        torch.cuda.synchronize()
    us = host[24:] * 1e6
    print("host us per iteration (act, env.step, record, total): median", np.median(us, 0).round(1),
          "p99", np.percentile(us, 99, 0).round(1), "max", us.max(0).round(1))
    for k, v in prof.items():
        v = np.array(v)
        print(f"  {k:16s} calls {v.size:5d}  max {v.max():9.1f} us  sum {v.sum():9.1f} us  >500us: {np.round(v[v > 500]).tolist()[:8]}")
    big = np.nonzero(us[:, 3] > 500)[0]
    print("iterations > 500 us:", [(int(i) + 24, us[i].round(0).tolist()) for i in big[:20]])


if __name__ == "__main__":
    main()
