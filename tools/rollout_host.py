"""Is the rollout loop host-bound?  Host enqueue time per step (the loop before its final
sync) vs the synchronized wall time per step, at 4096 envs (GPU box)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main(n=4096, steps=200, warmup=24):
    from legged_tracking_amd import config as CF, env as E, rollout as R
    dev = torch.device("cuda", 0)
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=32, cols=32)
    env = E.HistoryWrapper(E.TrajectoryTrackingEnv(sim_device=str(dev), cfg=cfg, seed=11, rank=0, world_size=1))
    ac = R.ActorCritic(env.num_obs, env.num_privileged_obs, env.num_obs_history, env.num_actions).to(dev)
    alg = R.PPO(ac, device=dev)
    T = 24
    alg.init_storage(n, T, [env.num_obs], [env.num_privileged_obs], [env.num_obs_history], [env.num_actions])
    env.reset()
    od = env.get_observations()
    st = {"obs": od["obs"], "priv": od["privileged_obs"], "hist": od["obs_history"]}
    parts = {"act": 0.0, "env": 0.0, "record": 0.0}

    def one(timed):
        if alg.storage.step == T:
            alg.storage.clear()
        t0 = time.perf_counter()
        a = alg.act(st["obs"], st["priv"], st["hist"])
        t1 = time.perf_counter()
        o, rew, done, info = env.step(a)
        t2 = time.perf_counter()
        st["obs"], st["priv"], st["hist"] = o["obs"], o["privileged_obs"], o["obs_history"]
        alg.process_env_step(rew, done, info)
        t3 = time.perf_counter()
        if timed:
            parts["act"] += t1 - t0
            parts["env"] += t2 - t1
            parts["record"] += t3 - t2

    with torch.inference_mode():
        for _ in range(warmup):
            one(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            one(True)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_wall = time.perf_counter() - t0
    us = lambda x: x / steps * 1e6  # noqa: E731
    print(f"n={n}: wall {us(t_wall):.1f} us/step, host enqueue {us(t_host):.1f} us/step "
          f"(act {us(parts['act']):.1f}, env.step {us(parts['env']):.1f}, record {us(parts['record']):.1f})")


if __name__ == "__main__":
    main()
