"""Run the bench workload step by step until an observation or reward is non-finite,
then save the pre-step state, actions and outputs of the offending envs
(gpurun_out/nan_hunt.npz) so the step can be replayed on the CPU oracle.

  python tools/nan_hunt.py [steps] [envs]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from legged_tracking_amd import config as CF, native, terrain as T
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    dev = torch.device("cuda", 0)
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=32, cols=32)
    c = CF.build_abi_config(cfg, n_envs=n)
    d = CF.derived(cfg)
    td = T.build(cfg, n, np.random.RandomState(11))
    g = native.Go1Native(c, str(dev))
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    rng = np.random.default_rng(100)
    g.state["friction"].copy_(torch.from_numpy(rng.uniform(0.1, 3.0, (n, 1)).astype(np.float32)))
    g.state["restitution"].copy_(torch.from_numpy(rng.uniform(0.0, 0.4, (n, 1)).astype(np.float32)))
    g.state["payload"].copy_(torch.from_numpy(rng.uniform(-1.0, 3.0, (n, 1)).astype(np.float32)))
    g.reset_envs(torch.ones(n, dtype=torch.bool, device=dev), rng_seed=11, rng_step=0)
    g.state["episode_length"].copy_(torch.from_numpy(rng.integers(0, 500, (n, 1)).astype(np.int32)))
    scales = CF.reward_scale_vector(d["reward_scales"])
    grav, gvec = CF.gravity_state(rng.uniform(-1, 1, 3))
    ring = torch.randn((64, n, 12), device=dev)
    stats = []
    for k in range(steps):
        pre = {name: t.clone() for name, t in g.state.t.items()}
        act = ring[k % 64]
        g.step(act, gvec, grav, scales, rng_seed=11, rng_step=1 + k)
        bad = ~(torch.isfinite(g.obs).all(1) & torch.isfinite(g.rew) & torch.isfinite(g.priv).all(1))
        if bad.any():
            ids = torch.nonzero(bad).flatten().cpu().numpy()
            print(f"step {k}: {len(ids)} env(s) with non-finite outputs: {ids[:16]}")
            out = {f"pre_{name}": t[ids].cpu().numpy() for name, t in pre.items()}
            out.update(ids=ids, step=k, actions=act[ids].cpu().numpy(), obs=g.obs[ids].cpu().numpy(),
                       rew=g.rew[ids].cpu().numpy(), reset=g.reset[ids].cpu().numpy(),
                       gvec=np.asarray(gvec), grav=np.asarray(grav))
            for name, t in g.state.t.items():
                out[f"post_{name}"] = t[ids].cpu().numpy()
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            np.savez(os.path.join(ROOT, "gpurun_out", "nan_hunt.npz"), **out)
            bo = g.obs[ids[0]].cpu().numpy()
            print("obs non-finite columns of the first env:", np.nonzero(~np.isfinite(bo))[0][:40])
            print("rew", g.rew[ids].cpu().numpy()[:8], "reset", g.reset[ids].cpu().numpy()[:8])
            for name in ("root", "dof_pos", "dof_vel", "base_rotation"):
                print("pre", name, pre[name][ids[0]].cpu().numpy())
            return 1
        qd_max = g.state["dof_vel"].abs().max().item()
        v_max = g.state["root"][:, 7:13].abs().max().item()
        stats.append((qd_max, v_max))
        if k % 200 == 0:
            a = np.array(stats[-200:])
            print(f"step {k} ok; max |qd| {a[:, 0].max():.1f} rad/s, max |base vel| {a[:, 1].max():.1f}", flush=True)
    print("no non-finite output in", steps, "steps")
    return 0


if __name__ == "__main__":
    sys.exit(main())
