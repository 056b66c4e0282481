"""Distribution of the f32 HIP integrator's one-step error against the f64 oracle, per env, and
what the worst envs have in common (contact on/off, joint limits) -- the evidence behind the
max-error bounds of tests/test_gpu_full_size.py and tests/test_gpu_parity.py.

  python tools/integrator_stats.py [n_envs] [terrain]      (GPU box)
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from legged_tracking_amd import config as CF, layout as L, native, terrain as T  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    terrain = sys.argv[2] if len(sys.argv) > 2 else "single_path"
    rows = 32 if n % 1024 == 0 else 4
    cfg = CF.readme_config(n_envs=n, terrain=terrain, rows=rows, cols=rows)
    c = CF.build_abi_config(cfg)
    td = T.build(cfg, n, np.random.RandomState(11))
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    rng = np.random.default_rng(9)
    st = O.NpState(n, cfg=c)
    st["friction"][:, 0] = rng.uniform(0.1, 3.0, n)
    st["payload"][:, 0] = rng.uniform(-1.0, 3.0, n)
    O.reset_envs(c, st, ter, np.ones(n, np.uint8), rng_seed=9, rng_step=0)
    st["episode_length"][:, 0] = rng.integers(0, 499, n)
    g = native.Go1Native(c, "cuda:0")
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    grav, gvec = CF.gravity_state([0.2, -0.1, 0.3])
    report = []
    lim = np.array([c.hard_limits[i] for i in range(24)], np.float64).reshape(12, 2)
    for t in range(6):  # a few steps, each from the same (GPU) state on both sides
        g.state.load(st.arrays)
        act = rng.normal(0, 1, (n, 12)).astype(np.float32)
        g.step(torch.from_numpy(act).cuda(), gvec, grav, scales, rng_seed=3, rng_step=100 + t)
        torch.cuda.synchronize()
        cf_gpu = g.contact_forces.cpu().numpy()
        out = O.step(c, st, ter, act, gvec, grav, scales, rng_seed=3, rng_step=100 + t, debug=False)
        gs = g.state.numpy()
        row = {"step": t}
        worst = {}
        for k in ("dof_pos", "dof_vel", "root"):
            err = np.abs(gs[k] - st[k]) / np.maximum(1.0, np.abs(st[k]))
            e = err.max(axis=1)
            row[k] = {"max": float(e.max()), "p99": float(np.percentile(e, 99)), "p999": float(np.percentile(e, 99.9)),
                      "n_gt_1e-2": int((e > 1e-2).sum()), "n_gt_1e-1": int((e > 1e-1).sum())}
            worst[k] = np.argsort(-e)[:8]
        # what distinguishes the worst envs: contact state disagreement / joint at a limit
        cg = np.linalg.norm(cf_gpu, axis=2) > 0
        co = np.linalg.norm(out["contact_forces"], axis=2) > 0
        flip = (cg != co).any(axis=1)
        at_lim = ((st["dof_pos"] < lim[:, 0] + 0.02) | (st["dof_pos"] > lim[:, 1] - 0.02)).any(axis=1)
        w = worst["dof_vel"]
        row["worst_dof_vel_envs"] = {"contact_flip": int(flip[w].sum()), "at_limit": int(at_lim[w].sum()),
                                     "of": len(w)}
        row["all_envs"] = {"contact_flip": int(flip.sum()), "at_limit": int(at_lim.sum()), "n": n}
        row["reset_agree"] = float((g.reset.cpu().numpy() == out["reset"].astype(bool)).mean())
        report.append(row)
        st = O.NpState(n, gs, c)
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
