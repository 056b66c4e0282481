"""The contact choices the step kernel holds for a control step, against choosing them every sim step (VERDICT r05
#4: "move the trunk-face vertex selection to every sim step, or add a test bounding the error of holding it").

The kernel (go1_device.h phys_substep) makes two discrete choices once per control step, on its first sim step, and
holds them for the other decimation - 1 = 3: the deepest point t of every capsule segment against the floor /
ceiling meshes (seg_deepest; the point then moves with its link, and its triangle is re-located under it) and the
trunk faces' two deepest terrain vertices (face_scan; the penalty force acts at them every sim step, face_force).
The f64 oracle does the same, and oracle.set_rescan_every_step makes either choice every sim step instead.

Workload: the bench's (README config, single_path tunnels): 256 envs reset and stepped by the oracle under N(0, 1)
actions, the states after 20, 40 and 60 steps (768, nearly all in terrain contact) with the torques of the next sim
step held, one control step (4 x 5 ms) each way.  Measured (f64): the capsules' held points change nothing in 760 of
the 768 envs and 2.8e-6 m / 4e-4 m/s at the 99th percentile; the faces' held vertices change nothing in 765 (only 5
envs have the trunk on the terrain).  The few large differences are trunks against a tunnel wall, where a wall
vertex entering the bottom face's footprint is pushed up along the face normal (capped at the box height: the
faces' known limitation) -- rescanned every step it is picked up a sim step earlier.  The
bounds below hold the 99th percentile and the share of identical envs (about 5x the measured values)."""
import numpy as np

from legged_tracking_amd import config as CF, layout as L, terrain as T
from oracle import oracle as O

N_ENVS = 256


def _states(seed=21):
    """States of the bench's workload: the README config on single_path tiles, 256 envs reset and stepped by the
    oracle under N(0, 1) actions; the states after 20, 40 and 60 steps with the torques of the next sim step"""
    cfg = CF.readme_config(n_envs=N_ENVS, terrain="single_path", rows=4, cols=4)
    td = T.build(cfg, N_ENVS, np.random.RandomState(11))
    held = CF.build_abi_config(cfg)
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    st = O.NpState(N_ENVS, cfg=held)
    rng = np.random.default_rng(seed)
    st["friction"][:, 0] = rng.uniform(0.1, 3.0, N_ENVS)
    O.reset_envs(held, st, ter, np.ones(N_ENVS, np.uint8), rng_seed=1, rng_step=0)
    st["episode_length"][:, 0] = rng.integers(0, 400, N_ENVS)
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    grav, gvec = CF.gravity_state([0.0, 0.0, 0.0])
    pool = []
    for k in range(61):
        before = st.copy()
        act = rng.normal(0, 1, (N_ENVS, 12)).astype(np.float32)
        out = O.step(held, st, ter, act, gvec, grav, scales, rng_seed=2, rng_step=k, debug=True)
        if k in (20, 40, 60):
            for e in range(N_ENVS):
                r = before["root"][e].astype(np.float64)
                body = dict(pos=r[0:3], quat=r[3:7], v=r[7:10], w=r[10:13],
                            q=before["dof_pos"][e].astype(np.float64), qd=before["dof_vel"][e].astype(np.float64))
                pool.append((td.tiles[td.env_tile[e]], td.env_terrain_origin[e], body,
                             out["torques"][0, e].astype(np.float64), float(before["friction"][e, 0])))
    return held, pool


def _run(pool, cfg, faces, segments):
    O.set_rescan_every_step(faces=faces, segments=segments)
    g = np.array([0.0, 0.0, -9.81])
    out, touched = [], 0
    try:
        for tile, origin, body, tau, mu in pool:
            b = {k: np.array(v, np.float64).copy() for k, v in body.items()}
            cf = O.physics(cfg, b, tau, 4, 0.005, g, mu, 0.0, 0.0, tile=tile, origin=origin)
            out.append(b)
            touched += np.abs(cf).max() > 0
    finally:
        O.set_rescan_every_step()
    return out, touched


def test_held_contact_choices_bounded_against_every_sim_step():
    cfg, pool = _states()
    n = len(pool)
    base, touched = _run(pool, cfg, False, False)
    assert touched >= 0.9 * n
    # p99 bounds per state component, and the least share of envs that must end bit-identical
    bounds = {"pos": 2e-4, "quat": 1e-3, "v": 0.02, "w": 0.2, "q": 0.01, "qd": 2.0}
    for faces, segments, min_same in ((True, False, 0.97), (False, True, 0.97), (True, True, 0.95)):
        res, _ = _run(pool, cfg, faces, segments)
        d = {k: np.array([np.abs(a[k] - b[k]).max() for a, b in zip(base, res)]) for k in bounds}
        same = int(np.sum(np.all([d[k] == 0 for k in d], axis=0)))
        p99 = {k: float(np.percentile(v, 99)) for k, v in d.items()}
        print(f"\nevery step: faces {faces}, capsules {segments}: {same} of {n} bit-identical; p99 "
              + ", ".join(f"{k} {v:.1e}" for k, v in p99.items()) + "; max "
              + ", ".join(f"{k} {v.max():.1e}" for k, v in d.items()))
        assert same >= min_same * n, same
        for k, b in bounds.items():
            assert p99[k] <= b, (faces, segments, k, p99[k])
