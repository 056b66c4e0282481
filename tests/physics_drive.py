"""Drive the native integrator through the step API (HIP or the f64 oracle) for the physical-
invariant tests (tests/test_physics_invariants.py).  Test infrastructure.

The step is the full fused env step; the scenarios keep everything but the physics inert:
motor strength 0 (zero joint torque), episode lengths far from the DR interval and the
time-out, the base far above the plane (no contact) unless the scenario is a stance."""
import numpy as np

from legged_tracking_amd import config as CF, layout as L, terrain as T
from oracle import oracle as O
from tests import physics_ref as P

N = 64
STEP_DT = 0.02  # decimation 4 x sim dt 0.005


def setup(n=N, seed=0, height=5.0, qd_sigma=0.2, v_sigma=0.5, w_sigma=1.0, strength=0.0, stance=False):
    cfg = CF.readme_config(n_envs=n, terrain="plane", rows=2, cols=2)
    cfg.domain_rand.randomize_motor_strength = False
    c = CF.build_abi_config(cfg)
    td = T.build(cfg, n, np.random.RandomState(11))
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    st = O.NpState(n, cfg=c)
    rng = np.random.default_rng(seed)
    st["friction"][:, 0] = 1.0
    O.reset_envs(c, st, ter, np.ones(n, np.uint8), rng_seed=seed, rng_step=0)
    dflt = np.array(L.DEFAULT_DOF_POS, np.float32)
    if stance:
        st["root"][:, 2] = 0.34
        st["root"][:, 3:7] = [0, 0, 0, 1]
        st["root"][:, 7:13] = 0.0
        st["dof_pos"][:] = dflt
        st["dof_vel"][:] = 0.0
    else:
        st["root"][:, 2] = height
        q = rng.normal(size=(n, 4))
        st["root"][:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
        st["root"][:, 7:10] = rng.normal(0, v_sigma, (n, 3))
        st["root"][:, 10:13] = rng.normal(0, w_sigma, (n, 3))
        st["dof_pos"][:] = dflt * rng.uniform(0.85, 1.15, (n, 12))
        st["dof_vel"][:] = rng.normal(0, qd_sigma, (n, 12))
    st["motor_strength"][:] = strength
    st["motor_offset"][:] = 0.0
    st["payload"][:] = 0.0
    st["episode_length"][:, 0] = 1  # no DR (every 300 steps) or time-out (500) within the runs
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    return c, td, ter, st, scales


def invariants(st, e, g):
    r = st["root"][e].astype(np.float64)
    return P.invariants(r[0:3], r[3:7], r[7:10], r[10:13], st["dof_pos"][e].astype(np.float64),
                        st["dof_vel"][e].astype(np.float64), g=g)


def all_invariants(st, g):
    return [invariants(st, e, g) for e in range(st.n)]


def oracle_roll(c, ter, st, scales, n_steps, gravity, actions=None):
    """n_steps oracle env steps; yields (state copy, contact forces) after each."""
    grav = np.asarray(gravity, np.float32)
    gvec = np.array([0, 0, -1], np.float32)
    for t in range(n_steps):
        a = np.zeros((st.n, 12), np.float32) if actions is None else actions
        out = O.step(c, st, ter, a, gvec, grav, scales, rng_seed=1, rng_step=t, debug=False)
        yield st, out["contact_forces"], out["reset"].astype(bool)


def hip_roll(c, td, st, scales, n_steps, gravity, actions=None):
    import torch
    from legged_tracking_amd import native
    g = native.Go1Native(c, "cuda:0")
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    g.state.load(st.arrays)
    grav = np.asarray(gravity, np.float32)
    gvec = np.array([0, 0, -1], np.float32)
    a = torch.zeros((st.n, 12), device="cuda:0") if actions is None else torch.as_tensor(actions, device="cuda:0")
    for t in range(n_steps):
        g.step(a, gvec, grav, scales, rng_seed=1, rng_step=t)
        torch.cuda.synchronize()
        s = O.NpState(st.n, g.state.numpy(), c)
        yield s, g.contact_forces.cpu().numpy(), g.reset.cpu().numpy().astype(bool)
    g.close()
