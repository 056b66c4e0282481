"""Helpers to replay the golden fixtures (tests/golden/*.npz) through the oracle or the HIP path."""
import os

import numpy as np

from legged_tracking_amd import config as CF
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STATE_KEYS = ("root", "dof_pos", "dof_vel", "last_actions", "last_dof_vel", "lag", "pos_err_hist", "vel_hist",
              "motor_strength", "motor_offset", "friction", "restitution", "payload", "episode_length",
              "curr_pose_index", "trajectory", "base_rotation", "collision_count", "episode_sums", "joint_pos_target")


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def fixture_config(d):
    terrain = str(d["meta/terrain"])
    n = d["s0/obs"].shape[0]
    cfg = CF.readme_config(n_envs=n, terrain=terrain, rows=4, cols=4)
    return cfg, CF.build_abi_config(cfg, n_envs=n)


def state_at(d, t, which="pre"):
    n = d["s0/obs"].shape[0]
    init = {k: d[f"s{t}/{which}/{k}"] for k in STATE_KEYS}
    return O.NpState(n, init)


def terrain_of(d):
    n = d["s0/obs"].shape[0]
    hs = d["static/env_height_samples"]
    if hs.shape[2] == 1:
        hs = np.zeros((n, 2, 80, 40), np.float32)
    return O.NpTerrain(hs, np.arange(n, dtype=np.int32), d["static/env_terrain_origin"], d["static/env_origins"])


def step_inputs(d, t):
    n = d["s0/obs"].shape[0]
    inj = dict(dof=d[f"s{t}/inj_dof"], root=d[f"s{t}/inj_root"], contact=d[f"s{t}/inj_contact"])
    scales = d[f"s{t}/reward_scales"].astype(np.float32)
    return dict(actions=d[f"s{t}/actions"], gravity_vec=d[f"s{t}/gravity_vec"], sim_gravity=d[f"s{t}/sim_gravity"],
                reward_scales=scales, uniforms=d[f"s{t}/uniforms"], inj=inj)
