"""The velocity-tracking step's C ABI and host configuration, without a GPU.

* include/go1_velocity.h vs the ctypes mirror (legged_tracking_amd/vel_abi.py): struct sizes reported by the
  compiled library, exported symbols;
* build_configs on scripts/train_velocity_tracking.py's configuration (BASELINE configs[1]) against the
  oracle's Params (oracle/vel_oracle.py, itself pinned by the reference's fixtures);
* the unsupported-configuration guard.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

from legged_tracking_amd import vel_abi as VA, velocity as VEL, velocity_config as V

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_struct_sizes_match_the_library():
    l = VEL.lib()
    out = (C.c_int64 * 3)()
    l.go1_vel_abi_sizes(out)
    assert list(out) == [C.sizeof(VA.Go1VelConfig), C.sizeof(VA.Go1VelState), C.sizeof(VA.Go1VelStepArgs)]
    assert l.go1_vel_abi_version() == VA.GO1_VEL_ABI_VERSION


def test_every_declared_symbol_is_exported():
    hdr = open(os.path.join(REPO, "include", "go1_velocity.h")).read()
    names = re.findall(r"^\s*(?:int|void|const char\*)\s+(go1_vel_\w+)\(", hdr, re.M)
    assert len(names) >= 8
    l = VEL.lib()
    for n in names:
        assert hasattr(l, n), n


def test_header_constants_match_the_mirror():
    hdr = open(os.path.join(REPO, "include", "go1_velocity.h")).read()
    consts = dict(re.findall(r"#define (GO1_VEL_\w+) (\d+)", hdr))
    for k in ("NUM_COMMANDS", "NUM_OBS", "MAX_TERMS", "SUM_EXTRA", "N_CATEGORIES", "N_KEYS", "MAX_BINS", "AUX"):
        assert int(consts["GO1_VEL_" + k]) == getattr(VA, "GO1_VEL_" + k), k
    enum = re.search(r"enum go1_vel_term \{(.*?)\};", hdr, re.S).group(1)
    ids = re.findall(r"GO1_VT_(\w+)", enum)
    assert [i.lower() for i in ids[:-1]] == list(VA.VTERM_IDS)


def test_configs_follow_the_reference_derivation():
    from oracle import vel_oracle as VO  # checker only
    cfg = V.train_velocity_config(n_envs=64)
    c, v, grid, w0, names, sum_keys = VEL.build_configs(cfg)
    P = VO.Params(cfg)
    assert names == P.names and sum_keys == P.sum_keys
    np.testing.assert_array_equal(grid, P.grid)
    np.testing.assert_array_equal(w0, P.w0)
    np.testing.assert_array_equal(np.array(v.noise_vec, np.float32), P.noise_vec)
    np.testing.assert_array_equal(np.array(v.cmd_scale, np.float32), P.cmd_scale)
    assert v.resample_interval == P.resample_interval == 500 and v.rand_interval == P.rand_interval == 200
    assert v.n_bins == 441 and v.n_task == 4 and v.history_len == 30 and v.reward_mode == 2
    assert np.float32(v.curriculum_ep_len) == np.float32(P.cur_ep_len)
    for k, key in enumerate(V.TASK_KEYS):
        assert sum_keys[v.task_slot[k]] == key
        assert np.float32(v.task_threshold[k]) == np.float32(P.thresholds[key] * P.scales[key])
    # the slots whose scaled rewards are <= 0 (pos / neg bucketing, :293-296)
    neg = {n for k, n in enumerate(names) if (v.nonpos_slots >> k) & 1}
    assert neg == {n for n in names if P.scales[n] * VA.VTERM_SIGN[n] < 0}
    assert "tracking_lin_vel" not in neg and "jump" in neg and "tracking_contacts_shaped_force" in neg and "torques" in neg
    np.testing.assert_array_equal(np.array(v.dof_pos_limits, np.float32).reshape(12, 2), P.soft)
    np.testing.assert_array_equal(np.array(v.default_dof_pos, np.float32), P.default)


def test_env_origins_follow_get_env_origins():
    d = np.load(os.path.join(REPO, "tests", "golden", "vel_plane.npz"))
    cfg = V.train_velocity_config(n_envs=d["static/env_origins"].shape[0])
    np.testing.assert_array_equal(VEL.plane_env_origins(len(d["static/env_origins"]), cfg), d["static/env_origins"])
    # a rank's slice of the global grid
    o = VEL.plane_env_origins(16, cfg, n_global=64, first=32)
    np.testing.assert_array_equal(o, d["static/env_origins"][32:48])


@pytest.mark.parametrize("edit,msg", [
    (lambda c: setattr(c.terrain, "mesh_type", "trimesh"), "mesh_type"),
    (lambda c: setattr(c.env, "observe_yaw", True), "observe_yaw"),
    (lambda c: setattr(c.domain_rand, "push_robots", True), "push_robots"),
    (lambda c: setattr(c.reward_scales, "feet_air_time", 1.0), "feet_air_time"),
    (lambda c: setattr(c.commands, "num_commands", 3), "num_commands"),
])
def test_unsupported_values_raise(edit, msg):
    cfg = V.train_velocity_config(n_envs=64)
    edit(cfg)
    with pytest.raises(NotImplementedError, match=msg):
        VEL.build_configs(cfg)
