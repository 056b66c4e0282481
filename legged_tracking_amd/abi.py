"""ctypes mirror of include/go1_mi355x.h (the C ABI).  Pure host code.

The struct layouts here must match the header field for field; tests/test_abi.py
checks sizes and offsets against the compiled library's expectations.
"""
import ctypes as C

GO1_ABI_VERSION = 6
GO1_NUM_DOF = 12
GO1_NUM_BODIES = 17
GO1_MAX_TERMS = 16
GO1_MAX_SUMS = GO1_MAX_TERMS + 3
GO1_NUM_PRIV = 2
GO1_LAG_SLOTS = 7


def lag_steps(decimation):
    """GO1_LAG_STEPS: env steps the stored lag keeps (go1_state.lag = 12 x this many floats)."""
    return (GO1_LAG_SLOTS + int(decimation) - 1) // int(decimation)
GO1_MAX_TRAJ = 16
GO1_U_NOISE = 47
GO1_MODEL_FLOATS = 178
GO1_ACTUATOR_FLOATS = 1313
GO1_GRID_X = 21
GO1_GRID_Y = 11
GO1_AUX = 32

# enum go1_term (include/go1_mi355x.h)
TERM_IDS = {name: i for i, name in enumerate((
    "torques", "dof_acc", "collision", "action_rate", "dof_pos_limits", "orientation", "ang_vel_xy",
    "reaching_z", "reaching_roll", "reaching_pitch", "exploration_lin", "exploration_yaw", "base_height",
    "large_vel", "e2e", "dof_vel", "dof_pos", "task_old", "reach_goal", "reach_goal_t", "reach_goal_T", "task",
    "exploration", "stalling", "linear_vel", "lin_vel_z", "feet_air_time", "survive", "reaching_yaw_abs"))}
GO1_T_COUNT = len(TERM_IDS)
GO1_T_NONE = 31


def episode_log_width(n_terms):
    """go1_step_args.episode_log row: n_terms + 3 sums, episode length, reached, goal distance."""
    return n_terms + 6


F = C.c_float
I32 = C.c_int32
P = C.c_void_p


class Go1Config(C.Structure):
    _fields_ = [
        ("n_envs", I32), ("terrain_kind", I32), ("camera_zero", I32), ("measure_front_half", I32),
        ("add_noise", I32), ("use_terminal_body_height", I32), ("custom_origins", I32), ("decimation", I32),
        ("n_internal", I32), ("rand_interval", I32), ("hf_nx", I32), ("hf_ny", I32), ("env_id_offset", I32),
        ("n_terms", I32), ("term_ids", I32 * GO1_MAX_TERMS), ("term_mask", C.c_uint32), ("reward_mode", I32),
        ("lin_vel_form", I32), ("terminate_end_of_trajectory", I32), ("use_terminal_body_rotation", I32),
        ("rotate_camera", I32), ("observe_heights", I32), ("timestep_in_obs", I32), ("num_obs", I32),
        ("u_per_env", I32), ("traj_kind", I32), ("traj_length", I32), ("traj_interp", I32),
        ("indefinite_slots", C.c_uint32), ("live_slots", C.c_uint32),
        ("sigma_rew_neg", F), ("small_vel_threshold", F), ("large_dist_threshold", F),
        ("traj_x_range", F), ("traj_y_range", F), ("traj_z_range", F), ("traj_roll_range", F),
        ("traj_pitch_range", F), ("traj_yaw_range", F), ("traj_x_mean", F), ("traj_y_mean", F),
        ("sim_dt", F), ("dt", F), ("action_scale", F), ("hip_scale_reduction", F), ("clip_actions", F),
        ("clip_obs", F), ("horizontal_scale", F), ("max_episode_length", F), ("terminal_body_height", F),
        ("switch_dist", F), ("base_height_target", F), ("tracking_sigma_lin", F), ("tracking_sigma_ang", F),
        ("target_lin_vel", F), ("target_ang_vel", F), ("lin_reaching_criterion", F),
        ("ang_reaching_criterion", F), ("t_reach", F), ("ceiling_height", F),
        ("obs_scale_dof_pos", F), ("obs_scale_dof_vel", F), ("obs_scale_heights", F),
        ("noise_gravity", F), ("noise_dof_pos", F), ("noise_dof_vel", F),
        ("camera_offset_x", F), ("camera_offset_norm", F),
        ("priv_friction_shift", F), ("priv_friction_scale", F), ("priv_rest_shift", F), ("priv_rest_scale", F),
        ("strength_range", F), ("strength_lo", F), ("offset_range", F), ("offset_lo", F),
        ("reset_dof_range", F), ("reset_dof_lo", F), ("reset_vel_range", F), ("reset_vel_lo", F),
        ("x_init_range2", F), ("x_init_lo", F), ("y_init_range2", F), ("y_init_lo", F), ("yaw_range2", F),
        ("yaw_lo", F), ("x_init_offset", F), ("y_init_offset", F),
        ("base_init_state", F * 13),
        ("traj_base_x", F), ("traj_base_y", F), ("traj_base_z", F), ("traj_roll", F), ("traj_pitch", F),
        ("traj_yaw", F),
        ("default_dof_pos", F * 12), ("dof_pos_limits", F * 24), ("torque_limits", F * 12),
        ("hard_limits", F * 24), ("height_grid_x", F * GO1_GRID_X), ("height_grid_y", F * GO1_GRID_Y),
        ("contact_stiffness", F), ("contact_damping", F), ("friction_damping", F), ("limit_stiffness", F),
        ("limit_damping", F), ("terrain_restitution", F), ("bounce_threshold", F), ("self_stiffness", F),
        ("self_damping", F),
        ("model", F * GO1_MODEL_FLOATS), ("actuator", F * GO1_ACTUATOR_FLOATS),
    ]


class Go1State(C.Structure):
    _fields_ = [(n, P) for n in (
        "root", "dof_pos", "dof_vel", "last_actions", "last_dof_vel", "lag", "pos_err_hist", "vel_hist",
        "motor_strength", "motor_offset", "friction", "restitution", "payload", "episode_length",
        "curr_pose_index", "trajectory", "base_rotation", "collision_count", "episode_sums",
        "joint_pos_target", "feet_air_time", "last_contacts")]


GO1_STATE_PLANES = 22
GO1_DTYPE_F32, GO1_DTYPE_I32 = 0, 1


class Go1Plane(C.Structure):
    """go1_plane: shape and strides (elements) of one state plane, checked by go1_bind."""
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64), ("row_stride", C.c_int64), ("col_stride", C.c_int64),
                ("dtype", I32), ("pad", I32)]


def plane_descs(tensors):
    """go1_plane[GO1_STATE_PLANES] for a {name: tensor} state, in go1_state order (torch shapes /
    strides as they are: go1_bind, not this helper, decides what it accepts)."""
    arr = (Go1Plane * GO1_STATE_PLANES)()
    for i, (name, _) in enumerate(Go1State._fields_):
        t = tensors[name]
        shape = tuple(t.shape) + (1,) * (2 - t.dim())
        stride = tuple(t.stride()) + (1,) * (2 - t.dim())
        arr[i] = Go1Plane(rows=shape[0], cols=shape[1], row_stride=stride[0], col_stride=stride[1],
                          dtype=GO1_DTYPE_I32 if str(t.dtype) == "torch.int32" else GO1_DTYPE_F32)
    return arr


class Go1Terrain(C.Structure):
    _fields_ = [("tiles", P), ("env_tile", P), ("env_terrain_origin", P), ("env_origins", P),
                ("n_tiles", I32), ("pad", I32)]


GO1_TUNNEL_REC = 40


class Go1TunnelParams(C.Structure):
    _fields_ = [("num_rows", I32), ("num_cols", I32), ("tile_x", I32), ("tile_y", I32), ("sub_x", I32),
                ("sub_y", I32), ("seed", C.c_uint32), ("pad", I32), ("horizontal_scale", C.c_double),
                ("vertical_scale", C.c_double), ("ceiling_height", C.c_double), ("p_flat", C.c_double),
                ("p_double", C.c_double)]


class Go1StepArgs(C.Structure):
    _fields_ = [
        ("actions", P), ("gravity_vec", F * 3), ("sim_gravity", F * 3), ("reward_scales", F * GO1_MAX_TERMS),
        ("rng_seed", C.c_uint64), ("rng_step", C.c_uint64), ("uniforms", P),
        ("inj_dof", P), ("inj_root", P), ("inj_contact", P),
        ("obs", P), ("priv", P), ("rew", P), ("reset", P), ("time_out", P), ("extras_time_outs", P),
        ("any_reset", P), ("contact_forces", P),
        ("dbg_torques", P), ("dbg_heights", P), ("dbg_terms", P), ("dbg_commands", P), ("dbg_reached", P),
        ("episode_log", P), ("aux", P), ("ev_begin", P), ("ev_end", P), ("obs_history", P), ("diverged_count", P),
        ("episode_log_count", P), ("episode_log_cap", I32), ("episode_log_tag", I32),
    ]


# state field widths and dtypes (must match go1_state order); None = set by the config:
# lag 12 x GO1_LAG_STEPS(decimation), trajectory 6 x traj_length, episode_sums n_terms + 3
STATE_SPEC = (
    ("root", 13, "f32"), ("dof_pos", 12, "f32"), ("dof_vel", 12, "f32"), ("last_actions", 12, "f32"),
    ("last_dof_vel", 12, "f32"), ("lag", None, "f32"), ("pos_err_hist", 24, "f32"), ("vel_hist", 24, "f32"),
    ("motor_strength", 12, "f32"), ("motor_offset", 12, "f32"), ("friction", 1, "f32"),
    ("restitution", 1, "f32"), ("payload", 1, "f32"), ("episode_length", 1, "i32"),
    ("curr_pose_index", 1, "i32"), ("trajectory", None, "f32"), ("base_rotation", 3, "f32"),
    ("collision_count", 1, "i32"), ("episode_sums", None, "f32"), ("joint_pos_target", 12, "f32"),
    ("feet_air_time", 4, "f32"), ("last_contacts", 4, "f32"),
)
assert tuple(n for n, _, _ in STATE_SPEC) == tuple(n for n, _ in Go1State._fields_)


def state_spec(cfg):
    """[(name, width, dtype)] of the state planes for a go1_config (or anything with n_terms,
    traj_length and decimation attributes)."""
    w = {"trajectory": 6 * int(cfg.traj_length), "episode_sums": int(cfg.n_terms) + 3,
         "lag": 12 * lag_steps(cfg.decimation)}
    return [(n, w.get(n, wd), dt) for n, wd, dt in STATE_SPEC]


def ptr(a):
    """Raw address of a numpy array or a torch tensor (None -> NULL)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data
