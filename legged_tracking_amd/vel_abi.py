"""ctypes mirror of include/go1_velocity.h (the velocity-tracking step's C ABI).  Pure host code.

Field for field as the header; tests/test_vel_abi.py checks the sizes against go1_vel_abi_sizes of the
compiled library.
"""
import ctypes as C

from . import vel_layout as VL

GO1_VEL_ABI_VERSION = 2
GO1_VEL_NUM_COMMANDS = VL.NUM_COMMANDS
GO1_VEL_NUM_OBS = VL.NUM_OBS
GO1_VEL_MAX_TERMS = VL.MAX_TERMS
GO1_VEL_SUM_EXTRA = VL.N_COMMAND_SUM_EXTRA
GO1_VEL_N_CATEGORIES = VL.N_CATEGORIES
GO1_VEL_N_KEYS = 15
GO1_VEL_MAX_BINS = 1024
GO1_VEL_AUX = 42
GO1_VEL_U_PER_ENV = VL.VU_PER_ENV
GO1_VEL_D_PER_ENV = VL.VD_PER_ENV
GO1_DTYPE_F64 = 2

# enum go1_vel_term
VTERM_IDS = {name: i for i, name in enumerate((
    "tracking_lin_vel", "tracking_ang_vel", "lin_vel_z", "ang_vel_xy", "orientation", "torques", "dof_acc",
    "action_rate", "collision", "dof_pos_limits", "jump", "tracking_contacts_shaped_force",
    "tracking_contacts_shaped_vel", "dof_pos", "dof_vel", "action_smoothness_1", "action_smoothness_2", "feet_slip",
    "feet_clearance_cmd_linear", "orientation_control", "raibert_heuristic"))}
GO1_VT_COUNT = len(VTERM_IDS)
# the fixed sign of each term's value (corl_rewards.py): +1 nonnegative, -1 nonpositive.  A slot's scaled
# reward then has the sign of scale x this, so the reference's pos / neg bucketing by the sign of the sum
# over envs (:293-296) is decided per slot at construction.
VTERM_SIGN = {"tracking_lin_vel": 1, "tracking_ang_vel": 1, "lin_vel_z": 1, "ang_vel_xy": 1, "orientation": 1,
              "torques": 1, "dof_acc": 1, "action_rate": 1, "collision": 1, "dof_pos_limits": 1, "jump": -1,
              "tracking_contacts_shaped_force": -1, "tracking_contacts_shaped_vel": -1, "dof_pos": 1, "dof_vel": 1,
              "action_smoothness_1": 1, "action_smoothness_2": 1, "feet_slip": 1, "feet_clearance_cmd_linear": 1,
              "orientation_control": 1, "raibert_heuristic": 1}

F = C.c_float
I32 = C.c_int32
D = C.c_double
P = C.c_void_p


class Go1VelConfig(C.Structure):
    _fields_ = [
        ("n_envs", I32), ("n_terms", I32), ("term_ids", I32 * GO1_VEL_MAX_TERMS), ("nonpos_slots", C.c_uint32),
        ("reward_mode", I32), ("resample_interval", I32), ("rand_interval", I32), ("add_noise", I32),
        ("use_terminal_body_height", I32), ("history_len", I32), ("n_bins", I32), ("gaitwise_curricula", I32),
        ("binary_phases", I32), ("n_task", I32), ("task_slot", I32 * 4), ("task_threshold", F * 4),
        ("curriculum_ep_len", F), ("max_episode_length", F), ("dt", F), ("clip_obs", F),
        ("cmd_scale", F * GO1_VEL_NUM_COMMANDS), ("noise_vec", F * GO1_VEL_NUM_OBS),
        ("obs_scale_dof_pos", F), ("obs_scale_dof_vel", F),
        ("priv_friction_shift", F), ("priv_friction_scale", F), ("priv_rest_shift", F), ("priv_rest_scale", F),
        ("strength_range", F), ("strength_lo", F), ("offset_range", F), ("offset_lo", F),
        ("reset_dof_range", F), ("reset_dof_lo", F), ("reset_vel_range", F), ("reset_vel_lo", F),
        ("yaw_range", F), ("yaw_lo", F),
        ("base_init_state", F * 13), ("default_dof_pos", F * 12), ("dof_pos_limits", F * 24),
        ("tracking_sigma", F), ("tracking_sigma_yaw", F), ("gait_force_sigma", F), ("gait_vel_sigma", F),
        ("kappa_gait_probs", F), ("base_height_target", F), ("sigma_rew_neg", F), ("terminal_body_height", F),
        ("pad", I32),
        ("local_range", D * GO1_VEL_N_KEYS), ("bin_sizes", D * GO1_VEL_N_KEYS),
    ]


VEL_STATE_SPEC = (
    ("root", 13, "f32"), ("dof_pos", 12, "f32"), ("dof_vel", 12, "f32"), ("last_actions", 12, "f32"),
    ("last_dof_vel", 12, "f32"), ("lag", 24, "f32"), ("pos_err_hist", 24, "f32"), ("vel_hist", 24, "f32"),
    ("motor_strength", 12, "f32"), ("motor_offset", 12, "f32"), ("friction", 1, "f32"), ("restitution", 1, "f32"),
    ("payload", 1, "f32"), ("episode_length", 1, "i32"), ("last_last_actions", 12, "f32"),
    ("last_joint_pos_target", 12, "f32"), ("last_last_joint_pos_target", 12, "f32"),
    ("commands", GO1_VEL_NUM_COMMANDS, "f32"), ("gait_indices", 1, "f32"), ("last_contacts", 4, "f32"),
    ("command_sums", None, "f32"), ("episode_sums", None, "f32"), ("command_bins", 1, "i32"),
    ("command_categories", 1, "i32"), ("curriculum_weights", None, "f64"),
)
GO1_VEL_STATE_PLANES = len(VEL_STATE_SPEC)


class Go1VelState(C.Structure):
    _fields_ = [(n, P) for n, _, _ in VEL_STATE_SPEC]


def vel_state_spec(n_terms, n_bins):
    """[(name, rows, width, dtype)]: rows None = n_envs (curriculum_weights has one row per category)."""
    w = {"command_sums": n_terms + GO1_VEL_SUM_EXTRA, "episode_sums": n_terms + 1, "curriculum_weights": n_bins}
    return [(n, GO1_VEL_N_CATEGORIES if n == "curriculum_weights" else None, w.get(n, wd), dt)
            for n, wd, dt in VEL_STATE_SPEC]


class Go1VelStepArgs(C.Structure):
    _fields_ = [
        ("actions", P), ("gravity_vec", F * 3), ("gravity_vec_after", F * 3), ("sim_gravity", F * 3),
        ("reward_scales", F * GO1_VEL_MAX_TERMS), ("rng_seed", C.c_uint64), ("rng_step", C.c_uint64),
        ("uniforms", P), ("uniforms_f64", P), ("uniforms_next", P), ("uniforms_f64_next", P),
        ("resample_next", I32), ("pad", I32),
        ("inj_dof", P), ("inj_root", P), ("inj_contact", P), ("inj_feet", P),
        ("obs", P), ("priv", P), ("rew", P), ("reset", P), ("time_out", P), ("extras_time_outs", P),
        ("contact_forces", P), ("obs_history_in", P), ("obs_history_out", P), ("aux", P),
        ("episode_log", P), ("episode_log_count", P), ("episode_log_cap", I32), ("episode_log_tag", I32),
        ("dbg_torques", P), ("dbg_terms", P), ("dbg_gait", P), ("ev_begin", P), ("ev_end", P),
        ("obs_history_in_ld", C.c_int64), ("obs_history_out_ld", C.c_int64),
    ]
