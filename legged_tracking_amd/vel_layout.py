"""Buffer layouts of the velocity-tracking step (BASELINE configs[1]), shared by the host code, the
C ABI (include/go1_velocity.h) and the tests.  Pure data -- no torch, no GPU.

Reference: go1_gym/envs/base/legged_robot_velocity_tracking.py (bare :N below), CoRLRewards
(go1_gym/envs/rewards/corl_rewards.py), RewardThresholdCurriculum (go1_gym/envs/base/curriculum.py).
"""

NUM_COMMANDS = 15          # x vel, y vel, yaw vel, body height, gait freq, phase, offset, bound, duration,
                           # footswing height, body pitch, body roll, stance width, stance length, aux coef
NUM_OBS = 70               # gravity 3, commands 15, dof pos 12, dof vel 12, actions 12, last actions 12, clock 4
NUM_PRIV = 2
N_CATEGORIES = 4           # pronk, trot, pace, bound (gaitwise_curricula, :1319-1321)
N_COMMAND_SUM_EXTRA = 5    # lin_vel_raw, ang_vel_raw, lin_vel_residual, ang_vel_residual, ep_timesteps (:1446)
MAX_TERMS = 24             # CoRLRewards terms with a nonzero scale (19 in train_velocity_tracking.py)

# ---- per-env f32 uniform draws (torch.rand / rand_like of one step), parity mode; Philox otherwise
VU_CAT_A = 0               # _resample_commands category draw, periodic resample (:760, via :704)
VU_CAT_B = 1               # the same, resample inside reset_idx (:182)
VU_DR_STRENGTH = 2         # _randomize_dof_props every rand_interval (:715-717): strength (1), offsets (12)
VU_RESET_STRENGTH = 15     # _randomize_dof_props in reset_idx (:183): strength (1), offsets (12)
VU_RESET_DOF = 28          # _reset_dofs (:974): 12
VU_RESET_YAW = 40          # _reset_root_states yaw (:1007-1009)
VU_RESET_VEL = 41          # _reset_root_states base velocities (:1014): 6
VU_NOISE = 47              # compute_observations noise (:394): NUM_OBS
VU_PER_ENV = VU_NOISE + NUM_OBS  # 117

# ---- per-env f64 draws of the curriculum's numpy RandomState (Curriculum.sample, curriculum.py:67-89)
VD_CHOICE_A = 0            # rng.choice uniform (periodic resample), then 15 rng.uniform cell draws
VD_CHOICE_B = 16           # the same for the resample in reset_idx
VD_PER_ENV = 32

# ---- velocity state planes (beside the physics planes of go1_state), SoA (n_envs, width)
def vel_state_spec(n_terms):
    return (
        ("commands", NUM_COMMANDS, "f32"),
        ("gait_indices", 1, "f32"),
        ("last_last_actions", 12, "f32"),
        ("last_joint_pos_target", 12, "f32"),
        ("last_last_joint_pos_target", 12, "f32"),
        ("command_sums", n_terms + N_COMMAND_SUM_EXTRA, "f32"),
        ("episode_sums", n_terms + 1, "f32"),     # reward_scales order, then "total" (:1433-1437)
        ("command_bins", 1, "i32"),
        ("command_categories", 1, "i32"),
    )


# CoRLRewards functions the velocity step implements, by name (go1_gym/envs/rewards/corl_rewards.py);
# a nonzero-scaled term outside this table raises (the reference prints a warning and skips a name
# the container lacks, :1426-1427; every train_velocity_tracking.py term exists)
VTERMS = ("tracking_lin_vel", "tracking_ang_vel", "lin_vel_z", "ang_vel_xy", "orientation", "torques",
          "dof_acc", "action_rate", "collision", "dof_pos_limits", "jump", "tracking_contacts_shaped_force",
          "tracking_contacts_shaped_vel", "dof_pos", "dof_vel", "action_smoothness_1", "action_smoothness_2",
          "feet_slip", "feet_contact_vel", "feet_contact_forces", "feet_clearance_cmd_linear", "feet_impact_vel",
          "orientation_control", "raibert_heuristic")
VTERM_IDS = {name: i for i, name in enumerate(VTERMS)}
