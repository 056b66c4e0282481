"""Canonical names, orders and buffer layouts shared by the host code, the C-ABI
and the tests.  Pure data -- no torch, no GPU.

Orders follow the reference:
  * DOF order FL, FR, RL, RR x (hip, thigh, calf)
    (go1_gym_deploy/envs/lcm_traj_agent.py:67-71; Isaac Gym sorts links by name).
  * Body order of the collapsed Go1 asset (resources/robots/go1/urdf/go1.urdf):
    base, then per leg hip, thigh, calf, foot (17 bodies; +1 arrow actor body per env
    in the reference's contact tensor, legged_robot_trajectory_tracking.py:1201).
  * Reward terms in vars(Cfg.reward_scales) order after zero scales are dropped
    (legged_robot_trajectory_tracking.py:1380-1397 with scripts/train.py:97-125).
"""

LEGS = ("FL", "FR", "RL", "RR")
DOF_NAMES = tuple(f"{leg}_{j}_joint" for leg in LEGS for j in ("hip", "thigh", "calf"))
BODY_NAMES = ("base",) + tuple(f"{leg}_{b}" for leg in LEGS for b in ("hip", "thigh", "calf", "foot"))
FEET_INDICES = (4, 8, 12, 16)
# penalize_contacts_on = ["thigh", "calf", "base"] (scripts/train.py:80), matched in that order
PENALISED_INDICES = (2, 6, 10, 14, 3, 7, 11, 15, 0)

# URDF joint limits per (hip, thigh, calf): go1.urdf:96, 138, 166
JOINT_LIMITS = ((-0.802851455917, 0.802851455917), (-1.0471975512, 4.18879020479),
                (-2.69653369433, -0.916297857297))
JOINT_VEL_LIMIT = (50.0, 28.0, 28.0)
TORQUE_LIMIT = 33.5
# default joint angles (go1_gym/envs/go1/go1_crawling.py:12-26)
DEFAULT_DOF_POS = (0.1, 0.8, -1.5, -0.1, 0.8, -1.5, 0.1, 1.0, -1.5, -0.1, 1.0, -1.5)
# body masses in Isaac Gym order (base absorbs the 0.001 kg imu link)
BODY_MASS_PHYSX = (4.801,) + (0.510299, 0.898919, 0.158015, 0.06) * 4

REWARD_KEYS = ("torques", "dof_acc", "collision", "action_rate", "dof_pos_limits", "base_height",
               "ang_vel_xy", "e2e", "exploration_lin", "exploration_yaw")
SUM_KEYS = REWARD_KEYS + ("total", "total_pos", "total_neg")
N_TERMS = len(REWARD_KEYS)
N_SUMS = len(SUM_KEYS)

# ---- observation layout (scripts/train.py:53, legged_robot_trajectory_tracking.py:368-423)
OBS_GRAVITY, OBS_CMD, OBS_DOF_POS, OBS_DOF_VEL, OBS_ACTIONS, OBS_HEIGHTS = 0, 3, 5, 17, 29, 41
N_HEIGHT_OBS = 220  # 2 layers x 10 front rows x 11 columns
NUM_OBS = 261
NUM_PRIV = 2
NUM_ACTIONS = 12
LAG_SLOTS = 7  # lag_timesteps + 1 (scripts/train.py:191, legged_robot_trajectory_tracking.py:1199)

# ---- canonical per-env uniform draws, U(0,1) f32, one row per env.
# The reference draws these from torch's RNG (fixtures record them); the HIP path
# draws them from a counter-based Philox stream keyed by (seed, env, step, slot),
# or reads them from a caller buffer in parity mode.
U_RESET_STRENGTH = 0   # _randomize_dof_props at reset: strength (1) then offsets (12)
U_RESET_DOF = 13       # _reset_dofs: 12
U_RESET_XY = 25        # _reset_root_states: x, y, yaw  (x,y only drawn for custom origins)
U_RESET_VEL = 28       # _reset_root_states: lin/ang vel 6
U_DR_STRENGTH = 34     # _randomize_dof_props every rand_interval: strength (1) + offsets (12)
U_NOISE = 47           # compute_observations noise: NUM_OBS
U_PER_ENV = U_NOISE + NUM_OBS  # 308

# ---- canonical per-env state the C-ABI reads and writes (SoA, one plane per field)
STATE_FIELDS = (
    # name, width, dtype
    ("root", 13, "f32"),            # pos3, quat xyzw 4, lin vel3 (world), ang vel3 (world)
    ("dof_pos", 12, "f32"),
    ("dof_vel", 12, "f32"),
    ("last_actions", 12, "f32"),
    ("last_dof_vel", 12, "f32"),
    ("lag", 24, "f32"),             # scaled actions of the last 2 steps (decimation 4), oldest first
    ("pos_err_hist", 24, "f32"),    # joint_pos_err_last, joint_pos_err_last_last
    ("vel_hist", 24, "f32"),        # joint_vel_last, joint_vel_last_last
    ("motor_strength", 12, "f32"),
    ("motor_offset", 12, "f32"),
    ("friction", 1, "f32"),
    ("restitution", 1, "f32"),
    ("payload", 1, "f32"),
    ("episode_length", 1, "i32"),
    ("curr_pose_index", 1, "i32"),
    ("trajectory", 6, "f32"),
    ("base_rotation", 3, "f32"),
    ("collision_count", 1, "i32"),
    ("episode_sums", N_SUMS, "f32"),
    ("joint_pos_target", 12, "f32"),
)


# ---- the reference's lag ring (lag_buffer: LAG_SLOTS tensors, pushed once per sim step, :973-974)
# and the stored form (go1_state.lag: the scaled actions of the last K = ceil(LAG_SLOTS / decimation)
# env steps, oldest first).  A step pushes its scaled action `decimation` times, so ring slot 6 - j
# (j pushes back) holds stored entry K - 1 - floor(j / decimation).
def lag_ring_to_stored(ring, decimation):
    """(n, LAG_SLOTS * 12) ring, slot 0 oldest -> (n, K * 12); raises if the ring is not of that form."""
    import numpy as np
    ring = np.asarray(ring).reshape(len(ring), LAG_SLOTS, 12)
    K = (LAG_SLOTS + decimation - 1) // decimation
    out = np.empty((ring.shape[0], K, 12), ring.dtype)
    for k in range(K):
        out[:, k] = ring[:, LAG_SLOTS - 1 - (K - 1 - k) * decimation]
    if not np.array_equal(lag_stored_to_ring(out.reshape(len(ring), -1), decimation).reshape(ring.shape), ring):
        raise ValueError("lag ring is not a sequence of per-step pushes of `decimation` copies")
    return out.reshape(len(ring), K * 12)


def lag_stored_to_ring(stored, decimation):
    """(n, K * 12) stored lag -> (n, LAG_SLOTS * 12) ring, slot 0 oldest."""
    import numpy as np
    K = (LAG_SLOTS + decimation - 1) // decimation
    stored = np.asarray(stored).reshape(len(stored), K, 12)
    ring = np.empty((stored.shape[0], LAG_SLOTS, 12), stored.dtype)
    for s in range(LAG_SLOTS):
        ring[:, s] = stored[:, K - 1 - (LAG_SLOTS - 1 - s) // decimation]
    return ring.reshape(len(stored), LAG_SLOTS * 12)
