/*
 * go1_mi355x.h -- C ABI of the MI355X-native Go1 trajectory-tracking step.
 *
 * This library replaces, for the hot path of Daffan/legged_tracking, the Isaac
 * Gym calls inside LeggedRobot.step() and the PyTorch post-physics code around
 * them (reference: go1_gym/envs/base/legged_robot_trajectory_tracking.py):
 *
 *   go1_step()        <- LeggedRobot.step                      :64-112
 *                         (_compute_torques :957-996, eval_actuator_network
 *                          :1311-1320, gym.set_dof_actuation_force_tensor /
 *                          simulate / fetch_results / refresh_dof_state_tensor
 *                          :82-88, post_physics_step :114-169)
 *   go1_reset_idx()   <- LeggedRobot.reset_idx(env_ids)        :218-296
 *   go1_reset_envs()     (the same, env ids as a mask)
 *                         (+ gym.set_*_tensor_indexed :1011-1013, :1050-1052)
 *   go1_set_terrain() <- Terrain env_height_samples / env_terrain_origin
 *                         (_get_env_origins :1808-1847)
 *   go1_tunnel_tiles() <- Terrain(cfg) tile generation (go1_gym/utils/tunnel.py:51-217,
 *                         tunnel_fn.py:99-163), seeded numpy stream reproduced on the device
 *
 * All device pointers are owned by the caller (PyTorch tensors); the library
 * never allocates or frees them.  Every call is asynchronous on the caller's
 * stream (hipStream_t passed as void*), never synchronises the host, and
 * returns 0 on success or a negative GO1_E* code; go1_last_error() returns a
 * thread-local message.  No C++ exceptions cross this boundary.
 * One host thread per handle.
 */
#ifndef GO1_MI355X_H
#define GO1_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GO1_ABI_VERSION 6

#define GO1_NUM_DOF 12
#define GO1_NUM_BODIES 17
#define GO1_MAX_TERMS 16   /* reward terms with a nonzero scale (Cfg.reward_scales, :1380-1397) */
#define GO1_MAX_SUMS (GO1_MAX_TERMS + 3) /* + total, total_pos, total_neg (:1400-1405) */
#define GO1_NUM_PRIV 2
#define GO1_LAG_SLOTS 7    /* the reference's lag ring: lag_timesteps + 1 slots, pushed once per sim step */
/* Stored lag: the scaled actions of the last GO1_LAG_STEPS(decimation) env steps.  Every env step pushes
 * its scaled action `decimation` times into the reference's 7-slot ring (:973-974), so the ring is
 * always those few actions, each repeated (slot 6 - j holds entry K - 1 - floor(j / decimation),
 * K = GO1_LAG_STEPS); storing them instead of the ring moves 2 x 48 B per env-step at decimation 4
 * instead of re-writing 7 x 48 B. */
#define GO1_LAG_STEPS(dec) ((GO1_LAG_SLOTS + (dec) - 1) / (dec))
#define GO1_MAX_TRAJ 16    /* waypoints per trajectory (Cfg.commands.traj_length) */
#define GO1_U_NOISE 47     /* parity-mode uniform slots: 0..46 reset / DR draws, then one per obs column
                              (compute_observations noise, :472-473), then the trajectory draws */
#define GO1_MODEL_FLOATS 178
#define GO1_ACTUATOR_FLOATS 1313 /* w1[32][6] b1[32] w2[32][32] b2[32] w3[32] b3[1] */
#define GO1_GRID_X 21
#define GO1_GRID_Y 11
#define GO1_AUX 32         /* base lin vel 3, base ang vel 3, commands 2, foot pos 12, torques 12 */
/* Episode-log row (go1_step_args.episode_log): n_terms + 3 episode sums, episode length,
 * reached, goal distance -> width n_terms + 6. */

/* Reward functions of the two reward containers the trajectory env can select
 * (Cfg.rewards.reward_container_name, :1373-1377): RewardsCrawling
 * (go1_gym/envs/rewards/reward_crawling.py) and TrajectoryTrackingRewards
 * (go1_gym/envs/rewards/trajectory_tracking_reward.py).  Functions with the same
 * name and body in both share an id; go1_config.term_ids lists, in reward_scales
 * order, the id of each nonzero-scaled term (GO1_T_NONE: the container has no such
 * function -- the reference warns, skips it and keeps a zero episode sum, :1390-1395). */
enum go1_term {
  GO1_T_TORQUES = 0,      /* both containers */
  GO1_T_DOF_ACC,
  GO1_T_COLLISION,
  GO1_T_ACTION_RATE,
  GO1_T_DOF_POS_LIMITS,
  GO1_T_ORIENTATION,
  GO1_T_ANG_VEL_XY,
  GO1_T_REACHING_Z,
  GO1_T_REACHING_ROLL,
  GO1_T_REACHING_PITCH,
  GO1_T_EXPLORATION_LIN,  /* RewardsCrawling exploration_lin == TrajectoryTrackingRewards reaching_linear_vel */
  GO1_T_EXPLORATION_YAW,  /* RewardsCrawling exploration_yaw == TrajectoryTrackingRewards reaching_yaw */
  GO1_T_BASE_HEIGHT,      /* RewardsCrawling only */
  GO1_T_LARGE_VEL,
  GO1_T_E2E,
  GO1_T_DOF_VEL,          /* TrajectoryTrackingRewards only */
  GO1_T_DOF_POS,
  GO1_T_TASK_OLD,
  GO1_T_REACH_GOAL,
  GO1_T_REACH_GOAL_T,     /* reach_goal_t: reached x episode length */
  GO1_T_REACH_GOAL_TR,    /* reach_goal_T: reached x (episode length > T_reach) */
  GO1_T_TASK,
  GO1_T_EXPLORATION,
  GO1_T_STALLING,
  GO1_T_LINEAR_VEL,
  GO1_T_LIN_VEL_Z,
  GO1_T_FEET_AIR_TIME,
  GO1_T_SURVIVE,
  GO1_T_REACHING_YAW_ABS,
  GO1_T_COUNT,
  GO1_T_NONE = 31
};

enum {
  GO1_OK = 0,
  GO1_E_ARG = -1,     /* bad argument / shape */
  GO1_E_HIP = -2,     /* HIP runtime error */
  GO1_E_STATE = -3,   /* call order: bind/terrain missing */
};

/* Static configuration, fixed for the life of a handle.  Values come from the
 * reference Cfg after config_go1() and scripts/train.py (see
 * legged_tracking_amd/config.py for the mapping and citations). */
typedef struct go1_config {
  int32_t n_envs;
  int32_t terrain_kind;        /* 0 plane (legged_robot_trajectory_tracking.py:1928-1932), 1 tunnel tiles */
  int32_t camera_zero;         /* Cfg.env.camera_zero (:400-404) */
  int32_t measure_front_half;  /* Cfg.terrain.measure_front_half (:395-399) */
  int32_t add_noise;           /* Cfg.noise.add_noise (:472-473) */
  int32_t use_terminal_body_height; /* (:205-209) */
  int32_t custom_origins;      /* trimesh origins draw x/y init noise (:1023-1033) */
  int32_t decimation;          /* 4 (go1_crawling.py:37) */
  int32_t n_internal;          /* physics sub-steps per sim step (native integrator) */
  int32_t rand_interval;       /* ceil(rand_interval_s / dt) (:1873) */
  int32_t hf_nx, hf_ny;        /* tile pixels: 80 x 40 for single_path */
  int32_t env_id_offset;       /* global id of local env 0 (rank * n_envs): keys the Philox streams */
  int32_t n_terms;             /* reward terms with a nonzero scale, <= GO1_MAX_TERMS */
  int32_t term_ids[GO1_MAX_TERMS]; /* go1_term of reward slot k, in Cfg.reward_scales order */
  uint32_t term_mask;          /* OR of (1 << id) over term_ids (the terms the kernel evaluates) */
  int32_t reward_mode;         /* 0 plain sum, 1 only_positive_rewards (:341-342), 2 ji22 style (:343-344) */
  int32_t lin_vel_form;        /* exploration_lin: 0 exp, 1 l1, 2 l2, 3 prod (reward_crawling.py:88-104) */
  int32_t terminate_end_of_trajectory; /* (:211-213; e2e bonus reward_crawling.py:64-66) */
  int32_t use_terminal_body_rotation;  /* (:215-216) */
  int32_t rotate_camera;       /* camera pitch 0 in the height scan (:1934-1936) */
  int32_t observe_heights;     /* (:388) */
  int32_t timestep_in_obs;     /* episode_length / max_episode_length after the actions (:375-377) */
  int32_t num_obs;             /* obs row width: 41 + timestep_in_obs + 2 x scanned points */
  int32_t u_per_env;           /* parity-mode uniform row width: GO1_U_NOISE + num_obs + trajectory draws */
  int32_t traj_kind;           /* 0 fixed_target, 1 random_target, 2 random_goal (trajectory_function.py) */
  int32_t traj_length;         /* waypoints per env, <= GO1_MAX_TRAJ */
  int32_t traj_interp;         /* num_interpolation (random_target) */
  uint32_t indefinite_slots;   /* bit k: reward slot k has no fixed sign (exploration, feet_air_time, the prod
                                  form of exploration_lin): its pos / neg bucket is the sign of the sum over
                                  all envs (:332-335), applied by a second launch (go1_step) */
  uint32_t live_slots;         /* bit k: slot k < n_terms has a reward function (term_ids[k] != GO1_T_NONE) */
  float sigma_rew_neg;         /* ji22 style */
  float small_vel_threshold, large_dist_threshold;
  float traj_x_range, traj_y_range, traj_z_range, traj_roll_range, traj_pitch_range, traj_yaw_range;
  float traj_x_mean, traj_y_mean;
  float sim_dt;                /* 0.005 (config.py:355) */
  float dt;                    /* decimation * sim_dt */
  float action_scale;          /* 0.25 */
  float hip_scale_reduction;   /* 0.5 */
  float clip_actions;          /* 10 (train.py:241) */
  float clip_obs;              /* 100 */
  float horizontal_scale;      /* 0.05 (>= 0.05 required with terrain_kind 1) */
  float max_episode_length;    /* ceil(episode_length_s / dt) = 500 */
  float terminal_body_height;  /* 0.0 */
  float switch_dist;           /* 0.3 (train.py:169) */
  float base_height_target;    /* 0.28 */
  float tracking_sigma_lin;    /* 0.05 */
  float tracking_sigma_ang;    /* 0.5 */
  float target_lin_vel;        /* 0.25 */
  float target_ang_vel;        /* pi/2 */
  float lin_reaching_criterion;/* 0.3 */
  float ang_reaching_criterion;/* pi/20 */
  float t_reach;               /* 0 */
  float ceiling_height;        /* used when !camera_zero (:406-409) */
  float obs_scale_dof_pos, obs_scale_dof_vel, obs_scale_heights;
  float noise_gravity, noise_dof_pos, noise_dof_vel; /* noise_vec entries (:1086-1166) */
  float camera_offset_x;       /* 0.12 (:1224) */
  float camera_offset_norm;    /* torch.norm(camera_offset) in f32 */
  float priv_friction_shift, priv_friction_scale, priv_rest_shift, priv_rest_scale;
  float strength_range, strength_lo;   /* torch: rand*(max-min)+min, as f32 */
  float offset_range, offset_lo;
  float reset_dof_range, reset_dof_lo; /* torch_rand_float(0.5, 1.5) */
  float reset_vel_range, reset_vel_lo; /* torch_rand_float(-0.5, 0.5) */
  float x_init_range2, x_init_lo, y_init_range2, y_init_lo, yaw_range2, yaw_lo;
  float x_init_offset, y_init_offset;
  float base_init_state[13];
  float traj_base_x, traj_base_y, traj_base_z, traj_roll, traj_pitch, traj_yaw;
  float default_dof_pos[12];
  float dof_pos_limits[24];    /* soft limits (lo, hi) per dof (:702-706) */
  float torque_limits[12];
  float hard_limits[24];       /* URDF limits for the native joint-limit model */
  float height_grid_x[GO1_GRID_X], height_grid_y[GO1_GRID_Y];
  /* native contact / joint-limit model (no reference equivalent: PhysX is closed) */
  float contact_stiffness, contact_damping, friction_damping, limit_stiffness, limit_damping;
  /* restitution (PhysX's restitution with the default average combine and bounce threshold): a point
   * approaching a surface faster than bounce_threshold gets a separating velocity target
   * e * |vn|, e = (state.restitution + terrain_restitution) / 2
   * (legged_robot_trajectory_tracking.py:676 / :1421-1428, config bounce_threshold_velocity :369) */
  float terrain_restitution, bounce_threshold;
  /* self-collision (asset.self_collisions == 0, go1_crawling.py:44): the calf and foot spheres against the
   * other legs' thigh / calf / foot spheres and the trunk box, explicit penalty springs; stiffness 0
   * disables them (self_collisions == 1) */
  float self_stiffness, self_damping;
  float model[GO1_MODEL_FLOATS];
  float actuator[GO1_ACTUATOR_FLOATS];
} go1_config;

/* Per-env state, SoA planes, each row-major (n_envs, width).  f32 unless noted. */
typedef struct go1_state {
  float* root;             /* 13: pos3, quat xyzw, lin vel3 (world), ang vel3 (world) */
  float* dof_pos;          /* 12 */
  float* dof_vel;          /* 12 */
  float* last_actions;     /* 12 */
  float* last_dof_vel;     /* 12 */
  float* lag;              /* 12 x GO1_LAG_STEPS(decimation): scaled actions of the last steps, oldest
                              first (the reference's 7-slot ring :973-974, stored compactly) */
  float* pos_err_hist;     /* 24: joint_pos_err_last, _last_last (:985-986) */
  float* vel_hist;         /* 24: joint_vel_last, _last_last */
  float* motor_strength;   /* 12 */
  float* motor_offset;     /* 12 */
  float* friction;         /* 1 */
  float* restitution;      /* 1 */
  float* payload;          /* 1 */
  int32_t* episode_length; /* 1 */
  int32_t* curr_pose_index;/* 1 */
  float* trajectory;       /* 6 x traj_length: waypoints (x y z roll pitch yaw) */
  float* base_rotation;    /* 3: rpy from the previous step (:929) */
  int32_t* collision_count;/* 1 */
  float* episode_sums;     /* n_terms + 3: reward_scales order, then total, total_pos, total_neg */
  float* joint_pos_target; /* 12 */
  float* feet_air_time;    /* 4 (feet_air_time reward, trajectory_tracking_reward.py:126-137) */
  float* last_contacts;    /* 4, 0 / 1 */
} go1_state;

/* Terrain: unique tiles (n_tiles, 2, hf_nx, hf_ny) f32 [layer 0 ceiling, 1 floor],
 * env -> tile index, env terrain origin (n_envs,3) and env origin (n_envs,3). */
typedef struct go1_terrain {
  const float* tiles;
  const int32_t* env_tile;
  const float* env_terrain_origin;
  const float* env_origins;
  int32_t n_tiles;
  int32_t pad;
} go1_terrain;

/* Per-call arguments of go1_step. */
typedef struct go1_step_args {
  const float* actions;        /* (n_envs, 12) */
  float gravity_vec[3];        /* normalized gravity used for projected_gravity (:134, :658) */
  float sim_gravity[3];        /* gravity applied by the integrator (:657-660) */
  float reward_scales[GO1_MAX_TERMS]; /* slot order (term_ids), already x dt, decayed (:1380-1385, :171-182) */
  uint64_t rng_seed;
  uint64_t rng_step;           /* Philox counter: one value per call */
  const float* uniforms;       /* parity mode: (n_envs, u_per_env); NULL -> Philox */
  /* parity mode: injected post-physics state instead of the native integrator */
  const float* inj_dof;        /* (decimation, n_envs, 12, 2) pos, vel after each sim step */
  const float* inj_root;       /* (n_envs, 13) after the last sim step */
  const float* inj_contact;    /* (n_envs, 17, 3) net contact forces */
  /* outputs */
  float* obs;                  /* (n_envs, num_obs) */
  float* priv;                 /* (n_envs, 2) */
  float* rew;                  /* (n_envs) */
  uint8_t* reset;              /* (n_envs) bool */
  uint8_t* time_out;           /* (n_envs) bool */
  uint8_t* extras_time_outs;   /* (n_envs) bool, rebound only on steps with a reset (:289-291);
                                  current after go1_sync_time_outs (see below) */
  int32_t* any_reset;          /* reserved (the library keeps its own flag words) */
  float* contact_forces;       /* (n_envs, 17, 3) or NULL */
  /* optional debug outputs (NULL = not written) */
  float* dbg_torques;          /* (decimation, n_envs, 12) */
  float* dbg_heights;          /* (n_envs, 2, 21, 11) measured heights before camera_zero */
  float* dbg_terms;            /* (n_envs, GO1_MAX_TERMS) unscaled reward terms, slot order */
  float* dbg_commands;         /* (n_envs, 2) */
  uint8_t* dbg_reached;        /* (n_envs) */
  /* optional host-facing outputs (NULL = not written) */
  float* episode_log;          /* (n_envs, n_terms + 6): rows of envs reset this step hold the
                                  reset_idx logging of extras["train/episode"] (:256-271): the n_terms + 3
                                  episode sums, episode length, reached, goal distance; every other row
                                  gets only its episode-length column (n_terms + 3) = 0 */
  float* aux;                  /* (n_envs, GO1_AUX): base_lin_vel, base_ang_vel, commands (post-reset),
                                  foot positions (world), torques of the last sim step: the
                                  TrajectoryTrackingEnv.step extras (trajectory_tracking/__init__.py:25-41) */
  /* optional hipEvent_t pair recorded around the fused step kernel alone (NULL = none) */
  void* ev_begin;
  void* ev_end;
  /* optional second copy of obs (NULL = not written): HistoryWrapper's obs_history for a history
     length of 1 (history_wrapper.py:18-24 builds it as a copy of obs every step) */
  float* obs_history;          /* (n_envs, num_obs) */
  /* optional (NULL = not counted): += the number of envs the native integrator's divergence guard
     reset this step (a non-finite state or a component beyond 1e4; no reference counterpart) */
  uint64_t* diverged_count;
  /* optional compact episode log (NULL = episode_log is the per-env (n_envs, n_terms + 6) layout):
     every env reset this step appends one row of n_terms + 8 floats -- the n_terms + 6 values above,
     then episode_log_tag and the env index -- at row atomicAdd(episode_log_count, ...) of episode_log
     (rows at or beyond episode_log_cap are dropped; size it n_envs x steps for none).  Rows of one
     step are in no particular order: order them by (tag, env) for the reference's logging order. */
  int32_t* episode_log_count;
  int32_t episode_log_cap;
  int32_t episode_log_tag;
} go1_step_args;

typedef struct go1_handle go1_handle;

/* Shape and strides (in elements) of one state plane as the caller's tensor has them
 * (PyTorch: t.shape, t.stride(), dtype), in go1_state field order.  go1_bind checks every plane
 * against the layout the kernels index -- (n_envs, width) row-major, dense, f32 / int32 as
 * go1_state notes -- and rejects a view that differs (GO1_E_ARG naming the plane): a
 * non-contiguous slice or transpose never reaches a kernel. */
#define GO1_STATE_PLANES 22
#define GO1_DTYPE_F32 0
#define GO1_DTYPE_I32 1
typedef struct go1_plane {
  int64_t rows, cols;             /* shape (n_envs, width) */
  int64_t row_stride, col_stride; /* elements; dense row-major = (cols, 1) */
  int32_t dtype;                  /* GO1_DTYPE_* */
  int32_t pad;
} go1_plane;

int go1_abi_version(void);
/* sizeof(go1_config), sizeof(go1_state), sizeof(go1_terrain), sizeof(go1_step_args):
 * lets a foreign binding (ctypes / cgo / JNI) verify its struct mirrors. */
void go1_abi_sizes(int64_t out[4]);
const char* go1_last_error(void);
/* Checks the config (GO1_E_ARG with go1_last_error for anything the kernels do not implement; among them a
 * heightfield finer than horizontal_scale = 0.05 m, where a capsule half-link could cross more grid lines than
 * the terrain search's candidates cover) and allocates the handle. */
int go1_create(const go1_config* cfg, go1_handle** out);
/* Binds the caller's state planes (never copied, allocated or freed).  planes: GO1_STATE_PLANES
 * descriptors, go1_state order, required. */
int go1_bind(go1_handle* h, const go1_state* state, const go1_plane* planes);
int go1_set_terrain(go1_handle* h, const go1_terrain* terrain);

/* Tunnel terrain generator on the device (no handle needed): the single_path tiles of a
 * num_rows x num_cols grid, bit-identical to the reference's Terrain(cfg) built after
 * np.random.seed(seed) (go1_gym/utils/tunnel.py:51-126, 189-217 with
 * TerrainFunctions.single_path, go1_gym/utils/tunnel_fn.py:99-163 and vec_plane_from_points :3-21).
 * Replaces the host numpy loop the reference runs once at env creation.
 *   extents: device int32 (n_sub, 4) = start_x, end_x, start_y, end_y of each sub-terrain's tunnel
 *            inside its tile (add_terrain_to_map :193-196), n_sub = num_rows * num_cols, row-major;
 *   records: device scratch, n_sub * GO1_TUNNEL_REC doubles (the drawn wedge parameters);
 *   tiles:   device output (n_sub, 2, tile_x, tile_y) f32, layer 0 ceiling, 1 floor (go1_terrain.tiles). */
#define GO1_TUNNEL_REC 40
typedef struct go1_tunnel_params {
  int32_t num_rows, num_cols;   /* Cfg.terrain.num_rows / num_cols */
  int32_t tile_x, tile_y;       /* int(terrain_length / hs), int(terrain_width / hs) */
  int32_t sub_x, sub_y;         /* SubTerrain shape: int(tile_y * terrain_ratio_y), int(tile_x * terrain_ratio_x) */
  uint32_t seed;                /* np.random.RandomState(seed) / np.random.seed(seed), 0 <= seed < 2^32 */
  int32_t pad;
  double horizontal_scale, vertical_scale, ceiling_height, p_flat, p_double;
} go1_tunnel_params;
int go1_tunnel_tiles(const go1_tunnel_params* p, const int32_t* extents, double* records, float* tiles,
                     void* stream);
int go1_step(go1_handle* h, const go1_step_args* args, void* stream);
/* Kernel variant.  go1_create selects a step kernel specialised for the README configuration
 * (scripts/train.py's README command: the integer flags of legged_tracking_amd/csrc/go1_spec.h
 * folded at compile time) when the config matches it, the generic kernel otherwise; both compute
 * identical results.  enable = 0 forces the generic kernel; enable = 1 fails (GO1_E_ARG) for a
 * config that does not match.  go1_is_specialized returns 1 when the specialised kernel runs. */
int go1_specialize(go1_handle* h, int enable);
int go1_is_specialized(go1_handle* h);
/* extras["time_outs"] (:289-291) is rebound to time_out only on steps with a reset.  The
 * rebinding for step k is applied by the kernel of step k+1 (no launch of its own); call
 * this to have extras_time_outs of the last go1_step current now (one tiny launch,
 * idempotent; the env's extras["time_outs"] read does it). */
int go1_sync_time_outs(go1_handle* h, void* stream);
/* The pending rebinding of the last step without applying it: out = {flag, pending, extras}
 * device pointers (int32 flag word, the step's uint8 time_out buffer, extras_time_outs), all 0
 * before the first step.  A consumer on the same stream that reads extras_time_outs before the
 * next go1_step uses `*flag ? pending[e] : extras[e]` and may write pending[e] into extras[e]
 * (go1_sync_time_outs does exactly that in a kernel of its own); the record kernel of the PPO
 * rollout (go1_rollout.h, go1_transition.time_outs_flag) does it while recording. */
int go1_time_outs_pending(go1_handle* h, int64_t out[3]);
/* reset_idx(env_ids) (:218-296) incl. the DR draws, for the n_ids device int32 env ids (local
 * indices 0 .. n_envs - 1; ids outside that range are skipped, duplicates reset the env once with
 * the same draws); uniforms NULL -> Philox(rng_seed, rng_step) keyed by global env id. */
int go1_reset_idx(go1_handle* h, const int32_t* ids, int32_t n_ids, const float* uniforms, uint64_t rng_seed,
                  uint64_t rng_step, void* stream);
/* The same for the envs whose mask[e] != 0 (one uint8 per env). */
int go1_reset_envs(go1_handle* h, const uint8_t* mask, const float* uniforms, uint64_t rng_seed,
                   uint64_t rng_step, void* stream);
/* Actuator-net torques for (n_rows, 6) inputs -> (n_rows) (eval_actuator_network :1311-1320). */
int go1_actuator_net(go1_handle* h, const float* x, float* out, int32_t n_rows, void* stream);
int go1_destroy(go1_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* GO1_MI355X_H */
