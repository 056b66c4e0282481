/*
 * go1_rollout.h -- C ABI of the MI355X PPO rollout kernels (legged_tracking_amd/csrc/rollout.hip).
 *
 * Replaces, for the rollout half of the hot path (go1_gym_learn/ppo_cse):
 *   go1_record_transition()  <- RolloutStorage.add_transitions     rollout_storage.py:57-71
 *                               + PPO.process_env_step bootstrap    ppo.py:79-92
 *   go1_gae()                <- RolloutStorage.compute_returns      rollout_storage.py:76-87
 *   go1_adv_normalize()      <- rollout_storage.py:89-90 (global normalisation; the
 *                               caller may all-reduce the 2 f64 statistics across ranks
 *                               between the two calls)
 *   go1_colsum()             <- the bias gradients of PPO.update's backward (ppo.py:155-157),
 *                               torch's grad_output.sum(0) in F.linear's backward
 *
 * All pointers are device pointers owned by the caller; every call is
 * asynchronous on the given HIP stream and returns 0 or a negative code.
 */
#ifndef GO1_ROLLOUT_H
#define GO1_ROLLOUT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GO1_OK_RT 0
#define GO1_RT_E_ARG -1
#define GO1_RT_E_HIP -2

/* One transition (rows of n_envs) and the storage slot it goes to. */
typedef struct go1_transition {
  const float* obs;               /* (n, num_obs) */
  const float* privileged_obs;    /* (n, num_priv) */
  const float* obs_history;       /* (n, num_obs_history) */
  const float* actions;           /* (n, num_actions) */
  const float* mu;                /* (n, num_actions) action mean */
  const float* sigma;             /* (n, num_actions) action std */
  const float* actions_log_prob;  /* (n) */
  const float* values;            /* (n) */
  const float* rewards;           /* (n) env rewards before bootstrapping */
  const uint8_t* dones;           /* (n) bool */
  const uint8_t* time_outs;       /* (n) bool or NULL (no bootstrap) */
  float *st_obs, *st_privileged_obs, *st_obs_history, *st_actions, *st_mu, *st_sigma, *st_actions_log_prob;
  float *st_values, *st_rewards;
  uint8_t* st_dones;
  int32_t num_obs, num_priv, num_obs_history, num_actions;
  /* Deferred extras["time_outs"] rebinding (go1_step rebinds only on steps with a reset,
   * legged_robot_trajectory_tracking.py:289-291, and defers it, see go1_time_outs_pending):
   * when time_outs_flag is non-NULL and *time_outs_flag != 0, the time-outs of this transition
   * are time_outs_pending, and they are also copied into time_outs_dst (the env's
   * extras["time_outs"] tensor, current afterwards).  NULL = time_outs is used as is. */
  const int32_t* time_outs_flag;
  const uint8_t* time_outs_pending;
  uint8_t* time_outs_dst;
  int64_t obs_history_ld;         /* row stride of obs_history in floats (0: num_obs_history), e.g. a window of
                                     the velocity env's wider history rows (go1_velocity.h obs_history_out_ld) */
} go1_transition;

/* Fused policy inference (ActorCritic.act / evaluate, actor_critic.py:121-150) for the
 * default AC_Args architecture: adaptation 261 -> 256 -> 128 -> 2, actor
 * [hist, latent] -> 512 -> 256 -> 128 -> num_actions, critic [hist, priv] -> 512 -> 256
 * -> 128 -> 1, ELU, to f32 accuracy on f16 matrix cores (3xF16 split products, see rollout.hip).
 * Weights split and packed by legged_tracking_amd/rollout.py (fragment order,
 * layers: a1 a2 a3 p1 p2 p3 p4 c1 c2 c3 c4). */
#define GO1_POLICY_LAYERS 11
typedef struct go1_policy_layer {
  /* [n/16][k/32][64 lanes][16] f16 (n padded to 16, k to 32): each weight w split into hi = f16(w)
     and lo = f16(w - hi); record (t, g, lane = 16 q + m) = hi, then lo, of W[16 t + m][32 g + 8 q + r],
     r = 0..7 (32 bytes: the lane's A fragments of v_mfma_f32_16x16x32_f16 for both halves) */
  const void* w;
  const float* b;  /* [n padded to 16] */
  const float* wf; /* (n, k) row-major f32, the unsplit weights: the f32 fallback of a workgroup whose
                      activations leave the f16 split's range (|x| >= 65504) */
} go1_policy_layer;
typedef struct go1_policy_args {
  const float* obs_history;    /* (n, hist_dim) */
  const float* privileged_obs; /* (n, num_priv) */
  float* action_mean;          /* (n, num_actions) */
  float* value;                /* (n) */
  float* latent;               /* (n, num_priv) or NULL: the adaptation module's output */
  /* optional in-kernel Normal(mean, std).sample() + log_prob (NULL actions = skip) */
  const float* std;            /* (num_actions) */
  float* actions;              /* (n, num_actions) */
  float* action_sigma;         /* (n, num_actions) */
  float* log_prob;             /* (n) */
  uint64_t rng_seed, rng_step; /* Philox key / counter, one counter value per call */
  int32_t env_id_offset;       /* global id of row 0 (rank * n) */
  int32_t n_envs, hist_dim, num_actions;
  int32_t num_priv;            /* privileged obs = latent width, 1 .. 8.  variant 1: 257 <= hist_dim <= 288 - num_priv
                                  (it walks exactly nine packed K groups; anything else is GO1_RT_E_ARG);
                                  variant 0 streams the inputs in chunks of 288 (hist_dim + num_priv <= 16384,
                                  the groups of 32 that hold the latent inside the last chunk) */
  int32_t variant;             /* 0: per-net workgroups of 32 envs (default), 1: one workgroup of 16 envs
                                  running all three nets; identical outputs (tests/test_rollout.py) */
  int32_t* overflow;           /* optional: += workgroups that recomputed in f32 (the range guard) */
  go1_policy_layer layers[GO1_POLICY_LAYERS];
  int64_t hist_ld;             /* row stride of obs_history in floats (0: hist_dim; >= hist_dim) */
} go1_policy_args;

const char* go1_rollout_last_error(void);
int go1_policy_forward(const go1_policy_args* args, void* stream);
int go1_record_transition(const go1_transition* tr, int32_t n_envs, float gamma, void* stream);
/* rewards/values/returns/advantages: (T, n) f32; dones (T, n) u8; last_values (n);
 * stats: 2 f64 (sum, sum of squares of the raw advantages), overwritten. */
int go1_gae(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
            float* returns, float* advantages, double* stats, int32_t T, int32_t n_envs, float gamma, float lam,
            void* stream);
/* advantages <- (a - mean) / (std + 1e-8); count = number of samples the stats cover (all ranks). */
int go1_adv_normalize(float* advantages, const double* stats, double count, int64_t total, void* stream);
/* out[c] = sum over rows of x[r][c], x row-major (rows, cols) f32, deterministic (fixed partition and order):
 * the PPO update's bias gradients (PPO.update, ppo.py:155-157 backward; torch's grad_output.sum(0)).
 * partial: scratch of parts x cols floats, 1 <= parts <= min(rows, 65535). */
int go1_colsum(const float* x, int64_t rows, int32_t cols, float* partial, int32_t parts, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GO1_ROLLOUT_H */
