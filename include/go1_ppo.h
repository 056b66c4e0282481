/*
 * go1_ppo.h -- C ABI of the MI355X PPO update engine (legged_tracking_amd/csrc/ppo_update.hip).
 *
 * Replaces, for the update half of the hot path (go1_gym_learn/ppo_cse/ppo.py:98-206, one mini-batch of
 * PPO.update), the torch autograd / hipBLASLt / torch.optim pipeline:
 *   go1_ppo_grad(phase 0)  <- ppo.py:107-158  ac.act / get_actions_log_prob / evaluate on the mini-batch,
 *                             the KL estimate, surrogate + clipped value loss - entropy, loss.backward()
 *   go1_ppo_step(phase 0)  <- ppo.py:119-132, 157-159  adaptive learning rate from the KL, clip_grad_norm_,
 *                             PPO.optimizer.step() (Adam over every parameter)
 *   go1_ppo_grad(phase 1)  <- ppo.py:169-194  adaptation_module(obs_history), F.mse_loss on the first 4/5 of
 *                             the rows (test loss on the rest), backward
 *   go1_ppo_step(phase 1)  <- ppo.py:196-198  adaptation_module_optimizer.step()
 *   go1_ppo_pack()         -  weights split into the f16 fragment images the GEMM kernels read
 * for the default AC_Args architecture (actor_critic.py:21-93): adaptation module hist -> 256 -> 128 -> priv,
 * actor [hist, latent] -> 512 -> 256 -> 128 -> actions, critic [hist, priv] -> 512 -> 256 -> 128 -> 1, ELU.
 *
 * Arithmetic: the GEMMs run on v_mfma_f32_16x16x32_f16 with every f32 operand split into hi + lo f16 halves
 * after an exact power-of-two scaling per tensor (3 MFMAs per product: hi*hi + hi*lo + lo*hi, f32
 * accumulation); everything else (biases, ELU, the loss, its gradient, reductions, Adam) is f32 / f64 VALU.
 * Reductions are fixed-order (partials per workgroup, summed in order): the update is deterministic.
 *
 * Buffers are owned by the caller (PyTorch tensors); every call is asynchronous on `stream` and may be
 * captured into a HIP graph (no host synchronisation, no allocation).  Hyper-parameters, learning rates,
 * step counts and loss sums live in device memory, so a captured graph follows later changes of them.
 */
#ifndef GO1_PPO_H
#define GO1_PPO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GO1_PPO_OK 0
#define GO1_PPO_E_ARG -1
#define GO1_PPO_E_HIP -2

/* fixed hidden widths of the supported architecture (AC_Args defaults) */
#define GO1_PPO_HA1 256
#define GO1_PPO_HA2 128
#define GO1_PPO_H1 512
#define GO1_PPO_H2 256
#define GO1_PPO_H3 128
/* aux sums at the head of the gradient buffer: surrogate, value, KL (phase 0); adaptation, adaptation
   test (phase 1); all-reduced together with the gradients */
#define GO1_PPO_AUX 8

typedef struct go1_ppo_dims {
  int32_t hist;     /* num_obs_history (>= 1) */
  int32_t priv;     /* num_privileged_obs = the adaptation module's output width, 1..8 */
  int32_t actions;  /* num_actions, 1..16 */
  int32_t mb;       /* mini-batch rows (num_envs * num_steps_per_env / num_mini_batches) */
  int64_t rows;     /* storage rows (num_steps_per_env * num_envs); every idx value < rows */
} go1_ppo_dims;

/* PPO_Args / Adam hyper-parameters, as floats in device memory (the caller rewrites them when they change) */
typedef struct go1_ppo_hyper {
  float clip_param, value_loss_coef, entropy_coef, max_grad_norm;
  float desired_kl;              /* <= 0: no adaptive schedule (desired_kl None or schedule != "adaptive") */
  float use_clipped_value_loss;  /* 0 / 1 */
  float selective;               /* selective_adaptation_module_loss: 0 / 1 (column 0 only) */
  float beta1, beta2, eps;       /* Adam (both optimizers) */
  float world;                   /* ranks the gradients are summed over (1 without a process group) */
  float adaptation_lr;           /* adaptation_module_learning_rate */
} go1_ppo_hyper;

typedef struct go1_ppo_bufs {
  /* rollout storage, (rows, width) row-major: RolloutStorage's (T, n, width) tensors flattened over (T, n) */
  const float* obs_history;
  int64_t hist_ld;               /* row stride of obs_history in floats (>= hist) */
  const float *privileged_obs, *actions, *values, *advantages, *returns, *actions_log_prob, *mu, *sigma;
  const int64_t* idx;            /* (mb) storage rows of the mini-batch (mini_batch_generator's permutation slice) */
  /* flat f32 parameters in state_dict order (adaptation_module.{0,2,4}, actor_body.{0,2,4,6},
     critic_body.{0,2,4,6}, each weight then bias; std last): go1_ppo_param_count() floats */
  float* params;
  float* grads;                  /* GO1_PPO_AUX + go1_ppo_param_count() floats: aux sums, then the flat gradient */
  float *exp_avg, *exp_avg_sq;   /* PPO.optimizer Adam state, flat like params */
  float *ad_exp_avg, *ad_exp_avg_sq; /* adaptation_module_optimizer Adam state, flat over the adaptation module */
  float* steps;                  /* [2] Adam step counts (torch's state['step']): main, adaptation */
  double* lr;                    /* [1] the adaptive learning rate of PPO.optimizer (f64, as the reference's floats) */
  const go1_ppo_hyper* hyper;    /* device memory */
  double* losses;                /* [4] running sums of the per-mini-batch means: value, surrogate, adaptation,
                                    adaptation test */
  void* work;                    /* go1_ppo_workspace_bytes() bytes, 256-byte aligned, zeroed once before first use */
} go1_ppo_bufs;

const char* go1_ppo_last_error(void);
/* number of parameters (floats), and of the adaptation module's (the leading slice) */
int go1_ppo_param_count(const go1_ppo_dims* d, int64_t* total, int64_t* adaptation);
int go1_ppo_workspace_bytes(const go1_ppo_dims* d, int64_t* bytes);
/* split + pack the GEMM weights from params (after any change of params outside go1_ppo_step) */
int go1_ppo_pack(const go1_ppo_dims* d, const go1_ppo_bufs* b, void* stream);
/* phase 0: main loss gradient into grads (+ aux sums); phase 1: adaptation-loss gradient into the adaptation
   slice of grads (+ aux).  At world > 1 the caller all-reduces grads[0 : GO1_PPO_AUX + count] (phase 0) or
   grads[0 : GO1_PPO_AUX + adaptation count] (phase 1) between go1_ppo_grad and go1_ppo_step. */
int go1_ppo_grad(const go1_ppo_dims* d, const go1_ppo_bufs* b, int32_t phase, void* stream);
/* phase 0: KL -> learning rate, gradient clip, Adam (all parameters), re-pack;
   phase 1: Adam of the adaptation module, re-pack of its weights */
int go1_ppo_step(const go1_ppo_dims* d, const go1_ppo_bufs* b, int32_t phase, void* stream);

/* test entry points of the two GEMM kernels (tests/test_ppo_engine.py): y = act(x W^T + b) (elu 0 / 1) and the
   weight gradient dw = sum_m d[m] x[m]^T, on the engine's 3xF16 MFMA path; n a multiple of 128.  The GEMM launch
   is repeated `reps` times (timing; same result) */
int go1_ppo_test_linear(const float* x, int64_t rows, int32_t k, const float* w, const float* bias, int32_t n,
                        int32_t elu, float* y, void* work, int64_t work_bytes, int32_t reps, void* stream);
int go1_ppo_test_wgrad(const float* x, const float* d, int64_t rows, int32_t k, int32_t n, float* dw, void* work,
                       int64_t work_bytes, int32_t reps, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GO1_PPO_H */
