// rollout.hip -- PPO rollout kernels for MI355X (gfx950): transition recording,
// GAE and the global advantage normalisation.  C ABI in include/go1_rollout.h.
//
// Reference (go1_gym_learn/ppo_cse):
//   go1_record_transition <- RolloutStorage.add_transitions  rollout_storage.py:57-71
//                            + PPO.process_env_step bootstrap  ppo.py:79-92
//   go1_gae               <- RolloutStorage.compute_returns   rollout_storage.py:76-87
//   go1_adv_normalize     <- rollout_storage.py:89-90 (mean / std over every rank's samples)
//
// The GAE recursion follows torch's f32 element-wise op order (no contraction:
// built with -ffp-contract=off), so returns / advantages are bit-identical to the
// reference's compute_returns; the normalisation statistics are accumulated in f64
// and may differ from torch's f32 reductions in the last ulp.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/go1_rollout.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}

#define RT_TRY(x)                                                                 \
  do {                                                                            \
    hipError_t _e = (x);                                                          \
    if (_e != hipSuccess) return fail(GO1_RT_E_HIP, hipGetErrorString(_e));       \
  } while (0)

// One thread per env: the reverse scan over T steps.  Reads rewards / dones /
// values once (coalesced along envs at each step), writes returns and raw
// advantages, and reduces (sum, sum of squares) of the advantages in f64.
__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
                                                  const float* __restrict__ values,
                                                  const float* __restrict__ last_values, float* __restrict__ returns,
                                                  float* __restrict__ advantages, double* __restrict__ stats, int T,
                                                  int n, float gamma, float lam) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  double s = 0.0, s2 = 0.0;
  if (e < n) {
    float adv = 0.0f;
    float next_v = last_values[e];
    for (int t = T - 1; t >= 0; --t) {
      const size_t i = (size_t)t * n + e;
      const float v = values[i];
      const float nt = 1.0f - (float)dones[i];
      // delta = r + nt * gamma * next_v - v   (torch: ((nt * gamma) * next_v), then +, then -)
      const float delta = (rewards[i] + (nt * gamma) * next_v) - v;
      // advantage = delta + nt * gamma * lam * advantage
      adv = delta + ((nt * gamma) * lam) * adv;
      const float ret = adv + v;
      returns[i] = ret;
      const float a = ret - v;  // advantages = returns - values (:89)
      advantages[i] = a;
      s += (double)a;
      s2 += (double)a * (double)a;
      next_v = v;
    }
  }
  // wave reduction, then one f64 atomic pair per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    s2 += __shfl_xor(s2, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(stats, s);
    atomicAdd(stats + 1, s2);
  }
}

// (a - mean) / (std + 1e-8) with the unbiased std of torch.std over `count` samples.
__global__ __launch_bounds__(256) void adv_norm_kernel(float* __restrict__ adv, const double* __restrict__ stats,
                                                       double count, size_t total) {
  const double mean_d = stats[0] / count;
  double var = (stats[1] - count * mean_d * mean_d) / (count - 1.0);
  var = var > 0.0 ? var : 0.0;
  const float mean = (float)mean_d;
  const float den = (float)sqrt(var) + 1e-8f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
    adv[i] = (adv[i] - mean) / den;
}

struct Seg {
  const float* src;
  float* dst;
  int64_t n;  // floats
};

// All per-step copies of add_transitions in one launch; the reward column gets the
// time-out bootstrap r + gamma * (v * time_out) (ppo.py:85-87), dones become u8.
__global__ __launch_bounds__(256) void record_kernel(go1_transition tr, int n, float gamma) {
  const Seg segs[7] = {{tr.obs, tr.st_obs, (int64_t)n * tr.num_obs},
                       {tr.privileged_obs, tr.st_privileged_obs, (int64_t)n * tr.num_priv},
                       {tr.obs_history, tr.st_obs_history, (int64_t)n * tr.num_obs_history},
                       {tr.actions, tr.st_actions, (int64_t)n * tr.num_actions},
                       {tr.mu, tr.st_mu, (int64_t)n * tr.num_actions},
                       {tr.sigma, tr.st_sigma, (int64_t)n * tr.num_actions},
                       {tr.actions_log_prob, tr.st_actions_log_prob, (int64_t)n}};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    const Seg g = segs[s];
    if (!g.src) continue;
    const bool vec = ((((uintptr_t)g.src) | ((uintptr_t)g.dst)) & 15) == 0;
    if (vec) {
      const int64_t n4 = g.n >> 2;
      const float4* s4 = reinterpret_cast<const float4*>(g.src);
      float4* d4 = reinterpret_cast<float4*>(g.dst);
      for (int64_t i = tid; i < n4; i += stride) d4[i] = s4[i];
      for (int64_t i = (n4 << 2) + tid; i < g.n; i += stride) g.dst[i] = g.src[i];
    } else {
      for (int64_t i = tid; i < g.n; i += stride) g.dst[i] = g.src[i];
    }
  }
  for (int64_t e = tid; e < n; e += stride) {
    const float v = tr.values[e];
    float r = tr.rewards[e];
    if (tr.time_outs) r = r + gamma * (v * (tr.time_outs[e] ? 1.0f : 0.0f));
    tr.st_rewards[e] = r;
    tr.st_values[e] = v;
    tr.st_dones[e] = tr.dones[e] ? 1 : 0;
  }
}

}  // namespace

extern "C" {

const char* go1_rollout_last_error(void) { return g_err.c_str(); }

int go1_record_transition(const go1_transition* tr, int32_t n_envs, float gamma, void* stream) {
  if (!tr || n_envs <= 0) return fail(GO1_RT_E_ARG, "go1_record_transition: bad argument");
  if (!tr->rewards || !tr->dones || !tr->values || !tr->st_rewards || !tr->st_dones || !tr->st_values)
    return fail(GO1_RT_E_ARG, "go1_record_transition: rewards / dones / values are required");
  int64_t big = (int64_t)n_envs * (tr->num_obs + tr->num_obs_history);
  int blocks = (int)((big / 4 + 255) / 256);
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(record_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *tr, n_envs, gamma);
  RT_TRY(hipGetLastError());
  return GO1_OK_RT;
}

int go1_gae(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
            float* returns, float* advantages, double* stats, int32_t T, int32_t n_envs, float gamma, float lam,
            void* stream) {
  if (!rewards || !dones || !values || !last_values || !returns || !advantages || !stats || T <= 0 || n_envs <= 0)
    return fail(GO1_RT_E_ARG, "go1_gae: bad argument");
  hipStream_t s = (hipStream_t)stream;
  RT_TRY(hipMemsetAsync(stats, 0, 2 * sizeof(double), s));
  hipLaunchKernelGGL(gae_kernel, dim3((n_envs + 255) / 256), dim3(256), 0, s, rewards, dones, values, last_values,
                     returns, advantages, stats, T, n_envs, gamma, lam);
  RT_TRY(hipGetLastError());
  return GO1_OK_RT;
}

int go1_adv_normalize(float* advantages, const double* stats, double count, int64_t total, void* stream) {
  if (!advantages || !stats || total < 0 || count < 2.0) return fail(GO1_RT_E_ARG, "go1_adv_normalize: bad argument");
  if (total == 0) return GO1_OK_RT;
  int64_t blocks = (total + 255) / 256;
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(adv_norm_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, advantages, stats,
                     count, (size_t)total);
  RT_TRY(hipGetLastError());
  return GO1_OK_RT;
}

}  // extern "C"
