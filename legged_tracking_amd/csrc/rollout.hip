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

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/go1_rollout.h"

namespace {

typedef float f4_t __attribute__((ext_vector_type(4)));

// Philox4x32-10 (Salmon et al. 2011), as in the env step kernel
__device__ __forceinline__ void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

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
  const int64_t hld = tr.obs_history_ld, hw = tr.num_obs_history;
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    const Seg g = segs[s];
    if (!g.src) continue;
    if (s == 2 && hld != hw) {  // a row-strided history window: rows of hw floats, hld apart
      if (((hw | hld) & 1) == 0 && ((((uintptr_t)g.src) | ((uintptr_t)g.dst)) & 7) == 0) {
        const int64_t w2 = hw >> 1, n2 = (int64_t)n * w2;
        for (int64_t i = tid; i < n2; i += stride) {
          const int64_t r = i / w2, c = i - r * w2;
          reinterpret_cast<float2*>(g.dst)[i] = *reinterpret_cast<const float2*>(g.src + r * hld + 2 * c);
        }
      } else {
        for (int64_t i = tid; i < g.n; i += stride) {
          const int64_t r = i / hw;
          g.dst[i] = g.src[r * hld + (i - r * hw)];
        }
      }
      continue;
    }
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
  const bool rebind = tr.time_outs_flag && *tr.time_outs_flag != 0;
  for (int64_t e = tid; e < n; e += stride) {
    const float v = tr.values[e];
    float r = tr.rewards[e];
    const uint8_t* to = rebind ? tr.time_outs_pending : tr.time_outs;
    if (to) {
      const uint8_t t = to[e];
      if (rebind && tr.time_outs_dst) tr.time_outs_dst[e] = t;
      r = r + gamma * (v * (t ? 1.0f : 0.0f));
    }
    tr.st_rewards[e] = r;
    tr.st_values[e] = v;
    tr.st_dones[e] = tr.dones[e] ? 1 : 0;
  }
}

// The same copies with one 16-byte chunk per thread and each workgroup on one segment (block ranges per
// segment, chosen on the host when every buffer is 16-byte aligned and the history is contiguous): every
// thread issues its single load at once instead of walking the segments one round trip after the other.
#define REC_MAX_SEGS 8
struct RecPlan {
  const float4* src[REC_MAX_SEGS];
  float4* dst[REC_MAX_SEGS];
  float4* dst2[REC_MAX_SEGS];  // a second destination (obs_history aliasing obs: one read feeds both rows)
  int64_t nf[REC_MAX_SEGS];    // floats
  int first[REC_MAX_SEGS + 1]; // first workgroup of each segment; first[nseg] = the env columns' first
  int nseg;
};
__global__ __launch_bounds__(256) void record_flat_kernel(RecPlan P, go1_transition tr, int n, float gamma) {
  const int b = blockIdx.x, t = threadIdx.x;
  if (b >= P.first[P.nseg]) {  // per-env columns: bootstrap reward, value, done
    const int64_t e = (int64_t)(b - P.first[P.nseg]) * 256 + t;
    if (e >= n) return;
    // every column requested before any is used (both time-out arrays: the flag picks one afterwards)
    const float v = tr.values[e];
    float r = tr.rewards[e];
    const uint8_t d = tr.dones[e];
    const uint8_t* tn_p = tr.time_outs ? tr.time_outs : tr.dones;
    const uint8_t* tp_p = tr.time_outs_pending ? tr.time_outs_pending : tr.dones;
    const uint8_t tn = tn_p[e], tp = tp_p[e];
    const bool rebind = tr.time_outs_flag && *tr.time_outs_flag != 0;
    if (rebind ? tr.time_outs_pending != nullptr : tr.time_outs != nullptr) {
      const uint8_t tt = rebind ? tp : tn;
      if (rebind && tr.time_outs_dst) tr.time_outs_dst[e] = tt;
      r = r + gamma * (v * (tt ? 1.0f : 0.0f));
    }
    tr.st_rewards[e] = r;
    tr.st_values[e] = v;
    tr.st_dones[e] = d ? 1 : 0;
    return;
  }
  int s = 0;  // the workgroup's segment (uniform)
  while (s + 1 < P.nseg && b >= P.first[s + 1]) ++s;
  const int64_t k = (int64_t)(b - P.first[s]) * 256 + t, n4 = P.nf[s] >> 2;
  const float4* src = P.src[s];
  float4* dst = P.dst[s];
  float4* dst2 = P.dst2[s];
  if (k < n4) {
    const float4 v = src[k];
    dst[k] = v;
    if (dst2) dst2[k] = v;
  }
  const int rem = (int)(P.nf[s] & 3);
  if (b == P.first[s] && t < rem) {  // the last nf % 4 floats
    const float x = reinterpret_cast<const float*>(src)[4 * n4 + t];
    reinterpret_cast<float*>(dst)[4 * n4 + t] = x;
    if (dst2) reinterpret_cast<float*>(dst2)[4 * n4 + t] = x;
  }
}

// ------------------------------------------------------------------ policy inference
// ActorCritic.act / evaluate (actor_critic.py:121-150) for 16 envs per workgroup of 16 waves:
//   adaptation: hist(261) -> 256 -> 128 -> 2 (latent)
//   actor:      [hist, latent](263) -> 512 -> 256 -> 128 -> 12 (action mean)
//   critic:     [hist, priv](263)   -> 512 -> 256 -> 128 -> 1  (value)
// ELU between layers.  f32 accuracy from f16 matrix cores ("3xF16"): every f32 weight and
// activation x is split into hi = f16(x) and lo = f16(x - hi) (22 significant bits together),
// and each 32-deep K group of a dot product is three v_mfma_f32_16x16x32_f16,
//   acc += Whi Xhi + Whi Xlo + Wlo Xhi
// with products exact in f32 and f32 accumulation; the dropped Wlo Xlo term is ~2^-22 of the
// product, below the f32 rounding of the sums.  On gfx950 a 16x16x32 f16 MFMA issues in the 16
// cycles of a 16x16x16 one (tools/probes/mfma_rate.hip: 16.3 cycles each, one wave), so the K=32 form
// does twice the work per MFMA cycle.  Weights are split and packed on the host into fragment order:
// 32 bytes per lane per (tile, K group) = 8 hi + 8 lo halves, L2-resident (2.8 MB for all three
// nets).  Activations live in LDS already split, as [k/8][env][8] halves (hi plane, then lo plane): a
// B fragment (k = 32 g + 8 q + r, env c) is one 16-byte read per plane, and a layer's output tile
// (rows 4 q + r of env c) one 8-byte write.
#ifndef GO1_POLICY_SCHED
#define GO1_POLICY_SCHED 1
#endif
constexpr int PIN = 288;  // 261 / 263 inputs padded to a multiple of 32
constexpr int PW = 16;    // waves per workgroup (four per SIMD)

typedef go1_policy_layer PolicyLayer;  // w packed [n/16][k/32][64 lanes][8 hi + 8 lo halves], b [n padded to 16]
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef _Float16 h16_t __attribute__((ext_vector_type(16)));
typedef float f8_t __attribute__((ext_vector_type(8)));  // one lane's weight fragment (32 bytes)

// split activation planes in LDS: element (k, env c) at [k / 8][c][k % 8] of hi, and of lo
struct ActV {
  h8_t* hi;
  h8_t* lo;
};
template <int K>
struct Act {
  h8_t hi[K / 8][16];
  h8_t lo[K / 8][16];
  __device__ ActV v() { return ActV{&hi[0][0], &lo[0][0]}; }
};

// ELU's negative branch through the hardware exponential (v_exp_f32): exp(x) - 1 loses relative accuracy
// only where |x| is tiny, where its absolute error stays ~6e-8 (the outputs are checked at 2e-5 of their
// scale against f64); expm1f's range reduction cost ~25 instructions per value on the workgroups' tails
__device__ __forceinline__ float elu(float x) { return x > 0.0f ? x : __expf(x) - 1.0f; }

// Normal(0, 1) draws of actions 4 q .. 4 q + 3 of global env gid: one Philox4x32-10 block keyed by
// (env, action group, step), two Box-Muller pairs on the hardware log2 / sqrt / sin / cos (v_sin / v_cos
// take revolutions).  The samples are the kernel's own stream (the reference draws from torch's generator).
__device__ __forceinline__ void normal4(uint32_t gid, int q, uint64_t step, uint64_t seed, float z[4]) {
  uint32_t ctr[4] = {gid, (uint32_t)q, (uint32_t)step, (uint32_t)(step >> 32)};
  philox4x32(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float u1 = ((float)(ctr[2 * p] >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
    const float u2 = (float)(ctr[2 * p + 1] >> 8) * (1.0f / 16777216.0f);       // [0, 1)
    const float r = __builtin_amdgcn_sqrtf(-2.0f * 0.69314718055994531f * __builtin_amdgcn_logf(u1));
    z[2 * p] = r * __builtin_amdgcn_cosf(u2);
    z[2 * p + 1] = r * __builtin_amdgcn_sinf(u2);
  }
}

// Range guard of the split: f16(x) overflows for |x| >= 65520 (and a NaN / inf input has no split), so a
// value outside (-65504, 65504) sets the workgroup's flag; the workgroup then recomputes its envs in
// f32 from the unsplit weights at its end (policy_fallback).  One compare per stored value.
__device__ __forceinline__ void ovf_check(float v, int* ovf) {
  if (!(fabsf(v) < 65504.0f)) *ovf = 1;
}
// four consecutive features 4 kq .. 4 kq + 3 of env c, split into the two planes
__device__ __forceinline__ void act_store4(ActV d, int kq, int c, f4_t v, int* ovf) {
  h4_t h, l;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ovf_check(v[r], ovf);
    h[r] = (_Float16)v[r];
    l[r] = (_Float16)(v[r] - (float)h[r]);
  }
  reinterpret_cast<h4_t*>(d.hi)[((kq >> 1) * 16 + c) * 2 + (kq & 1)] = h;
  reinterpret_cast<h4_t*>(d.lo)[((kq >> 1) * 16 + c) * 2 + (kq & 1)] = l;
}
__device__ __forceinline__ void act_store1(ActV d, int k, int c, float v, int* ovf) {
  ovf_check(v, ovf);
  const _Float16 h = (_Float16)v;
  reinterpret_cast<_Float16*>(d.hi)[((k >> 3) * 16 + c) * 8 + (k & 7)] = h;
  reinterpret_cast<_Float16*>(d.lo)[((k >> 3) * 16 + c) * 8 + (k & 7)] = (_Float16)(v - (float)h);
}

// acc += W x over one 32-deep K group: w = (8 hi, 8 lo) halves of the lane's A fragment
__device__ __forceinline__ f4_t mfma3(f8_t w, h8_t xh, h8_t xl, f4_t acc) {
  const h16_t wv = __builtin_bit_cast(h16_t, w);
  const h8_t wh = __builtin_shufflevector(wv, wv, 0, 1, 2, 3, 4, 5, 6, 7);
  const h8_t wl = __builtin_shufflevector(wv, wv, 8, 9, 10, 11, 12, 13, 14, 15);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xh, acc, 0, 0, 0);
}

template <int NT, int NL>
__device__ __forceinline__ void policy_load(const PolicyLayer* L, int G, int g, int tile0, int tstride, int lane,
                                            f8_t (&w)[NL][NT]) {
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int i = 0; i < NT; ++i)
      w[l][i] = reinterpret_cast<const f8_t*>(L[l].w)[((size_t)(tile0 + i * tstride) * G + g) * 64 + lane];
#if GO1_POLICY_SCHED
  // keep the prefetch where it is written: otherwise the scheduler sinks the loads next to
  // their MFMAs and the waits become vmcnt(1), exposing the L2 latency every group
  __builtin_amdgcn_sched_barrier(0);
#endif
}

template <int NT, int NL>
__device__ __forceinline__ void policy_group(const f8_t (&w)[NL][NT], const ActV* src, int g, int q, int c,
                                             f4_t (&acc)[NL][NT]) {
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const h8_t xh = src[l].hi[(4 * g + q) * 16 + c], xl = src[l].lo[(4 * g + q) * 16 + c];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[l][i] = mfma3(w[l][i], xh, xl, acc[l][i]);
  }
}

// NT output tiles (tile0 + i * tstride) of NL layers at the same depth (the actor and the critic
// advance together) for the 16 envs: acc = b + W x, ELU (act), store split to dst.  The G K groups
// are unrolled and the weight fragments run D groups ahead of the MFMAs: with three 8-cycle f16
// MFMAs per fragment the layers are bound by the L2 -> CU weight stream, which needs ~12
// 16-byte loads in flight per lane (64 B/clk/CU x the L2 latency, 16 waves).
// the first D weight groups of a policy_tiles phase, issued early: they depend on nothing the
// workgroup computes, so the adaptation module's can be in flight while the inputs are staged
template <int NT, int NL, int G, int D>
__device__ __forceinline__ void policy_prefetch(const PolicyLayer* L, int tile0, int tstride, int lane,
                                                f8_t (&w)[D][NL][NT]) {
#pragma unroll
  for (int g = 0; g < D && g < G; ++g) policy_load<NT, NL>(L, G, g, tile0, tstride, lane, w[g]);
}

template <int NT, int NL, int G, int D, bool PREFETCHED = false>
__device__ __forceinline__ void policy_tiles(const PolicyLayer* L, const ActV* src, int tile0, int tstride,
                                             const ActV* dst, bool act, int lane, int* ovf,
                                             f8_t (*pre)[NL][NT] = nullptr) {
  const int q = lane >> 4, c = lane & 15;
  f4_t acc[NL][NT];
  f8_t w[D][NL][NT];
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int i = 0; i < NT; ++i)
      acc[l][i] = *reinterpret_cast<const f4_t*>(L[l].b + 16 * (tile0 + i * tstride) + 4 * q);
  if constexpr (PREFETCHED) {
#pragma unroll
    for (int g = 0; g < D; ++g)
#pragma unroll
      for (int l = 0; l < NL; ++l)
#pragma unroll
        for (int i = 0; i < NT; ++i) w[g][l][i] = pre[g][l][i];
  } else {
    policy_prefetch<NT, NL, G, D>(L, tile0, tstride, lane, w);
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    policy_group<NT, NL>(w[g % D], src, g, q, c, acc);
    if (g + D < G) policy_load<NT, NL>(L, G, g + D, tile0, tstride, lane, w[g % D]);
  }
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      f4_t v = acc[l][i];
      if (act) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = elu(v[r]);
      }
      act_store4(dst[l], 4 * (tile0 + i * tstride) + q, c, v, ovf);
    }
}

// Partial product of one output tile over K groups [g0, g0 + NG), no bias: the K-split form of
// the narrow layers (one wave walking all of K would run a serial MFMA chain behind one L2
// round trip per group).  All NG weight fragments are loaded up front (one round trip).
template <int NG>
__device__ __forceinline__ f4_t tile_partial(const PolicyLayer& L, int Gs, int tile, int g0, ActV src, int lane) {
  const int q = lane >> 4, c = lane & 15;
  f8_t w[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) w[i] = reinterpret_cast<const f8_t*>(L.w)[((size_t)tile * Gs + g0 + i) * 64 + lane];
  f4_t acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < NG; ++i)
    acc = mfma3(w[i], src.hi[(4 * (g0 + i) + q) * 16 + c], src.lo[(4 * (g0 + i) + q) * 16 + c], acc);
  return acc;
}

// ---------------------------------------------------------------- range guard: f32 fallback
// y = act(W x + b) for one env, W (n_out, k_in) row-major f32, by the workgroup (output o on thread o)
__device__ void dense_f32(const float* __restrict__ W, const float* __restrict__ b, int n_out, int k_in,
                          const float* x, float* y, bool act) {
  for (int o = threadIdx.x; o < n_out; o += blockDim.x) {
    float acc = b[o];
    const float* w = W + (size_t)o * k_in;
    for (int k = 0; k < k_in; ++k) acc = fmaf(w[k], x[k], acc);
    y[o] = act ? elu(acc) : acc;
  }
  __syncthreads();
}

// The envs [e0, e0 + ne) of a workgroup whose split activations left the f16 range, recomputed in f32
// from the unsplit weights (layers[].wf): the adaptation module + actor (+ the Normal sample with the
// same Philox draws) and / or the critic.  `buf`: >= hist_dim + num_priv (rounded up to 32) + 768 floats of
// LDS no longer in use.
__device__ void policy_fallback(const go1_policy_args& P, int e0, int ne, bool actor, bool critic, float* buf) {
  const go1_policy_layer* L = P.layers;
  const int H = P.hist_dim, NP = P.num_priv, NA = P.num_actions;
  float* x = buf;
  float* ya = buf + ((H + NP + 31) & ~31);
  float* yb = ya + 512;
  for (int e = 0; e < ne; ++e) {
    const size_t ge = (size_t)(e0 + e);
    for (int k = threadIdx.x; k < H; k += blockDim.x) x[k] = P.obs_history[ge * P.hist_ld + k];
    __syncthreads();
    if (actor) {
      dense_f32(L[0].wf, L[0].b, 256, H, x, ya, true);
      dense_f32(L[1].wf, L[1].b, 128, 256, ya, yb, true);
      dense_f32(L[2].wf, L[2].b, NP, 128, yb, x + H, false);  // the latent, appended to the actor's input
      if (P.latent && (int)threadIdx.x < NP) P.latent[ge * NP + threadIdx.x] = x[H + threadIdx.x];
      dense_f32(L[3].wf, L[3].b, 512, H + NP, x, ya, true);
      dense_f32(L[4].wf, L[4].b, 256, 512, ya, yb, true);
      dense_f32(L[5].wf, L[5].b, 128, 256, yb, ya, true);
      dense_f32(L[6].wf, L[6].b, NA, 128, ya, yb, false);
      if (threadIdx.x == 0) {
        float lp_q[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        float zq[4];
        for (int f = 0; f < NA; ++f) {
          P.action_mean[ge * NA + f] = yb[f];
          if (P.actions) {
            const float sd = P.std[f];
            if ((f & 3) == 0) normal4((uint32_t)(ge + P.env_id_offset), f >> 2, P.rng_step, P.rng_seed, zq);
            const float z = zq[f & 3];
            P.actions[ge * NA + f] = yb[f] + sd * z;
            P.action_sigma[ge * NA + f] = sd;
            lp_q[f >> 2] += -0.5f * z * z - __logf(sd) - 0.91893853320467274f;
          }
        }
        if (P.actions) P.log_prob[ge] = (lp_q[0] + lp_q[1]) + (lp_q[2] + lp_q[3]);
      }
      __syncthreads();
    }
    if (critic) {
      for (int k = threadIdx.x; k < NP; k += blockDim.x) x[H + k] = P.privileged_obs[ge * NP + k];
      __syncthreads();
      dense_f32(L[7].wf, L[7].b, 512, H + NP, x, ya, true);
      dense_f32(L[8].wf, L[8].b, 256, 512, ya, yb, true);
      dense_f32(L[9].wf, L[9].b, 128, 256, yb, ya, true);
      dense_f32(L[10].wf, L[10].b, 1, 128, ya, yb, false);
      if (threadIdx.x == 0) P.value[ge] = yb[0];
      __syncthreads();
    }
  }
  if (threadIdx.x == 0 && P.overflow) atomicAdd(P.overflow, 1);
}

#ifdef GO1_POLICY_STAMPS  // diagnostic build only (tools/policy_stamps.py): s_memtime per wave per phase
#define PSTAMP_SLOTS 12
__device__ unsigned long long g_pstamps[512 * 16 * PSTAMP_SLOTS];
#define PSTAMP(k)                                                                                   \
  do {                                                                                              \
    unsigned long long t_;                                                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                   \
    if (blockIdx.x < 512) g_pstamps[(blockIdx.x * 16 + (threadIdx.x >> 6)) * PSTAMP_SLOTS + (k)] = t_; \
  } while (0)
#else
#define PSTAMP(k)
#endif

__global__ __launch_bounds__(64 * PW) void policy_kernel(go1_policy_args P) {
  __shared__ Act<PIN> xa, xc;  // actor / critic inputs (the adaptation module reads xa)
  __shared__ Act<512> h1[2];   // layer-1 outputs (actor, critic); layer 3 reuses them
  __shared__ Act<256> h2[2];   // layer-2 outputs; also the f32 scratch of the K-split partials
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int e0 = blockIdx.x * 16;
  PSTAMP(0);
  const int ne = min(16, P.n_envs - e0);
  const int NP = P.num_priv;
  const ActV va = xa.v(), vc = xc.v();
  __shared__ int s_ovf;
  if (tid == 0) s_ovf = 0;
#ifndef GO1_POLICY_NO_EARLY
  // the adaptation module's first weight groups are in flight while the inputs are staged
  f8_t w_ad[4][1][1];
  policy_prefetch<1, 1, PIN / 32, 4>(P.layers + 0, wave, PW, lane, w_ad);
#endif
  for (int idx = tid; idx < 16 * PIN; idx += 64 * PW) {
    const int e = idx / PIN, k = idx - e * PIN;
    float v = 0.0f;
    if (e < ne && k < P.hist_dim) v = P.obs_history[(size_t)(e0 + e) * P.hist_ld + k];
    act_store1(va, k, e, v, &s_ovf);
    act_store1(vc, k, e,
               (e < ne && k >= P.hist_dim && k < P.hist_dim + NP)
                   ? P.privileged_obs[(size_t)(e0 + e) * NP + (k - P.hist_dim)] : v, &s_ovf);
  }
  __syncthreads();
  PSTAMP(1);
  const PolicyLayer* Ls = P.layers;
  const ActV vh1[2] = {h1[0].v(), h1[1].v()}, vh2[2] = {h2[0].v(), h2[1].v()};
  // adaptation module (xa rows >= hist_dim are still zero)
#ifndef GO1_POLICY_NO_EARLY
  policy_tiles<1, 1, PIN / 32, 4, true>(Ls + 0, &va, wave, PW, &vh1[0], true, lane, &s_ovf, w_ad);  // 256
#else
  policy_tiles<1, 1, PIN / 32, 4>(Ls + 0, &va, wave, PW, &vh1[0], true, lane, &s_ovf);  // 256
#endif
  __syncthreads();
  PSTAMP(2);
  // 256 -> 128: waves w and w + 8 take the two K halves of tile w & 7; the upper half's partial
  // goes through LDS (h2[1], free until the actor/critic's second layer)
  {
    float(*scr)[16][16] = reinterpret_cast<float(*)[16][16]>(&h2[1]);
    const int q = lane >> 4, c = lane & 15, t = wave & 7, half = wave >> 3;
    f4_t acc = tile_partial<4>(Ls[1], 8, t, 4 * half, vh1[0], lane);
    if (half) {
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[t][4 * q + r][c] = acc[r];
    }
    __syncthreads();
    if (!half) {
      const f4_t b = *reinterpret_cast<const f4_t*>(Ls[1].b + 16 * t + 4 * q);
      f4_t v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = elu((b[r] + acc[r]) + scr[t][4 * q + r][c]);
      act_store4(vh2[0], 4 * t + q, c, v, &s_ovf);
    }
  }
  __syncthreads();
  PSTAMP(3);
  // 128 -> num_priv (the latent): one K group per wave (4 waves), partials summed by wave 0
  {
    float(*scr)[16][16] = reinterpret_cast<float(*)[16][16]>(&h2[1]);
    const int q = lane >> 4, c = lane & 15;
    if (wave < 4) {
      const f4_t acc = tile_partial<1>(Ls[2], 4, 0, wave, vh2[0], lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[wave][4 * q + r][c] = acc[r];
    }
    __syncthreads();
    if (wave == 0 && q < 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 4 * q + r;  // latent feature f: also the actor's input hist_dim + f
        if (f < NP) {
          float l = Ls[2].b[f];
#pragma unroll
          for (int w = 0; w < 4; ++w) l += scr[w][f][c];
          act_store1(va, P.hist_dim + f, c, l, &s_ovf);
          if (c < ne && P.latent) P.latent[(size_t)(e0 + c) * NP + f] = l;
        }
      }
    }
  }
  __syncthreads();
  PSTAMP(4);
  // actor and critic, layer by layer; wave w takes tiles w, w + 16, ... of both nets
  const PolicyLayer LA1[2] = {Ls[3], Ls[7]}, LA2[2] = {Ls[4], Ls[8]};
  {
    const ActV s1[2] = {va, vc};
    policy_tiles<2, 2, PIN / 32, 2>(LA1, s1, wave, PW, vh1, true, lane, &s_ovf);  // 512
  }
  __syncthreads();
  PSTAMP(5);
  policy_tiles<1, 2, 512 / 32, 3>(LA2, vh1, wave, PW, vh2, true, lane, &s_ovf);  // 256
  __syncthreads();
  PSTAMP(6);
  {  // 256 -> 128, one tile per wave: waves 0-7 the actor's, 8-15 the critic's
    const bool critic = wave >= 8;
    const PolicyLayer L3 = critic ? Ls[9] : Ls[5];
    const ActV src = critic ? h2[1].v() : h2[0].v(), dst = critic ? h1[1].v() : h1[0].v();
    policy_tiles<1, 1, 256 / 32, 4>(&L3, &src, wave & 7, 8, &dst, true, lane, &s_ovf);
  }
  __syncthreads();
  PSTAMP(7);
  // 128 -> num_actions (actor, waves 0-3) and 128 -> 1 (critic, waves 8-11): one K group per
  // wave, partials through LDS (h2, free once the third layer has read it)
  {
    float(*scr)[16][16] = reinterpret_cast<float(*)[16][16]>(&h2[0]);
    const int q = lane >> 4, c = lane & 15;
    const bool critic = wave >= 8;
    if ((wave & 7) < 4) {
      const f4_t part = tile_partial<1>(Ls[critic ? 10 : 6], 4, 0, wave & 7, critic ? h1[1].v() : h1[0].v(), lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[wave][4 * q + r][c] = part[r];
    }
  }
  __syncthreads();
  if (wave < 2) {
    const int q = lane >> 4, c = lane & 15;
    const PolicyLayer L = Ls[wave == 0 ? 6 : 10];
    f4_t acc = *reinterpret_cast<const f4_t*>(L.b + 4 * q);
    {
      float(*scr)[16][16] = reinterpret_cast<float(*)[16][16]>(&h2[0]);
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += scr[8 * wave + w][4 * q + r][c];
    }
    if (wave == 0 && P.actions) {
      // Normal(mean, std).sample() and its log_prob summed over the actions
      // (actor_critic.py:137-145), Box-Muller on Philox4x32-10 uniforms keyed by
      // (global env, action group q, step): row q, element r is action f = 4 q + r of env c (normal4)
      float lp = 0.0f;
      f4_t a4, s4;
      float z4[4];
      normal4((uint32_t)(e0 + c + P.env_id_offset), q, P.rng_step, P.rng_seed, z4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 4 * q + r;
        const bool real = f < P.num_actions;
        const float sd = real ? P.std[f] : 1.0f;
        const float z = z4[r];
        a4[r] = acc[r] + sd * z;
        s4[r] = sd;
        if (real) lp += -0.5f * z * z - __logf(sd) - 0.91893853320467274f;  // log sqrt(2 pi)
      }
      // sum over the four rows (actions 0-3, 4-7, 8-11, 12-15 of the env)
      auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(lp), __float_as_uint(lp), false, false);
      lp = __uint_as_float(x[0]) + __uint_as_float(x[1]);
      auto y = __builtin_amdgcn_permlane32_swap(__float_as_uint(lp), __float_as_uint(lp), false, false);
      lp = __uint_as_float(y[0]) + __uint_as_float(y[1]);
      if (c < ne) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 4 * q + r;
          if (f < P.num_actions) {
            P.actions[(size_t)(e0 + c) * P.num_actions + f] = a4[r];
            P.action_sigma[(size_t)(e0 + c) * P.num_actions + f] = s4[r];
          }
        }
        if (q == 0) P.log_prob[e0 + c] = lp;
      }
    }
    if (c < ne) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 4 * q + r;
        if (wave == 0 && f < P.num_actions) P.action_mean[(size_t)(e0 + c) * P.num_actions + f] = acc[r];
        if (wave == 1 && f == 0) P.value[e0 + c] = acc[r];
      }
    }
  }
  PSTAMP(8);
  __syncthreads();
  if (s_ovf) policy_fallback(P, e0, ne, true, true, reinterpret_cast<float*>(&h1[0]));
}

// ---------------------------------------------------------------- per-net workgroups
// policy_kernel streams all 2.8 MB of split weights through every CU (each workgroup serves 16 envs
// with all three nets), the L2 -> CU floor of that decomposition.  Here a workgroup runs ONE net for
// 32 envs as two 16-env B tiles that share every weight fragment: the first ceil(n / 32)
// workgroups run the adaptation module + actor (1.6 MB), the others the critic (1.2 MB), so a CU
// streams at most 1.6 MB for twice the envs.  K order, tile split and partial-sum order are those
// of policy_kernel, so the outputs are identical.
// weight groups (32 K values) in flight per wave, the 512-wide first layers and the 256-wide second
// (16-deep groups, round 2: (4, 8), (6, 12), (8, 12), (8, 16) all within 1 %)
#ifndef GO1_SPLIT_D1
#define GO1_SPLIT_D1 3
#endif
#ifndef GO1_SPLIT_D2
#define GO1_SPLIT_D2 6
#endif

template <int NT, int NL, int ET>
__device__ __forceinline__ void policy_group_e(const f8_t (&w)[NL][NT], const ActV (*src)[NL], int g, int q, int c,
                                               f4_t (&acc)[ET][NL][NT]) {
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int et = 0; et < ET; ++et) {
      const h8_t xh = src[et][l].hi[(4 * g + q) * 16 + c], xl = src[et][l].lo[(4 * g + q) * 16 + c];
#pragma unroll
      for (int i = 0; i < NT; ++i) acc[et][l][i] = mfma3(w[l][i], xh, xl, acc[et][l][i]);
    }
}

template <int NT, int NL, int ET, int G, int D, bool PREFETCHED = false>
__device__ __forceinline__ void policy_tiles_e(const PolicyLayer* L, const ActV (*src)[NL], int tile0, int tstride,
                                               const ActV (*dst)[NL], bool act, int lane, int* ovf,
                                               f8_t (*pre)[NL][NT] = nullptr) {
  const int q = lane >> 4, c = lane & 15;
  f4_t acc[ET][NL][NT];
  f8_t w[D][NL][NT];
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const f4_t b = *reinterpret_cast<const f4_t*>(L[l].b + 16 * (tile0 + i * tstride) + 4 * q);
#pragma unroll
      for (int et = 0; et < ET; ++et) acc[et][l][i] = b;
    }
  if constexpr (PREFETCHED) {
#pragma unroll
    for (int g = 0; g < D; ++g)
#pragma unroll
      for (int l = 0; l < NL; ++l)
#pragma unroll
        for (int i = 0; i < NT; ++i) w[g][l][i] = pre[g][l][i];
  } else {
    policy_prefetch<NT, NL, G, D>(L, tile0, tstride, lane, w);
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    policy_group_e<NT, NL, ET>(w[g % D], src, g, q, c, acc);
    if (g + D < G) policy_load<NT, NL>(L, G, g + D, tile0, tstride, lane, w[g % D]);
  }
#pragma unroll
  for (int et = 0; et < ET; ++et)
#pragma unroll
    for (int l = 0; l < NL; ++l)
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        f4_t v = acc[et][l][i];
        if (act) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = elu(v[r]);
        }
        act_store4(dst[et][l], 4 * (tile0 + i * tstride) + q, c, v, ovf);
      }
}

// tile_partial for ET env tiles sharing the weight fragments
// the NG weight fragments of a tile_partial_e, loaded ahead (they depend on nothing the workgroup computes)
template <int NG>
__device__ __forceinline__ void partial_load(const PolicyLayer& L, int Gs, int tile, int g0, int lane, f8_t (&w)[NG]) {
#pragma unroll
  for (int i = 0; i < NG; ++i) w[i] = reinterpret_cast<const f8_t*>(L.w)[((size_t)tile * Gs + g0 + i) * 64 + lane];
}

template <int NG, int ET>
__device__ __forceinline__ void tile_partial_e(const PolicyLayer& L, int Gs, int tile, int g0, const ActV* src, int lane,
                                               f4_t (&acc)[ET], const f8_t* pre = nullptr) {
  const int q = lane >> 4, c = lane & 15;
  f8_t w[NG];
  if (pre) {
#pragma unroll
    for (int i = 0; i < NG; ++i) w[i] = pre[i];
  } else {
    partial_load<NG>(L, Gs, tile, g0, lane, w);
  }
#pragma unroll
  for (int et = 0; et < ET; ++et) acc[et] = f4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < NG; ++i)
#pragma unroll
    for (int et = 0; et < ET; ++et)
      acc[et] = mfma3(w[i], src[et].hi[(4 * (g0 + i) + q) * 16 + c], src[et].lo[(4 * (g0 + i) + q) * 16 + c], acc[et]);
}

// LDS of policy_kernel_split: three env tiles of inputs and of 512-wide outputs.  Aliases (each used only
// after a barrier that ends the previous use): the 256-wide L2 outputs live in the input planes (dead once
// L1 has run); the adaptation module's L2 outputs in rows 256-383 of h1 (its L1 outputs hold rows 0-255)
// and its K-split partials in rows 384-511; the output layer's partials in the input planes.
struct SplitLds {
  Act<PIN> xin[3];
  Act<512> h1[3];
};
typedef float Scr[4][16][16];  // the output layer's K-split partials of one env tile

// Workgroup barrier over LDS only: waits for this wave's LDS operations, not for its global loads, so
// weight fragments requested ahead of a barrier stay in flight across it (__syncthreads' release fence
// waits for every memory operation).  policy_kernel_split never reads global memory it writes.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int ET, bool CRITIC>
__device__ __forceinline__ void split_body(const go1_policy_args& P, SplitLds& S, int e0, int ne, int* s_ovf) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int q = lane >> 4, c = lane & 15;
  const int NP = P.num_priv;
  ActV vx[ET][1], v1[ET][1], v2[ET][1];
#pragma unroll
  for (int et = 0; et < ET; ++et) {
    vx[et][0] = S.xin[et].v();
    v1[et][0] = S.h1[et].v();
    v2[et][0] = S.xin[et].v();  // L2 outputs over the dead inputs
  }
  // Every layer's first weight fragments are requested before the barrier that ends the previous phase
  // (they depend on nothing the workgroup computes), so a layer starts with its weights landed instead
  // of one L2 round trip after the barrier.
  const PolicyLayer* Ls = P.layers;
  const PolicyLayer* LN = Ls + (CRITIC ? 7 : 3);
  // First layers, K-streamed in chunks of CG groups (PIN inputs) through the input planes: the adaptation
  // module's L1 over the history (GA groups), the actor's / critic's L1 over [history, latent | priv] (GL
  // groups).  The actor's groups from gl = H / 32 on hold latent inputs: they run after the adaptation
  // module, from the last chunk's planes (the host guarantees they lie in it).  One chunk when the inputs
  // fit PIN (the README configuration); the velocity task's 30-deep history (2,100) takes eight.
  const int H = P.hist_dim, KIN = H + NP;
  const int GA = (H + 31) / 32, GL = (KIN + 31) / 32, gl = H / 32;
  constexpr int CG = PIN / 32;
  const int nch = (GL + CG - 1) / CG, g_last = CG * (nch - 1);
  const int g_pass = CRITIC ? GL : gl;  // L1 groups of the chunk pass
  // the f32 staging copy (h1 is free until the L1 epilogue); one chunk: the workgroup's rows are one
  // contiguous block of ne x H floats, copied with coalesced loads from one base pointer (all of the
  // thread's in flight) before the accumulators are live
  float* flat = reinterpret_cast<float*>(&S.h1[0]);
  const int fs = nch == 1 ? H : PIN;
  // L1 weight fragments, two groups ahead (two register sets, the group loop unrolled by two)
  f8_t wA0, wL00, wL01, wA1, wL10, wL11;
  auto load0 = [&](int g) {
    if constexpr (!CRITIC) wA0 = reinterpret_cast<const f8_t*>(Ls[0].w)[((size_t)wave * GA + g) * 64 + lane];
    wL00 = reinterpret_cast<const f8_t*>(LN[0].w)[((size_t)wave * GL + g) * 64 + lane];
    wL01 = reinterpret_cast<const f8_t*>(LN[0].w)[((size_t)(wave + PW) * GL + g) * 64 + lane];
  };
  auto load1 = [&](int g) {
    if constexpr (!CRITIC) wA1 = reinterpret_cast<const f8_t*>(Ls[0].w)[((size_t)wave * GA + g) * 64 + lane];
    wL10 = reinterpret_cast<const f8_t*>(LN[0].w)[((size_t)wave * GL + g) * 64 + lane];
    wL11 = reinterpret_cast<const f8_t*>(LN[0].w)[((size_t)(wave + PW) * GL + g) * 64 + lane];
  };
  // the first chunk's first two groups are requested before the inputs: they depend on nothing the workgroup
  // computes, so the weight stream starts under the input loads' latency instead of after the staging
#ifndef GO1_POLICY_L1_EARLY
#define GO1_POLICY_L1_EARLY 1
#endif
  if (GO1_POLICY_L1_EARLY) {
    const int gb0 = CRITIC ? min(CG, GL) : min(gl, min(CG, GL));
    if (0 < gb0) load0(0);
    if (1 < gb0) load1(1);
#if GO1_POLICY_SCHED
    __builtin_amdgcn_sched_barrier(0);
#endif
  }
  if (nch == 1) {
    constexpr int NI = (ET * 16 * PIN + 64 * PW - 1) / (64 * PW);
    const int64_t LD = P.hist_ld;
    const float* src = P.obs_history + (size_t)e0 * LD;
    const int total = ne * H;
    float v[NI];
    // unconditional loads at clamped indices: a load under a condition is waited for right after it is
    // issued (one HBM round trip per load instead of one for all)
    if (LD == H) {
#pragma unroll
      for (int i = 0; i < NI; ++i) v[i] = src[min(tid + i * 64 * PW, total - 1)];
    } else {  // rows of a wider buffer (row-strided window)
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = min(tid + i * 64 * PW, total - 1), r = j / H;
        v[i] = src[(size_t)r * LD + (j - r * H)];
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = tid + i * 64 * PW;
      if (j < total) flat[j] = v[i];
    }
    PSTAMP(9);
  }
  // the critic's privileged inputs into LDS behind the f32 copy (one clamped load per thread; the split
  // passes read them from there)
  float* pflat = flat + ET * 16 * PIN;
  static_assert(ET * 16 * (PIN + 8) * sizeof(float) <= sizeof(SplitLds::h1), "f32 staging exceeds h1");
  if constexpr (CRITIC) {
    const int t = min(tid, ET * 16 * NP - 1), e = t / NP;
    const float x = P.privileged_obs[(size_t)(e0 + min(e, ne - 1)) * NP + (t - e * NP)];
    if (tid < ET * 16 * NP) pflat[tid] = x;
  }
  f4_t accA[ET], accL[ET][2];
  {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f4_t b = *reinterpret_cast<const f4_t*>(LN[0].b + 16 * (wave + i * PW) + 4 * q);
#pragma unroll
      for (int et = 0; et < ET; ++et) accL[et][i] = b;
    }
    if constexpr (!CRITIC) {
      const f4_t b = *reinterpret_cast<const f4_t*>(Ls[0].b + 16 * wave + 4 * q);
#pragma unroll
      for (int et = 0; et < ET; ++et) accA[et] = b;
    }
  }
  for (int ch = 0; ch < nch; ++ch) {
    const int g0 = CG * ch, k0 = 32 * g0;
    // inputs of the chunk, in two passes through LDS: coalesced loads of each env's window (all of the
    // thread's in flight) into a flat f32 copy; then each lane splits eight consecutive features of one
    // env into one 16-byte record per plane, the lanes of a wave filling consecutive records
    // (element-wise split stores hit the same LDS banks 8-16 times over)
    // the f32 copy holds the history part of the chunk: rows of fs floats (one chunk: copied above)
    if (nch > 1) {
      // thread -> (env, column phase): TPE threads per env row, one row pointer per thread (per-element
      // addresses would be hoisted out of the chunk loop and spill)
      constexpr int TPE = (64 * PW) / (ET * 16), NI = (PIN + TPE - 1) / TPE;
      const int e = tid / TPE, kk = tid - e * TPE;
      const bool live = e < ET * 16;
      const bool row = live && e < ne;
      const float* src = P.obs_history + (size_t)(e0 + (row ? e : 0)) * P.hist_ld;
      float v[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {  // unconditional loads (index clamped), then the mask
        const int kc = kk + TPE * i, k = k0 + kc;
        const float x = src[min(k, H - 1)];
        v[i] = (row && kc < PIN && k < H) ? x : 0.0f;
      }
      if (live) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int kc = kk + TPE * i;
          if (kc < PIN) flat[e * PIN + kc] = v[i];
        }
      }
    }
    lds_barrier();
    if (ch == 0) PSTAMP(10);
    {
      constexpr int NC = PIN / 8, NTASK = ET * 16 * NC;
      for (int t = tid; t < NTASK; t += 64 * PW) {
        const int c = t & 15, rest = t >> 4, kc = rest % NC, et = rest / NC, e = 16 * et + c;
        h8_t hi8, lo8;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int kl = 8 * kc + r, k = k0 + kl;
          float x = 0.0f;
          if (e < ne) {
            if (k < H) x = flat[e * fs + kl];
            else if (CRITIC && k < KIN) x = pflat[e * NP + (k - H)];
          }
          ovf_check(x, s_ovf);
          hi8[r] = (_Float16)x;
          lo8[r] = (_Float16)(x - (float)hi8[r]);
        }
        S.xin[et].hi[kc][c] = hi8;
        S.xin[et].lo[kc][c] = lo8;
      }
    }
    lds_barrier();
    if (ch == 0) PSTAMP(1);
    // the chunk's groups (uniform runtime bounds, no predicated MFMAs): [g0, gb) feed the adaptation
    // module (actor) and L1; the next group's fragments are requested before this group's MFMAs
    {
      const int g1 = min(g0 + CG, GL), gb = CRITIC ? g1 : min(gl, g1);
      auto group = [&](int gi, const f8_t& a, const f8_t& l0, const f8_t& l1) {
#pragma unroll
        for (int et = 0; et < ET; ++et) {
          const h8_t xh = S.xin[et].hi[4 * gi + q][c], xl = S.xin[et].lo[4 * gi + q][c];
          if constexpr (!CRITIC) accA[et] = mfma3(a, xh, xl, accA[et]);
          accL[et][0] = mfma3(l0, xh, xl, accL[et][0]);
          accL[et][1] = mfma3(l1, xh, xl, accL[et][1]);
        }
      };
      if (ch > 0 || !GO1_POLICY_L1_EARLY) {  // the first chunk's were requested before the staging
        if (g0 < gb) load0(g0);
        if (g0 + 1 < gb) load1(g0 + 1);
      }
      for (int g = g0; g < gb; g += 2) {
        group(g - g0, wA0, wL00, wL01);
        if (g + 2 < gb) load0(g + 2);
        if (g + 1 < gb) {
          group(g + 1 - g0, wA1, wL10, wL11);
          if (g + 3 < gb) load1(g + 3);
        }
      }
      if constexpr (!CRITIC) {  // the history's last, partial group (adaptation module only; the actor's
        if (GA > gl && gl >= g0 && gl < g1) {  // L1 takes it with the latent)
          const f8_t a = reinterpret_cast<const f8_t*>(Ls[0].w)[((size_t)wave * GA + gl) * 64 + lane];
#pragma unroll
          for (int et = 0; et < ET; ++et)
            accA[et] = mfma3(a, S.xin[et].hi[4 * (gl - g0) + q][c], S.xin[et].lo[4 * (gl - g0) + q][c], accA[et]);
        }
      }
    }
    if (ch + 1 < nch) lds_barrier();  // the next chunk's staging overwrites the planes and the copy
  }
  // no barrier: the copy in h1 was last read before the last chunk's MFMAs (every wave has passed that
  // barrier), so each wave stores its first-layer outputs as soon as its own MFMAs are done, overlapping the
  // other waves' MFMAs (a barrier here made every wave run its ELUs at the same time)
  if constexpr (!CRITIC) {
    // adaptation module epilogue: ELU, split into h1 rows 0-255
#pragma unroll
    for (int et = 0; et < ET; ++et) {
      f4_t v = accA[et];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = elu(v[r]);
      act_store4(v1[et][0], 4 * wave + q, c, v, s_ovf);
    }
    // K-split partials of the adaptation module: 16 x 16 blocks in rows 384-511 of h1 (block t < 4 in
    // the hi plane, t >= 4 in the lo plane), free until the actor's L1 epilogue
    auto blk = [&](int et, int t) -> float(*)[16] {
      return reinterpret_cast<float(*)[16]>(t < 4 ? &S.h1[et].hi[384 / 8][0] : &S.h1[et].lo[384 / 8][0]) + 16 * (t & 3);
    };
    ActV va2[ET];  // adaptation L2 outputs: rows 256-383 of h1
#pragma unroll
    for (int et = 0; et < ET; ++et) va2[et] = ActV{&S.h1[et].hi[256 / 8][0], &S.h1[et].lo[256 / 8][0]};
    f8_t pa2[4];
    partial_load<4>(Ls[1], 8, wave & 7, 4 * (wave >> 3), lane, pa2);
    lds_barrier();
    PSTAMP(2);
    f8_t pa3[1];
    if (wave < 4) partial_load<1>(Ls[2], 4, 0, wave, lane, pa3);
    {  // 256 -> 128: waves w and w + 8 take the two K halves of tile w & 7
      const int t = wave & 7, half = wave >> 3;
      ActV src[ET];
#pragma unroll
      for (int et = 0; et < ET; ++et) src[et] = v1[et][0];
      f4_t acc[ET];
      tile_partial_e<4, ET>(Ls[1], 8, t, 4 * half, src, lane, acc, pa2);
      if (half) {
#pragma unroll
        for (int et = 0; et < ET; ++et)
#pragma unroll
          for (int r = 0; r < 4; ++r) blk(et, t)[4 * q + r][c] = acc[et][r];
      }
      lds_barrier();
      if (!half) {
        const f4_t b = *reinterpret_cast<const f4_t*>(Ls[1].b + 16 * t + 4 * q);
#pragma unroll
        for (int et = 0; et < ET; ++et) {
          f4_t v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = elu((b[r] + acc[et][r]) + blk(et, t)[4 * q + r][c]);
          act_store4(va2[et], 4 * t + q, c, v, s_ovf);
        }
      }
    }
    lds_barrier();
    PSTAMP(3);
    {  // 128 -> num_priv (the latent): one K group per wave (4 waves), partials summed by waves 0 .. ET-1
      if (wave < 4) {
        f4_t acc[ET];
        tile_partial_e<1, ET>(Ls[2], 4, 0, wave, va2, lane, acc, pa3);
#pragma unroll
        for (int et = 0; et < ET; ++et)
#pragma unroll
          for (int r = 0; r < 4; ++r) blk(et, wave)[4 * q + r][c] = acc[et][r];
      }
      lds_barrier();
      if (wave < ET && q < 2) {
        const int et = wave, e = 16 * et + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 4 * q + r;
          if (f < NP) {
            float l = Ls[2].b[f];
#pragma unroll
            for (int w = 0; w < 4; ++w) l += blk(et, w)[f][c];
            act_store1(S.xin[et].v(), H + f - 32 * g_last, c, l, s_ovf);  // the last chunk's planes
            if (e < ne && P.latent) P.latent[(size_t)(e0 + e) * NP + f] = l;
          }
        }
      }
    }
    lds_barrier();
    PSTAMP(4);
    // the actor's L1 groups that hold the latent
    for (int g = gl; g < GL; ++g) {
      const int gi = g - g_last;
      f8_t w[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) w[i] = reinterpret_cast<const f8_t*>(LN[0].w)[((size_t)(wave + i * PW) * GL + g) * 64 + lane];
#pragma unroll
      for (int et = 0; et < ET; ++et) {
        const h8_t xh = S.xin[et].hi[4 * gi + q][c], xl = S.xin[et].lo[4 * gi + q][c];
#pragma unroll
        for (int i = 0; i < 2; ++i) accL[et][i] = mfma3(w[i], xh, xl, accL[et][i]);
      }
    }
  } else {
    PSTAMP(2);
    PSTAMP(3);
    PSTAMP(4);
  }
  // actor (Ls 3-6) or critic (Ls 7-10), layer by layer; L1 epilogue: ELU, split into h1
#pragma unroll
  for (int et = 0; et < ET; ++et)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f4_t v = accL[et][i];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = elu(v[r]);
      act_store4(v1[et][0], 4 * (wave + i * PW) + q, c, v, s_ovf);
    }
  f8_t pl2[GO1_SPLIT_D2][1][1];
  policy_prefetch<1, 1, 512 / 32, GO1_SPLIT_D2>(LN + 1, wave, PW, lane, pl2);
  lds_barrier();
  PSTAMP(5);
  policy_tiles_e<1, 1, ET, 512 / 32, GO1_SPLIT_D2, true>(LN + 1, v1, wave, PW, v2, true, lane, s_ovf, pl2);  // 256
  f8_t pl3[4][1][1];
  if (wave < 8) policy_prefetch<1, 1, 256 / 32, 4>(LN + 2, wave, 8, lane, pl3);
  lds_barrier();
  PSTAMP(6);
  f8_t pl4[1];
  if (wave < 4) partial_load<1>(LN[3], 4, 0, wave, lane, pl4);
  if (wave < 8) policy_tiles_e<1, 1, ET, 256 / 32, 4, true>(LN + 2, v2, wave, 8, v1, true, lane, s_ovf, pl3);  // 128 -> h1
  lds_barrier();
  PSTAMP(7);
  // 128 -> num_actions / 1: one K group per wave, partials through LDS (the inputs' planes, dead now)
  Scr* scr = reinterpret_cast<Scr*>(&S.xin[0]);  // [et], over the dead input planes
  if (wave < 4) {
    ActV src[ET];
#pragma unroll
    for (int et = 0; et < ET; ++et) src[et] = v1[et][0];
    f4_t part[ET];
    tile_partial_e<1, ET>(LN[3], 4, 0, wave, src, lane, part, pl4);
#pragma unroll
    for (int et = 0; et < ET; ++et)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[et][wave][4 * q + r][c] = part[et][r];
  }
  lds_barrier();
  if (wave < ET) {
    const int et = wave, e = 16 * et + c;
    f4_t acc = *reinterpret_cast<const f4_t*>(LN[3].b + 4 * q);
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += scr[et][w][4 * q + r][c];
    if constexpr (!CRITIC) {
      if (P.actions) {
        float lp = 0.0f;
        f4_t a4, s4;
        float z4[4];
        normal4((uint32_t)(e0 + e + P.env_id_offset), q, P.rng_step, P.rng_seed, z4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 4 * q + r;
          const bool real = f < P.num_actions;
          const float sd = real ? P.std[f] : 1.0f;
          const float z = z4[r];
          a4[r] = acc[r] + sd * z;
          s4[r] = sd;
          if (real) lp += -0.5f * z * z - __logf(sd) - 0.91893853320467274f;  // log sqrt(2 pi)
        }
        auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(lp), __float_as_uint(lp), false, false);
        lp = __uint_as_float(x[0]) + __uint_as_float(x[1]);
        auto y = __builtin_amdgcn_permlane32_swap(__float_as_uint(lp), __float_as_uint(lp), false, false);
        lp = __uint_as_float(y[0]) + __uint_as_float(y[1]);
        if (e < ne) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int f = 4 * q + r;
            if (f < P.num_actions) {
              P.actions[(size_t)(e0 + e) * P.num_actions + f] = a4[r];
              P.action_sigma[(size_t)(e0 + e) * P.num_actions + f] = s4[r];
            }
          }
          if (q == 0) P.log_prob[e0 + e] = lp;
        }
      }
      if (e < ne) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 4 * q + r;
          if (f < P.num_actions) P.action_mean[(size_t)(e0 + e) * P.num_actions + f] = acc[r];
        }
      }
    } else if (e < ne && q == 0) {
      P.value[e0 + e] = acc[0];
    }
  }
  PSTAMP(8);
  __syncthreads();
  if (*s_ovf) policy_fallback(P, e0, ne, !CRITIC, CRITIC, reinterpret_cast<float*>(&S.h1[0]));
}

// envs per workgroup: actor workgroups (adaptation module + actor, 1.6 MB of split weights) take SPLIT_ET_A
// env tiles, critic workgroups (1.2 MB) SPLIT_ET_C, so the two kinds take about as long (4096 envs: actor
// 65.8 k / critic 58.5 k cycles; with 3 + 3 tiles the actor workgroups grew to 84 k: 39 against 32.5 us)
#ifndef GO1_SPLIT_ET_A
#define GO1_SPLIT_ET_A 2
#endif
#ifndef GO1_SPLIT_ET_C
#define GO1_SPLIT_ET_C 3
#endif
constexpr int SE_A = 16 * GO1_SPLIT_ET_A, SE_C = 16 * GO1_SPLIT_ET_C;

__global__ __launch_bounds__(64 * PW) void policy_kernel_split(go1_policy_args P) {
  __shared__ SplitLds S;
  __shared__ int s_ovf;
  PSTAMP(0);
  if (threadIdx.x == 0) s_ovf = 0;
  const int na = (P.n_envs + SE_A - 1) / SE_A;
  if ((int)blockIdx.x < na) {
    const int e0 = blockIdx.x * SE_A;
    split_body<GO1_SPLIT_ET_A, false>(P, S, e0, min(SE_A, P.n_envs - e0), &s_ovf);
  } else {
    const int e0 = (blockIdx.x - na) * SE_C;
    split_body<GO1_SPLIT_ET_C, true>(P, S, e0, min(SE_C, P.n_envs - e0), &s_ovf);
  }
}

}  // namespace

// ------------------------------------------------------------------ column sums (bias gradients)
// out[c] = sum_r x[r][c] of a row-major (R, C) f32 matrix, deterministic: pass 1 sums row partition p of 64
// columns per workgroup (4 row groups x 64 columns, each lane a fixed stride-4 row order, the 4 groups added
// in order through LDS) into partial[p][c]; pass 2 adds the partitions in order.  The PPO update's bias
// gradients (dL/db = column sums of dL/dy over the 24,576-sample mini-batch): torch's sum(0) takes 18-24 us
// for 24,576 x 512 (tools/reduce_bench.py), 2-3x the HBM time of the 50 MB it reads.
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ x, int64_t R, int C, int64_t RP,
                                                          float* __restrict__ partial) {
  __shared__ float s[4][64];
  const int t = threadIdx.x, cl = t & 63, rg = t >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int64_t r0 = (int64_t)blockIdx.y * RP, r1 = r0 + RP < R ? r0 + RP : R;
  float acc = 0.0f;
  if (c < C) {
    // eight rows in flight per lane (independent loads), added in row order
    int64_t r = r0 + rg;
    for (; r + 28 < r1; r += 32) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = x[(r + 4 * k) * C + c];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
    for (; r < r1; r += 4) acc += x[r * C + c];
  }
  s[rg][cl] = acc;
  __syncthreads();
  if (rg == 0 && c < C) partial[(int64_t)blockIdx.y * C + c] = ((s[0][cl] + s[1][cl]) + s[2][cl]) + s[3][cl];
}
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ partial, int P, int C,
                                                           float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float acc = 0.0f;
  int p = 0;
  for (; p + 8 <= P; p += 8) {  // eight partitions in flight, added in order
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = partial[(int64_t)(p + k) * C + c];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  for (; p < P; ++p) acc += partial[(int64_t)p * C + c];
  out[c] = acc;
}

extern "C" {

#ifdef GO1_POLICY_STAMPS
int go1_policy_stamps(void* host, size_t bytes) {
  if (bytes > sizeof(g_pstamps)) bytes = sizeof(g_pstamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pstamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

const char* go1_rollout_last_error(void) { return g_err.c_str(); }

int go1_record_transition(const go1_transition* tr, int32_t n_envs, float gamma, void* stream) {
  if (!tr || n_envs <= 0) return fail(GO1_RT_E_ARG, "go1_record_transition: bad argument");
  if (!tr->rewards || !tr->dones || !tr->values || !tr->st_rewards || !tr->st_dones || !tr->st_values)
    return fail(GO1_RT_E_ARG, "go1_record_transition: rewards / dones / values are required");
  if (tr->obs_history && tr->obs_history_ld != 0 && tr->obs_history_ld < tr->num_obs_history)
    return fail(GO1_RT_E_ARG, "go1_record_transition: obs_history_ld < num_obs_history");
  go1_transition T = *tr;
  if (T.obs_history_ld == 0) T.obs_history_ld = T.num_obs_history;
  {  // the flat form when every buffer is 16-byte aligned and the history contiguous
    const Seg segs[7] = {{T.obs, T.st_obs, (int64_t)n_envs * T.num_obs},
                         {T.privileged_obs, T.st_privileged_obs, (int64_t)n_envs * T.num_priv},
                         {T.obs_history, T.st_obs_history, (int64_t)n_envs * T.num_obs_history},
                         {T.actions, T.st_actions, (int64_t)n_envs * T.num_actions},
                         {T.mu, T.st_mu, (int64_t)n_envs * T.num_actions},
                         {T.sigma, T.st_sigma, (int64_t)n_envs * T.num_actions},
                         {T.actions_log_prob, T.st_actions_log_prob, (int64_t)n_envs}};
    const char* fe = std::getenv("GO1_RECORD_FLAT");  // "0": the segment-walking kernel (A/B)
    bool flat = T.obs_history_ld == T.num_obs_history && !(fe && fe[0] == '0');
    for (int i = 0; i < 7; ++i)
      if (segs[i].src && segs[i].n > 0)
        flat = flat && ((((uintptr_t)segs[i].src) | ((uintptr_t)segs[i].dst)) & 15) == 0;
    if (flat) {
      RecPlan P;
      memset(&P, 0, sizeof(P));
      const bool alias = T.obs && T.obs_history == T.obs && T.num_obs == T.num_obs_history;
      int blk = 0;
      for (int i = 0; i < 7; ++i) {
        if (!segs[i].src || segs[i].n <= 0 || (i == 2 && alias)) continue;
        const int s = P.nseg++;
        P.src[s] = reinterpret_cast<const float4*>(segs[i].src);
        P.dst[s] = reinterpret_cast<float4*>(segs[i].dst);
        P.dst2[s] = (i == 0 && alias) ? reinterpret_cast<float4*>(T.st_obs_history) : nullptr;
        P.nf[s] = segs[i].n;
        P.first[s] = blk;
        blk += (int)std::max<int64_t>(1, ((segs[i].n >> 2) + 255) / 256);
      }
      P.first[P.nseg] = blk;
      blk += (n_envs + 255) / 256;
      hipLaunchKernelGGL(record_flat_kernel, dim3(blk), dim3(256), 0, (hipStream_t)stream, P, T, n_envs, gamma);
      RT_TRY(hipGetLastError());
      return GO1_OK_RT;
    }
  }
  int64_t big = (int64_t)n_envs * (tr->num_obs + tr->num_obs_history);
  int blocks = (int)((big / 4 + 255) / 256);
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(record_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, T, n_envs, gamma);
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

int go1_policy_forward(const go1_policy_args* args, void* stream) {
  if (!args || args->n_envs <= 0 || !args->obs_history || !args->privileged_obs || !args->action_mean ||
      !args->value)
    return fail(GO1_RT_E_ARG, "go1_policy_forward: bad argument");
  if (args->num_priv < 1 || args->num_priv > 8 || args->hist_dim < 1 || args->num_actions > 16)
    return fail(GO1_RT_E_ARG, "go1_policy_forward: input / latent / action width outside the compiled architecture");
  {
    // variant 1 stages all inputs at once (PIN); variant 0 streams them in chunks of PIN, and the actor's
    // groups that hold the latent must lie in the last chunk (its planes receive the latent)
    const int kin = args->hist_dim + args->num_priv, gl = args->hist_dim / 32, GL = (kin + 31) / 32;
    const int g_last = (PIN / 32) * ((GL + PIN / 32 - 1) / (PIN / 32) - 1);
    // variant 1 stages all inputs at once (kin <= PIN) and walks PIN / 32 K groups of the packed first layers
    // (compile-time G): the packing (ceil(k / 32) groups per output tile) must have exactly that many, or its
    // reads leave the buffer.  Together: 257 <= hist_dim <= 288 - num_priv.
    if (args->variant == 1 && (kin > PIN || (args->hist_dim + 31) / 32 != PIN / 32))
      return fail(GO1_RT_E_ARG, "go1_policy_forward: variant 1 needs hist_dim in 257.." +
                                    std::to_string(PIN - args->num_priv) + " (288 - num_priv; 9 packed K groups), got " +
                                    std::to_string(args->hist_dim));
    if (gl < g_last || kin > 16384)
      return fail(GO1_RT_E_ARG, "go1_policy_forward: history width not supported by the chunked first layers");
  }
  for (int i = 0; i < GO1_POLICY_LAYERS; ++i)
    if (!args->layers[i].w || !args->layers[i].b || !args->layers[i].wf)
      return fail(GO1_RT_E_ARG, "go1_policy_forward: missing layer (split, bias and f32 weights are required)");
  if (args->variant != 0 && args->variant != 1) return fail(GO1_RT_E_ARG, "go1_policy_forward: variant");
  if (args->hist_ld != 0 && args->hist_ld < args->hist_dim)
    return fail(GO1_RT_E_ARG, "go1_policy_forward: hist_ld < hist_dim");
  go1_policy_args P = *args;
  if (P.hist_ld == 0) P.hist_ld = P.hist_dim;
  if (P.variant == 0)
    hipLaunchKernelGGL(policy_kernel_split, dim3((P.n_envs + SE_A - 1) / SE_A + (P.n_envs + SE_C - 1) / SE_C),
                       dim3(64 * PW), 0, (hipStream_t)stream, P);
  else
    hipLaunchKernelGGL(policy_kernel, dim3((P.n_envs + 15) / 16), dim3(64 * PW), 0, (hipStream_t)stream, P);
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

int go1_colsum(const float* x, int64_t rows, int32_t cols, float* partial, int32_t parts, float* out, void* stream) {
  if (!x || !partial || !out || rows < 1 || cols < 1 || parts < 1 || parts > 65535 || parts > rows)
    return fail(GO1_RT_E_ARG, "go1_colsum: bad argument");
  const int64_t rp = (rows + parts - 1) / parts;
  hipLaunchKernelGGL(colsum_part_kernel, dim3((unsigned)((cols + 63) / 64), (unsigned)parts), dim3(256), 0,
                     (hipStream_t)stream, x, rows, cols, rp, partial);
  RT_TRY(hipGetLastError());
  hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     partial, parts, cols, out);
  RT_TRY(hipGetLastError());
  return GO1_OK_RT;
}

}  // extern "C"
