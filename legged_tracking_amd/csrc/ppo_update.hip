// ppo_update.hip -- the PPO update (go1_gym_learn/ppo_cse/ppo.py:98-206) as hand-written HIP for MI355X
// (gfx950).  C ABI in include/go1_ppo.h; host mirror legged_tracking_amd/rollout.py (PPO.update).
//
// One mini-batch of PPO.update is a fixed chain of launches (go1_ppo_grad / go1_ppo_step), every one of them
// stream-ordered and graph-capturable:
//
//   phase 0 (ppo.py:107-159)                                  phase 1 (ppo.py:169-198)
//   xw<F>   adaptation L1  hist(gathered) -> a1a (256)        xw<F>   adaptation L1 (new weights) -> a1a
//   xw<F>   adaptation L2  a1a -> a2a (128)                   xw<F>   adaptation L2 -> a2a
//   adapt<FWD>  adaptation L3  a2a -> latent (priv)           adapt<MSE>  L3, mse loss vs privileged_obs on the
//   xw<F>   actor L1 [hist, latent], critic L1 [hist, priv]               first 4/5 of the rows, backward to a2a
//   xw<F>   actor / critic L2, L3                             xw<D>   delta a1a
//   head    actor L4 + critic L4, log-prob, ratio, clipped    wgrad   adaptation L1, L2 weight gradients
//           surrogate, clipped value loss, KL, entropy        reduce  -> grads (adaptation slice), aux
//           gradient; backward through L4 -> delta a3         finalize, adam (adaptation optimizer), pack
//   xw<D>   delta a2 (= W3^T delta3 * ELU'), delta a1
//   adapt<BWD> d latent = W1[:, hist:]^T delta1, backward through adaptation L3 -> delta a2a
//   xw<D>   delta a1a
//   wgrad   every weight gradient of the GEMM layers (one grouped launch, split over row chunks)
//   reduce  partials -> flat gradient (+ loss / KL sums); [all-reduce at world > 1]
//   norm, finalize (KL -> learning rate, clip_grad_norm_), adam (all parameters), pack
//
// GEMMs ("xw": activations x weights^T, "wgrad": delta^T x activations) run on v_mfma_f32_16x16x32_f16 with
// f32 accuracy from the 3xF16 split (hi = f16(x), lo = f16(x - hi), products hi*hi + hi*lo + lo*hi, f32
// accumulation; the dropped lo*lo term is ~2^-22 of a product).  Every operand tensor is first scaled by an
// exact power of two that puts its largest magnitude in [2^14, 2^15): f16's range is then never left, and the
// lo halves stay normal for every element within 2^17 of the tensor's maximum (gradients of a mean over
// 24,576 samples are ~1e-5..1e-8: unscaled they would fall into f16's subnormals).  Producers record max |x|
// (one atomicMax per wave); consumers derive the scale from it; the product is unscaled in the epilogue.
// Weights are split once per optimiser step into fragment images (forward and transposed) by the pack kernel.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <string>

#include "../../include/go1_ppo.h"

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}
#define PPO_TRY(x)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) return fail(GO1_PPO_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

typedef float f4_t __attribute__((ext_vector_type(4)));
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef __fp16 hp2_t __attribute__((ext_vector_type(2)));

constexpr int TB = 128;      // GEMM tile: 128 rows x 128 features per workgroup (4 waves of 64 x 64)
constexpr int HA1 = GO1_PPO_HA1, HA2 = GO1_PPO_HA2, H1 = GO1_PPO_H1, H2 = GO1_PPO_H2, H3 = GO1_PPO_H3;
constexpr int NAUX = GO1_PPO_AUX;
constexpr int NORM_BLOCKS = 256;

// ------------------------------------------------------------------ scaling and the 3xF16 split
// max |x| is tracked as the bit pattern of a non-negative float (ordered like an unsigned int; a NaN's bits
// exceed inf's, so a NaN operand disables the scaling and propagates).  scale exponent: max * 2^e in [2^14, 2^15).
__device__ __forceinline__ int scale_exp(uint32_t bits) {
  if (bits == 0u || bits >= 0x7f800000u) return 0;
  const int ef = (int)(bits >> 23);
  const int e = ef ? ef - 127 : (31 - __clz((int)bits)) - 149;
  const int s = 14 - e;
  return s < -126 ? -126 : (s > 126 ? 126 : s);
}
__device__ __forceinline__ float pow2f(int e) { return __int_as_float((e + 127) << 23); }  // e in [-126, 127]

__device__ __forceinline__ uint32_t absbits(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// x * s split into f16 hi / lo halves.  hi rounds toward zero (v_cvt_pkrtz: one instruction per pair), so
// x - hi is exact and |lo| < ulp16(hi); lo rounds toward zero too: |x - hi - lo| < 2^-21 |x|.
__device__ __forceinline__ void split4(f4_t v, float s, h4_t& hi, h4_t& lo) {
  v *= s;
  const hp2_t h01 = __builtin_amdgcn_cvt_pkrtz(v[0], v[1]);
  const hp2_t h23 = __builtin_amdgcn_cvt_pkrtz(v[2], v[3]);
  const hp2_t l01 = __builtin_amdgcn_cvt_pkrtz(v[0] - (float)h01[0], v[1] - (float)h01[1]);
  const hp2_t l23 = __builtin_amdgcn_cvt_pkrtz(v[2] - (float)h23[0], v[3] - (float)h23[1]);
  hi = __builtin_bit_cast(h4_t, __builtin_shufflevector(h01, h23, 0, 1, 2, 3));
  lo = __builtin_bit_cast(h4_t, __builtin_shufflevector(l01, l23, 0, 1, 2, 3));
}

__device__ __forceinline__ f4_t mfma3(h8_t wh, h8_t wl, h8_t xh, h8_t xl, f4_t acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xh, acc, 0, 0, 0);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ELU (alpha = 1) as torch's kernel: x > 0 ? x : expm1(x); its derivative from the output a: 1 or a + 1 = exp(x)
// expm1 for z <= 0 in ~14 instructions (ocml's expm1f is ~40, which made the ELU epilogue VALU-bound):
// z in [-0.5, 0]: degree-9 Taylor polynomial (truncation < 2^-27 relative); z < -0.5: exp(z) - 1 on v_exp_f32
// (|result| > 0.39, so the exp's ~1 ulp error stays ~2^-23 relative).  Within 2 ulp of expm1f on z <= 0.
__device__ __forceinline__ float expm1_neg(float z) {
  float p = 1.0f / 362880.0f;
  p = fmaf(p, z, 1.0f / 40320.0f);
  p = fmaf(p, z, 1.0f / 5040.0f);
  p = fmaf(p, z, 1.0f / 720.0f);
  p = fmaf(p, z, 1.0f / 120.0f);
  p = fmaf(p, z, 1.0f / 24.0f);
  p = fmaf(p, z, 1.0f / 6.0f);
  p = fmaf(p, z, 0.5f);
  const float small = fmaf(p * z, z, z);
  const float big = __builtin_amdgcn_exp2f(z * 1.44269504f) - 1.0f;
  return z >= -0.5f ? small : big;
}
__device__ __forceinline__ float elu(float z) {
  const float e = expm1_neg(fminf(z, 0.0f));  // unconditionally: a select, not a branch per value
  return z > 0.0f ? z : e;
}
__device__ __forceinline__ float delu_from_out(float a) { return a > 0.0f ? 1.0f : a + 1.0f; }

// ------------------------------------------------------------------ xw: C = act(A W^T + b) / (A W^T) * ELU'
// A: activations (M rows, row stride lda, k0 columns; the first layers read the gathered mini-batch rows G).
// W: the weight image of the pack kernel, [K / 32 groups][plane hi, lo][q = 0..3][n rows][8 halves]: lane (q, c)
// of a 16-row tile reads its A fragment of v_mfma_f32_16x16x32_f16 (row c, k = 8 q .. 8 q + 7) as one 16-byte
// load per plane.  MFMA roles: weights are the A operand (16 features), activations the B operand (16 rows); a
// lane's accumulator holds features 4 q .. 4 q + 3 of row c, stored as one 16-byte row-major write.
// Staging: the next 32-deep K group of the 128-row A tile is loaded (16-byte loads) while the current one is
// multiplied, split into hi / lo planes [q][row][8] in LDS; the weight fragments of a group are loaded at its
// start.  About 150 registers: two or three workgroups per CU overlap each other's loads and MFMAs.
struct XwProb {
  const float* a;
  int64_t lda;
  int32_t k0;                   // real columns (elements k >= k0 of a row are read as 0)
  const uint32_t* amax;
  const uint32_t* amax2;        // optional second max (G's latent columns)
  const h8_t* w;
  const int32_t* wexp;
  int32_t G;                    // K groups of 32 in the weight image
  int32_t n;                    // output features (multiple of TB)
  const float* bias;            // F epilogue
  const float* aprev;           // D epilogue: the forward activation whose ELU' multiplies
  int64_t ldp;
  float* c;
  int64_t ldc;
  uint32_t* cmax;
  float* colsum;                // D: [tiles_m][n] column sums of C
  int32_t tiles_n, tile0;
};
struct XwLaunch {
  XwProb p[2];
  int32_t nprob, M, total;
};

enum { EPI_LIN = 0, EPI_ELU = 1, EPI_DELU = 2 };

#ifndef PPO_XW_LB
#define PPO_XW_LB 2
#endif
#ifndef PPO_XW_V
#define PPO_XW_V 1  // 0: weight fragments loaded at the start of their K group; 1: one group ahead; 2: through LDS
#endif

#ifdef PPO_STAMPS  // diagnostic build only (tools/xw_stamps.py): s_memrealtime per workgroup at kernel start,
                   // after the first staged group, after the K loop and after the epilogue
__device__ unsigned long long g_xw_stamps[8192][4];
#define XW_STAMP(i)                                                                                   \
  do {                                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_xw_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define XW_STAMP(i)
#endif

template <int EPI>
__global__ __launch_bounds__(256, PPO_XW_LB) void xw_kernel(XwLaunch L) {
  XW_STAMP(0);
  __shared__ h8_t sA[2][2][4][TB];  // [buffer][plane][q][row]: 32 KiB
  __shared__ float sRed[2][64];
  __shared__ uint32_t sMax[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, q = lane >> 4, c = lane & 15;
  int t = blockIdx.x;
  if ((L.total & 7) == 0) t = (t & 7) * (L.total >> 3) + (t >> 3);  // one XCD walks consecutive row tiles
  const XwProb& P = (L.nprob > 1 && t >= L.p[1].tile0) ? L.p[1] : L.p[0];
  const int lt = t - P.tile0, mt = lt / P.tiles_n, nt = lt - mt * P.tiles_n;
  const int wm = w & 1, wn = w >> 1, M = L.M;
  int eA = 0, eW = 0;  // the operands' scale exponents: read after the first group's loads are issued
  float sa = 1.0f;
  // staging: per instruction 8 rows x 32 k; lane -> row (lane >> 1) & 7, float4 k4 = 2 (lane >> 4) + (lane & 1)
  const int srow = (lane >> 1) & 7, k4 = ((lane >> 4) << 1) | (lane & 1);
  const int mrow0 = mt * TB + w * 32 + srow;  // row of instruction it: mrow0 + 8 it
  // every load is unconditional (rows clamped to M - 1, columns to the row's last 16 bytes) and out-of-range
  // values are zeroed afterwards: a load under a branch makes hipcc wait for it (vmcnt(0)) right away
  const float* arow[4];
  float rmask[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int m = mrow0 + 8 * it;
    arow[it] = P.a + (size_t)min(m, M - 1) * P.lda;
    rmask[it] = m < M ? 1.0f : 0.0f;
  }
  const int kmax = (int)P.lda - 4;
  f4_t st[4];
  int stk = 0;  // first column of the staged group: the masks are applied in store(), after the MFMAs, so that the
                // loads stay in flight across them
  auto load = [&](int g) {
    const int k = g * 32 + 4 * k4, kc = min(k, kmax);
    stk = k;
#pragma unroll
    for (int it = 0; it < 4; ++it) st[it] = *reinterpret_cast<const f4_t*>(arow[it] + kc);
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      f4_t v = st[it];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (stk + i < P.k0) ? v[i] * rmask[it] : 0.0f;
      h4_t hi, lo;
      split4(v, sa, hi, lo);
      const int row = w * 32 + it * 8 + srow;
      reinterpret_cast<h4_t*>(&sA[buf][0][k4 >> 1][row])[k4 & 1] = hi;
      reinterpret_cast<h4_t*>(&sA[buf][1][k4 >> 1][row])[k4 & 1] = lo;
    }
  };
  const size_t npad = (size_t)P.n;
  const h8_t* wrow = P.w + (size_t)q * npad + nt * TB + wn * 64 + c;  // + (g * 2 + plane) * 4 * npad + 16 tn
  f4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (f4_t){0.0f, 0.0f, 0.0f, 0.0f};
  // the F epilogue's bias, loaded now: a load at the epilogue would be waited for right there
  f4_t bias4[4];
#pragma unroll
  for (int tn = 0; tn < 4; ++tn)
    bias4[tn] = EPI != EPI_DELU ? *reinterpret_cast<const f4_t*>(P.bias + nt * TB + wn * 64 + tn * 16 + 4 * q)
                                : (f4_t){0.0f, 0.0f, 0.0f, 0.0f};
  const int G = P.G;
  auto loadw = [&](int g, h8_t (&wh)[4], h8_t (&wl)[4]) {
    const h8_t* wg = wrow + (size_t)g * 8 * npad;
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      wh[tn] = wg[tn * 16];
      wl[tn] = wg[4 * npad + tn * 16];
    }
  };
  auto mma = [&](int cur, const h8_t (&wh)[4], const h8_t (&wl)[4]) {
#pragma unroll
    for (int tm = 0; tm < 4; ++tm) {
      const h8_t xh = sA[cur][0][q][wm * 64 + tm * 16 + c];
      const h8_t xl = sA[cur][1][q][wm * 64 + tm * 16 + c];
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) acc[tn][tm] = mfma3(wh[tn], wl[tn], xh, xl, acc[tn][tm]);
    }
  };
  load(0);
#if PPO_XW_V == 1
  // weight fragments and the A tile of the next group in flight across this group's MFMAs: every load is
  // unconditional (the last group re-loads itself), the LDS store of the staged group follows the MFMAs
  h8_t wh0[4], wl0[4], wh1[4], wl1[4];
  loadw(0, wh0, wl0);
#endif
  // the max |x| records (one dependent round trip) after the first group's loads are in flight
  eA = scale_exp(P.amax2 ? max(*P.amax, *P.amax2) : *P.amax);
  eW = *P.wexp;
  sa = pow2f(eA);
  store(0);
#if PPO_XW_V == 1
  __syncthreads();
  auto body = [&](int g, int cur, h8_t (&wh)[4], h8_t (&wl)[4], h8_t (&nwh)[4], h8_t (&nwl)[4]) {
    const int gn = min(g + 1, G - 1);
#ifndef PPO_XW_NOW  // timing experiments only: PPO_XW_NOW / NOA / NOMMA drop the weight loads / A loads / MFMAs
    loadw(gn, nwh, nwl);
#else
    (void)nwh; (void)nwl;
#endif
#ifndef PPO_XW_NOA
    load(gn);
#endif
#ifndef PPO_XW_NOMMA
    mma(cur, wh, wl);
#else
    if (g < 0) mma(cur, wh, wl);
#endif
    store(cur ^ 1);
    __syncthreads();
  };
  XW_STAMP(1);
  for (int g = 0; g < G; g += 2) {
    body(g, 0, wh0, wl0, wh1, wl1);
    if (g + 1 < G) body(g + 1, 1, wh1, wl1, wh0, wl0);
  }
  XW_STAMP(2);
#elif PPO_XW_V == 2
  // weight tile through LDS: each thread stages 4 x 16 bytes of the next group's 16 KiB image with the A tile
  __shared__ h8_t sW[2][2][4][TB];  // [buffer][plane][q][n]
  const h8_t* wsrc = P.w + nt * TB + (tid & 31) + (size_t)(tid >> 5) * npad;  // chunk (plane, q) = tid >> 5
  h8_t wst[4];
  auto loadw2 = [&](int g) {
    const h8_t* p = wsrc + (size_t)g * 8 * npad;
#pragma unroll
    for (int i = 0; i < 4; ++i) wst[i] = p[32 * i];
  };
  auto storew2 = [&](int buf) {
    h8_t* d = &sW[buf][0][0][0] + (size_t)(tid >> 5) * TB + (tid & 31);
#pragma unroll
    for (int i = 0; i < 4; ++i) d[32 * i] = wst[i];
  };
  loadw2(0);
  storew2(0);
  __syncthreads();
  for (int g = 0; g < G; ++g) {
    const int cur = g & 1;
    const int gn = min(g + 1, G - 1);  // unconditional: the last group re-loads itself into the idle buffer
    loadw2(gn);
    load(gn);
    h8_t wh[4], wl[4];
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      wh[tn] = sW[cur][0][q][wn * 64 + tn * 16 + c];
      wl[tn] = sW[cur][1][q][wn * 64 + tn * 16 + c];
    }
    mma(cur, wh, wl);
    store(cur ^ 1);
    storew2(cur ^ 1);
    __syncthreads();
  }
#else
  __syncthreads();
  for (int g = 0; g < G; ++g) {
    const int cur = g & 1;
    h8_t wh[4], wl[4];
    loadw(g, wh, wl);
    const bool more = g + 1 < G;
    if (more) load(g + 1);
    mma(cur, wh, wl);
    if (more) store(cur ^ 1);
    __syncthreads();
  }
#endif
  // epilogue.  The D form's ELU' operand: the next column block's rows are requested while this one is
  // finished (clamped rows, unconditional: a load under the row test would be waited for at once); rows past
  // M only skip their store.
  const int sh = -(eA + eW);
  uint32_t amax = 0u;
  f4_t csum[4];
  f4_t ap[2][4];
  auto load_ap = [&](int tn, f4_t (&a)[4]) {
    const int n = nt * TB + wn * 64 + tn * 16 + 4 * q;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm) {
      const int mc = min(mt * TB + wm * 64 + tm * 16 + c, M - 1);
      a[tm] = *reinterpret_cast<const f4_t*>(P.aprev + (size_t)mc * P.ldp + n);
    }
  };
  if (EPI == EPI_DELU) load_ap(0, ap[0]);
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) {
    if (EPI == EPI_DELU && tn + 1 < 4) load_ap(tn + 1, ap[(tn + 1) & 1]);
    csum[tn] = (f4_t){0.0f, 0.0f, 0.0f, 0.0f};
    const int n = nt * TB + wn * 64 + tn * 16 + 4 * q;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm) {
      const int m = mt * TB + wm * 64 + tm * 16 + c;
      const bool in = m < M;
      f4_t v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = ldexpf(acc[tn][tm][i], sh);
      if (EPI == EPI_DELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = in ? v[i] * delu_from_out(ap[tn & 1][tm][i]) : 0.0f;
        csum[tn] += v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float z = v[i] + bias4[tn][i];
          v[i] = EPI == EPI_ELU ? elu(z) : z;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) amax = max(amax, in ? absbits(v[i]) : 0u);
#ifdef PPO_XW_NOSTORE  // timing experiment: no C stores
      if (v[0] != v[0] && v[1] == 12345.0f)
#endif
      if (in) *reinterpret_cast<f4_t*>(P.c + (size_t)m * P.ldc + n) = v;
    }
  }
  amax = wave_max_u32(amax);
  if (lane == 0) sMax[w] = amax;  // one atomic per workgroup (a single address takes them one at a time)
  __syncthreads();
  if (tid == 0 && P.cmax) atomicMax(P.cmax, max(max(sMax[0], sMax[1]), max(sMax[2], sMax[3])));
  XW_STAMP(3);
  if (EPI == EPI_DELU && P.colsum) {
    // column sums of this tile in a fixed order: the 16 rows of a lane group (xor tree), then wm = 0 + wm = 1
#pragma unroll
    for (int tn = 0; tn < 4; ++tn)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float s = csum[tn][i];
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 8);
        csum[tn][i] = s;
      }
    if (wm == 1 && c == 0)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn)
#pragma unroll
        for (int i = 0; i < 4; ++i) sRed[wn][tn * 16 + 4 * q + i] = csum[tn][i];
    __syncthreads();
    if (wm == 0 && c == 0)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int f = tn * 16 + 4 * q + i;
          P.colsum[(size_t)mt * P.n + nt * TB + wn * 64 + f] = csum[tn][i] + sRed[wn][f];
        }
  }
}

// ------------------------------------------------------------------ wgrad: partial[s] = sum over a row chunk of
// delta[m]^T x[m].  Both operands are row-major with the reduction (row) index strided, so they are staged as
// split f16 row-major LDS images [32 rows][128 columns] (16-byte chunks XOR-swizzled per row) and read back
// transposed with ds_read_b64_tr_b16: lane i of a 16-lane group receives column i of a 4-row block, i.e. 4
// consecutive rows (the MFMA K index) of one column.  MFMA roles: x columns (k) are the A operand rows,
// delta columns (n) the B operand columns: a lane's accumulator holds k = 4 q .. 4 q + 3 of one n, stored as
// one 16-byte write into partial[s][n][k].
struct WgProb {
  const float* x;
  int64_t ldx;
  int32_t k0;         // real x columns
  const uint32_t* xmax;
  const uint32_t* xmax2;  // optional second max (G's latent columns)
  const float* d;
  int64_t ldd;
  const uint32_t* dmax;
  float* part;        // [S][n][kpad]
  int64_t pstride;    // floats per chunk s
  int32_t kpad;       // row length of the partial (multiple of TB)
  int32_t tiles_k, tiles_n, tile0;
};
struct WgLaunch {
  WgProb p[8];
  int32_t nprob, M, S, chunk, total;
};

typedef __fp16 v4hp_t __attribute__((__vector_size__(8)));  // the ds_read_tr16 builtin's operand type
typedef __attribute__((address_space(3))) v4hp_t lds_v4hp_t;

__device__ __forceinline__ int swz(int r) { return ((r & 3) | ((r >> 1) & 4)) << 1; }
// byte offset of the 4 halves at (row r, column 4 j) in a [32][128-half] image with swizzled 16-byte chunks
__device__ __forceinline__ int img_off(int r, int j4) { return r * 256 + 16 * ((j4 >> 1) ^ swz(r)) + 8 * (j4 & 1); }

__device__ __forceinline__ h8_t tr_frag(const char* base, int col0, int q, int i) {
  // rows 8 q .. 8 q + 7 of column col0 + i: two transposed 4-row reads
  const int r = i >> 2, p = i & 3;
  const int j4 = (col0 >> 2) + p;
  const h4_t a = __builtin_bit_cast(
      h4_t, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_v4hp_t*)(base + img_off(8 * q + r, j4))));
  const h4_t b = __builtin_bit_cast(
      h4_t, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_v4hp_t*)(base + img_off(8 * q + 4 + r, j4))));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgLaunch L) {
  __shared__ __attribute__((aligned(16))) char sX[2][2][32 * 256];  // [buffer][plane] 8 KiB images
  __shared__ __attribute__((aligned(16))) char sD[2][2][32 * 256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, q = lane >> 4, c = lane & 15;
  int b = blockIdx.x, s, t;
  if ((L.S & 7) == 0) {
    const int bb = b >> 3;
    s = (b & 7) + 8 * (bb / L.total);
    t = bb % L.total;
  } else {
    s = b / L.total;
    t = b % L.total;
  }
  int pi = 0;
#pragma unroll
  for (int i = 1; i < 8; ++i)
    if (i < L.nprob && t >= L.p[i].tile0) pi = i;
  const WgProb& P = L.p[pi];
  const int lt = t - P.tile0, tk = lt / P.tiles_n, tn = lt - tk * P.tiles_n;
  const int wk = w & 1, wn = w >> 1;
  const int m_lo = s * L.chunk, m_hi = min(L.M, m_lo + L.chunk);
  const int eX = scale_exp(P.xmax2 ? max(*P.xmax, *P.xmax2) : *P.xmax), eD = scale_exp(*P.dmax);
  const float sx = pow2f(eX), sd = pow2f(eD);
  // k-tiles of this wave that hold real columns (the first layers' K is not a multiple of 128)
  const int kw0 = tk * TB + wk * 64;
  const int nkt = max(0, min(4, (P.k0 - kw0 + 15) >> 4));
  // staging: instruction j covers rows 2 j, 2 j + 1 of the wave's 8; lane -> row + (lane >> 5), float4 lane & 31
  const int col4 = lane & 31;
  const int kx = tk * TB + 4 * col4, kxc = min(kx, (int)P.ldx - 4);
  const int rsub = w * 8 + (lane >> 5);  // + 2 j
  const float* xb = P.x + kxc;
  const float* db = P.d + tn * TB + 4 * col4;
  // two register slots: the rows of group g + 1 are in flight while group g is multiplied, and group g + 2 is
  // requested before group g + 1 is split into LDS (every load unconditional: rows clamped, the last group
  // re-loaded past the end; out-of-range values zeroed in store(), after the MFMAs)
  f4_t sxv[2][4], sdv[2][4];
  int sm0[2] = {0, 0};
  const int ng = (m_hi - m_lo + 31) >> 5;
  auto load = [&](int slot, int g) {
    const int m0 = m_lo + min(g, ng - 1) * 32;
    sm0[slot] = m0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int mc = min(m0 + rsub + 2 * j, L.M - 1);
      sxv[slot][j] = *reinterpret_cast<const f4_t*>(xb + (size_t)mc * P.ldx);
      sdv[slot][j] = *reinterpret_cast<const f4_t*>(db + (size_t)mc * P.ldd);
    }
  };
  auto store = [&](int slot, int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = rsub + 2 * j;
      const float rm = sm0[slot] + r < m_hi ? 1.0f : 0.0f;
      f4_t vx = sxv[slot][j], vd = sdv[slot][j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vx[i] = kx + i < P.k0 ? vx[i] * rm : 0.0f;
        vd[i] = vd[i] * rm;
      }
      const int off = img_off(r, col4);
      h4_t hi, lo;
      split4(vx, sx, hi, lo);
      *reinterpret_cast<h4_t*>(&sX[buf][0][off]) = hi;
      *reinterpret_cast<h4_t*>(&sX[buf][1][off]) = lo;
      split4(vd, sd, hi, lo);
      *reinterpret_cast<h4_t*>(&sD[buf][0][off]) = hi;
      *reinterpret_cast<h4_t*>(&sD[buf][1][off]) = lo;
    }
  };
  f4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int bq = 0; bq < 4; ++bq) acc[a][bq] = (f4_t){0.0f, 0.0f, 0.0f, 0.0f};
  auto mma = [&](int cur) {
    if (nkt > 0) {
      h8_t dh[4], dl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dh[j] = tr_frag(sD[cur][0], wn * 64 + j * 16, q, c);
        dl[j] = tr_frag(sD[cur][1], wn * 64 + j * 16, q, c);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < nkt) {
          const h8_t xh = tr_frag(sX[cur][0], wk * 64 + i * 16, q, c);
          const h8_t xl = tr_frag(sX[cur][1], wk * 64 + i * 16, q, c);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma3(xh, xl, dh[j], dl[j], acc[i][j]);
        }
      }
    }
  };
  if (ng > 0) {
    load(0, 0);
    store(0, 0);
    load(1, 1);
    __syncthreads();
    for (int g = 0; g < ng; g += 2) {
      // slot 1 holds group g + 1; slot 0 is free
      load(0, g + 2);
      mma(0);
      store(1, 1);
      __syncthreads();
      if (g + 1 < ng) {
        // slot 0 holds group g + 2; slot 1 is free
        load(1, g + 3);
        mma(1);
        store(0, 0);
        __syncthreads();
      }
    }
  }
  const int sh = -(eX + eD);
  float* part = P.part + (size_t)s * P.pstride;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= nkt) continue;
    const int k = kw0 + i * 16 + 4 * q;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = tn * TB + wn * 64 + j * 16 + c;
      f4_t v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ldexpf(acc[i][j][e], sh);
      *reinterpret_cast<f4_t*>(part + (size_t)n * P.kpad + k) = v;
    }
  }
}

// ------------------------------------------------------------------ the mini-batch rows of the storage
// One thread per element (no per-row dependent loads):
//   G[m] = [obs_history[idx[m]] (H), latent (P, written by adapt_kernel<0>), privileged_obs[idx[m]] (P), 0 ...]
//   B[m] = [actions (A), mu (A), sigma (A), actions_log_prob, advantages, returns, values]   (the head's inputs)
// G is the first layers' operand in 16-byte-loadable rows: the actor reads [hist, latent] (H + P columns), the
// critic [hist, latent, priv] against weights whose latent columns are zero, the adaptation module [hist].
struct GatherArgs {
  const float* hist;
  int64_t hld;
  const float *priv, *act, *mu, *sigma, *logp, *adv, *ret, *val;
  const int64_t* idx;
  int32_t M, H, P, A, ldg, bw;
  float* G;
  float* B;
  uint32_t* mx;
};

// A wave gathers four rows at a time (rows strided over the grid): the four storage indices come in one load,
// then every element load of the four rows is issued (clamped addresses, selects afterwards) before any store.
// One atomicMax per workgroup: a max per row-block would serialise ~M atomics on one address.
constexpr int GATHER_BLOCKS_MAX = 1024;
__global__ __launch_bounds__(256) void gather_kernel(GatherArgs g) {
  __shared__ uint32_t red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int M = g.M, H = g.H, P = g.P, A = g.A, ldg = g.ldg, bw = g.bw;
  const int nwaves = gridDim.x * 4;
  uint32_t mb = 0u;
  for (int m0 = (blockIdx.x * 4 + w) * 4; m0 < M; m0 += nwaves * 4) {
    const int64_t ri = g.idx[min(m0 + (lane & 3), M - 1)];
    int64_t r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = __shfl(ri, j);
    for (int k0 = 0; k0 < ldg; k0 += 64) {
      const int k = k0 + lane;
      const int kh = min(k, H - 1), kp = min(max(k - H - P, 0), P - 1);
      const bool in_h = k < H, in_p = k >= H + P && k < H + 2 * P;
      float vh[4], vp[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vh[j] = g.hist[r[j] * g.hld + kh];
        vp[j] = g.priv[r[j] * P + kp];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = in_h ? vh[j] : (in_p ? vp[j] : 0.0f);
        if (m0 + j < M && k < ldg) {
          g.G[(size_t)(m0 + j) * ldg + k] = v;
          mb = max(mb, absbits(v));
        }
      }
    }
    // B rows: [actions A, mu A, sigma A, logp, adv, ret, values, 0 ...] (bw <= 64 columns)
    {
      const int k = lane;
      const int seg = k < A ? 0 : (k < 2 * A ? 1 : (k < 3 * A ? 2 : 3));
      const int ka = min(k - seg * A, A - 1);
      const float* srcA = seg == 0 ? g.act : (seg == 1 ? g.mu : g.sigma);
      const int t = k - 3 * A;  // 0: logp, 1: adv, 2: ret, 3: values
      const float* srcS = t == 0 ? g.logp : (t == 1 ? g.adv : (t == 2 ? g.ret : g.val));
      float va[4], vs[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        va[j] = srcA[r[j] * A + max(ka, 0)];
        vs[j] = srcS[r[j]];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = seg < 3 ? va[j] : (t < 4 ? vs[j] : 0.0f);
        if (m0 + j < M && k < bw) g.B[(size_t)(m0 + j) * bw + k] = v;
      }
    }
  }
  mb = wave_max_u32(mb);
  if (lane == 0) red[w] = mb;
  __syncthreads();
  if (threadIdx.x == 0) {
    mb = max(max(red[0], red[1]), max(red[2], red[3]));
    if (mb) atomicMax(g.mx, mb);
  }
}

__device__ __forceinline__ float half_sum(float v) {  // sum over the 32 lanes of a half-wave
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}
__device__ __forceinline__ float quarter_sum(float v) {  // sum over the 16 lanes of a quarter-wave
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
  return v;
}

// ------------------------------------------------------------------ the actor / critic heads and the loss
// A half-wave per mini-batch row (two rows per wave step, rows strided over the grid), lanes along the 128
// features of a3 (4 per lane, lane + 32 j).  mu = W4 a3 + b4, V = W4c a3c + b4c (half-wave sums), then
// Normal(mu, std).log_prob, the ratio, the clipped surrogate, the clipped value loss and the KL (ppo.py:107-158)
// and their gradients with torch's semantics (max / clamp backward: ties split the gradient in halves, clamp
// passes it on the closed interval); lane a < A owns action a.  Backward through L4: delta3 = (W4^T dmu) *
// ELU'(a3) for the lane's features, with per-lane sums of dW4, db3 (and the critic's) over the rows; the block's
// eight half-waves are summed (in a fixed order) into one partial row [block][HSTR] for reduce_kernel.
struct HeadArgs {
  int32_t M, A, bw;
  const float* B;  // gathered [actions, mu, sigma, logp, adv, ret, values] rows
  const float* a3p;
  const float* a3c;
  const float* w4p;
  const float* b4p;
  const float* w4c;
  const float* b4c;
  const float* std_;
  const go1_ppo_hyper* hyper;
  float* d3p;
  float* d3c;
  uint32_t* d3pmax;
  uint32_t* d3cmax;
  float* part;
  int32_t hstr;
};
// partial layout: dW4p [A][128], db4p [A], db3p [128], dW4c [128], db4c, db3c [128], dstd [A], Ls, Lv, KL
__host__ __device__ constexpr int head_stride(int A) { return A * 128 + A + 128 + 128 + 1 + 128 + A + 3; }
constexpr int HEAD_BLOCKS = 512;

template <int NA>
__global__ __launch_bounds__(256) void head_kernel(HeadArgs H) {
  __shared__ float red[4][head_stride(NA)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, half = lane >> 5, l = lane & 31;
  const int gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
  const int A = H.A;
  const go1_ppo_hyper hp = *H.hyper;
  const float invM = 1.0f / (float)H.M, eps = hp.clip_param;
  const float LOG_SQRT_2PI = 0.91893853320467274f;  // math.log(math.sqrt(2 * math.pi))
  const float* __restrict__ a3p = H.a3p;
  const float* __restrict__ a3c = H.a3c;
  const float* __restrict__ Bv = H.B;
  float w4[4][NA], w4c[4], gw4[4][NA], gw4c[4], db3[4], db3c[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      w4[j][a] = a < A ? H.w4p[a * H3 + l + 32 * j] : 0.0f;
      gw4[j][a] = 0.0f;
    }
    w4c[j] = H.w4c[l + 32 * j];
    gw4c[j] = db3[j] = db3c[j] = 0.0f;
  }
  const float sgm = l < A ? H.std_[l] : 1.0f;  // lane a's std
  const float b4 = l < A ? H.b4p[l] : 0.0f, b4c = H.b4c[0];
  float db4 = 0.0f, dstd = 0.0f, db4cs = 0.0f, ls = 0.0f, lv = 0.0f, kls = 0.0f;
  uint32_t mxp = 0u, mxc = 0u;
  for (int m = 2 * gw + half; m < H.M + half; m += 2 * nw) {
    const bool valid = m < H.M;
    const int mr = valid ? m : H.M - 1;  // an out-of-range half computes row M - 1 and discards it
    float x[4], y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = a3p[(size_t)mr * H3 + l + 32 * j];
      y[j] = a3c[(size_t)mr * H3 + l + 32 * j];
    }
    const float* br = Bv + (size_t)mr * H.bw;
    const float xa = l < A ? br[l] : 0.0f, om = l < A ? br[A + l] : 0.0f, os = l < A ? br[2 * A + l] : 1.0f;
    const float old_logp = br[3 * A], adv = br[3 * A + 1], ret = br[3 * A + 2], tvv = br[3 * A + 3];
    float mua = 0.0f;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      float s = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) s = fmaf(w4[j][a], x[j], s);
      s = half_sum(s);
      if (a == l) mua = s;
    }
    mua += b4;
    float V = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) V = fmaf(w4c[j], y[j], V);
    V = half_sum(V) + b4c;
    float lpa = 0.0f, kla = 0.0f, dx = 0.0f;
    if (l < A) {
      dx = xa - mua;
      const float var = sgm * sgm;
      // Normal.log_prob: -((value - loc) ** 2) / (2 * var) - log(scale) - log(sqrt(2 pi))
      lpa = (-(dx * dx) / (2.0f * var) - logf(sgm)) - LOG_SQRT_2PI;
      // KL (ppo.py:121-124): log(sigma / old_sigma + 1e-5) + (old_sigma^2 + (old_mu - mu)^2) / (2 sigma^2) - 0.5
      const float dm = om - mua;
      kla = (logf(sgm / os + 1.0e-5f) + (os * os + dm * dm) / (2.0f * (sgm * sgm))) - 0.5f;
    }
    const float logp = half_sum(lpa), kl = half_sum(kla);
    const float ratio = expf(logp - old_logp);
    const float s1 = -adv * ratio;
    const float rc = fminf(fmaxf(ratio, 1.0f - eps), 1.0f + eps);
    const float s2 = -adv * rc;
    const float w1 = s1 > s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float w2 = s2 > s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float inr = (ratio >= 1.0f - eps && ratio <= 1.0f + eps) ? 1.0f : 0.0f;
    const float dlogp = valid ? (invM * (w1 * -adv + w2 * (-adv * inr))) * ratio : 0.0f;
    float dmu_a = 0.0f;
    if (l < A) {
      const float var = sgm * sgm;
      dmu_a = dlogp * (dx / var);
      dstd += dlogp * ((dx * dx) / (var * sgm) - 1.0f / sgm);
      db4 += dmu_a;
    }
    float dV, vl;
    if (hp.use_clipped_value_loss != 0.0f) {
      const float vc = tvv + fminf(fmaxf(V - tvv, -eps), eps);
      const float e1 = V - ret, e2 = vc - ret;
      const float l1 = e1 * e1, l2 = e2 * e2;
      vl = fmaxf(l1, l2);
      const float u1 = l1 > l2 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f);
      const float u2 = l2 > l1 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f);
      const float dvi = V - tvv;
      const float vin = (dvi >= -eps && dvi <= eps) ? 1.0f : 0.0f;
      dV = hp.value_loss_coef * invM * (u1 * 2.0f * e1 + u2 * 2.0f * e2 * vin);
    } else {
      const float e = ret - V;
      vl = e * e;
      dV = hp.value_loss_coef * invM * (-2.0f * e);
    }
    if (!valid) dV = 0.0f;
    if (l == 0 && valid) {
      ls += fmaxf(s1, s2);
      lv += vl;
      kls += kl;
      db4cs += dV;
    }
    // backward through L4: every lane needs every dmu_a of its half
    float g[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) g[a] = a < A ? __shfl(dmu_a, a, 32) : 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float tt = 0.0f;
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        tt = fmaf(w4[j][a], g[a], tt);
        gw4[j][a] = fmaf(g[a], x[j], gw4[j][a]);
      }
      const float dp = tt * delu_from_out(x[j]);
      const float dc = (w4c[j] * dV) * delu_from_out(y[j]);
      gw4c[j] = fmaf(dV, y[j], gw4c[j]);
      db3[j] += dp;
      db3c[j] += dc;
      if (valid) {
        H.d3p[(size_t)m * H3 + l + 32 * j] = dp;
        H.d3c[(size_t)m * H3 + l + 32 * j] = dc;
        mxp = max(mxp, absbits(dp));
        mxc = max(mxc, absbits(dc));
      }
    }
  }
  mxp = wave_max_u32(mxp);
  mxc = wave_max_u32(mxc);
  if (lane == 0) {
    atomicMax(H.d3pmax, mxp);
    atomicMax(H.d3cmax, mxc);
  }
  // the two halves of the wave, then the block's four waves in LDS (fixed order)
  auto comb = [](float v) { return v + __shfl_xor(v, 32); };
  const int o_db4p = A * 128, o_db3p = o_db4p + A, o_dW4c = o_db3p + 128, o_db4c = o_dW4c + 128,
            o_db3c = o_db4c + 1, o_dstd = o_db3c + 128, o_loss = o_dstd + A;
  float* rw = red[wv];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = l + 32 * j;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const float v = comb(gw4[j][a]);
      if (half == 0 && a < A) rw[a * 128 + k] = v;
    }
    const float v1 = comb(db3[j]), v2 = comb(gw4c[j]), v3 = comb(db3c[j]);
    if (half == 0) {
      rw[o_db3p + k] = v1;
      rw[o_dW4c + k] = v2;
      rw[o_db3c + k] = v3;
    }
  }
  const float s_db4 = comb(db4), s_dstd = comb(dstd), s_db4c = comb(db4cs), s_ls = comb(ls), s_lv = comb(lv),
              s_kl = comb(kls);
  if (half == 0 && l < A) {
    rw[o_db4p + l] = s_db4;
    rw[o_dstd + l] = s_dstd;
  }
  if (lane == 0) {
    rw[o_db4c] = s_db4c;
    rw[o_loss + 0] = s_ls;
    rw[o_loss + 1] = s_lv;
    rw[o_loss + 2] = s_kl;
  }
  __syncthreads();
  float* part = H.part + (size_t)blockIdx.x * H.hstr;
  for (int e = threadIdx.x; e < H.hstr; e += 256) {
    float v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    // the entropy term -entropy_coef * mean(sum_a (0.5 + 0.5 log 2 pi + log std_a)): d / d std_a = -coef / std_a
    if (blockIdx.x == 0 && e >= o_dstd && e < o_dstd + A) v += -hp.entropy_coef / H.std_[e - o_dstd];
    part[e] = v;
  }
}

// ------------------------------------------------------------------ the adaptation module's output layer
// MODE 0: latent = W3a a2a + b3a, written into the latent columns of G (the actor's input).  MODE 1 (phase 1):
// the same, then F.mse_loss against privileged_obs (G's priv columns) on rows < num_train (test loss on the
// rest) and its gradient.  MODE 0 / 1: a quarter-wave per row (four rows per wave step), lanes along the 128
// features of a2a (8 consecutive per lane).  MODE 2 (phase 0): d latent = W1p[:, hist:]^T delta1p (the actor's
// first layer, latent columns): a wave per row, lanes along its 512 outputs (8 per lane), two rows per step.
// MODE 1 / 2 then back-propagate through W3a: delta2a = (W3a^T g) * ELU'(a2a) with partial sums of dW3a, db3a,
// db2a.  Partial row [block][LSTR]: dW3a [P][128], db3a [P], db2a [128], loss train, loss test.
struct AdaptArgs {
  int32_t M, P, hist, num_train, ldg;
  const float* a2a;
  const float* w3a;
  const float* b3a;
  float* G;           // latent columns at hist .. hist + P (MODE 0 writes), priv at hist + P .. (MODE 1 reads)
  uint32_t* latmax;
  const float* d1p;   // MODE 2: [M][512]
  const float* w1p;   // MODE 2: (512, hist + P)
  const go1_ppo_hyper* hyper;
  float* d2a;
  uint32_t* d2amax;
  float* part;
  int32_t lstr;
};
__host__ __device__ constexpr int adapt_stride(int P) { return P * 128 + P + 128 + 2; }
constexpr int ADAPT_BLOCKS = 512;

template <int MODE>
__global__ __launch_bounds__(256) void adapt_kernel(AdaptArgs D) {
  __shared__ float red[4][adapt_stride(8)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
  const int P = D.P;
  const go1_ppo_hyper hp = *D.hyper;
  const int nsel = hp.selective != 0.0f ? 1 : P;
  const float* __restrict__ a2a = D.a2a;
  // MODE 0 / 1: quarter q4 = lane >> 4 owns a row, lane l = lane & 15 features 8 l .. 8 l + 7;
  // MODE 2: the wave owns a row pair, lane features k = lane, lane + 64 of a2a, outputs 8 lane .. of delta1p
  const int q4 = lane >> 4, l = lane & 15;
  constexpr int NF = MODE == 2 ? 2 : 8;  // a2a features per lane
  float w3[NF][8], gw3[NF][8], db2[NF];
#pragma unroll
  for (int u = 0; u < NF; ++u) {
    const int k = MODE == 2 ? lane + 64 * u : 8 * l + u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      w3[u][j] = j < P ? D.w3a[j * HA2 + k] : 0.0f;
      gw3[u][j] = 0.0f;
    }
    db2[u] = 0.0f;
  }
  float db3 = 0.0f, lt = 0.0f, lte = 0.0f;  // db3: lane j < P (MODE 2) / quarter-lane j < P (MODE 0 / 1)
  uint32_t mx = 0u;
  if (MODE == 0 || MODE == 1) {
    float b3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) b3[j] = j < P ? D.b3a[j] : 0.0f;
    const float inv = 1.0f / (float)(D.num_train * nsel);
    for (int m = 4 * gw + q4; m < D.M + q4; m += 4 * nw) {
      const bool valid = m < D.M;
      const int mr = valid ? m : D.M - 1;
      const f4_t x0 = *reinterpret_cast<const f4_t*>(a2a + (size_t)mr * HA2 + 8 * l);
      const f4_t x1 = *reinterpret_cast<const f4_t*>(a2a + (size_t)mr * HA2 + 8 * l + 4);
      const float x[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      float yl = 0.0f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = 0.0f;
#pragma unroll
        for (int u = 0; u < 8; ++u) s = fmaf(w3[u][j], x[u], s);
        s = quarter_sum(s) + b3[j];
        if (j == l) yl = s;
      }
      float* grow = D.G + (size_t)mr * D.ldg + D.hist;
      if (MODE == 0) {
        if (valid && l < P) {
          grow[l] = yl;
          mx = max(mx, absbits(yl));
        }
        continue;
      }
      // F.mse_loss(pred[:nt, sel], target[:nt, sel]) (ppo.py:187-190): sel = every column, or column 0
      float gl = 0.0f;
      if (valid && l < nsel) {
        const float e = yl - grow[P + l];
        if (m < D.num_train) {
          gl = 2.0f * e * inv;
          lt += e * e;
        } else {
          lte += e * e;
        }
      }
      db3 += gl;
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = j < P ? __shfl(gl, j, 16) : 0.0f;
      float d[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float tt = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          tt = fmaf(w3[u][j], g[j], tt);
          gw3[u][j] = fmaf(g[j], x[u], gw3[u][j]);
        }
        d[u] = tt * delu_from_out(x[u]);
        db2[u] += d[u];
        mx = max(mx, valid ? absbits(d[u]) : 0u);
      }
      if (valid) {
        *reinterpret_cast<f4_t*>(D.d2a + (size_t)m * HA2 + 8 * l) = (f4_t){d[0], d[1], d[2], d[3]};
        *reinterpret_cast<f4_t*>(D.d2a + (size_t)m * HA2 + 8 * l + 4) = (f4_t){d[4], d[5], d[6], d[7]};
      }
    }
  } else {
    float w1l[8][8];  // W1p[n][hist + j] for the lane's 8 outputs n = 8 lane .. 8 lane + 7
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) w1l[u][j] = j < P ? D.w1p[(size_t)(8 * lane + u) * (D.hist + P) + D.hist + j] : 0.0f;
    const float* __restrict__ d1p = D.d1p;
    for (int m0 = gw; m0 < D.M; m0 += 2 * nw) {
      const int mb = m0 + nw;
      const bool vb = mb < D.M;
      const int rows[2] = {m0, vb ? mb : m0};
      float dd[2][8], x[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f4_t d0 = *reinterpret_cast<const f4_t*>(d1p + (size_t)rows[t] * H1 + 8 * lane);
        const f4_t d1 = *reinterpret_cast<const f4_t*>(d1p + (size_t)rows[t] * H1 + 8 * lane + 4);
        dd[t][0] = d0[0]; dd[t][1] = d0[1]; dd[t][2] = d0[2]; dd[t][3] = d0[3];
        dd[t][4] = d1[0]; dd[t][5] = d1[1]; dd[t][6] = d1[2]; dd[t][7] = d1[3];
        x[t][0] = a2a[(size_t)rows[t] * HA2 + lane];
        x[t][1] = a2a[(size_t)rows[t] * HA2 + lane + 64];
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t == 1 && !vb) break;
        float g[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float s = 0.0f;
#pragma unroll
          for (int u = 0; u < 8; ++u) s = fmaf(w1l[u][j], dd[t][u], s);
          g[j] = j < P ? wave_sum(s) : 0.0f;
          if (j == lane) db3 += g[j];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float tt = 0.0f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            tt = fmaf(w3[u][j], g[j], tt);
            gw3[u][j] = fmaf(g[j], x[t][u], gw3[u][j]);
          }
          const float d = tt * delu_from_out(x[t][u]);
          db2[u] += d;
          D.d2a[(size_t)rows[t] * HA2 + lane + 64 * u] = d;
          mx = max(mx, absbits(d));
        }
      }
    }
  }
  mx = wave_max_u32(mx);
  if (MODE == 0) {
    if (lane == 0) atomicMax(D.latmax, mx);
    return;
  }
  if (lane == 0) atomicMax(D.d2amax, mx);
  // quarters (MODE 1) combined by xor 16, 32; then the block's waves in LDS
  auto comb = [](float v) {
    if (MODE == 1) {
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
    }
    return v;
  };
  const int o_db3 = P * 128, o_db2 = o_db3 + P, o_loss = o_db2 + 128;
  float* rw = red[wv];
  const bool writer = MODE == 2 || q4 == 0;
#pragma unroll
  for (int u = 0; u < NF; ++u) {
    const int k = MODE == 2 ? lane + 64 * u : 8 * l + u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = comb(gw3[u][j]);
      if (writer && j < P) rw[j * 128 + k] = v;
    }
    const float v = comb(db2[u]);
    if (writer) rw[o_db2 + k] = v;
  }
  const float s_db3 = comb(db3), s_lt = comb(lt), s_lte = comb(lte);
  if (writer && (MODE == 2 ? lane : l) < P) rw[o_db3 + (MODE == 2 ? lane : l)] = s_db3;
  if (lane == 0) {
    rw[o_loss] = MODE == 1 ? s_lt : 0.0f;
    rw[o_loss + 1] = MODE == 1 ? s_lte : 0.0f;
  }
  if (MODE == 1) {  // the loss sums live on lanes l < nsel of each quarter: sum them across the quarter too
    float a = quarter_sum(l < nsel ? lt : 0.0f), b = quarter_sum(l < nsel ? lte : 0.0f);
    a += __shfl_xor(a, 16);
    a += __shfl_xor(a, 32);
    b += __shfl_xor(b, 16);
    b += __shfl_xor(b, 32);
    if (lane == 0) {
      rw[o_loss] = a;
      rw[o_loss + 1] = b;
    }
  }
  __syncthreads();
  float* part = D.part + (size_t)blockIdx.x * D.lstr;
  for (int e = threadIdx.x; e < D.lstr; e += 256) part[e] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
}

// ------------------------------------------------------------------ reduce: dst[r][c] = sum_p src[p][r][c]
// Segment table over every gradient tensor (and the aux sums); 256 threads per 64 output elements, the
// partials split four ways across the waves, summed in a fixed order.
struct Seg {
  float* dst;
  const float* src;
  int64_t lds, pstride, ldd;          // source row stride, partial stride, destination row stride
  int32_t rows, cols, nparts, start;  // start: first flat element of the segment in the launch
};
constexpr int MAX_SEGS = 32;
struct SegTable {
  Seg s[MAX_SEGS];
  int32_t nseg, total;
};

__global__ __launch_bounds__(256) void reduce_kernel(SegTable T) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  float acc = 0.0f;
  int si = -1, r = 0, cc = 0;
  if (e < T.total) {
    si = 0;
    for (int i = 1; i < T.nseg; ++i)
      if (e >= T.s[i].start) si = i;
    const Seg& S = T.s[si];
    const int le = e - S.start;
    r = le / S.cols;
    cc = le - r * S.cols;
    const float* src = S.src + (size_t)r * S.lds + cc;
    // parts w, w + 4, w + 8, ...: eight independent chains (loads in flight), summed in a fixed order
    float a[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    int p = w;
    for (; p + 28 < S.nparts; p += 32)
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += src[(size_t)(p + 4 * j) * S.pstride];
    for (int j = 0; p < S.nparts; p += 4, ++j) a[j & 7] += src[(size_t)p * S.pstride];
    acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && si >= 0) {
    const Seg& S = T.s[si];
    S.dst[(size_t)r * S.ldd + cc] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  }
}

// ------------------------------------------------------------------ norm, finalize, Adam
__global__ __launch_bounds__(256) void norm_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = g[i];
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// Adam scalars for one optimiser step, written by finalize_kernel: [0] gradient scale (clip / world), [1] -step
// size, [2] sqrt(bias correction 2), [3] eps, [4] 1 - beta1, [5] beta2, [6] 1 - beta2
struct Finalize {
  int32_t phase, M, num_train, nsel_all;
  const go1_ppo_hyper* hyper;
  const float* aux;
  const double* norm_part;
  double* lr;
  float* steps;
  double* losses;
  float* scal;
  uint32_t* zero[3];  // max slots to clear for the launches that follow: zero[i][0 .. nz[i])
  int32_t nz[3];
};

__global__ __launch_bounds__(256) void finalize_kernel(Finalize F) {
  __shared__ double red[256];
  const go1_ppo_hyper hp = *F.hyper;
  const double world = hp.world > 0.0f ? (double)hp.world : 1.0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if ((int)threadIdx.x < F.nz[i]) F.zero[i][threadIdx.x] = 0u;
  double s = 0.0;
  if (F.phase == 0) s = F.norm_part[threadIdx.x];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  double lr;
  float gscale;
  if (F.phase == 0) {
    // adaptive learning rate (ppo.py:119-132) from the KL mean over every rank's rows
    const float kl_mean = (float)((double)F.aux[2] / world) / (float)F.M;
    lr = F.lr[0];
    if (hp.desired_kl > 0.0f) {
      const double dk = (double)hp.desired_kl, k = (double)kl_mean;
      if (k > dk * 2.0)
        lr = fmax(1e-5, lr / 1.5);
      else if (k < dk / 2.0 && k > 0.0)
        lr = fmin(1e-2, lr * 1.5);
      F.lr[0] = lr;
    }
    // clip_grad_norm_ (ppo.py:157) of the rank-averaged gradient: clip_coef = max_norm / (norm + 1e-6), <= 1
    const float total = (float)(sqrt(red[0]) / world);
    const float coef = hp.max_grad_norm / (total + 1.0e-6f);
    gscale = (float)((double)fminf(coef, 1.0f) / world);
    F.losses[0] += (double)((float)((double)F.aux[1] / world) / (float)F.M);  // value loss
    F.losses[1] += (double)((float)((double)F.aux[0] / world) / (float)F.M);  // surrogate loss
  } else {
    lr = (double)hp.adaptation_lr;
    gscale = (float)(1.0 / world);
    const int nsel = hp.selective != 0.0f ? 1 : F.nsel_all;
    F.losses[2] += (double)((float)((double)F.aux[3] / world) / (float)(F.num_train * nsel));
    const int ntest = F.M - F.num_train;
    F.losses[3] += ntest > 0 ? (double)((float)((double)F.aux[4] / world) / (float)(ntest * nsel)) : 0.0;
  }
  // torch Adam (single-tensor form): step += 1; bias_correction1 = 1 - beta1 ** step; step_size = lr / bc1;
  // denom = sqrt(exp_avg_sq) / sqrt(bc2) + eps
  const float step = F.steps[F.phase] + 1.0f;
  F.steps[F.phase] = step;
  const double b1 = (double)hp.beta1, b2 = (double)hp.beta2;
  const double bc1 = 1.0 - pow(b1, (double)step), bc2 = 1.0 - pow(b2, (double)step);
  F.scal[0] = gscale;
  F.scal[1] = (float)(-(lr / bc1));
  F.scal[2] = (float)sqrt(bc2);
  F.scal[3] = hp.eps;
  F.scal[4] = (float)(1.0 - b1);
  F.scal[5] = hp.beta2;
  F.scal[6] = (float)(1.0 - b2);
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m1, float* __restrict__ m2, int64_t n,
                                                   const float* __restrict__ scal) {
  const float gs = scal[0], nss = scal[1], bc2s = scal[2], eps = scal[3], w1 = scal[4], b2 = scal[5], c2 = scal[6];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gr = g[i] * gs;
    float a = m1[i];
    a = a + w1 * (gr - a);             // exp_avg.lerp_(grad, 1 - beta1)
    float v = m2[i] * b2;              // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    v = v + (c2 * gr) * gr;
    const float den = sqrtf(v) / bc2s + eps;
    p[i] = p[i] + (nss * a) / den;     // param.addcdiv_(exp_avg, denom, value=-step_size)
    m1[i] = a;
    m2[i] = v;
  }
}

// ------------------------------------------------------------------ weight max and the fragment images
struct PackW {
  const float* w;  // source (n, k - gap) with row stride ldw; image column kk reads source column kk (kk < gap_at),
                   // nothing (gap_at <= kk < gap_at + gap: zero weights), kk - gap (beyond)
  int32_t n, k, ldw, gap_at, gap, G, npad;
  h8_t* img;       // forward image [G][2][4][npad][8]
  h8_t* imgt;      // transposed image [ceil(n / 32)][2][4][kpadT][8] or NULL
  int32_t Gt, npadt;
  uint32_t* wmax;
  int32_t* wexp;
  int32_t start;   // first element of this tensor in the launch
};
constexpr int MAX_PACK = 8;
struct PackTable {
  PackW t[MAX_PACK];
  int32_t nt, total;
};

// grid (blocks, tensors): block-level max, one atomic per block and tensor
__global__ __launch_bounds__(256) void wmax_kernel(PackTable T) {
  __shared__ uint32_t red[4];
  const PackW& W = T.t[blockIdx.y];
  const int ks = W.k - W.gap, n = W.n * ks;
  uint32_t mx = 0u;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int r = e / ks;
    mx = max(mx, absbits(W.w[(size_t)r * W.ldw + (e - r * ks)]));
  }
  mx = wave_max_u32(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    mx = max(max(red[0], red[1]), max(red[2], red[3]));
    if (mx) atomicMax(W.wmax, mx);
  }
}

__global__ __launch_bounds__(256) void pack_kernel(PackTable T) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= T.total) return;
  int ti = 0;
  for (int i = 1; i < T.nt; ++i)
    if (e >= T.t[i].start) ti = i;
  const PackW& W = T.t[ti];
  const int le = e - W.start, n = le / W.k, k = le - n * W.k;
  const int es = scale_exp(*W.wmax);
  if (le == 0) *W.wexp = es;
  const bool in_gap = k >= W.gap_at && k < W.gap_at + W.gap;
  const float x = in_gap ? 0.0f : ldexpf(W.w[(size_t)n * W.ldw + (k < W.gap_at ? k : k - W.gap)], es);
  const _Float16 hi = (_Float16)__builtin_amdgcn_cvt_pkrtz(x, 0.0f)[0];
  const _Float16 lo = (_Float16)__builtin_amdgcn_cvt_pkrtz(x - (float)hi, 0.0f)[0];
  {
    const int g = k >> 5, q = (k >> 3) & 3, r = k & 7;
    _Float16* base = reinterpret_cast<_Float16*>(W.img);
    base[(((size_t)(g * 2 + 0) * 4 + q) * W.npad + n) * 8 + r] = hi;
    base[(((size_t)(g * 2 + 1) * 4 + q) * W.npad + n) * 8 + r] = lo;
  }
  if (W.imgt) {
    const int g = n >> 5, q = (n >> 3) & 3, r = n & 7;
    _Float16* base = reinterpret_cast<_Float16*>(W.imgt);
    base[(((size_t)(g * 2 + 0) * 4 + q) * W.npadt + k) * 8 + r] = hi;
    base[(((size_t)(g * 2 + 1) * 4 + q) * W.npadt + k) * 8 + r] = lo;
  }
}

__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, int64_t rows, int32_t cols,
                                                     int64_t ld, uint32_t* __restrict__ out) {
  uint32_t mx = 0u;
  const int64_t total = rows * (int64_t)cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cols;
    mx = max(mx, absbits(x[r * ld + (i - r * cols)]));
  }
  mx = wave_max_u32(mx);
  if ((threadIdx.x & 63) == 0) atomicMax(out, mx);
}

__global__ void zero_u32_kernel(uint32_t* p, int n) {
  if ((int)threadIdx.x < n) p[threadIdx.x] = 0u;
}

// ------------------------------------------------------------------ workspace layout
enum MaxSlot {
  MX_G = 0,  // the gathered mini-batch rows (obs_history, privileged_obs)
  MX_LAT, MX_A1A, MX_A2A, MX_P1, MX_P2, MX_P3, MX_C1, MX_C2, MX_C3,
  MX_D3P, MX_D3C, MX_D2P, MX_D2C, MX_D1P, MX_D1C, MX_D2A, MX_D1A,
  MX_N
};
enum WSlot { W_A0 = 0, W_A2, W_P0, W_P2, W_P4, W_C0, W_C2, W_C4, W_N };

struct Lay {
  int H, P, A, M, MP, MT, HB, ldg, bw;
  int S[2], chunk[2];  // weight-gradient row split per phase (about two workgroups per CU in one round)
  int64_t np_total, np_adapt;
  // parameter offsets (floats) in state_dict order
  int64_t pw[11], pb[11], pstd;
  // workspace byte offsets
  size_t maxes, wmax, wexp, scal, normp, G, Bb, a1a, a2a, p1, p2, p3, c1, c2, c3, d3p, d3c, d2p, d2c, d1p, d1c, d2a,
      d1a, cs1a, cs1p, cs1c, cs2p, cs2c, hpart, apart, wpart[W_N], img[W_N], imgt[W_N], total;
  int64_t wpart_stride[W_N];
  int wn[W_N], wk[W_N];  // rows / GEMM columns of each weight image
};

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

bool make_layout(const go1_ppo_dims* d, Lay& L, std::string& err) {
  if (!d || d->hist < 1 || d->priv < 1 || d->priv > 8 || d->actions < 1 || d->actions > 16 || d->mb < 1 ||
      d->rows < d->mb) {
    err = "go1_ppo: dims outside the supported architecture (hist >= 1, priv 1..8, actions 1..16, mb <= rows)";
    return false;
  }
  L.H = d->hist;
  L.P = d->priv;
  L.A = d->actions;
  L.M = d->mb;
  L.MT = cdiv(L.M, TB);
  L.MP = L.MT * TB;
  L.HB = std::min(HEAD_BLOCKS, cdiv(L.M, 4));
  L.ldg = cdiv(L.H + 2 * L.P, 4) * 4;  // [hist, latent, priv]
  L.bw = cdiv(3 * L.A + 4, 4) * 4;     // [actions, mu, sigma, logp, adv, ret, values]
  // parameters
  const int64_t H = L.H, P = L.P, A = L.A;
  const int64_t wsz[11] = {HA1 * H, HA2 * HA1, P * HA2, H1 * (H + P), H2 * H1, H3 * H2, A * H3,
                           H1 * (H + P), H2 * H1, H3 * H2, 1 * H3};
  const int64_t bsz[11] = {HA1, HA2, P, H1, H2, H3, A, H1, H2, H3, 1};
  int64_t o = 0;
  for (int i = 0; i < 11; ++i) {
    L.pw[i] = o;
    o += wsz[i];
    L.pb[i] = o;
    o += bsz[i];
    if (i == 2) L.np_adapt = o;
  }
  L.pstd = o;
  o += A;
  L.np_total = o;
  // workspace
  size_t b = 0;
  auto take = [&](size_t bytes) {
    const size_t at = b;
    b += (bytes + 255) & ~(size_t)255;
    return at;
  };
  const size_t F = sizeof(float), MPs = (size_t)L.MP;
  L.maxes = take(64 * 4);
  L.wmax = take(16 * 4);
  L.wexp = take(16 * 4);
  L.scal = take(32 * 4);
  L.normp = take(NORM_BLOCKS * 8);
  L.G = take(MPs * L.ldg * F);
  L.Bb = take(MPs * L.bw * F);
  L.a1a = take(MPs * HA1 * F);
  L.a2a = take(MPs * HA2 * F);
  L.p1 = take(MPs * H1 * F);
  L.p2 = take(MPs * H2 * F);
  L.p3 = take(MPs * H3 * F);
  L.c1 = take(MPs * H1 * F);
  L.c2 = take(MPs * H2 * F);
  L.c3 = take(MPs * H3 * F);
  L.d3p = take(MPs * H3 * F);
  L.d3c = take(MPs * H3 * F);
  L.d2p = take(MPs * H2 * F);
  L.d2c = take(MPs * H2 * F);
  L.d1p = take(MPs * H1 * F);
  L.d1c = take(MPs * H1 * F);
  L.d2a = take(MPs * HA2 * F);
  L.d1a = take(MPs * HA1 * F);
  L.cs1a = take((size_t)L.MT * HA1 * F);
  L.cs1p = take((size_t)L.MT * H1 * F);
  L.cs1c = take((size_t)L.MT * H1 * F);
  L.cs2p = take((size_t)L.MT * H2 * F);
  L.cs2c = take((size_t)L.MT * H2 * F);
  L.hpart = take((size_t)HEAD_BLOCKS * head_stride(L.A) * F);
  L.apart = take((size_t)ADAPT_BLOCKS * adapt_stride(L.P) * F);
  // weight-gradient partials [S][n][kpad] and weight images (4 bytes per element: hi + lo halves)
  const int wn[W_N] = {HA1, HA2, H1, H2, H3, H1, H2, H3};
  // the row split of each phase's grouped weight-gradient launch: at most 512 workgroups (two per CU with the
  // launch's 64 KiB of LDS: one more would start a second round), chunks of >= 64 rows
  {
    const int wk0[W_N] = {L.H, HA1, L.H + L.P, H1, H2, L.H + 2 * L.P, H1, H2};
    int tiles[2] = {0, 0};
    for (int i = 0; i < W_N; ++i) {
      const int t = cdiv(wk0[i], TB) * (wn[i] / TB);
      tiles[0] += t;
      if (i == W_A0 || i == W_A2) tiles[1] += t;
    }
    for (int ph = 0; ph < 2; ++ph) {
      int S = 512 / tiles[ph];
      S = std::max(1, std::min(std::min(S, 64), L.M / 64));
      L.chunk[ph] = cdiv(cdiv(L.M, S), 32) * 32;
      L.S[ph] = cdiv(L.M, L.chunk[ph]);
    }
  }
  // GEMM columns: the actor's first layer reads [hist, latent], the critic's [hist, latent, priv] (zero weights on
  // the latent columns), the adaptation module's [hist]
  const int wk[W_N] = {L.H, HA1, L.H + L.P, H1, H2, L.H + 2 * L.P, H1, H2};
  for (int i = 0; i < W_N; ++i) {
    L.wn[i] = wn[i];
    L.wk[i] = wk[i];
    const int kpad = cdiv(wk[i], TB) * TB;
    L.wpart_stride[i] = (int64_t)wn[i] * kpad;
    const int S = (i == W_A0 || i == W_A2) ? std::max(L.S[0], L.S[1]) : L.S[0];
    L.wpart[i] = take((size_t)S * wn[i] * kpad * F);
    L.img[i] = take((size_t)cdiv(wk[i], 32) * 32 * wn[i] * 4);
    // transposed images for the layers the backward crosses: a2 (adaptation L2), p2, p4, c2, c4
    const bool tr = i == W_A2 || i == W_P2 || i == W_P4 || i == W_C2 || i == W_C4;
    L.imgt[i] = tr ? take((size_t)cdiv(wn[i], 32) * 32 * wk[i] * 4) : 0;
  }
  L.total = b;
  return true;
}

// parameter indices: a0 a2 a4 | p0 p2 p4 p6 | c0 c2 c4 c6
enum { IA0 = 0, IA2, IA4, IP0, IP2, IP4, IP6, IC0, IC2, IC4, IC6 };
// one weight image per W slot: slot -> parameter index
constexpr int kWParam[W_N] = {IA0, IA2, IP0, IP2, IP4, IC0, IC2, IC4};

struct Ctx {
  const go1_ppo_dims* d;
  const go1_ppo_bufs* b;
  Lay L;
  char* ws;
  hipStream_t s;
  template <class T>
  T* at(size_t off) const {
    return reinterpret_cast<T*>(ws + off);
  }
  uint32_t* mx(int slot) const { return at<uint32_t>(L.maxes) + slot; }
  const float* W(int i) const { return b->params + L.pw[i]; }
  const float* B(int i) const { return b->params + L.pb[i]; }
  float* gW(int i) const { return b->grads + NAUX + L.pw[i]; }
  float* gB(int i) const { return b->grads + NAUX + L.pb[i]; }
};

XwProb xw_prob(const Ctx& C, const float* a, int64_t lda, int k0, const uint32_t* amax, int wslot, bool transposed,
               int n, const float* bias, const float* aprev, int64_t ldp, float* out, int64_t ldc, uint32_t* cmax,
               float* colsum, const uint32_t* amax2 = nullptr) {
  XwProb p{};
  p.a = a;
  p.lda = lda;
  p.k0 = k0;
  p.amax = amax;
  p.amax2 = amax2;
  p.w = C.at<h8_t>(transposed ? C.L.imgt[wslot] : C.L.img[wslot]);
  p.wexp = C.at<int32_t>(C.L.wexp) + wslot;
  p.G = cdiv(transposed ? C.L.wn[wslot] : C.L.wk[wslot], 32);
  p.n = n;
  p.bias = bias;
  p.aprev = aprev;
  p.ldp = ldp;
  p.c = out;
  p.ldc = ldc;
  p.cmax = cmax;
  p.colsum = colsum;
  p.tiles_n = n / TB;
  return p;
}

int launch_xw(const Ctx& C, int epi, XwProb p0, const XwProb* p1) {
  XwLaunch L{};
  L.p[0] = p0;
  L.p[0].tile0 = 0;
  L.nprob = 1;
  L.M = C.L.M;
  int total = C.L.MT * p0.tiles_n;
  if (p1) {
    L.p[1] = *p1;
    L.p[1].tile0 = total;
    L.nprob = 2;
    total += C.L.MT * p1->tiles_n;
  }
  L.total = total;
  if (epi == EPI_ELU)
    hipLaunchKernelGGL(xw_kernel<EPI_ELU>, dim3(total), dim3(256), 0, C.s, L);
  else if (epi == EPI_DELU)
    hipLaunchKernelGGL(xw_kernel<EPI_DELU>, dim3(total), dim3(256), 0, C.s, L);
  else
    hipLaunchKernelGGL(xw_kernel<EPI_LIN>, dim3(total), dim3(256), 0, C.s, L);
  PPO_TRY(hipGetLastError());
  return GO1_PPO_OK;
}

WgProb wg_prob(const Ctx& C, int wslot, const float* x, int64_t ldx, int k0, const uint32_t* xmax, const float* d,
               int64_t ldd, int n, const uint32_t* dmax, const uint32_t* xmax2 = nullptr) {
  WgProb p{};
  p.x = x;
  p.ldx = ldx;
  p.k0 = k0;
  p.xmax = xmax;
  p.xmax2 = xmax2;
  p.d = d;
  p.ldd = ldd;
  p.dmax = dmax;
  p.part = C.at<float>(C.L.wpart[wslot]);
  p.pstride = C.L.wpart_stride[wslot];
  p.kpad = cdiv(k0, TB) * TB;
  p.tiles_k = p.kpad / TB;
  p.tiles_n = n / TB;
  return p;
}

int launch_wg(const Ctx& C, WgProb* ps, int np, int phase) {
  WgLaunch L{};
  int total = 0;
  for (int i = 0; i < np; ++i) {
    L.p[i] = ps[i];
    L.p[i].tile0 = total;
    total += ps[i].tiles_k * ps[i].tiles_n;
  }
  L.nprob = np;
  L.M = C.L.M;
  L.S = C.L.S[phase];
  L.chunk = C.L.chunk[phase];
  L.total = total;
  hipLaunchKernelGGL(wgrad_kernel, dim3(total * L.S), dim3(256), 0, C.s, L);
  PPO_TRY(hipGetLastError());
  return GO1_PPO_OK;
}

struct SegBuilder {
  SegTable T{};
  void add(float* dst, const float* src, int rows, int cols, int64_t lds, int nparts, int64_t pstride,
           int64_t ldd = -1) {
    Seg& s = T.s[T.nseg++];
    s.dst = dst;
    s.src = src;
    s.rows = rows;
    s.cols = cols;
    s.lds = lds;
    s.ldd = ldd < 0 ? cols : ldd;
    s.nparts = nparts;
    s.pstride = pstride;
    s.start = T.total;
    T.total += rows * cols;
  }
};

int launch_reduce(const Ctx& C, SegBuilder& B) {
  if (B.T.nseg > MAX_SEGS) return fail(GO1_PPO_E_ARG, "go1_ppo: segment table overflow");
  hipLaunchKernelGGL(reduce_kernel, dim3(cdiv(B.T.total, 64)), dim3(256), 0, C.s, B.T);
  PPO_TRY(hipGetLastError());
  return GO1_PPO_OK;
}

// weight-gradient segment of W slot i (partials [S][n][kpad]) into the flat gradient of parameter pi (row stride ldd)
void seg_w(const Ctx& C, SegBuilder& B, int wslot, int pi, int ldd, int phase) {
  const int n = C.L.wn[wslot], k = C.L.wk[wslot];
  const int kpad = cdiv(k, TB) * TB;
  B.add(C.gW(pi), C.at<float>(C.L.wpart[wslot]), n, k, kpad, C.L.S[phase], C.L.wpart_stride[wslot], ldd);
}

int pack_weights(const Ctx& C, bool adaptation_only, bool zero_max) {
  const Lay& L = C.L;
  PackTable T{};
  const int nw = adaptation_only ? 2 : W_N;
  uint32_t* wmax = C.at<uint32_t>(L.wmax);
  for (int i = 0; i < nw; ++i) {
    PackW& p = T.t[T.nt++];
    const int pi = kWParam[i];
    p.w = C.W(pi);
    p.n = L.wn[i];
    p.k = L.wk[i];
    p.ldw = (pi == IC0) ? L.H + L.P : L.wk[i];
    p.gap_at = (pi == IC0) ? L.H : 0;  // the critic's image: zero weights on G's latent columns
    p.gap = (pi == IC0) ? L.P : 0;
    p.G = cdiv(L.wk[i], 32);
    p.npad = L.wn[i];
    p.img = C.at<h8_t>(L.img[i]);
    p.imgt = L.imgt[i] ? C.at<h8_t>(L.imgt[i]) : nullptr;
    p.Gt = cdiv(L.wn[i], 32);
    p.npadt = L.wk[i];
    p.wmax = wmax + i;
    p.wexp = C.at<int32_t>(L.wexp) + i;
    p.start = T.total;
    T.total += L.wn[i] * L.wk[i];
  }
  if (zero_max) {  // otherwise finalize_kernel cleared them
    hipLaunchKernelGGL(zero_u32_kernel, dim3(1), dim3(64), 0, C.s, wmax, nw);
    PPO_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(wmax_kernel, dim3(32, T.nt), dim3(256), 0, C.s, T);
  PPO_TRY(hipGetLastError());
  hipLaunchKernelGGL(pack_kernel, dim3(cdiv(T.total, 256)), dim3(256), 0, C.s, T);
  PPO_TRY(hipGetLastError());
  return GO1_PPO_OK;
}

int check_ctx(const go1_ppo_dims* d, const go1_ppo_bufs* b, Ctx& C, void* stream) {
  std::string err;
  if (!make_layout(d, C.L, err)) return fail(GO1_PPO_E_ARG, err);
  if (!b || !b->params || !b->grads || !b->work || !b->hyper)
    return fail(GO1_PPO_E_ARG, "go1_ppo: params, grads, hyper and work are required");
  if ((((uintptr_t)b->work) & 255) != 0) return fail(GO1_PPO_E_ARG, "go1_ppo: work must be 256-byte aligned");
  C.d = d;
  C.b = b;
  C.ws = (char*)b->work;
  C.s = (hipStream_t)stream;
  return GO1_PPO_OK;
}

AdaptArgs adapt_args(const Ctx& C) {
  const Lay& L = C.L;
  AdaptArgs AD{};
  AD.M = L.M;
  AD.P = L.P;
  AD.hist = L.H;
  AD.num_train = (L.M / 5) * 4;  // int(data_size // 5 * 4) (ppo.py:166)
  AD.ldg = L.ldg;
  AD.a2a = C.at<float>(L.a2a);
  AD.w3a = C.W(IA4);
  AD.b3a = C.B(IA4);
  AD.G = C.at<float>(L.G);
  AD.latmax = C.mx(MX_LAT);
  AD.d1p = C.at<float>(L.d1p);
  AD.w1p = C.W(IP0);
  AD.hyper = C.b->hyper;
  AD.d2a = C.at<float>(L.d2a);
  AD.d2amax = C.mx(MX_D2A);
  AD.part = C.at<float>(L.apart);
  AD.lstr = adapt_stride(L.P);
  return AD;
}

// the adaptation module's forward through L1, L2 (ELU) from the gathered rows
int adapt_forward(const Ctx& C) {
  const Lay& L = C.L;
  int rc;
  float *G = C.at<float>(L.G), *a1a = C.at<float>(L.a1a), *a2a = C.at<float>(L.a2a);
  if ((rc = launch_xw(C, EPI_ELU,
                      xw_prob(C, G, L.ldg, L.H, C.mx(MX_G), W_A0, false, HA1, C.B(IA0), nullptr, 0, a1a, HA1,
                              C.mx(MX_A1A), nullptr),
                      nullptr)))
    return rc;
  return launch_xw(C, EPI_ELU,
                   xw_prob(C, a1a, HA1, HA1, C.mx(MX_A1A), W_A2, false, HA2, C.B(IA2), nullptr, 0, a2a, HA2,
                           C.mx(MX_A2A), nullptr),
                   nullptr);
}

// delta a1a = (W2a^T delta2a) * ELU'(a1a)
int adapt_backward_l2(const Ctx& C) {
  const Lay& L = C.L;
  return launch_xw(C, EPI_DELU,
                   xw_prob(C, C.at<float>(L.d2a), HA2, HA2, C.mx(MX_D2A), W_A2, true, HA1, nullptr, C.at<float>(L.a1a),
                           HA1, C.at<float>(L.d1a), HA1, C.mx(MX_D1A), C.at<float>(L.cs1a)),
                   nullptr);
}

void adapt_segments(const Ctx& C, SegBuilder& SB, int phase) {
  const Lay& L = C.L;
  const int P = L.P, as = adapt_stride(P);
  const float* ap = C.at<float>(L.apart);
  seg_w(C, SB, W_A0, IA0, L.H, phase);
  SB.add(C.gB(IA0), C.at<float>(L.cs1a), 1, HA1, 0, L.MT, HA1);
  seg_w(C, SB, W_A2, IA2, HA1, phase);
  SB.add(C.gB(IA2), ap + P * 128 + P, 1, HA2, 0, L.HB, as);
  SB.add(C.gW(IA4), ap, 1, P * 128, 0, L.HB, as);
  SB.add(C.gB(IA4), ap + P * 128, 1, P, 0, L.HB, as);
}

int grad_phase0(const Ctx& C) {
  const Lay& L = C.L;
  const go1_ppo_bufs* b = C.b;
  const int H = L.H, P = L.P;
  if (!b->obs_history || !b->privileged_obs || !b->actions || !b->values || !b->advantages || !b->returns ||
      !b->actions_log_prob || !b->mu || !b->sigma || !b->idx || b->hist_ld < H)
    return fail(GO1_PPO_E_ARG, "go1_ppo_grad: storage tensors and idx are required");
  int rc;
  // the mini-batch rows (the max slots were cleared by the previous step's finalize_kernel, or are fresh)
  float *G = C.at<float>(L.G), *Bb = C.at<float>(L.Bb);
  {
    GatherArgs ga{};
    ga.hist = b->obs_history;
    ga.hld = b->hist_ld;
    ga.priv = b->privileged_obs;
    ga.act = b->actions;
    ga.mu = b->mu;
    ga.sigma = b->sigma;
    ga.logp = b->actions_log_prob;
    ga.adv = b->advantages;
    ga.ret = b->returns;
    ga.val = b->values;
    ga.idx = b->idx;
    ga.M = L.M;
    ga.H = H;
    ga.P = P;
    ga.A = L.A;
    ga.ldg = L.ldg;
    ga.bw = L.bw;
    ga.G = G;
    ga.B = Bb;
    ga.mx = C.mx(MX_G);
    hipLaunchKernelGGL(gather_kernel, dim3(std::min(cdiv(L.M, 16), GATHER_BLOCKS_MAX)), dim3(256), 0, C.s, ga);
    PPO_TRY(hipGetLastError());
  }
  float *a1a = C.at<float>(L.a1a);
  float *p1 = C.at<float>(L.p1), *p2 = C.at<float>(L.p2), *p3 = C.at<float>(L.p3);
  float *c1 = C.at<float>(L.c1), *c2 = C.at<float>(L.c2), *c3 = C.at<float>(L.c3);
  float *d3p = C.at<float>(L.d3p), *d3c = C.at<float>(L.d3c), *d2p = C.at<float>(L.d2p), *d2c = C.at<float>(L.d2c);
  float *d1p = C.at<float>(L.d1p), *d1c = C.at<float>(L.d1c), *d2a = C.at<float>(L.d2a), *d1a = C.at<float>(L.d1a);
  // ---- forward: adaptation module (ppo.py:110 ac.act -> update_distribution -> adaptation_module)
  if ((rc = adapt_forward(C))) return rc;
  AdaptArgs AD = adapt_args(C);
  hipLaunchKernelGGL(adapt_kernel<0>, dim3(L.HB), dim3(256), 0, C.s, AD);
  PPO_TRY(hipGetLastError());
  // ---- forward: actor [hist, latent] and critic [hist, latent (zero weights), priv]
  {
    XwProb pa = xw_prob(C, G, L.ldg, H + P, C.mx(MX_G), W_P0, false, H1, C.B(IP0), nullptr, 0, p1, H1, C.mx(MX_P1),
                        nullptr, C.mx(MX_LAT));
    XwProb pc = xw_prob(C, G, L.ldg, H + 2 * P, C.mx(MX_G), W_C0, false, H1, C.B(IC0), nullptr, 0, c1, H1,
                        C.mx(MX_C1), nullptr, C.mx(MX_LAT));
    if ((rc = launch_xw(C, EPI_ELU, pa, &pc))) return rc;
    pa = xw_prob(C, p1, H1, H1, C.mx(MX_P1), W_P2, false, H2, C.B(IP2), nullptr, 0, p2, H2, C.mx(MX_P2), nullptr);
    pc = xw_prob(C, c1, H1, H1, C.mx(MX_C1), W_C2, false, H2, C.B(IC2), nullptr, 0, c2, H2, C.mx(MX_C2), nullptr);
    if ((rc = launch_xw(C, EPI_ELU, pa, &pc))) return rc;
    pa = xw_prob(C, p2, H2, H2, C.mx(MX_P2), W_P4, false, H3, C.B(IP4), nullptr, 0, p3, H3, C.mx(MX_P3), nullptr);
    pc = xw_prob(C, c2, H2, H2, C.mx(MX_C2), W_C4, false, H3, C.B(IC4), nullptr, 0, c3, H3, C.mx(MX_C3), nullptr);
    if ((rc = launch_xw(C, EPI_ELU, pa, &pc))) return rc;
  }
  // ---- heads, loss, backward through L4 (ppo.py:111-155)
  HeadArgs HD{};
  HD.M = L.M;
  HD.A = L.A;
  HD.bw = L.bw;
  HD.B = Bb;
  HD.a3p = p3;
  HD.a3c = c3;
  HD.w4p = C.W(IP6);
  HD.b4p = C.B(IP6);
  HD.w4c = C.W(IC6);
  HD.b4c = C.B(IC6);
  HD.std_ = b->params + L.pstd;
  HD.hyper = b->hyper;
  HD.d3p = d3p;
  HD.d3c = d3c;
  HD.d3pmax = C.mx(MX_D3P);
  HD.d3cmax = C.mx(MX_D3C);
  HD.part = C.at<float>(L.hpart);
  HD.hstr = head_stride(L.A);
  if (L.A <= 12)
    hipLaunchKernelGGL(head_kernel<12>, dim3(L.HB), dim3(256), 0, C.s, HD);
  else
    hipLaunchKernelGGL(head_kernel<16>, dim3(L.HB), dim3(256), 0, C.s, HD);
  PPO_TRY(hipGetLastError());
  // ---- backward through L3, L2 (delta = W^T delta_next * ELU'(a))
  {
    XwProb pa = xw_prob(C, d3p, H3, H3, C.mx(MX_D3P), W_P4, true, H2, nullptr, p2, H2, d2p, H2, C.mx(MX_D2P),
                        C.at<float>(L.cs2p));
    XwProb pc = xw_prob(C, d3c, H3, H3, C.mx(MX_D3C), W_C4, true, H2, nullptr, c2, H2, d2c, H2, C.mx(MX_D2C),
                        C.at<float>(L.cs2c));
    if ((rc = launch_xw(C, EPI_DELU, pa, &pc))) return rc;
    pa = xw_prob(C, d2p, H2, H2, C.mx(MX_D2P), W_P2, true, H1, nullptr, p1, H1, d1p, H1, C.mx(MX_D1P),
                 C.at<float>(L.cs1p));
    pc = xw_prob(C, d2c, H2, H2, C.mx(MX_D2C), W_C2, true, H1, nullptr, c1, H1, d1c, H1, C.mx(MX_D1C),
                 C.at<float>(L.cs1c));
    if ((rc = launch_xw(C, EPI_DELU, pa, &pc))) return rc;
  }
  // ---- the latent's gradient into the adaptation module, its L3 and L2 backward
  hipLaunchKernelGGL(adapt_kernel<2>, dim3(L.HB), dim3(256), 0, C.s, AD);
  PPO_TRY(hipGetLastError());
  if ((rc = adapt_backward_l2(C))) return rc;
  // ---- weight gradients of the GEMM layers, one grouped launch
  {
    WgProb ps[8];
    ps[0] = wg_prob(C, W_P0, G, L.ldg, H + P, C.mx(MX_G), d1p, H1, H1, C.mx(MX_D1P), C.mx(MX_LAT));
    ps[1] = wg_prob(C, W_C0, G, L.ldg, H + 2 * P, C.mx(MX_G), d1c, H1, H1, C.mx(MX_D1C), C.mx(MX_LAT));
    ps[2] = wg_prob(C, W_P2, p1, H1, H1, C.mx(MX_P1), d2p, H2, H2, C.mx(MX_D2P));
    ps[3] = wg_prob(C, W_C2, c1, H1, H1, C.mx(MX_C1), d2c, H2, H2, C.mx(MX_D2C));
    ps[4] = wg_prob(C, W_P4, p2, H2, H2, C.mx(MX_P2), d3p, H3, H3, C.mx(MX_D3P));
    ps[5] = wg_prob(C, W_C4, c2, H2, H2, C.mx(MX_C2), d3c, H3, H3, C.mx(MX_D3C));
    ps[6] = wg_prob(C, W_A0, G, L.ldg, H, C.mx(MX_G), d1a, HA1, HA1, C.mx(MX_D1A));
    ps[7] = wg_prob(C, W_A2, a1a, HA1, HA1, C.mx(MX_A1A), d2a, HA2, HA2, C.mx(MX_D2A));
    if ((rc = launch_wg(C, ps, 8, 0))) return rc;
  }
  // ---- partials -> flat gradient (+ aux: surrogate, value, KL sums)
  SegBuilder SB;
  const int hs = head_stride(L.A), A = L.A;
  const float* hp = C.at<float>(L.hpart);
  const int o_db4p = A * 128, o_db3p = o_db4p + A, o_dW4c = o_db3p + 128, o_db4c = o_dW4c + 128, o_db3c = o_db4c + 1,
            o_dstd = o_db3c + 128, o_loss = o_dstd + A;
  SB.add(b->grads, hp + o_loss, 1, 3, 0, L.HB, hs);
  adapt_segments(C, SB, 0);
  seg_w(C, SB, W_P0, IP0, H + P, 0);
  SB.add(C.gB(IP0), C.at<float>(L.cs1p), 1, H1, 0, L.MT, H1);
  seg_w(C, SB, W_P2, IP2, H1, 0);
  SB.add(C.gB(IP2), C.at<float>(L.cs2p), 1, H2, 0, L.MT, H2);
  seg_w(C, SB, W_P4, IP4, H2, 0);
  SB.add(C.gB(IP4), hp + o_db3p, 1, H3, 0, L.HB, hs);
  SB.add(C.gW(IP6), hp, 1, A * 128, 0, L.HB, hs);
  SB.add(C.gB(IP6), hp + o_db4p, 1, A, 0, L.HB, hs);
  {  // the critic's first layer: G's hist columns, then its priv columns (the latent columns' gradient is dropped)
    const int kpad = cdiv(H + 2 * P, TB) * TB;
    const float* wp = C.at<float>(L.wpart[W_C0]);
    SB.add(C.gW(IC0), wp, H1, H, kpad, L.S[0], L.wpart_stride[W_C0], H + P);
    SB.add(C.gW(IC0) + H, wp + H + P, H1, P, kpad, L.S[0], L.wpart_stride[W_C0], H + P);
  }
  SB.add(C.gB(IC0), C.at<float>(L.cs1c), 1, H1, 0, L.MT, H1);
  seg_w(C, SB, W_C2, IC2, H1, 0);
  SB.add(C.gB(IC2), C.at<float>(L.cs2c), 1, H2, 0, L.MT, H2);
  seg_w(C, SB, W_C4, IC4, H2, 0);
  SB.add(C.gB(IC4), hp + o_db3c, 1, H3, 0, L.HB, hs);
  SB.add(C.gW(IC6), hp + o_dW4c, 1, 128, 0, L.HB, hs);
  SB.add(C.gB(IC6), hp + o_db4c, 1, 1, 0, L.HB, hs);
  SB.add(b->grads + NAUX + L.pstd, hp + o_dstd, 1, A, 0, L.HB, hs);
  return launch_reduce(C, SB);
}

int grad_phase1(const Ctx& C) {
  const Lay& L = C.L;
  const go1_ppo_bufs* b = C.b;
  const int P = L.P;
  int rc;
  // the gathered rows G are this mini-batch's (phase 0); the maxima phase 1 recomputes were cleared by step 0
  if ((rc = adapt_forward(C))) return rc;
  AdaptArgs AD = adapt_args(C);
  hipLaunchKernelGGL(adapt_kernel<1>, dim3(L.HB), dim3(256), 0, C.s, AD);
  PPO_TRY(hipGetLastError());
  if ((rc = adapt_backward_l2(C))) return rc;
  {
    WgProb ps[2];
    ps[0] = wg_prob(C, W_A0, C.at<float>(L.G), L.ldg, L.H, C.mx(MX_G), C.at<float>(L.d1a), HA1, HA1, C.mx(MX_D1A));
    ps[1] = wg_prob(C, W_A2, C.at<float>(L.a1a), HA1, HA1, C.mx(MX_A1A), C.at<float>(L.d2a), HA2, HA2,
                    C.mx(MX_D2A));
    if ((rc = launch_wg(C, ps, 2, 1))) return rc;
  }
  SegBuilder SB;
  const int as = adapt_stride(P);
  const float* ap = C.at<float>(L.apart);
  SB.add(b->grads + 3, ap + P * 128 + P + 128, 1, 2, 0, L.HB, as);  // aux[3], aux[4]: adaptation loss sums
  adapt_segments(C, SB, 1);
  return launch_reduce(C, SB);
}

int step_phase(const Ctx& C, int phase) {
  const Lay& L = C.L;
  const go1_ppo_bufs* b = C.b;
  if (!b->steps || !b->lr || !b->losses || !b->exp_avg || !b->exp_avg_sq || !b->ad_exp_avg || !b->ad_exp_avg_sq)
    return fail(GO1_PPO_E_ARG, "go1_ppo_step: Adam state, steps, lr and losses are required");
  const float* g = b->grads + NAUX;
  const int64_t n = phase == 0 ? L.np_total : L.np_adapt;
  if (phase == 0) {
    hipLaunchKernelGGL(norm_kernel, dim3(NORM_BLOCKS), dim3(256), 0, C.s, g, n, C.at<double>(L.normp));
    PPO_TRY(hipGetLastError());
  }
  Finalize F{};
  F.phase = phase;
  F.M = L.M;
  F.num_train = (L.M / 5) * 4;
  F.nsel_all = L.P;
  F.hyper = b->hyper;
  F.aux = b->grads;
  F.norm_part = C.at<double>(L.normp);
  F.lr = b->lr;
  F.steps = b->steps;
  F.losses = b->losses;
  F.scal = C.at<float>(L.scal) + 8 * phase;
  // phase 0 clears the maxima phase 1 recomputes and the weight maxima of the pack that follows; phase 1 clears
  // every activation / gradient maximum (the next mini-batch) and the adaptation weights' maxima
  if (phase == 0) {
    F.zero[0] = C.mx(MX_A1A), F.nz[0] = 2;
    F.zero[1] = C.mx(MX_D2A), F.nz[1] = 2;
    F.zero[2] = C.at<uint32_t>(L.wmax), F.nz[2] = (int)W_N;
  } else {
    F.zero[0] = C.mx(MX_G), F.nz[0] = (int)MX_N;
    F.zero[1] = C.at<uint32_t>(L.wmax), F.nz[1] = 2;
    F.zero[2] = C.at<uint32_t>(L.wmax), F.nz[2] = 0;
  }
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, C.s, F);
  PPO_TRY(hipGetLastError());
  float* m1 = phase == 0 ? b->exp_avg : b->ad_exp_avg;
  float* m2 = phase == 0 ? b->exp_avg_sq : b->ad_exp_avg_sq;
  const int nblk = (int)((n + 255) / 256);
  hipLaunchKernelGGL(adam_kernel, dim3(nblk > 1024 ? 1024 : nblk), dim3(256), 0, C.s, b->params, g, m1, m2, n,
                     (const float*)F.scal);
  PPO_TRY(hipGetLastError());
  return pack_weights(C, phase == 1, false);
}

}  // namespace

extern "C" {

const char* go1_ppo_last_error(void) { return g_err.c_str(); }

int go1_ppo_param_count(const go1_ppo_dims* d, int64_t* total, int64_t* adaptation) {
  Lay L;
  std::string err;
  if (!make_layout(d, L, err)) return fail(GO1_PPO_E_ARG, err);
  if (total) *total = L.np_total;
  if (adaptation) *adaptation = L.np_adapt;
  return GO1_PPO_OK;
}

int go1_ppo_workspace_bytes(const go1_ppo_dims* d, int64_t* bytes) {
  Lay L;
  std::string err;
  if (!make_layout(d, L, err)) return fail(GO1_PPO_E_ARG, err);
  if (bytes) *bytes = (int64_t)L.total;
  return GO1_PPO_OK;
}

int go1_ppo_pack(const go1_ppo_dims* d, const go1_ppo_bufs* b, void* stream) {
  Ctx C;
  int rc = check_ctx(d, b, C, stream);
  if (rc) return rc;
  return pack_weights(C, false, true);
}

int go1_ppo_grad(const go1_ppo_dims* d, const go1_ppo_bufs* b, int32_t phase, void* stream) {
  Ctx C;
  int rc = check_ctx(d, b, C, stream);
  if (rc) return rc;
  if (phase == 0) return grad_phase0(C);
  if (phase == 1) return grad_phase1(C);
  return fail(GO1_PPO_E_ARG, "go1_ppo_grad: phase 0 or 1");
}

int go1_ppo_step(const go1_ppo_dims* d, const go1_ppo_bufs* b, int32_t phase, void* stream) {
  Ctx C;
  int rc = check_ctx(d, b, C, stream);
  if (rc) return rc;
  if (phase != 0 && phase != 1) return fail(GO1_PPO_E_ARG, "go1_ppo_step: phase 0 or 1");
  return step_phase(C, phase);
}

#ifdef PPO_STAMPS
extern "C" int go1_ppo_xw_stamps(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xw_stamps), sizeof(g_xw_stamps), 0, hipMemcpyDeviceToHost) != hipSuccess;
}
#endif
// ---- test entry points: one GEMM of each kind on caller tensors (x rows 16-byte aligned: k % 4 == 0 or padded)
int go1_ppo_test_linear(const float* x, int64_t rows, int32_t k, const float* w, const float* bias, int32_t n,
                        int32_t elu, float* y, void* work, int64_t work_bytes, int32_t reps, void* stream) {
  if (!x || !w || !bias || !y || !work || rows < 1 || k < 1 || n < TB || n % TB != 0)
    return fail(GO1_PPO_E_ARG, "go1_ppo_test_linear: bad argument (n a multiple of 128)");
  const int G = cdiv(k, 32), ldx = cdiv(k, 4) * 4;
  const size_t need = 1024 + (size_t)G * 32 * n * 4 + (size_t)rows * ldx * 4;
  if ((size_t)work_bytes < need) return fail(GO1_PPO_E_ARG, "go1_ppo_test_linear: work too small");
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)work;
  uint32_t* mx = (uint32_t*)ws;  // [0] x max, [1] w max, [2] y max
  int32_t* wexp = (int32_t*)(ws + 64);
  h8_t* img = (h8_t*)(ws + 1024);
  float* xp = (float*)(ws + 1024 + (size_t)G * 32 * n * 4);  // x with rows padded to 16 bytes
  PPO_TRY(hipMemsetAsync(ws, 0, need, s));
  PPO_TRY(hipMemcpy2DAsync(xp, ldx * 4, x, (size_t)k * 4, (size_t)k * 4, rows, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(absmax_kernel, dim3(256), dim3(256), 0, s, x, rows, k, (int64_t)k, mx);
  PackTable T{};
  PackW& p = T.t[0];
  T.nt = 1;
  p.w = w;
  p.n = n;
  p.k = k;
  p.ldw = k;
  p.G = G;
  p.npad = n;
  p.img = img;
  p.wmax = mx + 1;
  p.wexp = wexp;
  T.total = n * k;
  hipLaunchKernelGGL(wmax_kernel, dim3(32, 1), dim3(256), 0, s, T);
  hipLaunchKernelGGL(pack_kernel, dim3(cdiv(T.total, 256)), dim3(256), 0, s, T);
  XwLaunch L{};
  XwProb& q = L.p[0];
  q.a = xp;
  q.lda = ldx;
  q.k0 = k;
  q.amax = mx;
  q.w = img;
  q.wexp = wexp;
  q.G = G;
  q.n = n;
  q.bias = bias;
  q.c = y;
  q.ldc = n;
  q.cmax = mx + 2;
  q.tiles_n = n / TB;
  L.nprob = 1;
  L.M = (int)rows;
  L.total = cdiv((int)rows, TB) * q.tiles_n;
  for (int i = 0; i < (reps > 1 ? reps : 1); ++i) {
    if (elu)
      hipLaunchKernelGGL(xw_kernel<EPI_ELU>, dim3(L.total), dim3(256), 0, s, L);
    else
      hipLaunchKernelGGL(xw_kernel<EPI_LIN>, dim3(L.total), dim3(256), 0, s, L);
  }
  PPO_TRY(hipGetLastError());
  return GO1_PPO_OK;
}

int go1_ppo_test_wgrad(const float* x, const float* d, int64_t rows, int32_t k, int32_t n, float* dw, void* work,
                       int64_t work_bytes, int32_t reps, void* stream) {
  if (!x || !d || !dw || !work || rows < 1 || k < 1 || n < TB || n % TB != 0)
    return fail(GO1_PPO_E_ARG, "go1_ppo_test_wgrad: bad argument (n a multiple of 128)");
  const int kpad = cdiv(k, TB) * TB, ldx = cdiv(k, 4) * 4;
  int S = (int)(cdiv((int)rows, TB) * TB / 256);
  S = S >= 16 ? 16 : (S >= 8 ? 8 : (S < 1 ? 1 : S));
  const int chunk = cdiv(cdiv((int)rows, S), 32) * 32;
  S = cdiv((int)rows, chunk);
  const size_t need = 1024 + (size_t)S * n * kpad * 4 + (size_t)rows * ldx * 4;
  if ((size_t)work_bytes < need) return fail(GO1_PPO_E_ARG, "go1_ppo_test_wgrad: work too small");
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)work;
  uint32_t* mx = (uint32_t*)ws;
  float* part = (float*)(ws + 1024);
  float* xp = part + (size_t)S * n * kpad;
  PPO_TRY(hipMemsetAsync(ws, 0, 1024, s));
  PPO_TRY(hipMemcpy2DAsync(xp, ldx * 4, x, (size_t)k * 4, (size_t)k * 4, rows, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(absmax_kernel, dim3(256), dim3(256), 0, s, x, rows, k, (int64_t)k, mx);
  hipLaunchKernelGGL(absmax_kernel, dim3(256), dim3(256), 0, s, d, rows, n, (int64_t)n, mx + 1);
  WgLaunch L{};
  WgProb& p = L.p[0];
  p.x = xp;
  p.ldx = ldx;
  p.k0 = k;
  p.xmax = mx;
  p.d = d;
  p.ldd = n;
  p.dmax = mx + 1;
  p.part = part;
  p.pstride = (int64_t)n * kpad;
  p.kpad = kpad;
  p.tiles_k = kpad / TB;
  p.tiles_n = n / TB;
  L.nprob = 1;
  L.M = (int)rows;
  L.S = S;
  L.chunk = chunk;
  L.total = p.tiles_k * p.tiles_n;
  for (int i = 0; i < (reps > 1 ? reps : 1); ++i)
    hipLaunchKernelGGL(wgrad_kernel, dim3(L.total * S), dim3(256), 0, s, L);
  PPO_TRY(hipGetLastError());
  SegBuilder SB;
  SB.add(dw, part, n, k, kpad, S, (int64_t)n * kpad);
  hipLaunchKernelGGL(reduce_kernel, dim3(cdiv(SB.T.total, 64)), dim3(256), 0, s, SB.T);
  PPO_TRY(hipGetLastError());
  return GO1_PPO_OK;
}

}  // extern "C"
