// go1_terrain.hip -- the single_path tunnel terrain generated on the MI355X.
//
// Replaces the reference's init-time numpy loop over sub-terrains:
//   go1_gym/utils/tunnel.py:51-126 (Terrain.__init__: one difficulty draw, then a top and a bottom
//   SubTerrain per sub-terrain, the ceiling flip and 0.05 m clamp :96-98, the 0.8 m ceiling / 0.5 m
//   floor outside the tunnel :80-81) and :189-217 (add_terrain_to_map: the tunnel placed at
//   [start_x, end_x) x [start_y, end_y) of its tile), with
//   go1_gym/utils/tunnel_fn.py:99-163 (TerrainFunctions.single_path: up to two pyramidal wedges per
//   layer, heights from vec_plane_from_points :3-21, walls on the floor's border, int truncation).
//
// Two launches on the caller's stream:
//   1. tunnel_draw_kernel (one wave): numpy's legacy RandomState stream -- MT19937 with
//      mt19937_seed seeding, random_sample doubles (a >> 5, b >> 6) / 2^53, uniform(low, high) =
//      low + (high - low) u -- drawn in the reference's order (the draw count of a layer depends on
//      its own p2 draw, so the stream is sequential); the wave twists the 624-word state in
//      parallel batches of 64 and every lane walks the stream in lockstep.  Output: one record of
//      wedge parameters per sub-terrain (GO1_TUNNEL_REC doubles).
//   2. tunnel_tile_kernel (one 256-thread block per sub-terrain): 16 lanes build the 2 layers x
//      2 wedges x 4 face planes (numpy's np.cross / np.sum operation order, f64), then the block
//      rasterises both 80 x 40 layers of the tile, coalesced f32 stores.
// Every f64 operation is the one numpy performs, in numpy's order, compiled without contraction
// (-ffp-contract=off), so a seed yields the reference's tiles bit for bit
// (tests/test_gpu_terrain.py against terrain.make_single_path, itself pinned to the reference's
// tiles by tests/test_terrain.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/go1_mi355x.h"

#pragma clang fp contract(off)

int go1_internal_fail(int code, const std::string& msg);  // go1_step.hip: sets go1_last_error()

namespace {

constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MT_MATRIX_A = 0x9908b0dfu, MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu;

// record layout (doubles): [0] difficulty, then per layer (0 top, 1 bottom) at 1 + 16 layer:
// p1, p2, num_y, off_y[2], off_x[2], mean_x[2], mean_z[2], pw[2], pl[2], (pad)
constexpr int REC_LAYER = 16;
static_assert(1 + 2 * REC_LAYER <= GO1_TUNNEL_REC, "record layout");

struct MtWave {
  uint32_t* key;  // LDS, MT_N words
  uint32_t* out;  // LDS, MT_N tempered words
  int pos;        // wave-uniform
};

// mt19937_gen of numpy (randomkit): key[i] = key[i + 397 mod 624] ^ twist(key[i], key[i + 1]),
// in place and in index order.  Batches of 64 consecutive indices are exact: within a batch every
// lane reads before any lane writes (one wave, in order), key[i + 1] is still old (same or a later
// batch) except for i = 623, whose key[0] was rewritten in the first batch as in the sequential
// loop, and key[i - 227] (i >= 227) was rewritten in an earlier batch (batch length 64 < 227).
__device__ void mt_twist(MtWave& s, int lane) {
  for (int b = 0; b < MT_N; b += 64) {
    const int i = b + lane;
    uint32_t nv = 0;
    if (i < MT_N) {
      const uint32_t y = (s.key[i] & MT_UPPER) | (s.key[i + 1 < MT_N ? i + 1 : 0] & MT_LOWER);
      nv = s.key[i + MT_M < MT_N ? i + MT_M : i + MT_M - MT_N] ^ (y >> 1) ^ ((y & 1u) ? MT_MATRIX_A : 0u);
    }
    __syncthreads();  // (one-wave block) every lane's reads of this batch are done
    if (i < MT_N) s.key[i] = nv;
    __syncthreads();
  }
  for (int i = lane; i < MT_N; i += 64) {  // tempering (mt19937_next32)
    uint32_t y = s.key[i];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    s.out[i] = y;
  }
  __syncthreads();
  s.pos = 0;
}

__device__ uint32_t mt_next32(MtWave& s, int lane) {
  if (s.pos == MT_N) mt_twist(s, lane);
  return s.out[s.pos++];
}

// legacy random_sample / next_double: (a * 2^26 + b) / 2^53
__device__ double mt_next_double(MtWave& s, int lane) {
  const int32_t a = (int32_t)(mt_next32(s, lane) >> 5), b = (int32_t)(mt_next32(s, lane) >> 6);
  return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// RandomState.uniform(low, high): random_uniform(lower, range) = lower + range * u with
// range = high - low (mtrand.pyx), one double per element in C order
__device__ double uniform(MtWave& s, int lane, double lo, double hi) { return lo + (hi - lo) * mt_next_double(s, lane); }

__global__ __launch_bounds__(64) void tunnel_draw_kernel(go1_tunnel_params p, double* __restrict__ rec) {
  __shared__ uint32_t s_key[MT_N], s_out[MT_N];
  const int lane = threadIdx.x;
  MtWave s{s_key, s_out, MT_N};
  if (lane == 0) {  // mt19937_seed (legacy seeding of an integer seed)
    uint32_t v = p.seed;
    for (int i = 0; i < MT_N; ++i) {
      s_key[i] = v;
      v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();
  // SubTerrain extent in metres (tunnel_fn.py:102): l = pixel_x hs, w = pixel_y hs
  const double w = (double)p.sub_y * p.horizontal_scale;
  // mean_x = np.linspace(-w/2, w/2, 3)[1:-1] (tunnel_fn.py:127): start + 1 * step
  const double start = -w / 2.0, stop = w / 2.0;
  const double step = (stop - start) / 2.0;
  const double cx = 1.0 * step + start;
  const int n_sub = p.num_rows * p.num_cols;
  for (int k = 0; k < n_sub; ++k) {
    double* R = rec + (size_t)k * GO1_TUNNEL_REC;
    const double diff = uniform(s, lane, 0.0, 1.0);  // difficulty (tunnel.py:90), unused by single_path
    if (lane == 0) R[0] = diff;
#pragma unroll
    for (int layer = 0; layer < 2; ++layer) {
      const bool top = layer == 0;
      const double p1 = uniform(s, lane, 0.0, 1.0), p2 = uniform(s, lane, 0.0, 1.0);
      const int num_y = p2 < p.p_double ? 2 : 1;
      // tunnel_fn.py:111-124: offsets y then x, each a (num_y, 1) draw (register arrays, static
      // indices: the draws are uniform branches on num_y)
      const double oy = top ? 0.6 : 0.4, ox = top ? 0.3 : 0.2;
      double offy[2] = {0.0, 0.0}, offx[2] = {0.0, 0.0}, mx[2] = {0.0, 0.0}, mz[2] = {0.0, 0.0};
      double pw[2] = {0.0, 0.0}, pl[2] = {0.0, 0.0};
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (i < num_y) offy[i] = uniform(s, lane, -oy, oy);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (i < num_y) offx[i] = uniform(s, lane, -ox, ox);
      double hmax, hmin;
      if (p1 < p.p_flat) { hmax = top ? 0.4 : 0.15; hmin = top ? 0.7 : 0.3; }
      else { hmax = 0.0; hmin = 0.0; }
      const double lw_lo = top ? 0.2 : 0.1, lw_hi = top ? 0.4 : 0.3;
      // mean_x (after meshgrid) += offset_x; mean_z = uniform(mean_x) * (hmax - hmin) + hmin
      // (uniform(low=mean_x, high=1.0): range = 1.0 - mean_x, element-wise)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (i < num_y) {
          mx[i] = cx + offx[i];
          const double u = mx[i] + (1.0 - mx[i]) * mt_next_double(s, lane);
          mz[i] = u * (hmax - hmin) + hmin;
        }
      // pw, pl = uniform(lw_low, lw_high, size=(2, num_y)): row 0 then row 1
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (i < num_y) pw[i] = uniform(s, lane, lw_lo, lw_hi);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (i < num_y) pl[i] = uniform(s, lane, lw_lo, lw_hi);
      if (lane == 0) {
        double* L = R + 1 + REC_LAYER * layer;
        L[0] = p1; L[1] = p2; L[2] = (double)num_y;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          L[3 + i] = offy[i]; L[5 + i] = offx[i]; L[7 + i] = mx[i]; L[9 + i] = mz[i];
          L[11 + i] = pw[i]; L[13 + i] = pl[i];
        }
      }
    }
  }
}

// np.linspace(start, stop, num)[k] (numpy 2.x function_base.py): k * ((stop - start) / (num - 1))
// + start, the last element exactly stop
__device__ __forceinline__ double linspace_at(double start, double stop, int num, int k) {
  if (k == num - 1) return stop;
  const double step = (stop - start) / (double)(num - 1);
  return (double)k * step + start;
}

struct Face {
  double dc, ac, bc;  // d / c, a / c, b / c (vec_plane_from_points :15-18)
};

__global__ __launch_bounds__(256) void tunnel_tile_kernel(go1_tunnel_params p, const double* __restrict__ rec,
                                                          const int32_t* __restrict__ extents,
                                                          float* __restrict__ tiles) {
  __shared__ Face s_face[2][2][4];  // layer, wedge, face
  __shared__ int s_num_y[2];
  const int k = blockIdx.x;
  const double* r = rec + (size_t)k * GO1_TUNNEL_REC;
  const int tid = threadIdx.x;
  if (tid < 16) {
    const int layer = tid >> 3, wedge = (tid >> 2) & 1, face = tid & 3;
    const double* L = r + 1 + REC_LAYER * layer;
    const int num_y = (int)L[2];
    if (wedge < num_y) {
      const double mx = L[7 + wedge], my = L[3 + wedge], mz = L[9 + wedge];
      const double pw = L[11 + wedge], pl = L[13 + wedge];
      // wedge_points (tunnel_fn.py:134-141): corners (+-pw + mean_x, +-pl + mean_y, 0), apex = means;
      // faces [[0, 1, apex], [1, 2, apex], [2, 3, apex], [3, 0, apex]] (:142-148)
      const double cxs[4] = {pw + mx, -pw + mx, -pw + mx, pw + mx};
      const double cys[4] = {pl + my, pl + my, -pl + my, -pl + my};
      const int i1 = face, i2 = (face + 1) & 3;
      const double p1[3] = {cxs[i1], cys[i1], 0.0}, p2[3] = {cxs[i2], cys[i2], 0.0}, p3[3] = {mx, my, mz};
      const double v1[3] = {p3[0] - p1[0], p3[1] - p1[1], p3[2] - p1[2]};
      const double v2[3] = {p3[0] - p2[0], p3[1] - p2[1], p3[2] - p2[2]};
      // np.cross: each component a product minus a product, rounded separately
      const double t0 = v1[1] * v2[2], u0 = v1[2] * v2[1];
      const double t1 = v1[2] * v2[0], u1 = v1[0] * v2[2];
      const double t2 = v1[0] * v2[1], u2 = v1[1] * v2[0];
      const double a = t0 - u0, b = t1 - u1, c = t2 - u2;
      // np.sum(cp * p3, axis=-1): products, then a left-to-right sum
      const double d = (a * p3[0] + b * p3[1]) + c * p3[2];
      s_face[layer][wedge][face] = Face{d / c, a / c, b / c};
    }
    if (tid == 0 || tid == 8) s_num_y[layer] = num_y;
  }
  __syncthreads();
  const int nx = p.tile_x, ny = p.tile_y, pix = nx * ny;
  const int sx = extents[4 * k], ex = extents[4 * k + 1], sy = extents[4 * k + 2], ey = extents[4 * k + 3];
  const int px = p.sub_x, py = p.sub_y;  // SubTerrain height_field_raw shape (pixel_x, pixel_y)
  const double hs = p.horizontal_scale, vs = p.vertical_scale;
  const double l = (double)px * hs, w = (double)py * hs;
  const double unit = (double)(int64_t)(1.0 / vs);
  const double ceil_out = unit * p.ceiling_height, floor_out = 0.5 * unit;  // tunnel.py:80-81
  const double ceil_raw = p.ceiling_height / vs, ceil_min = 0.05 / vs;   // tunnel.py:96-98
  float* out = tiles + (size_t)k * 2 * pix;
  for (int idx = tid; idx < 2 * pix; idx += 256) {
    const int layer = idx / pix, x = (idx % pix) / ny, y = idx % ny;
    double v;
    if (x >= sx && x < ex && y >= sy && y < ey) {
      // tile[layer, sx + a, sy + b] = height_field_raw.T[a, b] = height_field_raw[b, a]
      const int a = x - sx, b = y - sy;
      // points_coord[b, a] = (linspace(-w/2, w/2, pixel_y)[a], linspace(-l/2, l/2, pixel_x)[b])
      const double qx = linspace_at(-w / 2.0, w / 2.0, py, a), qy = linspace_at(-l / 2.0, l / 2.0, px, b);
      double h;
      if (layer == 1 && (b == 0 || b == px - 1 || a == 0 || a == py - 1)) {
        h = 0.5;  // tunnel_fn.py:155-159
      } else {
        h = 0.0;
        for (int wd = 0; wd < s_num_y[layer]; ++wd) {
          double hm = 0.0;
          for (int f = 0; f < 4; ++f) {
            const Face& F = s_face[layer][wd][f];
            double t = F.dc - F.ac * qx;
            t = t - F.bc * qy;
            t = t < 0.0 ? 0.0 : t;  // np.clip(., 0, inf)
            hm = f == 0 ? t : (t < hm ? t : hm);  // min over the wedge's faces
          }
          h = wd == 0 ? hm : (hm > h ? hm : h);  // max over wedges
        }
      }
      const double raw = (double)(int64_t)(h / vs);  // (height_field_raw / vertical_scale).astype(int)
      if (layer == 0) {
        v = ceil_raw - raw;
        v = v < ceil_min ? ceil_min : v;
      } else {
        v = raw;
      }
    } else {
      v = layer == 0 ? ceil_out : floor_out;
    }
    out[idx] = (float)(v * vs);  // (tiles * vertical_scale).astype(np.float32)
  }
}

}  // namespace

extern "C" int go1_tunnel_tiles(const go1_tunnel_params* p, const int32_t* extents, double* records, float* tiles,
                                void* stream) {
  if (!p || !extents || !records || !tiles) return go1_internal_fail(GO1_E_ARG, "go1_tunnel_tiles: null argument");
  if (p->num_rows <= 0 || p->num_cols <= 0 || p->tile_x <= 0 || p->tile_y <= 0 || p->sub_x < 2 || p->sub_y < 2)
    return go1_internal_fail(GO1_E_ARG, "go1_tunnel_tiles: bad grid shape");
  if (!(p->vertical_scale > 0.0) || !(p->horizontal_scale > 0.0))
    return go1_internal_fail(GO1_E_ARG, "go1_tunnel_tiles: scales must be > 0");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(tunnel_draw_kernel, dim3(1), dim3(64), 0, s, *p, records);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    hipLaunchKernelGGL(tunnel_tile_kernel, dim3(p->num_rows * p->num_cols), dim3(256), 0, s, *p, records, extents,
                       tiles);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return go1_internal_fail(GO1_E_HIP, std::string("go1_tunnel_tiles: ") + hipGetErrorString(e));
  return 0;
}
