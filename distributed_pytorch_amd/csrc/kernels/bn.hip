// K4/K5/K6 — BatchNorm2d (training + eval) fused with ReLU and the optional 2x2/s2 max-pool.
//
// Replaces native_batch_norm / relu_ / max_pool2d_with_indices and their backwards
// (model.py:16,24,25).  Activations are NHWC fp32; C % 4 == 0.
//
// The conv that feeds a BN is computed WITHOUT its bias: training-mode BN subtracts the batch
// mean, so the bias cancels exactly in the output; it only enters running_mean (added in the
// finalize kernel) and the eval-mode shift.  Its gradient (mathematically 0) is produced from
// the same per-channel sums PyTorch would reduce (see bn_bwd_finalize).
//
// Forward:  stats partials per row-block (shifted sums, optionally summing split-K conv slabs
//           on the fly and writing z) -> finalize (Chan merge, running-stat update with unbiased
//           var, momentum, num_batches_tracked) -> apply+relu(+pool).
// Backward: only z (the conv output) is stored; y = relu(z*scale+shift), the pool argmax (first
//           max in window scan order, as torch's CPU kernel) and x_hat are recomputed:
//           reduce pass (sum dy, sum dy*xhat, sum xhat; optionally summing split-K dgrad slabs
//           of g and writing g) -> finalize -> apply pass writing dz.
//
// Activation modes (ACT): 0 = ReLU (VGG, optional fused 2x2 max-pool), 1 = none (ResNet
// downsample / pre-add BN), 2 = ReLU(BN(z) + residual) (ResNet block output; backward also emits
// the residual-branch gradient).  The ReLU mask is recomputed from z (and the residual).
//
// Reductions: a RT-thread (1024) block covers RPB rows x all channels (threads per row = C/4
// float4 lanes, RT/(C/4) rows in flight, 4 rows' loads issued together), keeps per-thread partials
// in registers, combines them with an LDS tree, and writes ONE partial per (block, channel) —
// deterministic, no atomics.  ~256 blocks: one wave of full CUs, few partials to merge.  The
// backward reduce uses RTB (256) -thread blocks, ~512 of them (see RTB).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

extern "C" {  // bn_wide.hip: bf16 apply passes with 16-byte lanes (return 1: not applicable)
int dpa_bn_apply_wide(const unsigned short* z, const unsigned short* res, unsigned short* out, unsigned char* mask,
                      const float* scale, const float* shift, long M, int C, int act, hipStream_t st,
                      const float* rscale, const float* rshift);
int dpa_bn_bwd_apply_wide(const unsigned short* g, const unsigned short* g2, const unsigned short* z,
                          unsigned short* dz, const float* scale, const float* shift, const float* coef, long M, int C,
                          int act, hipStream_t st);
int dpa_bn_bwd_reduce_wide(const unsigned short* g, const unsigned short* g2, const unsigned short* z,
                           const unsigned short* res, const unsigned char* mask, unsigned short* dyout,
                           const float* scale, const float* shift, const float* mean, const float* invstd,
                           float* part, int Mo, int C, int act, int rpb, int* sig, int sig_val, hipStream_t st);
}

namespace {

constexpr int RT = 1024;  // forward-statistics block size
// Backward reduce geometry, by tensor size (M rows x C/4 float4 lanes):
// * up to WIDE_MIN_F4 lanes (every VGG-11 layer at batch 256): 256-thread blocks with a 4 KB LDS
//   tree, ~512 of them.  In the VGG engine the reduce runs beside the weight-gradient convs of the
//   other stream; a 1024-thread / 48 KB block could not be placed on a CU holding conv blocks and
//   waited for whole CUs to drain (3-6x slower in the step); 512 blocks: +2.2 % step throughput
//   over 1024 and +0.7 % over 256 (fewer partial rows for the finalize).
// * larger tensors (ResNet-50 at batch 128: 3.2M-25.7M lanes per BN; autograd runs them on one
//   stream): 1024-thread blocks, ~256 of them — 512 x 256 left ResNet-50 at 7,035 img/s against
//   7,485 (measured A/B, 2048 x 256: 7,454).
constexpr int RTB = 256;
constexpr int BWD_BLOCKS = 512;
// Four bf16 rows' loads in flight per thread in the apply passes and the wide reduce (A/B:
// ResNet-50 +0.6 % over one / two rows).
constexpr bool g_bn_unr = true;
constexpr long WIDE_MIN_F4 = 3L << 20;
constexpr int BWD_WIDE_BLOCKS = 256;
// bf: bf16 tensors (the generic path, its 16-byte-lane reduce): the 1024-thread geometry at every
// size (ResNet-50 A/B: 9,240 -> 9,330 img/s); fp32 (the VGG engine) by size as above.
inline bool bwd_wide(long M, int C, bool bf = false) { return bf || M * (long)(C >> 2) > WIDE_MIN_F4; }
inline int bwd_rt(long M, int C, bool bf = false) { return bwd_wide(M, C, bf) ? RT : RTB; }
inline int bwd_blocks(long M, int C, bool bf = false) { return bwd_wide(M, C, bf) ? BWD_WIDE_BLOCKS : BWD_BLOCKS; }

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// element-4 accessors: activations / gradients are fp32 (VGG engine, x3) or bf16 (generic bf16
// path: z, g, residual and their gradients stored in bf16, math in fp32)
__device__ __forceinline__ float4 ld4(const float* p, long i4) { return reinterpret_cast<const float4*>(p)[i4]; }
__device__ __forceinline__ float4 ld4(const u16* p, long i4) {
  const ushort4 h = reinterpret_cast<const ushort4*>(p)[i4];
  return make_float4(bf16_f(h.x), bf16_f(h.y), bf16_f(h.z), bf16_f(h.w));
}
__device__ __forceinline__ void st4(float* p, long i4, float4 v) { reinterpret_cast<float4*>(p)[i4] = v; }
__device__ __forceinline__ void st4(u16* p, long i4, float4 v) {
  reinterpret_cast<ushort4*>(p)[i4] = make_ushort4(bf16_rne(v.x), bf16_rne(v.y), bf16_rne(v.z), bf16_rne(v.w));
}

struct RedGeom {
  int C4, TPR, RPI, CG;  // float4 lanes per row, threads per row, rows per iteration, channel groups/thread
};

__host__ __device__ inline RedGeom red_geom(int C, int rt = RT) {
  RedGeom g;
  g.C4 = C >> 2;
  g.TPR = g.C4 < rt ? g.C4 : rt;
  g.RPI = rt / g.TPR;
  g.CG = (g.C4 + g.TPR - 1) / g.TPR;
  return g;
}

// rows per block so that the grid has ~`blocks` blocks (at least one full iteration per block)
__host__ inline int red_rows_per_block(int M, int C, int rt = RT, int blocks = 256) {
  const RedGeom g = red_geom(C, rt);
  int rpb = (M + blocks - 1) / blocks;
  rpb = ((rpb + g.RPI - 1) / g.RPI) * g.RPI;
  return rpb < g.RPI ? g.RPI : rpb;
}

inline int bwd_rows_per_block(int M, int C, bool bf = false) {
  return red_rows_per_block(M, C, bwd_rt(M, C, bf), bwd_blocks(M, C, bf));
}

// In-block tree over the RPI row lanes of each channel lane (fixed order): on return sh[t] for
// lane_r == 0 holds the block sum.  Caller has stored sh[t] and synchronised.
template <int NARR, int T = RT>
__device__ __forceinline__ void tree_rows(float4 (*sh)[T], int t, int lane_r, int TPR, int RPI) {
  int p2 = 1;
  while (p2 < RPI) p2 <<= 1;
  for (int o = p2 >> 1; o >= 1; o >>= 1) {
    if (lane_r < o && lane_r + o < RPI) {
#pragma unroll
      for (int q = 0; q < NARR; ++q) sh[q][t] = f4add(sh[q][t], sh[q][t + o * TPR]);
    }
    __syncthreads();
  }
}

// as tree_rows, maxima instead of sums
template <int T = RT>
__device__ __forceinline__ void tree_rows_max(float4 (*sh)[T], int t, int lane_r, int TPR, int RPI) {
  int p2 = 1;
  while (p2 < RPI) p2 <<= 1;
  for (int o = p2 >> 1; o >= 1; o >>= 1) {
    if (lane_r < o && lane_r + o < RPI) {
      const float4 a = sh[0][t], b = sh[0][t + o * TPR];
      sh[0][t] = make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
    }
    __syncthreads();
  }
}

#define F4GET(v, k) ((k) == 0 ? (v).x : (k) == 1 ? (v).y : (k) == 2 ? (v).z : (v).w)

// fp64 lanes of the backward sums (bn_bwd_reduce_kernel)
struct __attribute__((aligned(16))) dbl4 {
  double x, y, z, w;
};
template <int T>
__device__ __forceinline__ void tree_rows_d(dbl4* sh, int t, int lane_r, int TPR, int RPI) {
  int p2 = 1;
  while (p2 < RPI) p2 <<= 1;
  for (int o = p2 >> 1; o >= 1; o >>= 1) {
    if (lane_r < o && lane_r + o < RPI) {
      const dbl4 a = sh[t], b = sh[t + o * TPR];
      sh[t] = dbl4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
    }
    __syncthreads();
  }
}


// ---- output writer: NP == 0 -> fp32 float4 store; NP in {1,3} -> bf16 planes x = x0 (+ x1 + x2);
// NP 2 -> the fp16 pair of x * s (common.h split_val) -- the next conv reads MFMA-ready operands.

template <int NP>
__device__ __forceinline__ void store4(float* f, u16* pl, long ps, long i4, float4 v, float s = 1.f) {
  if constexpr (NP == 0) {
    reinterpret_cast<float4*>(f)[i4] = v;
  } else {
    const float vv[4] = {v.x, v.y, v.z, v.w};
    u16 o[4][3];
#pragma unroll
    for (int k = 0; k < 4; ++k) split_val<NP>(vv[k], o[k], s);
#pragma unroll
    for (int p = 0; p < NP; ++p)
      reinterpret_cast<ushort4*>(pl + p * ps)[i4] = make_ushort4(o[0][p], o[1][p], o[2][p], o[3][p]);
  }
}
// activation planes: the fixed scale of fp16 pairs
template <int NP>
__device__ __forceinline__ void store4a(float* f, u16* pl, long ps, long i4, float4 v) {
  store4<NP>(f, pl, ps, i4, v, NP == 2 ? H2_SA : 1.f);
}

// ---- forward statistics: per (row-block, channel) (mean, M2) via sums shifted by the block's
// first row.  If nsplit > 1, src holds nsplit slabs of [M][C] that are summed here and written
// to z (the split-K reduction of the producing conv, fused).
template <typename TZ>
__global__ __launch_bounds__(RT) void bn_stats_kernel(const TZ* __restrict__ src, TZ* __restrict__ z, int nsplit,
                                                      float2* __restrict__ part, int M, int C, int rpb) {
  const RedGeom g = red_geom(C);
  const int t = threadIdx.x;
  const int lane_c = t % g.TPR, lane_r = t / g.TPR;
  const bool active = lane_r < g.RPI;
  const int r0 = blockIdx.x * rpb;
  const int r1 = min(M, r0 + rpb);
  const long slab4 = (long)M * g.C4;
  __shared__ float4 sh[2][RT];
  auto acc = [](float4 v, float4 K, float4& a1, float4& a2) {
    const float d0 = v.x - K.x, d1 = v.y - K.y, d2 = v.z - K.z, d3 = v.w - K.w;
    a1.x += d0;
    a1.y += d1;
    a1.z += d2;
    a1.w += d3;
    a2.x = fmaf(d0, d0, a2.x);
    a2.y = fmaf(d1, d1, a2.y);
    a2.z = fmaf(d2, d2, a2.z);
    a2.w = fmaf(d3, d3, a2.w);
  };
  for (int cg = 0; cg < g.CG; ++cg) {
    const int c4 = lane_c + cg * g.TPR;
    const bool cval = active && c4 < g.C4;
    float4 K = make_float4(0.f, 0.f, 0.f, 0.f), a1 = K, a2 = K;
    if (cval) {
      // shift = the block's first row (summed over splits)
      K = ld4(src, (long)r0 * g.C4 + c4);
      for (int s = 1; s < nsplit; ++s) K = f4add(K, ld4(src, s * slab4 + (long)r0 * g.C4 + c4));
      int r = r0 + lane_r;
      if (nsplit == 1) {  // 4 rows' loads in flight
        for (; r + 3 * g.RPI < r1; r += 4 * g.RPI) {
          float4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = ld4(src, (long)(r + u * g.RPI) * g.C4 + c4);
#pragma unroll
          for (int u = 0; u < 4; ++u) acc(v[u], K, a1, a2);
        }
      }
      for (; r < r1; r += g.RPI) {
        const long i = (long)r * g.C4 + c4;
        float4 v = ld4(src, i);
        for (int s = 1; s < nsplit; ++s) v = f4add(v, ld4(src, s * slab4 + i));
        if (nsplit > 1) st4(z, i, v);
        acc(v, K, a1, a2);
      }
    }
    sh[0][t] = a1;
    sh[1][t] = a2;
    __syncthreads();
    tree_rows<2>(sh, t, lane_r, g.TPR, g.RPI);
    if (cval && lane_r == 0) {
      a1 = sh[0][t];
      a2 = sh[1][t];
      const float n = (float)(r1 - r0), inv = 1.f / n;
      float2* o = part + (long)blockIdx.x * C + c4 * 4;
      o[0] = make_float2(K.x + a1.x * inv, fmaxf(a2.x - a1.x * a1.x * inv, 0.f));
      o[1] = make_float2(K.y + a1.y * inv, fmaxf(a2.y - a1.y * a1.y * inv, 0.f));
      o[2] = make_float2(K.z + a1.z * inv, fmaxf(a2.z - a1.z * a1.z * inv, 0.f));
      o[3] = make_float2(K.w + a1.w * inv, fmaxf(a2.w - a1.w * a1.w * inv, 0.f));
    }
    __syncthreads();
  }
}

struct Welford {
  float n, mean, m2;
};

__device__ __forceinline__ Welford merge(Welford a, Welford b) {
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float n = a.n + b.n;
  const float d = b.mean - a.mean;
  const float f = b.n / n;
  Welford r;
  r.n = n;
  r.mean = a.mean + d * f;
  r.m2 = a.m2 + b.m2 + d * d * a.n * f;
  return r;
}

// 8 channels x 32 partial-groups per block (32-B coalesced partial reads, 4 loads in flight per
// thread), Chan merge, then scale/shift + running-stat update.
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float2* __restrict__ part, int nblk, int rpb, int M,
                                                          int C, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ bias, float* __restrict__ rmean,
                                                          float* __restrict__ rvar, long long* __restrict__ nbt,
                                                          float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                          float* __restrict__ scale, float* __restrict__ shift,
                                                          float momentum, float eps) {
  // 4 channels per block, 64 partial-row groups of each, fixed-order Chan merges
  constexpr int CPB = 4, G = 256 / CPB;
  const int cl = threadIdx.x % CPB, grp = threadIdx.x / CPB;
  const int c = blockIdx.x * CPB + cl;
  Welford acc{0.f, 0.f, 0.f};
  if (c < C) {
    // 16 partial rows per thread in flight (conv0's ~1024 epilogue partials: one memory latency
    // instead of four), merged in the same order
    for (int k = grp; k < nblk; k += 16 * G) {
      float2 p[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) p[u] = k + G * u < nblk ? part[(long)(k + G * u) * C + c] : make_float2(0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int kk = k + G * u;
        if (kk < nblk) acc = merge(acc, Welford{(float)min(rpb, M - kk * rpb), p[u].x, p[u].y});
      }
    }
  }
  __shared__ Welford sh[256];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o >= CPB; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] = merge(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  if (grp == 0 && c < C) {
    const Welford w = sh[cl];
    const float var = w.m2 / w.n;
    const float inv = rsqrtf(var + eps);
    const float gm = gamma[c];
    mean_out[c] = w.mean;
    invstd_out[c] = inv;
    scale[c] = gm * inv;
    shift[c] = beta[c] - w.mean * gm * inv;
    if (rmean) {
      const float b = bias ? bias[c] : 0.f;
      const float unb = w.n > 1.f ? w.m2 / (w.n - 1.f) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * (w.mean + b);
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
    }
    if (c == 0 && nbt) nbt[0] += 1;
  }
}

// Finalize from CHANNEL-MAJOR (mean, M2) partials part[c][k] (a conv epilogue's statistics,
// conv_x3.hip epi_col_stats: up to thousands of row tiles per channel).  One block per channel:
// 256 threads stride the channel's contiguous partials with 8 loads in flight, then a fixed-order
// tree merge.
__global__ __launch_bounds__(256) void bn_finalize_cm_kernel(const float2* __restrict__ part, int nblk, int rpb, int M,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta,
                                                             const float* __restrict__ bias, float* __restrict__ rmean,
                                                             float* __restrict__ rvar, long long* __restrict__ nbt,
                                                             float* __restrict__ mean_out,
                                                             float* __restrict__ invstd_out, float* __restrict__ scale,
                                                             float* __restrict__ shift, float momentum, float eps) {
  const int c = blockIdx.x, t = threadIdx.x;
  const float2* pc = part + (long)c * nblk;
  Welford acc{0.f, 0.f, 0.f};
  // 8 partials per thread in flight (guarded: the ResNet-50 epilogue partials, ~400-1600 per
  // channel, are 2-7 per thread -- a rolled tail loop paid one memory latency each), same order
  for (int k = t; k < nblk; k += 8 * 256) {
    float2 p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = k + 256 * u < nblk ? pc[k + 256 * u] : make_float2(0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int kk = k + 256 * u;
      if (kk < nblk) acc = merge(acc, Welford{(float)min(rpb, M - kk * rpb), p[u].x, p[u].y});
    }
  }
  __shared__ Welford sh[256];
  sh[t] = acc;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if (t < o) sh[t] = merge(sh[t], sh[t + o]);
    __syncthreads();
  }
  if (t == 0) {
    const Welford w = sh[0];
    const float var = w.m2 / w.n;
    const float inv = rsqrtf(var + eps);
    const float gm = gamma[c];
    mean_out[c] = w.mean;
    invstd_out[c] = inv;
    scale[c] = gm * inv;
    shift[c] = beta[c] - w.mean * gm * inv;
    if (rmean) {
      const float b = bias ? bias[c] : 0.f;
      const float unb = w.n > 1.f ? w.m2 / (w.n - 1.f) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * (w.mean + b);
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
    }
    if (c == 0 && nbt) nbt[0] += 1;
  }
}

// Eval-mode affine: y = gamma*(z + b - rm)/sqrt(rv+eps) + beta = z*scale + shift
__global__ void bn_eval_params_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ bias, const float* __restrict__ rmean,
                                      const float* __restrict__ rvar, float* __restrict__ scale,
                                      float* __restrict__ shift, int C, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float s = gamma[c] * rsqrtf(rvar[c] + eps);
  scale[c] = s;
  shift[c] = beta[c] + ((bias ? bias[c] : 0.f) - rmean[c]) * s;
}

__device__ __forceinline__ float4 affine_relu(float4 v, float4 sc, float4 sh) {
  return make_float4(fmaxf(fmaf(v.x, sc.x, sh.x), 0.f), fmaxf(fmaf(v.y, sc.y, sh.y), 0.f),
                     fmaxf(fmaf(v.z, sc.z, sh.z), 0.f), fmaxf(fmaf(v.w, sc.w, sh.w), 0.f));
}

// a = act(z*scale + shift [+ res]), optionally 2x2/s2 max-pooled (ACT 0 only).
// z: [N,H,W,C]  a: [N,H/2,W/2,C] or [N,H,W,C]
// mask (ACT 2, optional): one byte per 4 channels, bit k = (BN(z) + res > 0) of channel 4*c4 + k --
// the backward reads it instead of re-reading the residual (0.25 instead of 2-4 bytes per element)
template <bool POOL, int NP, int ACT, typename TZ>
__global__ __launch_bounds__(256) void bn_apply_kernel(const TZ* __restrict__ z, float* __restrict__ a,
                                                       u16* __restrict__ a3, long ps,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const TZ* __restrict__ res,
                                                       int N, int H, int W, int C,
                                                       unsigned char* __restrict__ mask) {
  const int C4 = C >> 2;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const long total = (long)N * Ho * Wo * C4;
  const long stride = (long)gridDim.x * blockDim.x;
  auto body = [&](long i, int c4, float4 sc, float4 sh) {
    if (!POOL) {
      if constexpr (ACT == 0) {
        store4a<NP>(a, a3, ps, i, affine_relu(ld4(z, i), sc, sh));
      } else {
        const float4 v = ld4(z, i);
        float4 u = make_float4(fmaf(v.x, sc.x, sh.x), fmaf(v.y, sc.y, sh.y), fmaf(v.z, sc.z, sh.z),
                               fmaf(v.w, sc.w, sh.w));
        if constexpr (ACT == 2) {
          const float4 r = ld4(res, i);
          const float4 t = make_float4(u.x + r.x, u.y + r.y, u.z + r.z, u.w + r.w);
          if (mask)
            mask[i] = (unsigned char)((t.x > 0.f) | ((t.y > 0.f) << 1) | ((t.z > 0.f) << 2) | ((t.w > 0.f) << 3));
          u = make_float4(fmaxf(t.x, 0.f), fmaxf(t.y, 0.f), fmaxf(t.z, 0.f), fmaxf(t.w, 0.f));
        }
        store4a<NP>(a, a3, ps, i, u);
      }
    } else {
      const unsigned t = (unsigned)(i / C4);  // pooled pixel (VGG sizes: < 2^32)
      const unsigned ow = t % (unsigned)Wo, t2 = t / (unsigned)Wo;
      const unsigned oh = t2 % (unsigned)Ho, n = t2 / (unsigned)Ho;
      const long base = (((long)n * H + 2 * oh) * W + 2 * ow) * C4 + c4;
      const float4 v00 = affine_relu(ld4(z, base), sc, sh);
      const float4 v01 = affine_relu(ld4(z, base + C4), sc, sh);
      const float4 v10 = affine_relu(ld4(z, base + (long)W * C4), sc, sh);
      const float4 v11 = affine_relu(ld4(z, base + (long)W * C4 + C4), sc, sh);
      store4a<NP>(a, a3, ps, i,
                  make_float4(fmaxf(fmaxf(v00.x, v01.x), fmaxf(v10.x, v11.x)),
                              fmaxf(fmaxf(v00.y, v01.y), fmaxf(v10.y, v11.y)),
                              fmaxf(fmaxf(v00.z, v01.z), fmaxf(v10.z, v11.z)),
                              fmaxf(fmaxf(v00.w, v01.w), fmaxf(v10.w, v11.w))));
    }
  };
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (stride % C4 == 0) {  // every element of this thread has the same channel group (launcher's grid)
    const int c4 = (int)(i0 % C4);
    const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
    const float4 sh = reinterpret_cast<const float4*>(shift)[c4];
    long i = i0;
    // four rows' loads in flight per thread (memory-level parallelism of the bf16 passes)
    if (sizeof(TZ) == 2 && g_bn_unr)  // bf16 rows (8 bytes per thread); fp32 as before
    for (; i + 3 * stride < total; i += 4 * stride) {
      body(i, c4, sc, sh);
      body(i + stride, c4, sc, sh);
      body(i + 2 * stride, c4, sc, sh);
      body(i + 3 * stride, c4, sc, sh);
    }
    for (; i < total; i += stride) body(i, c4, sc, sh);
  } else {
    for (long i = i0; i < total; i += stride) {
      const int c4 = (int)(i % C4);
      body(i, c4, reinterpret_cast<const float4*>(scale)[c4], reinterpret_cast<const float4*>(shift)[c4]);
    }
  }
}

// gradient through the activation at one element: u = BN output, r = residual (ACT 2)
template <int ACT>
__device__ __forceinline__ float act_grad(float u, float r, float g) {
  if constexpr (ACT == 0) return u > 0.f ? g : 0.f;
  else if constexpr (ACT == 1) return g;
  else return (u + r) > 0.f ? g : 0.f;
}

// route the pooled grad to the first max of the window (scan order 00,01,10,11), relu mask
__device__ __forceinline__ void route1(float z00, float z01, float z10, float z11, float sc, float sh, float g,
                                       float& d00, float& d01, float& d10, float& d11) {
  const float y00 = fmaxf(fmaf(z00, sc, sh), 0.f), y01 = fmaxf(fmaf(z01, sc, sh), 0.f);
  const float y10 = fmaxf(fmaf(z10, sc, sh), 0.f), y11 = fmaxf(fmaf(z11, sc, sh), 0.f);
  int arg = 0;
  float mx = y00;
  if (y01 > mx) { mx = y01; arg = 1; }
  if (y10 > mx) { mx = y10; arg = 2; }
  if (y11 > mx) { mx = y11; arg = 3; }
  d00 = (arg == 0 && y00 > 0.f) ? g : 0.f;
  d01 = (arg == 1 && y01 > 0.f) ? g : 0.f;
  d10 = (arg == 2 && y10 > 0.f) ? g : 0.f;
  d11 = (arg == 3 && y11 > 0.f) ? g : 0.f;
}

// Per-channel backward finalize from the complete sums: dgamma, dbeta, dbias and the dz coefficients
// of the CENTRED form dz = k1*dy + c2*(z - mean) + k3 (coef rows: k1, c2, k3, mean).  The centred form
// keeps the x-hat term's rounding relative to |z - mean| instead of |z|: the expanded
// c2*z + (k3 - c2*mean) cancels when |mean| >> sigma, which trained layers reach, and its rounding
// then grew every lower layer's gradients (docs/PERF_NOTES.md round 6; torch's CPU backward also
// forms (z - mean)).  Returns the channel's dz bound |k1| max|dy| + |c2| max|z - mean| + |k3|.
__device__ __forceinline__ float bwd_coef(int c, int C, float sdy, float sdx, float sx, float mdy, float mz,
                                          float Mfull, const float* __restrict__ gamma,
                                          const float* __restrict__ mean, const float* __restrict__ invstd,
                                          float* __restrict__ dgamma, float* __restrict__ dbeta,
                                          float* __restrict__ dbias, float* __restrict__ coef) {
  const float iv = invstd[c], gm = gamma[c];
  const float k1 = gm * iv;
  const float k2x = -k1 * sdx / Mfull;  // coefficient of xhat
  const float k3 = -k1 * sdy / Mfull;
  const float c2 = k2x * iv;
  dgamma[c] = sdx;
  dbeta[c] = sdy;
  if (dbias) dbias[c] = k2x * sx;  // = sum over rows of dz (analytically 0)
  coef[c] = k1;
  coef[C + c] = c2;      // coefficient of z - mean
  coef[2 * C + c] = k3;  // constant
  coef[3 * C + c] = mean[c];
  // (rounding of the fma chain stays far inside the 2^14 -> 65504 headroom of the scale)
  return fabsf(k1) * mdy + fabsf(c2) * mz + fabsf(k3);
}

// The same from fp64 sums of dy, dy (z - mean) and (z - mean) (bn_bwd_reduce_kernel): the arithmetic in
// double, the outputs rounded once.
__device__ __forceinline__ float bwd_coef_d(int c, int C, double sdy, double sdc, double sxc, float mdy, float mz,
                                            double Mfull, const float* __restrict__ gamma,
                                            const float* __restrict__ mean, const float* __restrict__ invstd,
                                            float* __restrict__ dgamma, float* __restrict__ dbeta,
                                            float* __restrict__ dbias, float* __restrict__ coef) {
  const double iv = invstd[c], gm = gamma[c];
  const double sdx = sdc * iv;  // sum dy * xhat
  const double k1 = gm * iv;
  const double k2x = -k1 * sdx / Mfull;
  const double k3 = -k1 * sdy / Mfull;
  const double c2 = k2x * iv;
  dgamma[c] = (float)sdx;
  dbeta[c] = (float)sdy;
  if (dbias) dbias[c] = (float)(k2x * sxc * iv);
  coef[c] = (float)k1;
  coef[C + c] = (float)c2;
  coef[2 * C + c] = (float)k3;
  coef[3 * C + c] = mean[c];
  return (float)(fabs(k1) * mdy + fabs(c2) * mz + fabs(k3));
}

// Backward reduce: per (row-block, channel) sums of dy, dy*(z - mean), (z - mean) and maxima of |dy|,
// |z| (the data-gradient bound of fp16-pair planes, bn_bwd_finalize_kernel).  Rows are OUTPUT rows of
// the layer (pooled positions when POOL).  The three sums leave each thread's short run of rows
// (2-8 rows in the VGG geometry) in FP64: the block tree, the partials and the finalize sum in
// double (torch's CPU batch norm accumulates in double too): the BN parameter gradients are sums
// over up to 262,144 rows that cancel heavily once the network trains, and fp32 accumulation left
// dgamma / dbeta several times further from fp64 than stock torch fp32 at a trained state
// (docs/PERF_NOTES.md round 6; fp64 arithmetic per element measured 1.5 % slower in the step).  part: [block][3][C] doubles, then [block][2][C]
// floats (the maxima) at float offset gridDim.x * 6 * C.  If nsplit > 1, gsrc holds the split-K slabs of g and
// the summed g is written to gout (consumed by the apply pass).  g2 (optional, nsplit == 1): a second
// contribution to the same gradient, summed on load here and in the apply pass instead of by a
// separate add pass (ResNet: a block input's two gradient contributions, ops/functional.GradJoin).
// dyout (ACT 2, optional): the gradient through the add+ReLU, dy = relu'(u + r) * (g + g2), is
// stored here (it is the residual's gradient dres); the apply pass then reads dy alone (ACT 1)
// instead of g, g2 and the mask again.
// part layout: [block][3][C]
template <bool POOL, int ACT, typename TZ, int RTB>
__global__ __launch_bounds__(RTB) void bn_bwd_reduce_kernel(const TZ* __restrict__ gsrc, TZ* __restrict__ gout,
                                                            int nsplit, const TZ* __restrict__ z,
                                                            const TZ* __restrict__ res,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            float* __restrict__ part, int N, int H, int W, int C,
                                                            int rpb, int* sig, int sig_val,
                                                            const TZ* __restrict__ g2,
                                                            const unsigned char* __restrict__ mask,
                                                            TZ* __restrict__ dyout, unsigned* __restrict__ bound) {
  start_signal(sig, sig_val);
  if (bound != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *bound = 0u;  // re-armed for this layer's
                                                                               // finalize (the next kernel)
  const RedGeom gg = red_geom(C, RTB);
  const int t = threadIdx.x;
  const int lane_c = t % gg.TPR, lane_r = t / gg.TPR;
  const bool active = lane_r < gg.RPI;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const int Mo = N * Ho * Wo;
  const int r0 = blockIdx.x * rpb;
  const int r1 = min(Mo, r0 + rpb);
  const long slab4 = (long)Mo * gg.C4;
  __shared__ dbl4 shd[RTB];  // one tree buffer, used for the three sums in turn (and the maxima,
                             // as float4 in its first half)
  float4(*sh)[RTB] = reinterpret_cast<float4(*)[RTB]>(shd);
  for (int cg = 0; cg < gg.CG; ++cg) {
    const int c4 = lane_c + cg * gg.TPR;
    const bool cval = active && c4 < gg.C4;
    float sdy[4] = {0, 0, 0, 0}, sdx[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0};  // dy, dy (z - mu), z - mu
    float mdy[4] = {0, 0, 0, 0}, mz[4] = {0, 0, 0, 0};  // max |dy|, max |z|
    if (cval) {
      const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
      const float4 sh = reinterpret_cast<const float4*>(shift)[c4];
      const float4 mu = reinterpret_cast<const float4*>(mean)[c4];
      const float4 is = reinterpret_cast<const float4*>(invstd)[c4];
      int r = r0 + lane_r;
      // UNR rows' loads in flight: the 1024-thread geometry of large tensors (ResNet-50; two rows
      // +6 %, four for 8-byte bf16 rows); the 256-thread blocks that run beside the VGG
      // weight-gradient convs keep one row.  Rows are summed in order (deterministic).
      auto rows = [&](auto unr) {
        constexpr int UNR = decltype(unr)::value;
        for (; r + (UNR - 1) * gg.RPI < r1; r += UNR * gg.RPI) {
          long gi[UNR];
          float4 gv[UNR], zv[UNR], rv[UNR];
          unsigned mv[UNR];
          const bool mk = ACT == 2 && mask;
#pragma unroll
          for (int u = 0; u < UNR; ++u) {
            gi[u] = (long)(r + u * gg.RPI) * gg.C4 + c4;
            gv[u] = ld4(gsrc, gi[u]);
            if (g2) gv[u] = f4add(gv[u], ld4(g2, gi[u]));
            zv[u] = ld4(z, gi[u]);
            rv[u] = ACT == 2 && !mk ? ld4(res, gi[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
            mv[u] = mk ? mask[gi[u]] : 0u;
          }
#pragma unroll
          for (int u = 0; u < UNR; ++u) {
            float dyu[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float zz = F4GET(zv[u], k);
              const float dy = mk ? (((mv[u] >> k) & 1u) ? F4GET(gv[u], k) : 0.f)
                                  : act_grad<ACT>(fmaf(zz, F4GET(sc, k), F4GET(sh, k)), F4GET(rv[u], k),
                                                  F4GET(gv[u], k));
              const float zc = zz - F4GET(mu, k);
              sdy[k] += dy;
              sdx[k] = fmaf(dy, zc, sdx[k]);
              sx[k] += zc;
              mdy[k] = fmaxf(mdy[k], fabsf(dy));
              mz[k] = fmaxf(mz[k], fabsf(zz - F4GET(mu, k)));
              dyu[k] = dy;
            }
            if (ACT == 2 && dyout) st4(dyout, gi[u], make_float4(dyu[0], dyu[1], dyu[2], dyu[3]));
          }
        }
      };
      if (RTB == RT && !POOL && nsplit == 1) {
        if (sizeof(TZ) == 2 && g_bn_unr) rows(std::integral_constant<int, 4>());
        rows(std::integral_constant<int, 2>());
      }
      for (; r < r1; r += gg.RPI) {
        const long gi = (long)r * gg.C4 + c4;
        float4 gv = ld4(gsrc, gi);
        for (int s = 1; s < nsplit; ++s) gv = f4add(gv, ld4(gsrc, s * slab4 + gi));
        if (nsplit > 1) st4(gout, gi, gv);
        if (g2) gv = f4add(gv, ld4(g2, gi));  // a second gradient contribution (nsplit == 1 only)
        if (!POOL) {
          const float4 zv = ld4(z, gi);
          const bool mk = ACT == 2 && mask;
          const float4 rv = ACT == 2 && !mk ? ld4(res, gi) : make_float4(0.f, 0.f, 0.f, 0.f);
          const unsigned m = mk ? mask[gi] : 0u;
          float dyv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float zz = F4GET(zv, k);
            const float dy = mk ? (((m >> k) & 1u) ? F4GET(gv, k) : 0.f)
                                : act_grad<ACT>(fmaf(zz, F4GET(sc, k), F4GET(sh, k)), F4GET(rv, k), F4GET(gv, k));
            const float zc = zz - F4GET(mu, k);
            sdy[k] += dy;
            sdx[k] = fmaf(dy, zc, sdx[k]);
            sx[k] += zc;
            mdy[k] = fmaxf(mdy[k], fabsf(dy));
            mz[k] = fmaxf(mz[k], fabsf(zz - F4GET(mu, k)));
            dyv[k] = dy;
          }
          if (ACT == 2 && dyout) st4(dyout, gi, make_float4(dyv[0], dyv[1], dyv[2], dyv[3]));
        } else {
          const int ow = r % Wo;
          const int tt = r / Wo;
          const int oh = tt % Ho;
          const int n = tt / Ho;
          const long base = (((long)n * H + 2 * oh) * W + 2 * ow) * gg.C4 + c4;
          const float4 z00 = ld4(z, base), z01 = ld4(z, base + gg.C4), z10 = ld4(z, base + (long)W * gg.C4),
                       z11 = ld4(z, base + (long)W * gg.C4 + gg.C4);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float d00, d01, d10, d11;
            route1(F4GET(z00, k), F4GET(z01, k), F4GET(z10, k), F4GET(z11, k), F4GET(sc, k), F4GET(sh, k),
                   F4GET(gv, k), d00, d01, d10, d11);
            const float m = F4GET(mu, k);
            const float x00 = F4GET(z00, k) - m, x01 = F4GET(z01, k) - m;
            const float x10 = F4GET(z10, k) - m, x11 = F4GET(z11, k) - m;
            sdy[k] += (d00 + d01) + (d10 + d11);  // (at most one routed term is non-zero)
            sdx[k] = fmaf(d00, x00, fmaf(d01, x01, fmaf(d10, x10, fmaf(d11, x11, sdx[k]))));
            sx[k] += (x00 + x01) + (x10 + x11);
            mdy[k] = fmaxf(mdy[k], fmaxf(fmaxf(fabsf(d00), fabsf(d01)), fmaxf(fabsf(d10), fabsf(d11))));
            const float mf = F4GET(mu, k);
            mz[k] = fmaxf(mz[k], fmaxf(fmaxf(fabsf(F4GET(z00, k) - mf), fabsf(F4GET(z01, k) - mf)),
                                       fmaxf(fabsf(F4GET(z10, k) - mf), fabsf(F4GET(z11, k) - mf))));
          }
        }
      }
    }
    const dbl4 dv[3] = {dbl4{(double)sdy[0], (double)sdy[1], (double)sdy[2], (double)sdy[3]},
                        dbl4{(double)sdx[0], (double)sdx[1], (double)sdx[2], (double)sdx[3]},
                        dbl4{(double)sx[0], (double)sx[1], (double)sx[2], (double)sx[3]}};
    double* od = reinterpret_cast<double*>(part) + (long)blockIdx.x * 3 * C + c4 * 4;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      shd[t] = dv[q];
      __syncthreads();
      tree_rows_d<RTB>(shd, t, lane_r, gg.TPR, gg.RPI);
      if (cval && lane_r == 0) *reinterpret_cast<dbl4*>(od + q * C) = shd[t];
      __syncthreads();
    }
    const float4 vals[2] = {make_float4(mdy[0], mdy[1], mdy[2], mdy[3]), make_float4(mz[0], mz[1], mz[2], mz[3])};
    float* o = part + (long)gridDim.x * 6 * C + (long)blockIdx.x * 2 * C + c4 * 4;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      sh[0][t] = vals[q];
      __syncthreads();
      tree_rows_max<RTB>(sh, t, lane_r, gg.TPR, gg.RPI);
      if (cval && lane_r == 0) *reinterpret_cast<float4*>(o + q * C) = sh[0][t];
      __syncthreads();
    }
  }
}

// Per channel: sum the block partials (fixed order -> deterministic), emit dgamma, dbeta, dbias and
// the dz coefficients: dz = k1*dy + k2*z + k3.   8 channels x 32 groups per block.
// Q: rows per block partial (5: with the maxima of |dy| and |z|, bn_bwd_reduce_kernel; 3: bn_wide.hip's
// reduce).  bound (Q 5, optional): |dz| <= |k1| max|dy| + |k2| max|z| + |k3| per channel, maximised over
// the channels into the word (an fp32 bit pattern; non-negative floats order like their bits), the
// scale of the fp16-pair dz planes and of the convs that read them.
// Backward finalize: BF_CPB channels per 256-thread block, 256/BF_CPB partial rows of each in
// flight (a thread's loads are issued 16 rows at a time), fixed-order LDS tree.
template <int BF_CPB, int Q>
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                              float Mfull, const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ dbias, float* __restrict__ coef,
                                                              unsigned* __restrict__ bound) {
  constexpr int G = 256 / BF_CPB;  // partial-row groups per channel
  const int cl = threadIdx.x % BF_CPB, grp = threadIdx.x / BF_CPB;
  const int c = blockIdx.x * BF_CPB + cl;
  const bool mx = Q == 5 && bound != nullptr;
  float a = 0.f, b = 0.f, x = 0.f, mdy = 0.f, mz = 0.f;
  if (c < C) {
    // 16 partial rows per thread in flight (one memory latency for the engine's 512-row partials
    // instead of two); out-of-range rows add +0.f (exact: the sums start at +0), same order
    for (int k = grp; k < nblk; k += 16 * G) {
      // (the maxima are loaded like the sums, without a branch: a conditional load per row would
      // wait for each row's load in turn -- 16 memory latencies instead of one)
      float pa[16], pb[16], px[16], pm[16], pz[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        // out-of-range rows load row 0 (always valid) and are masked after the load: no branch
        const bool v = k + G * u < nblk;
        const float* p = part + (long)(v ? k + G * u : 0) * Q * C + c;
        const float l0 = p[0], l1 = p[C], l2 = p[2 * C];
        pa[u] = v ? l0 : 0.f;
        pb[u] = v ? l1 : 0.f;
        px[u] = v ? l2 : 0.f;
        if constexpr (Q == 5) {
          const float l3 = p[3 * C], l4 = p[4 * C];
          pm[u] = v ? l3 : 0.f;  // maxima of magnitudes: 0 is their identity
          pz[u] = v ? l4 : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        a += pa[u];
        b += pb[u];
        x += px[u];
        if constexpr (Q == 5) {
          mdy = fmaxf(mdy, pm[u]);
          mz = fmaxf(mz, pz[u]);
        }
      }
    }
  }
  __shared__ float sh[5][256];
  sh[0][threadIdx.x] = a;
  sh[1][threadIdx.x] = b;
  sh[2][threadIdx.x] = x;
  sh[3][threadIdx.x] = mdy;
  sh[4][threadIdx.x] = mz;
  __syncthreads();
  for (int o = 128; o >= BF_CPB; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + o];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + o];
      sh[2][threadIdx.x] += sh[2][threadIdx.x + o];
      if (mx) {
        sh[3][threadIdx.x] = fmaxf(sh[3][threadIdx.x], sh[3][threadIdx.x + o]);
        sh[4][threadIdx.x] = fmaxf(sh[4][threadIdx.x], sh[4][threadIdx.x + o]);
      }
    }
    __syncthreads();
  }
  float B = 0.f;
  if (grp == 0 && c < C) {
    const float b = bwd_coef(c, C, sh[0][cl], sh[1][cl], sh[2][cl], mx ? sh[3][cl] : 0.f, mx ? sh[4][cl] : 0.f, Mfull,
                             gamma, mean, invstd, dgamma, dbeta, dbias, coef);
    if (mx) B = b;
  }
  if (mx) {  // the block's channels' largest bound, one atomic per block
    __syncthreads();
    if (grp == 0) sh[0][cl] = B;
    __syncthreads();
    if (threadIdx.x == 0) {
      float m = 0.f;
      for (int q = 0; q < BF_CPB; ++q) m = fmaxf(m, sh[0][q]);
      if (!(m < 3.0e38f)) m = 3.0e38f;  // inf / NaN gradients: the largest finite bound (scale 2^-114)
      atomicMax(bound, __float_as_uint(m));
    }
  }
}

// The finalize of bn_bwd_reduce_kernel's partials: fp64 sums [block][3][C] (dy, dy (z - mean),
// z - mean) and fp32 maxima [block][2][C] at float offset nblk * 6 * C.  Same geometry and fixed order
// as bn_bwd_finalize_kernel, the sums and the coefficient arithmetic in double (bwd_coef_d).
template <int BF_CPB>
__global__ __launch_bounds__(256) void bn_bwd_finalize_d_kernel(const float* __restrict__ part, int nblk, int C,
                                                                float Mfull, const float* __restrict__ gamma,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                float* __restrict__ dbias, float* __restrict__ coef,
                                                                unsigned* __restrict__ bound) {
  constexpr int G = 256 / BF_CPB;  // partial-row groups per channel
  const int cl = threadIdx.x % BF_CPB, grp = threadIdx.x / BF_CPB;
  const int c = blockIdx.x * BF_CPB + cl;
  const bool mx = bound != nullptr;
  const double* pd = reinterpret_cast<const double*>(part);
  const float* pf = part + (long)nblk * 6 * C;
  double a = 0.0, b = 0.0, x = 0.0;
  float mdy = 0.f, mz = 0.f;
  if (c < C) {
    for (int k = grp; k < nblk; k += 16 * G) {  // 16 rows per thread in flight, branch-free masking
      double pa[16], pb[16], px[16];
      float pm[16], pz[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const bool v = k + G * u < nblk;
        const long row = v ? k + G * u : 0;
        const double* p = pd + row * 3 * C + c;
        const float* q = pf + row * 2 * C + c;
        const double l0 = p[0], l1 = p[C], l2 = p[2 * C];
        const float l3 = q[0], l4 = q[C];
        pa[u] = v ? l0 : 0.0;
        pb[u] = v ? l1 : 0.0;
        px[u] = v ? l2 : 0.0;
        pm[u] = v ? l3 : 0.f;
        pz[u] = v ? l4 : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        a += pa[u];
        b += pb[u];
        x += px[u];
        mdy = fmaxf(mdy, pm[u]);
        mz = fmaxf(mz, pz[u]);
      }
    }
  }
  __shared__ double shd[3][256];
  __shared__ float shf[2][256];
  shd[0][threadIdx.x] = a;
  shd[1][threadIdx.x] = b;
  shd[2][threadIdx.x] = x;
  shf[0][threadIdx.x] = mdy;
  shf[1][threadIdx.x] = mz;
  __syncthreads();
  for (int o = 128; o >= BF_CPB; o >>= 1) {
    if ((int)threadIdx.x < o) {
      shd[0][threadIdx.x] += shd[0][threadIdx.x + o];
      shd[1][threadIdx.x] += shd[1][threadIdx.x + o];
      shd[2][threadIdx.x] += shd[2][threadIdx.x + o];
      shf[0][threadIdx.x] = fmaxf(shf[0][threadIdx.x], shf[0][threadIdx.x + o]);
      shf[1][threadIdx.x] = fmaxf(shf[1][threadIdx.x], shf[1][threadIdx.x + o]);
    }
    __syncthreads();
  }
  float B = 0.f;
  if (grp == 0 && c < C)
    B = bwd_coef_d(c, C, shd[0][cl], shd[1][cl], shd[2][cl], shf[0][cl], shf[1][cl], Mfull, gamma, mean, invstd,
                   dgamma, dbeta, dbias, coef);
  if (mx) {  // the block's channels' largest bound, one atomic per block
    __syncthreads();
    if (grp == 0) shf[0][cl] = B;
    __syncthreads();
    if (threadIdx.x == 0) {
      float m = 0.f;
      for (int q = 0; q < BF_CPB; ++q) m = fmaxf(m, shf[0][q]);
      if (!(m < 3.0e38f)) m = 3.0e38f;  // inf / NaN gradients: the largest finite bound (scale 2^-114)
      atomicMax(bound, __float_as_uint(m));
    }
  }
}

template <bool POOL, int NP, int ACT, typename TZ>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const TZ* __restrict__ g, const TZ* __restrict__ z,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ coef, float* __restrict__ dz,
                                                           u16* __restrict__ dz3, long ps,
                                                           const TZ* __restrict__ res, TZ* __restrict__ dres,
                                                           int N, int H, int W, int C, const TZ* __restrict__ g2,
                                                           const unsigned char* __restrict__ mask,
                                                           const unsigned* __restrict__ bound) {
  const int C4 = C >> 2;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const long total = (long)N * Ho * Wo * C4;
  const long stride = (long)gridDim.x * blockDim.x;
  // fp16-pair planes (NP 2): the scale of the bound the finalize wrote
  const float dsc = NP == 2 ? h2_scale_of_bound(__uint_as_float(*bound)) : 1.f;
  struct Co {
    float4 sc, sh, k1, k2, k3, mu;
  };
  auto coefs = [&](int c4) {  // (centred form: dz = k1 dy + k2 (z - mu) + k3, bwd_coef)
    return Co{reinterpret_cast<const float4*>(scale)[c4], reinterpret_cast<const float4*>(shift)[c4],
              reinterpret_cast<const float4*>(coef)[c4], reinterpret_cast<const float4*>(coef + C)[c4],
              reinterpret_cast<const float4*>(coef + 2 * C)[c4], reinterpret_cast<const float4*>(coef + 3 * C)[c4]};
  };
  auto body = [&](long i, int c4, const Co& q) {
    float4 gv = ld4(g, i);
    if (g2) gv = f4add(gv, ld4(g2, i));
    if (!POOL) {
      const float4 zv = ld4(z, i);
      const bool mk = ACT == 2 && mask;
      const float4 rv = ACT == 2 && !mk ? ld4(res, i) : make_float4(0.f, 0.f, 0.f, 0.f);
      const unsigned m = mk ? mask[i] : 0u;
      float r[4], dyv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float zz = F4GET(zv, k);
        const float dy = mk ? (((m >> k) & 1u) ? F4GET(gv, k) : 0.f)
                            : act_grad<ACT>(fmaf(zz, F4GET(q.sc, k), F4GET(q.sh, k)), F4GET(rv, k), F4GET(gv, k));
        dyv[k] = dy;
        // explicit fma order: every ACT instantiation rounds alike (the dy pass's ACT 1 apply is
        // bitwise the ACT 2 one it replaces)
        r[k] = fmaf(F4GET(q.k1, k), dy, fmaf(F4GET(q.k2, k), zz - F4GET(q.mu, k), F4GET(q.k3, k)));
      }
      store4<NP>(dz, dz3, ps, i, make_float4(r[0], r[1], r[2], r[3]), dsc);
      if constexpr (ACT == 2) st4(dres, i, make_float4(dyv[0], dyv[1], dyv[2], dyv[3]));
    } else {
      const unsigned t = (unsigned)(i / C4);  // pooled pixel (VGG sizes: < 2^32)
      const unsigned ow = t % (unsigned)Wo, t2 = t / (unsigned)Wo;
      const unsigned oh = t2 % (unsigned)Ho, n = t2 / (unsigned)Ho;
      const long base = (((long)n * H + 2 * oh) * W + 2 * ow) * C4 + c4;
      const long idx[4] = {base, base + C4, base + (long)W * C4, base + (long)W * C4 + C4};
      float4 zq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) zq[u] = ld4(z, idx[u]);
      float out[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float d[4];
        route1(F4GET(zq[0], k), F4GET(zq[1], k), F4GET(zq[2], k), F4GET(zq[3], k), F4GET(q.sc, k), F4GET(q.sh, k),
               F4GET(gv, k), d[0], d[1], d[2], d[3]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          out[u][k] = fmaf(F4GET(q.k1, k), d[u], fmaf(F4GET(q.k2, k), F4GET(zq[u], k) - F4GET(q.mu, k), F4GET(q.k3, k)));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        store4<NP>(dz, dz3, ps, idx[u], make_float4(out[u][0], out[u][1], out[u][2], out[u][3]), dsc);
    }
  };
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (stride % C4 == 0) {  // every element of this thread has the same channel group (launcher's grid)
    const int c4 = (int)(i0 % C4);
    const Co q = coefs(c4);
    long i = i0;
    if (sizeof(TZ) == 2 && g_bn_unr)  // bf16 rows (8 bytes per thread); fp32 as before
    for (; i + 3 * stride < total; i += 4 * stride) {  // four rows' loads in flight per thread
      body(i, c4, q);
      body(i + stride, c4, q);
      body(i + 2 * stride, c4, q);
      body(i + 3 * stride, c4, q);
    }
    for (; i < total; i += stride) body(i, c4, q);
  } else {
    for (long i = i0; i < total; i += stride) {
      const int c4 = (int)(i % C4);
      body(i, c4, coefs(c4));
    }
  }
}

int grid_1d(long n) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

// grid for a channel-interleaved elementwise pass over n float4 groups of C4 channel groups: when
// the grid is capped, round it so the grid stride is a multiple of C4 (each thread then keeps one
// channel group: per-channel coefficients loaded once, no 64-bit modulo per element)
int grid_ch(long n, int C4) {
  int g = grid_1d(n);
  if ((long)g * 256 < n && C4 > 256 && C4 % 256 == 0) {
    const int m = C4 / 256;
    g = (g + m - 1) / m * m;
  }
  return g;
}


// ---------------- host launchers (TZ = float: fp32 activations; u16: bf16 activations) ----------------
template <typename TZ>
int bn_fwd_stats_host(const TZ* src, int nsplit, TZ* z, float* part, int M, int C, const float* gamma,
                      const float* beta, const float* bias, float* rmean, float* rvar, long long* nbt, float* mean,
                      float* invstd, float* scale, float* shift, float momentum, float eps, hipStream_t st) {
  const int rpb = red_rows_per_block(M, C);
  const int nblk = (M + rpb - 1) / rpb;
  bn_stats_kernel<TZ><<<nblk, RT, 0, st>>>(src, z, nsplit < 1 ? 1 : nsplit, reinterpret_cast<float2*>(part), M, C,
                                           rpb);
  bn_finalize_kernel<<<cdiv(C, 4), 256, 0, st>>>(reinterpret_cast<const float2*>(part), nblk, rpb, M, C, gamma, beta,
                                                  bias, rmean, rvar, nbt, mean, invstd, scale, shift, momentum, eps);
  return (int)hipGetLastError();
}

template <bool POOL, int NP, typename TZ>
void bn_apply_launch(int act, int grid, hipStream_t st, const TZ* z, float* a, u16* a3, long ps, const float* scale,
                     const float* shift, const TZ* res, int N, int H, int W, int C, unsigned char* mask) {
  if constexpr (POOL) {
    bn_apply_kernel<true, NP, 0, TZ><<<grid, 256, 0, st>>>(z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
  } else {
    if (act == 0)
      bn_apply_kernel<false, NP, 0, TZ><<<grid, 256, 0, st>>>(z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
    else if (act == 1)
      bn_apply_kernel<false, NP, 1, TZ><<<grid, 256, 0, st>>>(z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
    else
      bn_apply_kernel<false, NP, 2, TZ><<<grid, 256, 0, st>>>(z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
  }
}

template <typename TZ>
int bn_apply_host(const TZ* z, float* a, u16* a3, int np, const float* scale, const float* shift, int N, int H, int W,
                  int C, int pool, int act, const TZ* res, hipStream_t st, unsigned char* mask = nullptr) {
  if constexpr (sizeof(TZ) == 2) {  // bf16 in, one bf16 plane out: 16-byte lanes (bn_wide.hip)
    if (!pool && np == 1) {
      const int rc = dpa_bn_apply_wide(z, res, a3, mask, scale, shift, (long)N * H * W, C, act, st, nullptr, nullptr);
      if (rc != 1) return rc;
    }
  }
  const long total = (long)N * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 4);
  const long ps = total * 4;
  const int grid = grid_ch(total, C / 4);
  if (np == 2) {  // fp16-pair activation planes (the fp32 VGG engine: fp32 z, ReLU)
    if constexpr (sizeof(TZ) == 4) {
      if (act != 0) return -2;
      if (pool) bn_apply_launch<true, 2, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
      else bn_apply_launch<false, 2, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
      return (int)hipGetLastError();
    } else {
      return -2;
    }
  }
  if (pool) {
    if (np == 0) bn_apply_launch<true, 0, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
    else if (np == 1) bn_apply_launch<true, 1, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
    else bn_apply_launch<true, 3, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
  } else {
    if (np == 0) bn_apply_launch<false, 0, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
    else if (np == 1) bn_apply_launch<false, 1, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
    else bn_apply_launch<false, 3, TZ>(act, grid, st, z, a, a3, ps, scale, shift, res, N, H, W, C, mask);
  }
  return (int)hipGetLastError();
}

template <bool POOL, int NP, typename TZ>
void bn_bwd_apply_launch(int act, int grid, hipStream_t st, const TZ* g, const TZ* z, const float* scale,
                         const float* shift, const float* coef, float* dz, u16* dz3, long ps, const TZ* res, TZ* dres,
                         int N, int H, int W, int C, const TZ* g2, const unsigned char* mask,
                         const unsigned* bound = nullptr) {
  if constexpr (POOL) {
    bn_bwd_apply_kernel<true, NP, 0, TZ><<<grid, 256, 0, st>>>(g, z, scale, shift, coef, dz, dz3, ps, res, dres, N, H,
                                                                W, C, g2, mask, bound);
  } else {
    if (act == 0)
      bn_bwd_apply_kernel<false, NP, 0, TZ><<<grid, 256, 0, st>>>(g, z, scale, shift, coef, dz, dz3, ps, res, dres, N,
                                                                   H, W, C, g2, mask, bound);
    else if (act == 1)
      bn_bwd_apply_kernel<false, NP, 1, TZ><<<grid, 256, 0, st>>>(g, z, scale, shift, coef, dz, dz3, ps, res, dres, N,
                                                                   H, W, C, g2, mask, bound);
    else
      bn_bwd_apply_kernel<false, NP, 2, TZ><<<grid, 256, 0, st>>>(g, z, scale, shift, coef, dz, dz3, ps, res, dres, N,
                                                                   H, W, C, g2, mask, bound);
  }
}

// Backward statistics: reduce pass (summing split-K dgrad slabs of g into g when nsplit > 1) and
// finalize (dgamma, dbeta, dbias, apply coefficients).  Returns a HIP error code.
template <typename TZ>
int bn_bwd_stats(const TZ* gsrc, int nsplit, TZ* g, const TZ* z, const float* scale, const float* shift,
                 const float* mean, const float* invstd, const float* gamma, float* part, float* coef, float* dgamma,
                 float* dbeta, float* dbias, int N, int H, int W, int C, int pool, int act, const TZ* res,
                 hipStream_t st, int* sig = nullptr, int sig_val = 0, const TZ* g2 = nullptr,
                 const unsigned char* mask = nullptr, TZ* dyout = nullptr, unsigned* bound = nullptr) {
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const int Mo = N * Ho * Wo;
  constexpr bool bf = sizeof(TZ) == 2;
  const int rpb = bwd_rows_per_block(Mo, C, bf);
  int nblk = (Mo + rpb - 1) / rpb;
  const bool wide = bwd_wide(Mo, C, bf);
  int nw = 0;  // bf16 in the 1024-thread geometry: 16-byte lanes (bn_wide.hip); 0 = not applicable
  if constexpr (sizeof(TZ) == 2) {
    if (wide && !pool && nsplit == 1) {
      nw = dpa_bn_bwd_reduce_wide(gsrc, g2, z, res, mask, dyout, scale, shift, mean, invstd, part, Mo, C, act, rpb,
                                  sig, sig_val, st);
      if (nw < 0) return -nw;  // a failed launch (not "not applicable")
    }
  }
#define RED(P, A)                                                                                               \
  if (wide)                                                                                                       \
    bn_bwd_reduce_kernel<P, A, TZ, RT><<<nblk, RT, 0, st>>>(gsrc, g, nsplit, z, res, scale, shift, mean, invstd, part, \
                                                            N, H, W, C, rpb, sig, sig_val, g2, mask, dyout, bound);     \
  else                                                                                                            \
    bn_bwd_reduce_kernel<P, A, TZ, RTB><<<nblk, RTB, 0, st>>>(gsrc, g, nsplit, z, res, scale, shift, mean, invstd,  \
                                                              part, N, H, W, C, rpb, sig, sig_val, g2, mask, dyout, bound)
  if (nw > 0) {
    nblk = nw;
  } else if (pool) {
    RED(true, 0);
  } else if (act == 0) {
    RED(false, 0);
  } else if (act == 1) {
    RED(false, 1);
  } else {
    RED(false, 2);
  }
#undef RED
  if (nw > 0)  // (bn_wide.hip's rows: the three sums)
    bn_bwd_finalize_kernel<8, 3><<<cdiv(C, 8), 256, 0, st>>>(part, nblk, C, (float)N * H * W, gamma, mean, invstd,
                                                             dgamma, dbeta, dbias, coef, nullptr);
  else
    bn_bwd_finalize_d_kernel<8><<<cdiv(C, 8), 256, 0, st>>>(part, nblk, C, (float)N * H * W, gamma, mean, invstd,
                                                            dgamma, dbeta, dbias, coef, bound);
  return (int)hipGetLastError();
}

// ---- first layer: BN backward apply fused with the 3x3/s1/p1 weight gradient on the network input.
// Layer 0 of VGG (model.py:18-25 with in_channels 3) has no data gradient, so its dz is read only by
// its weight gradient: dW[co][r][s][ci] = sum_{n,h,w} dz[n,h,w,co] * x[n,h+r-1,w+s-1,ci].  Here each
// thread computes dz for a 2x2 pool window x 4 channels (the apply kernel's routing + coefficients,
// never stored) and accumulates the 27 (tap, input channel) products of each in fp32 registers.
// x (fp32 NHWC, 4 channels, the 4th zero) is staged once per block in LDS with its zero halo.
// Geometry: H = W = 32, 2x2 pool, C = 64, <= 3 live input channels; block = one image band of WB0_RPB
// pooled rows; 256 threads = 16 channel quads x 16 pooled columns, a quad's 16 column lanes form one
// 16-lane row of a wave.  Block partials [blocks][C][27] are summed in a fixed order by
// wgrad0_reduce_kernel (deterministic, no atomics).
constexpr int WB0_RPB = 8;          // pooled rows per block
constexpr int WB0_XR = 2 * WB0_RPB + 2;  // staged input rows (with halo)
constexpr int WB0_XC = 34;          // staged input columns (32 + halo)

__global__ __launch_bounds__(256) void bn_bwd_wgrad0_kernel(const float* __restrict__ g, const float* __restrict__ z,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ coef,
                                                            const float* __restrict__ x, float* __restrict__ wpart) {
  constexpr int H = 32, W = 32, C = 64, C4 = 16, Ho = 16, Wo = 16;
  constexpr int bands = Ho / WB0_RPB;
  __shared__ float4 xs[WB0_XR][WB0_XC];
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const int ow = lane & 15;
  const int c4 = wv * 4 + (lane >> 4);
  const int n = blockIdx.x / bands, band = blockIdx.x % bands;
  const int oh0 = band * WB0_RPB;
  const int h_lo = 2 * oh0 - 1;  // first staged input row
  // stage x rows h_lo .. h_lo + XR - 1, columns -1 .. 32 (zero outside the image)
  for (int e = t; e < WB0_XR * WB0_XC; e += 256) {
    const int rr = e / WB0_XC, cc = e % WB0_XC;
    const int h = h_lo + rr, w = cc - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h >= 0 && h < H && w >= 0 && w < W) v = reinterpret_cast<const float4*>(x)[((long)n * H + h) * W + w];
    xs[rr][cc] = v;
  }
  __syncthreads();
  const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
  const float4 sh = reinterpret_cast<const float4*>(shift)[c4];
  const float4 k1 = reinterpret_cast<const float4*>(coef)[c4];
  const float4 k2 = reinterpret_cast<const float4*>(coef + C)[c4];
  const float4 k3 = reinterpret_cast<const float4*>(coef + 2 * C)[c4];
  const float4 mu = reinterpret_cast<const float4*>(coef + 3 * C)[c4];  // (centred form, bwd_coef)
  float acc[4][27];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < 27; ++j) acc[k][j] = 0.f;
  for (int oh = oh0; oh < oh0 + WB0_RPB; ++oh) {
    const float4 gv = reinterpret_cast<const float4*>(g)[(((long)n * Ho + oh) * Wo + ow) * C4 + c4];
    const long base = (((long)n * H + 2 * oh) * W + 2 * ow) * C4 + c4;
    float4 zq[4];
    zq[0] = reinterpret_cast<const float4*>(z)[base];
    zq[1] = reinterpret_cast<const float4*>(z)[base + C4];
    zq[2] = reinterpret_cast<const float4*>(z)[base + W * C4];
    zq[3] = reinterpret_cast<const float4*>(z)[base + W * C4 + C4];
    float d[4][4];  // [window position][channel]
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float r[4];
      route1(F4GET(zq[0], k), F4GET(zq[1], k), F4GET(zq[2], k), F4GET(zq[3], k), F4GET(sc, k), F4GET(sh, k),
             F4GET(gv, k), r[0], r[1], r[2], r[3]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q][k] = F4GET(k1, k) * r[q] + F4GET(k2, k) * (F4GET(zq[q], k) - F4GET(mu, k)) + F4GET(k3, k);
    }
    // the 4x4 input neighbourhood of the 2x2 window: rows 2oh-1 .. 2oh+2, columns 2ow-1 .. 2ow+2
    const int xr = 2 * oh - 1 - h_lo;  // staged row of input row 2oh-1
    float4 nb[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) nb[a][b] = xs[xr + a][2 * ow + b];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int dh = q >> 1, dw = q & 1;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) {
          const float4 xv = nb[dh + r][dw + s2];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[k][(r * 3 + s2) * 3 + 0] = fmaf(d[q][k], xv.x, acc[k][(r * 3 + s2) * 3 + 0]);
            acc[k][(r * 3 + s2) * 3 + 1] = fmaf(d[q][k], xv.y, acc[k][(r * 3 + s2) * 3 + 1]);
            acc[k][(r * 3 + s2) * 3 + 2] = fmaf(d[q][k], xv.z, acc[k][(r * 3 + s2) * 3 + 2]);
          }
        }
    }
  }
  // sum over the 16 column lanes of each channel quad (fixed xor order), lane ow == 0 writes
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < 27; ++j) {
      float v = acc[k][j];
      v += __shfl_xor(v, 8, 16);
      v += __shfl_xor(v, 4, 16);
      v += __shfl_xor(v, 2, 16);
      v += __shfl_xor(v, 1, 16);
      acc[k][j] = v;
    }
  if (ow == 0) {
    float* o = wpart + (long)blockIdx.x * C * 27 + (long)(4 * c4) * 27;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 27; ++j) o[k * 27 + j] = acc[k][j];
  }
}

// dw[co][r][s][0..CP) (KRSC, CP = padded input channels; channels >= 3 get 0) = fixed-order sum of
// the block partials [nblk][C][27].  One block per output channel: 32 groups x 32 lanes.
__global__ __launch_bounds__(1024) void wgrad0_reduce_kernel(const float* __restrict__ wpart, int nblk, int C,
                                                             float* __restrict__ dw, int CP) {
  __shared__ float sh[32][32];
  const int co = blockIdx.x, j = threadIdx.x & 31, grp = threadIdx.x >> 5;
  float a = 0.f;
  if (j < 27) {
    int b = grp;
    for (; b + 3 * 32 < nblk; b += 4 * 32) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = wpart[((long)(b + 32 * u) * C + co) * 27 + j];
#pragma unroll
      for (int u = 0; u < 4; ++u) a += v[u];
    }
    for (; b < nblk; b += 32) a += wpart[((long)b * C + co) * 27 + j];
  }
  sh[grp][j] = a;
  __syncthreads();
  for (int o = 16; o >= 1; o >>= 1) {
    if (grp < o) sh[grp][j] += sh[grp + o][j];
    __syncthreads();
  }
  for (int e = threadIdx.x; e < 9 * CP; e += 1024) {
    const int rs = e / CP, ci = e % CP;
    dw[(long)co * 9 * CP + e] = ci < 3 ? sh[0][rs * 3 + ci] : 0.f;
  }
}


template <typename TZ>
int bn_bwd_host(const TZ* gsrc, int nsplit, TZ* g, const TZ* z, const float* scale, const float* shift,
                const float* mean, const float* invstd, const float* gamma, float* part, float* coef, float* dgamma,
                float* dbeta, float* dbias, float* dz, u16* dz3, int np, int N, int H, int W, int C, int pool, int act,
                const TZ* res, TZ* dres, hipStream_t st, int* sig, int sig_val, const TZ* g2,
                const unsigned char* mask, unsigned* bound) {
  if (nsplit < 1) nsplit = 1;
  if (np == 2 && (sizeof(TZ) != 4 || bound == nullptr || act != 0)) return -2;  // fp16 pairs: the VGG engine
  // add+ReLU: the reduce pass stores dy (= dres) and the apply pass reads it alone as an identity
  // activation (measured faster than re-reading g, g2 and the mask / residual)
  const bool dyp = act == 2 && nsplit == 1 && !pool && dres != nullptr;
  const int rc0 = bn_bwd_stats<TZ>(gsrc, nsplit, g, z, scale, shift, mean, invstd, gamma, part, coef, dgamma, dbeta,
                                   dbias, N, H, W, C, pool, act, res, st, sig, sig_val, g2, mask, dyp ? dres : nullptr,
                                   np == 2 ? bound : nullptr);
  if (rc0) return rc0;
  if (dyp) {
    act = 1;
    gsrc = dres;
    g2 = nullptr;
    mask = nullptr;
    res = nullptr;
    dres = nullptr;
  }
  if (dz == nullptr && dz3 == nullptr) return -2;
  const int Mo = N * (pool ? (H / 2) * (W / 2) : H * W);
  const TZ* gg = nsplit > 1 ? g : gsrc;
  if constexpr (sizeof(TZ) == 2) {  // bf16 in, one bf16 plane out: 16-byte lanes (bn_wide.hip)
    if (!pool && np == 1 && act != 2) {
      const int rc = dpa_bn_bwd_apply_wide(gg, g2, z, dz3, scale, shift, coef, (long)Mo, C, act, st);
      if (rc != 1) return rc;
    }
  }
  const long total = (long)Mo * (C / 4);
  const long ps = (long)N * H * W * C;
  const int grid = grid_ch(total, C / 4);
#define BAP(P, NPT) \
  bn_bwd_apply_launch<P, NPT, TZ>(act, grid, st, gg, z, scale, shift, coef, dz, dz3, ps, res, dres, N, H, W, C, g2, mask)
  if (np == 2) {
    if constexpr (sizeof(TZ) == 4) {
      if (pool)
        bn_bwd_apply_launch<true, 2, TZ>(act, grid, st, gg, z, scale, shift, coef, dz, dz3, ps, res, dres, N, H, W, C,
                                         g2, mask, bound);
      else
        bn_bwd_apply_launch<false, 2, TZ>(act, grid, st, gg, z, scale, shift, coef, dz, dz3, ps, res, dres, N, H, W,
                                          C, g2, mask, bound);
    }
    return (int)hipGetLastError();
  }
  if (pool) {
    if (np == 0) BAP(true, 0);
    else if (np == 1) BAP(true, 1);
    else BAP(true, 3);
  } else {
    if (np == 0) BAP(false, 0);
    else if (np == 1) BAP(false, 1);
    else BAP(false, 3);
  }
#undef BAP
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {
// floats of partial workspace needed by fwd stats (2 per (block, channel)) / bwd (5 per ...)
// (backward: rows of the fp32 or the bf16 geometry, whichever has more; the bf16 wide reduce of
// bn_wide.hip uses the bf16 geometry's rows per block)
long dpa_bn_part_floats(int M, int C, int bwd) {
  if (!bwd) {
    const int rpb = red_rows_per_block(M, C);
    return (long)((M + rpb - 1) / rpb) * C * 2;
  }
  const int r32 = bwd_rows_per_block(M, C, false), r16 = bwd_rows_per_block(M, C, true);
  // fp32 geometry: [block][3][C] fp64 sums + [block][2][C] maxima (8 floats per (block, channel));
  // bf16 wide reduce (bn_wide.hip): [block][3][C] fp32
  return std::max((long)((M + r32 - 1) / r32) * 8, (long)((M + r16 - 1) / r16) * 5) * C;
}

// z [M][C] (or nsplit fp32 slabs of it in src; then z is written) -> partials -> finalize.
// zbf: z/src are bf16 (nsplit must be 1).
int dpa_bn_fwd_stats(const void* src, int nsplit, void* z, float* part, int M, int C, const float* gamma,
                     const float* beta, const float* bias, float* rmean, float* rvar, long long* nbt, float* mean,
                     float* invstd, float* scale, float* shift, float momentum, float eps, int zbf, hipStream_t st) {
  if (C % 4 || (zbf && nsplit > 1)) return -2;
  if (zbf)
    return bn_fwd_stats_host<u16>((const u16*)src, nsplit, (u16*)z, part, M, C, gamma, beta, bias, rmean, rvar, nbt,
                                  mean, invstd, scale, shift, momentum, eps, st);
  return bn_fwd_stats_host<float>((const float*)src, nsplit, (float*)z, part, M, C, gamma, beta, bias, rmean, rvar,
                                  nbt, mean, invstd, scale, shift, momentum, eps, st);
}

// Finalize from (mean, M2) partials of nblk row blocks of rpb rows each (the producer is not
// bn_stats_kernel, e.g. the first-layer conv's epilogue, first_layer.hip).
int dpa_bn_finalize(const float* part, int nblk, int rpb, int M, int C, const float* gamma, const float* beta,
                    const float* bias, float* rmean, float* rvar, long long* nbt, float* mean, float* invstd,
                    float* scale, float* shift, float momentum, float eps, hipStream_t st) {
  bn_finalize_kernel<<<cdiv(C, 4), 256, 0, st>>>(reinterpret_cast<const float2*>(part), nblk, rpb, M, C, gamma, beta,
                                                  bias, rmean, rvar, nbt, mean, invstd, scale, shift, momentum, eps);
  return (int)hipGetLastError();
}

// Finalize from channel-major partials part[c][k] (conv epilogue statistics).
int dpa_bn_finalize_cm(const float* part, int nblk, int rpb, int M, int C, const float* gamma, const float* beta,
                       const float* bias, float* rmean, float* rvar, long long* nbt, float* mean, float* invstd,
                       float* scale, float* shift, float momentum, float eps, hipStream_t st) {
  bn_finalize_cm_kernel<<<C, 256, 0, st>>>(reinterpret_cast<const float2*>(part), nblk, rpb, M, gamma, beta, bias,
                                           rmean, rvar, nbt, mean, invstd, scale, shift, momentum, eps);
  return (int)hipGetLastError();
}

int dpa_bn_eval_params(const float* gamma, const float* beta, const float* bias, const float* rmean,
                       const float* rvar, float* scale, float* shift, int C, float eps, hipStream_t st) {
  bn_eval_params_kernel<<<cdiv(C, 256), 256, 0, st>>>(gamma, beta, bias, rmean, rvar, scale, shift, C, eps);
  return (int)hipGetLastError();
}

// out: fp32 a (np == 0), bf16 planes a3 [np][...] (np in {1, 3}) or fp16 pairs (np 2, scale H2_SA).  act: 0 relu (pool allowed),
// 1 none, 2 relu(. + res).  zbf: z and res are bf16.
int dpa_bn_apply(const void* z, float* a, u16* a3, int np, const float* scale, const float* shift, int N, int H,
                 int W, int C, int pool, int act, const void* res, int zbf, hipStream_t st, unsigned char* mask) {
  if (C % 4 || act < 0 || act > 2 || (act != 0 && pool) || (act == 2 && !res)) return -2;
  if (mask && act != 2) return -2;
  if (zbf)
    return bn_apply_host<u16>((const u16*)z, a, a3, np, scale, shift, N, H, W, C, pool, act, (const u16*)res, st,
                              mask);
  return bn_apply_host<float>((const float*)z, a, a3, np, scale, shift, N, H, W, C, pool, act, (const float*)res, st,
                              mask);
}

// gsrc: grad of the layer output (pooled shape if pool), or nsplit fp32 slabs of it (then the sum is
// written to g).  Writes dz [N,H,W,C] (fp32, or bf16 planes dz3) and dgamma/dbeta/dbias; act 2 also
// the residual gradient dres.  zbf: gsrc/g/z/res/dres are bf16 (nsplit must be 1).  g2 (optional,
// same type and shape as g, nsplit 1): the gradient is gsrc + g2, summed on load.
int dpa_bn_bwd(const void* gsrc, int nsplit, void* g, const void* z, const float* scale, const float* shift,
               const float* mean, const float* invstd, const float* gamma, float* part, float* coef, float* dgamma,
               float* dbeta, float* dbias, float* dz, u16* dz3, int np, int N, int H, int W, int C, int pool, int act,
               const void* res, void* dres, int zbf, hipStream_t st, int* sig, int sig_val, const void* g2,
               const unsigned char* mask, unsigned* bound) {
  if (C % 4 || act < 0 || act > 2 || (act != 0 && pool) || (act == 2 && ((!res && !mask) || !dres))) return -2;
  if (mask && act != 2) return -2;
  if (zbf && nsplit > 1) return -2;
  if (g2 && nsplit > 1) return -2;  // a second gradient operand is summed on load of an unsplit g only
  if (zbf)
    return bn_bwd_host<u16>((const u16*)gsrc, nsplit, (u16*)g, (const u16*)z, scale, shift, mean, invstd, gamma, part,
                            coef, dgamma, dbeta, dbias, dz, dz3, np, N, H, W, C, pool, act, (const u16*)res,
                            (u16*)dres, st, sig, sig_val, (const u16*)g2, mask, bound);
  return bn_bwd_host<float>((const float*)gsrc, nsplit, (float*)g, (const float*)z, scale, shift, mean, invstd, gamma,
                            part, coef, dgamma, dbeta, dbias, dz, dz3, np, N, H, W, C, pool, act, (const float*)res,
                            (float*)dres, st, sig, sig_val, (const float*)g2, mask, bound);
}

// Layer-0 backward (see bn_bwd_wgrad0_kernel): BN statistics, then the fused apply + weight gradient.
// g [N,16,16,64] (or nsplit slabs of it in gsrc), z [N,32,32,64], x [N,32,32,4] fp32, dw [64,3,3,CP].
long dpa_wgrad0_part_floats(int N) { return (long)N * (16 / WB0_RPB) * 64 * 27; }

int dpa_bn_bwd_wgrad0(const float* gsrc, int nsplit, float* g, const float* z, const float* scale,
                      const float* shift, const float* mean, const float* invstd, const float* gamma, float* part,
                      float* coef, float* dgamma, float* dbeta, float* dbias, const float* x, float* wpart,
                      float* dw, int CP, int N, hipStream_t st, int* sig, int sig_val) {
  if (nsplit < 1) nsplit = 1;
  if (CP < 3) return -2;
  const int rc = bn_bwd_stats<float>(gsrc, nsplit, g, z, scale, shift, mean, invstd, gamma, part, coef, dgamma, dbeta,
                                     dbias, N, 32, 32, 64, 1, 0, nullptr, st, sig, sig_val);
  if (rc) return rc;
  const float* gg = nsplit > 1 ? g : gsrc;
  const int nblk = N * (16 / WB0_RPB);
  bn_bwd_wgrad0_kernel<<<nblk, 256, 0, st>>>(gg, z, scale, shift, coef, x, wpart);
  wgrad0_reduce_kernel<<<64, 1024, 0, st>>>(wpart, nblk, 64, dw, CP);
  return (int)hipGetLastError();
}

DPA_H2_OVF_ACCESSOR(dpa_h2_ovf_bn)

}  // extern "C"
