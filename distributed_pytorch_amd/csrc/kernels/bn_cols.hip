// Training BatchNorm2d (+ReLU, +2x2/s2 max-pool) of a SMALL activation in one launch with no
// cross-block hand-off: the VGG tail layers (4x4 and 2x2 maps at batch 256; model.py:16,24,25).
//
// bn_fused.hip runs these layers as channel slices x R row blocks that meet per slice (tickets,
// a bounded spin, an agent-scope hand-off): ~12-20 us per layer in the step for 2-8 MB tensors,
// mostly the rendezvous and its latency chain (profiles/r4_null_step_timeline.txt).  Here a block
// owns CW = 4 channels over ALL rows of the layer, so nothing leaves the block between the
// statistics and the apply:
//
//   * thread t holds row units t, t + 256, ... (a unit is one pixel, or one 2x2 pool window =
//     4 pixels) of its 4 channels in registers, summing the split-K slabs of the producing conv in
//     split order on load (and writing z when there are several);
//   * exact two-pass statistics from the registers: the block's fixed-order LDS tree gives the
//     mean, a second pass the centred sum of squares; then the finalize (running statistics with
//     the folded conv bias, unbiased variance, num_batches_tracked) and the apply:
//     relu(fma(z, scale, shift)) (max over the window), written as fp32 or bf16 operand planes --
//     or nothing when the consumer applies it (the head kernel, a conv with BN on load);
//   * grid = C / 4 blocks; each lane's 16-byte loads are strided by the row pitch (scattered, but
//     the tensors are L2/MALL-resident right after the conv that wrote them).
// Deterministic (fixed orders throughout), no atomics, no residency assumption.
#include "common.h"

namespace {

constexpr int CT = 256;  // threads per block
constexpr int CW = 4;    // channels per block

__device__ __forceinline__ float4 ld4f(const float* p, long i4) { return reinterpret_cast<const float4*>(p)[i4]; }
__device__ __forceinline__ float f4g(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// block-wide fixed-order sum of 4 lanes' values (LDS tree over the 256 threads)
__device__ __forceinline__ float4 block_sum4(float4 v, float4* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
#pragma unroll
  for (int o = CT / 2; o >= 1; o >>= 1) {
    if (t < o) {
      const float4 a = sh[t], b = sh[t + o];
      sh[t] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
    __syncthreads();
  }
  const float4 r = sh[0];
  __syncthreads();
  return r;
}

// U: row units per thread (compile-time register tile); POOL: a unit is a 2x2 window; NP: 0 fp32
// output, 1 / 3 bf16 planes; out == nullptr: statistics and coefficients only
template <int U, bool POOL, int NP>
__global__ __launch_bounds__(CT) void bn_cols_fwd_kernel(const float* __restrict__ src, int nsplit, long slab,
                                                         float* __restrict__ zw, int N, int H, int W, int C,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         const float* __restrict__ bias, float* __restrict__ rmean,
                                                         float* __restrict__ rvar, long long* __restrict__ nbt,
                                                         float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                         float* __restrict__ scale_out, float* __restrict__ shift_out,
                                                         float* __restrict__ out, u16* __restrict__ out3, long ps,
                                                         float momentum, float eps) {
  constexpr int Q = POOL ? 4 : 1;  // pixels per unit
  const int C4 = C >> 2, c4 = blockIdx.x;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const int units = N * Ho * Wo;
  const int t = threadIdx.x;
  __shared__ float4 sh[CT];
  float4 v[U][Q];
  // pixel (row of z) of sub-position q of unit u
  auto pix = [&](int u, int q) -> long {
    if constexpr (!POOL) {
      return u;
    } else {
      const int ow = u % Wo, r = u / Wo, oh = r % Ho, n = r / Ho;
      return ((long)n * H + 2 * oh + (q >> 1)) * W + 2 * ow + (q & 1);
    }
  };
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int u = t + j * CT;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (u < units) {
        const long i4 = pix(u, q) * C4 + c4;
        a = ld4f(src, i4);
        for (int k = 1; k < nsplit; ++k) {  // split-K slabs, in split order
          const float4 b = ld4f(src + k * slab, i4);
          a = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
        }
        if (nsplit > 1) reinterpret_cast<float4*>(zw)[i4] = a;
      }
      v[j][q] = a;
      s = make_float4(s.x + a.x, s.y + a.y, s.z + a.z, s.w + a.w);
    }
  }
  const float cnt = (float)units * Q;
  const float4 tot = block_sum4(s, sh);
  const float4 mu = make_float4(tot.x / cnt, tot.y / cnt, tot.z / cnt, tot.w / cnt);
  float4 s2 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (t + j * CT < units) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float4 d = make_float4(v[j][q].x - mu.x, v[j][q].y - mu.y, v[j][q].z - mu.z, v[j][q].w - mu.w);
        s2 = make_float4(fmaf(d.x, d.x, s2.x), fmaf(d.y, d.y, s2.y), fmaf(d.z, d.z, s2.z), fmaf(d.w, d.w, s2.w));
      }
    }
  }
  const float4 m2 = block_sum4(s2, sh);
  // finalize (bn_finalize_kernel's expressions)
  float sc[4], shf[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * c4 + k;
    const float m = f4g(mu, k), M2 = f4g(m2, k);
    const float var = M2 / cnt;
    const float inv = rsqrtf(var + eps);
    const float gm = gamma[c];
    sc[k] = gm * inv;
    shf[k] = beta[c] - m * gm * inv;
    if (t == 0) {
      mean_out[c] = m;
      invstd_out[c] = inv;
      scale_out[c] = sc[k];
      shift_out[c] = shf[k];
      if (rmean) {
        const float b = bias ? bias[c] : 0.f;
        const float unb = cnt > 1.f ? M2 / (cnt - 1.f) : var;
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * (m + b);
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
      }
    }
  }
  if (t == 0 && c4 == 0 && nbt) nbt[0] += 1;
  if (out == nullptr && out3 == nullptr) return;
  // apply: relu(fma(z, scale, shift)), max over the window
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int u = t + j * CT;
    if (u >= units) continue;
    float y[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float m = fmaxf(fmaf(f4g(v[j][0], k), sc[k], shf[k]), 0.f);
#pragma unroll
      for (int q = 1; q < Q; ++q) m = fmaxf(m, fmaxf(fmaf(f4g(v[j][q], k), sc[k], shf[k]), 0.f));
      y[k] = m;
    }
    const long o4 = (long)u * C4 + c4;
    if constexpr (NP == 0) {
      reinterpret_cast<float4*>(out)[o4] = make_float4(y[0], y[1], y[2], y[3]);
    } else {
      u16 o[4][3];
#pragma unroll
      for (int k = 0; k < 4; ++k) split_val<NP>(y[k], o[k]);
#pragma unroll
      for (int p = 0; p < NP; ++p)
        reinterpret_cast<ushort4*>(out3 + p * ps)[o4] = make_ushort4(o[0][p], o[1][p], o[2][p], o[3][p]);
    }
  }
}


// ---- backward: the same block geometry.  dy through the ReLU (and the 2x2 window's first max, in
// scan order 00, 01, 10, 11, as bn.hip's route1), sums of dy, dy * xhat, xhat from registers
// (fixed-order tree), bn_bwd_finalize_kernel's coefficients, then dz = fma(k1, dy, fma(k2, z, k3))
// for every pixel.  gsrc: dL/d(layer output) (pooled shape when POOL), or nsplit slabs of it.
template <int U, bool POOL, int NP>
__global__ __launch_bounds__(CT) void bn_cols_bwd_kernel(const float* __restrict__ gsrc, int nsplit, long gslab,
                                                         const float* __restrict__ z, int N, int H, int W, int C,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ gamma, float* __restrict__ dgamma,
                                                         float* __restrict__ dbeta, float* __restrict__ dbias,
                                                         float* __restrict__ dz, u16* __restrict__ dz3, long ps,
                                                         int* sig, int sig_val) {
  start_signal(sig, sig_val);
  constexpr int Q = POOL ? 4 : 1;
  const int C4 = C >> 2, c4 = blockIdx.x;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const int units = N * Ho * Wo;
  const int t = threadIdx.x;
  __shared__ float4 sh[CT];
  const float4 sc = reinterpret_cast<const float4*>(scale)[c4], sf = reinterpret_cast<const float4*>(shift)[c4];
  const float4 mu = reinterpret_cast<const float4*>(mean)[c4], is = reinterpret_cast<const float4*>(invstd)[c4];
  float4 zv[U][Q], gv[U];
  auto pix = [&](int u, int q) -> long {
    if constexpr (!POOL) {
      return u;
    } else {
      const int ow = u % Wo, r = u / Wo, oh = r % Ho, n = r / Ho;
      return ((long)n * H + 2 * oh + (q >> 1)) * W + 2 * ow + (q & 1);
    }
  };
  // dy of sub-position q of unit j, channel k
  auto dyk = [&](int j, int q, int k) -> float {
    const float g = f4g(gv[j], k), s_ = f4g(sc, k), h_ = f4g(sf, k);
    if constexpr (!POOL) {
      return fmaf(f4g(zv[j][0], k), s_, h_) > 0.f ? g : 0.f;
    } else {
      float y[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) y[p] = fmaxf(fmaf(f4g(zv[j][p], k), s_, h_), 0.f);
      int arg = 0;
      float mx = y[0];
      if (y[1] > mx) { mx = y[1]; arg = 1; }
      if (y[2] > mx) { mx = y[2]; arg = 2; }
      if (y[3] > mx) { mx = y[3]; arg = 3; }
      return (arg == q && y[q] > 0.f) ? g : 0.f;
    }
  };
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int u = t + j * CT;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < Q; ++q) zv[j][q] = g;
    if (u < units) {
      const long g4 = (long)u * C4 + c4;
      g = ld4f(gsrc, g4);
      for (int k = 1; k < nsplit; ++k) {
        const float4 b = ld4f(gsrc + k * gslab, g4);
        g = make_float4(g.x + b.x, g.y + b.y, g.z + b.z, g.w + b.w);
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) zv[j][q] = ld4f(z, pix(u, q) * C4 + c4);
    }
    gv[j] = g;
  }
  float a[3][4] = {};
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (t + j * CT >= units) continue;
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float dy = dyk(j, q, k);
        const float xh = (f4g(zv[j][q], k) - f4g(mu, k)) * f4g(is, k);
        a[0][k] += dy;
        a[1][k] = fmaf(dy, xh, a[1][k]);
        a[2][k] += xh;
      }
  }
  float4 tot[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) tot[i] = block_sum4(make_float4(a[i][0], a[i][1], a[i][2], a[i][3]), sh);
  const float Mfull = (float)units * Q;
  float k1[4], k2[4], k3[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * c4 + k;
    const float sdy = f4g(tot[0], k), sdx = f4g(tot[1], k), sx = f4g(tot[2], k);
    const float iv = f4g(is, k), gm = gamma[c];
    const float kk1 = gm * iv;
    const float k2x = -kk1 * sdx / Mfull;
    const float kk3 = -kk1 * sdy / Mfull;
    k1[k] = kk1;
    k2[k] = k2x * iv;
    k3[k] = kk3 - k2x * iv * f4g(mu, k);
    if (t == 0) {
      dgamma[c] = sdx;
      dbeta[c] = sdy;
      if (dbias) dbias[c] = k2x * sx;
    }
  }
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int u = t + j * CT;
    if (u >= units) continue;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      float r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = fmaf(k1[k], dyk(j, q, k), fmaf(k2[k], f4g(zv[j][q], k), k3[k]));
      const long o4 = pix(u, q) * C4 + c4;
      if constexpr (NP == 0) {
        reinterpret_cast<float4*>(dz)[o4] = make_float4(r[0], r[1], r[2], r[3]);
      } else {
        u16 o[4][3];
#pragma unroll
        for (int k = 0; k < 4; ++k) split_val<NP>(r[k], o[k]);
#pragma unroll
        for (int p = 0; p < NP; ++p)
          reinterpret_cast<ushort4*>(dz3 + p * ps)[o4] = make_ushort4(o[0][p], o[1][p], o[2][p], o[3][p]);
      }
    }
  }
}

template <int U, bool POOL>
void launch_np(int np, int grid, hipStream_t st, const float* src, int nsplit, long slab, float* zw, int N, int H,
               int W, int C, const float* gamma, const float* beta, const float* bias, float* rmean, float* rvar,
               long long* nbt, float* mean, float* invstd, float* scale, float* shift, float* out, u16* out3, long ps,
               float momentum, float eps) {
#define BC_ARGS                                                                                                 \
  src, nsplit, slab, zw, N, H, W, C, gamma, beta, bias, rmean, rvar, nbt, mean, invstd, scale, shift, out, out3, ps, \
      momentum, eps
  if (np == 0)
    bn_cols_fwd_kernel<U, POOL, 0><<<grid, CT, 0, st>>>(BC_ARGS);
  else if (np == 1)
    bn_cols_fwd_kernel<U, POOL, 1><<<grid, CT, 0, st>>>(BC_ARGS);
  else
    bn_cols_fwd_kernel<U, POOL, 3><<<grid, CT, 0, st>>>(BC_ARGS);
#undef BC_ARGS
}

// register tile per thread: the smallest U in {1, 2, 4, 8, 16} holding every unit (0: too large)
int cols_units(int units, bool pool) {
  const int need = (units + CT - 1) / CT;
  const int umax = pool ? 4 : 16;  // (a pool unit is 4 pixels: 16 float4 per thread at most)
  for (int u = 1; u <= umax; u *= 2)
    if (need <= u) return u;
  return 0;
}

template <int U, bool POOL>
void launch_bwd_np(int np, int grid, hipStream_t st, const float* gsrc, int nsplit, long gslab, const float* z, int N,
                   int H, int W, int C, const float* scale, const float* shift, const float* mean, const float* invstd,
                   const float* gamma, float* dgamma, float* dbeta, float* dbias, float* dz, u16* dz3, long ps,
                   int* sig, int sig_val) {
#define BB_ARGS \
  gsrc, nsplit, gslab, z, N, H, W, C, scale, shift, mean, invstd, gamma, dgamma, dbeta, dbias, dz, dz3, ps, sig, sig_val
  if (np == 0)
    bn_cols_bwd_kernel<U, POOL, 0><<<grid, CT, 0, st>>>(BB_ARGS);
  else if (np == 1)
    bn_cols_bwd_kernel<U, POOL, 1><<<grid, CT, 0, st>>>(BB_ARGS);
  else
    bn_cols_bwd_kernel<U, POOL, 3><<<grid, CT, 0, st>>>(BB_ARGS);
#undef BB_ARGS
}

}  // namespace

extern "C" {
// 1 when this layer (units = output pixels, or pool windows) fits the column-block forward BN
int dpa_bn_cols_ok(int units, int C, int pool) { return C % 4 == 0 && cols_units(units, pool != 0) > 0; }

// src: z [N,H,W,C] fp32, or nsplit slabs of it (then z is written to zw); writes mean, invstd,
// scale, shift, the running statistics (rmean may be null: none) and nbt; out (fp32) or out3 (bf16
// planes [np][...], plane stride ps) receives relu(BN(z)) (2x2 max-pooled); both null: no apply.
int dpa_bn_cols_fwd(const float* src, int nsplit, float* zw, int N, int H, int W, int C, int pool,
                    const float* gamma, const float* beta, const float* bias, float* rmean, float* rvar,
                    long long* nbt, float* mean, float* invstd, float* scale, float* shift, float* out,
                    unsigned short* out3, int np, long ps, float momentum, float eps, hipStream_t st) {
  const int units = N * (pool ? (H / 2) * (W / 2) : H * W);
  const int U = C % 4 ? 0 : cols_units(units, pool != 0);
  if (!U || (pool && (H % 2 || W % 2))) return -6;
  const long slab = (long)N * H * W * C;
  const int grid = C / 4;
  if (nsplit < 1) nsplit = 1;
#define L(UU, P)                                                                                                  \
  launch_np<UU, P>(np, grid, st, src, nsplit, slab, zw, N, H, W, C, gamma, beta, bias, rmean, rvar, nbt, mean, invstd, \
                   scale, shift, out, out3, ps, momentum, eps)
  if (pool) {
    switch (U) {
      case 1: L(1, true); break;
      case 2: L(2, true); break;
      default: L(4, true); break;
    }
  } else {
    switch (U) {
      case 1: L(1, false); break;
      case 2: L(2, false); break;
      case 4: L(4, false); break;
      case 8: L(8, false); break;
      default: L(16, false); break;
    }
  }
#undef L
  return (int)hipGetLastError();
}

// Backward of the same layers: gsrc = dL/d(layer output) (pooled shape when pool) or nsplit slabs of
// it; writes dgamma, dbeta, dbias (optional) and dz [N,H,W,C] as fp32 or bf16 planes (np, stride ps).
int dpa_bn_cols_bwd(const float* gsrc, int nsplit, const float* z, int N, int H, int W, int C, int pool,
                    const float* scale, const float* shift, const float* mean, const float* invstd,
                    const float* gamma, float* dgamma, float* dbeta, float* dbias, float* dz, unsigned short* dz3,
                    int np, long ps, int* sig, int sig_val, hipStream_t st) {
  const int units = N * (pool ? (H / 2) * (W / 2) : H * W);
  const int U = C % 4 ? 0 : cols_units(units, pool != 0);
  if (!U || (pool && (H % 2 || W % 2))) return -6;
  const long gslab = (long)units * C;
  const int grid = C / 4;
  if (nsplit < 1) nsplit = 1;
#define L(UU, P)                                                                                                \
  launch_bwd_np<UU, P>(np, grid, st, gsrc, nsplit, gslab, z, N, H, W, C, scale, shift, mean, invstd, gamma, dgamma, \
                       dbeta, dbias, dz, dz3, ps, sig, sig_val)
  if (pool) {
    switch (U) {
      case 1: L(1, true); break;
      case 2: L(2, true); break;
      default: L(4, true); break;
    }
  } else {
    switch (U) {
      case 1: L(1, false); break;
      case 2: L(2, false); break;
      case 4: L(4, false); break;
      case 8: L(8, false); break;
      default: L(16, false); break;
    }
  }
#undef L
  return (int)hipGetLastError();
}
}  // extern "C"
