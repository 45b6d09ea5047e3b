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
// Forward:  stats partials (shifted sums per 64-row chunk) -> finalize (Chan merge, running-stat
//           update with unbiased var, momentum, num_batches_tracked) -> apply+relu(+pool).
// Backward: nothing but z (the conv output) is stored; y = relu(z*scale+shift), the pool argmax
//           (first max in window scan order, as torch's CPU kernel) and x_hat are recomputed:
//           reduce pass (sum dy, sum dy*xhat, sum xhat) -> finalize -> apply pass writing dz.
#include "common.h"

namespace {
constexpr int CHUNK = 64;  // rows per stats partial

// ---- forward statistics: per (chunk, channel) shifted sums -> (mean, M2) ----
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ z, float2* __restrict__ part, int M,
                                                       int C) {
  const int C4 = C >> 2;
  const int per_block = 256 / C4;  // chunks per block (C4 <= 256 divides 256 for C in {4..1024} powers of 2)
  const int t = threadIdx.x;
  if (t >= per_block * C4) return;
  const int c4 = t % C4;
  const int chunk = blockIdx.x * per_block + t / C4;
  const int r0 = chunk * CHUNK;
  if (r0 >= M) return;
  const int r1 = min(M, r0 + CHUNK);
  const float4* zp = reinterpret_cast<const float4*>(z) + (long)r0 * C4 + c4;
  const float4 x0 = zp[0];
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  for (int r = r0; r < r1; ++r) {
    const float4 v = zp[(long)(r - r0) * C4];
    const float d0 = v.x - x0.x, d1 = v.y - x0.y, d2 = v.z - x0.z, d3 = v.w - x0.w;
    s1.x += d0;
    s1.y += d1;
    s1.z += d2;
    s1.w += d3;
    s2.x += d0 * d0;
    s2.y += d1 * d1;
    s2.z += d2 * d2;
    s2.w += d3 * d3;
  }
  const float n = (float)(r1 - r0), inv = 1.f / n;
  float2* o = part + (long)chunk * C + c4 * 4;
  o[0] = make_float2(x0.x + s1.x * inv, fmaxf(s2.x - s1.x * s1.x * inv, 0.f));
  o[1] = make_float2(x0.y + s1.y * inv, fmaxf(s2.y - s1.y * s1.y * inv, 0.f));
  o[2] = make_float2(x0.z + s1.z * inv, fmaxf(s2.z - s1.z * s1.z * inv, 0.f));
  o[3] = make_float2(x0.w + s1.w * inv, fmaxf(s2.w - s1.w * s1.w * inv, 0.f));
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

// One block per channel: Chan-merge the chunk partials, derive scale/shift, update running stats.
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float2* __restrict__ part, int nchunks, int M, int C,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ bias, float* __restrict__ rmean,
                                                          float* __restrict__ rvar, long long* __restrict__ nbt,
                                                          float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                          float* __restrict__ scale, float* __restrict__ shift,
                                                          float momentum, float eps) {
  const int c = blockIdx.x;
  Welford acc{0.f, 0.f, 0.f};
  for (int k = threadIdx.x; k < nchunks; k += 256) {
    const float2 p = part[(long)k * C + c];
    const int cnt = min(CHUNK, M - k * CHUNK);
    acc = merge(acc, Welford{(float)cnt, p.x, p.y});
  }
  __shared__ Welford sh[256];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] = merge(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const Welford w = sh[0];
    const float var = w.m2 / w.n;
    const float inv = rsqrtf(var + eps);
    const float g = gamma[c];
    mean_out[c] = w.mean;
    invstd_out[c] = inv;
    scale[c] = g * inv;
    shift[c] = beta[c] - w.mean * g * inv;
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

// a = relu(z*scale + shift), optionally 2x2/s2 max-pooled.  z: [N,H,W,C]  a: [N,H/2,W/2,C] or [N,H,W,C]
template <bool POOL>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ z, float* __restrict__ a,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int N, int H, int W, int C) {
  const int C4 = C >> 2;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const long total = (long)N * Ho * Wo * C4;
  const long stride = (long)gridDim.x * blockDim.x;
  const float4* z4 = reinterpret_cast<const float4*>(z);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c4 = (int)(i % C4);
    const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
    const float4 sh = reinterpret_cast<const float4*>(shift)[c4];
    if (!POOL) {
      reinterpret_cast<float4*>(a)[i] = affine_relu(z4[i], sc, sh);
    } else {
      long t = i / C4;
      const int ow = (int)(t % Wo);
      t /= Wo;
      const int oh = (int)(t % Ho);
      const int n = (int)(t / Ho);
      const long base = (((long)n * H + 2 * oh) * W + 2 * ow) * C4 + c4;
      const float4 v00 = affine_relu(z4[base], sc, sh);
      const float4 v01 = affine_relu(z4[base + C4], sc, sh);
      const float4 v10 = affine_relu(z4[base + (long)W * C4], sc, sh);
      const float4 v11 = affine_relu(z4[base + (long)W * C4 + C4], sc, sh);
      reinterpret_cast<float4*>(a)[i] =
          make_float4(fmaxf(fmaxf(v00.x, v01.x), fmaxf(v10.x, v11.x)), fmaxf(fmaxf(v00.y, v01.y), fmaxf(v10.y, v11.y)),
                      fmaxf(fmaxf(v00.z, v01.z), fmaxf(v10.z, v11.z)), fmaxf(fmaxf(v00.w, v01.w), fmaxf(v10.w, v11.w)));
    }
  }
}

// --- backward helpers: per scalar channel, route pooled grad to the first max, apply relu mask ---
// returns dy for the 4 window positions (00,01,10,11)
__device__ __forceinline__ void route1(float z00, float z01, float z10, float z11, float sc, float sh, float g,
                                       float& d00, float& d01, float& d10, float& d11) {
  const float y00 = fmaxf(fmaf(z00, sc, sh), 0.f), y01 = fmaxf(fmaf(z01, sc, sh), 0.f);
  const float y10 = fmaxf(fmaf(z10, sc, sh), 0.f), y11 = fmaxf(fmaf(z11, sc, sh), 0.f);
  int arg = 0;
  float mx = y00;
  if (y01 > mx) { mx = y01; arg = 1; }
  if (y10 > mx) { mx = y10; arg = 2; }
  if (y11 > mx) { mx = y11; arg = 3; }
  // relu backward: gradient passes where the relu output is > 0
  d00 = (arg == 0 && y00 > 0.f) ? g : 0.f;
  d01 = (arg == 1 && y01 > 0.f) ? g : 0.f;
  d10 = (arg == 2 && y10 > 0.f) ? g : 0.f;
  d11 = (arg == 3 && y11 > 0.f) ? g : 0.f;
}

#define F4GET(v, k) ((k) == 0 ? (v).x : (k) == 1 ? (v).y : (k) == 2 ? (v).z : (v).w)

// Reduce pass: per (row chunk, c4) sums of dy, dy*xhat, xhat.  For POOL, rows are pooled positions
// (each covers 4 full-resolution rows).  part layout: [chunk][3][C]
template <bool POOL>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ g, const float* __restrict__ z,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            float* __restrict__ part, int N, int H, int W, int C) {
  const int C4 = C >> 2;
  const int per_block = 256 / C4;
  const int t = threadIdx.x;
  if (t >= per_block * C4) return;
  const int c4 = t % C4;
  const int chunk = blockIdx.x * per_block + t / C4;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const int Mo = N * Ho * Wo;
  const int r0 = chunk * CHUNK;
  if (r0 >= Mo) return;
  const int r1 = min(Mo, r0 + CHUNK);
  const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
  const float4 sh = reinterpret_cast<const float4*>(shift)[c4];
  const float4 mu = reinterpret_cast<const float4*>(mean)[c4];
  const float4 is = reinterpret_cast<const float4*>(invstd)[c4];
  const float4* z4 = reinterpret_cast<const float4*>(z);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float sdy[4] = {0, 0, 0, 0}, sdx[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0};
  for (int r = r0; r < r1; ++r) {
    const float4 gv = g4[(long)r * C4 + c4];
    if (!POOL) {
      const float4 zv = z4[(long)r * C4 + c4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float zz = F4GET(zv, k);
        const float y = fmaf(zz, F4GET(sc, k), F4GET(sh, k));
        const float dy = y > 0.f ? F4GET(gv, k) : 0.f;
        const float xh = (zz - F4GET(mu, k)) * F4GET(is, k);
        sdy[k] += dy;
        sdx[k] += dy * xh;
        sx[k] += xh;
      }
    } else {
      const int ow = r % Wo;
      const int tt = r / Wo;
      const int oh = tt % Ho;
      const int n = tt / Ho;
      const long base = (((long)n * H + 2 * oh) * W + 2 * ow) * C4 + c4;
      const float4 z00 = z4[base], z01 = z4[base + C4], z10 = z4[base + (long)W * C4], z11 = z4[base + (long)W * C4 + C4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float d00, d01, d10, d11;
        route1(F4GET(z00, k), F4GET(z01, k), F4GET(z10, k), F4GET(z11, k), F4GET(sc, k), F4GET(sh, k), F4GET(gv, k),
               d00, d01, d10, d11);
        const float m = F4GET(mu, k), iv = F4GET(is, k);
        const float x00 = (F4GET(z00, k) - m) * iv, x01 = (F4GET(z01, k) - m) * iv;
        const float x10 = (F4GET(z10, k) - m) * iv, x11 = (F4GET(z11, k) - m) * iv;
        sdy[k] += (d00 + d01) + (d10 + d11);
        sdx[k] += (d00 * x00 + d01 * x01) + (d10 * x10 + d11 * x11);
        sx[k] += (x00 + x01) + (x10 + x11);
      }
    }
  }
  float* o = part + (long)chunk * 3 * C + c4 * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    o[k] = sdy[k];
    o[C + k] = sdx[k];
    o[2 * C + k] = sx[k];
  }
}

// Per channel: sum the chunk partials (fixed order -> deterministic), emit dgamma, dbeta, dbias and
// the dz coefficients: dz = k1*dy + k2*z + k3.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nchunks, int C,
                                                              float Mfull, const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ dbias, float* __restrict__ coef) {
  const int c = blockIdx.x;
  float a = 0.f, b = 0.f, x = 0.f;
  for (int k = threadIdx.x; k < nchunks; k += 256) {
    const float* p = part + (long)k * 3 * C + c;
    a += p[0];
    b += p[C];
    x += p[2 * C];
  }
  __shared__ float sh[3][256];
  sh[0][threadIdx.x] = a;
  sh[1][threadIdx.x] = b;
  sh[2][threadIdx.x] = x;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + o];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + o];
      sh[2][threadIdx.x] += sh[2][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float sdy = sh[0][0], sdx = sh[1][0], sx = sh[2][0];
    const float iv = invstd[c], g = gamma[c];
    const float k1 = g * iv;
    const float k2x = -k1 * sdx / Mfull;  // coefficient of xhat
    const float k3 = -k1 * sdy / Mfull;
    dgamma[c] = sdx;
    dbeta[c] = sdy;
    if (dbias) dbias[c] = k1 * (sdy - sdy) + k2x * sx;  // = sum over rows of dz
    coef[c] = k1;
    coef[C + c] = k2x * iv;                   // coefficient of z
    coef[2 * C + c] = k3 - k2x * iv * mean[c];  // constant
  }
}

template <bool POOL>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ g, const float* __restrict__ z,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ coef, float* __restrict__ dz,
                                                           int N, int H, int W, int C) {
  const int C4 = C >> 2;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const long total = (long)N * Ho * Wo * C4;
  const long stride = (long)gridDim.x * blockDim.x;
  const float4* z4 = reinterpret_cast<const float4*>(z);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* o4 = reinterpret_cast<float4*>(dz);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c4 = (int)(i % C4);
    const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
    const float4 sh = reinterpret_cast<const float4*>(shift)[c4];
    const float4 k1 = reinterpret_cast<const float4*>(coef)[c4];
    const float4 k2 = reinterpret_cast<const float4*>(coef + C)[c4];
    const float4 k3 = reinterpret_cast<const float4*>(coef + 2 * C)[c4];
    const float4 gv = g4[i];
    if (!POOL) {
      const float4 zv = z4[i];
      float r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float zz = F4GET(zv, k);
        const float dy = fmaf(zz, F4GET(sc, k), F4GET(sh, k)) > 0.f ? F4GET(gv, k) : 0.f;
        r[k] = F4GET(k1, k) * dy + F4GET(k2, k) * zz + F4GET(k3, k);
      }
      o4[i] = make_float4(r[0], r[1], r[2], r[3]);
    } else {
      long t = i / C4;
      const int ow = (int)(t % Wo);
      t /= Wo;
      const int oh = (int)(t % Ho);
      const int n = (int)(t / Ho);
      const long base = (((long)n * H + 2 * oh) * W + 2 * ow) * C4 + c4;
      const long idx[4] = {base, base + C4, base + (long)W * C4, base + (long)W * C4 + C4};
      float4 zq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) zq[q] = z4[idx[q]];
      float out[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float d[4];
        route1(F4GET(zq[0], k), F4GET(zq[1], k), F4GET(zq[2], k), F4GET(zq[3], k), F4GET(sc, k), F4GET(sh, k),
               F4GET(gv, k), d[0], d[1], d[2], d[3]);
#pragma unroll
        for (int q = 0; q < 4; ++q) out[q][k] = F4GET(k1, k) * d[q] + F4GET(k2, k) * F4GET(zq[q], k) + F4GET(k3, k);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) o4[idx[q]] = make_float4(out[q][0], out[q][1], out[q][2], out[q][3]);
    }
  }
}

int grid_1d(long n) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

int dpa_bn_nchunks(int M) { return (M + CHUNK - 1) / CHUNK; }

// z [M][C] -> partials [nchunks][C] float2 -> finalize
int dpa_bn_fwd_stats(const float* z, float* part, int M, int C, const float* gamma, const float* beta,
                     const float* bias, float* rmean, float* rvar, long long* nbt, float* mean, float* invstd,
                     float* scale, float* shift, float momentum, float eps, hipStream_t st) {
  if (C % 4 || (256 % (C / 4)) != 0) return -2;
  const int nchunks = (M + CHUNK - 1) / CHUNK;
  const int per_block = 256 / (C / 4);
  bn_stats_kernel<<<cdiv(nchunks, per_block), 256, 0, st>>>(z, reinterpret_cast<float2*>(part), M, C);
  bn_finalize_kernel<<<C, 256, 0, st>>>(reinterpret_cast<const float2*>(part), nchunks, M, C, gamma, beta, bias, rmean,
                                        rvar, nbt, mean, invstd, scale, shift, momentum, eps);
  return (int)hipGetLastError();
}

int dpa_bn_eval_params(const float* gamma, const float* beta, const float* bias, const float* rmean,
                       const float* rvar, float* scale, float* shift, int C, float eps, hipStream_t st) {
  bn_eval_params_kernel<<<cdiv(C, 256), 256, 0, st>>>(gamma, beta, bias, rmean, rvar, scale, shift, C, eps);
  return (int)hipGetLastError();
}

int dpa_bn_apply(const float* z, float* a, const float* scale, const float* shift, int N, int H, int W, int C,
                 int pool, hipStream_t st) {
  if (C % 4) return -2;
  const long total = (long)N * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 4);
  if (pool)
    bn_apply_kernel<true><<<grid_1d(total), 256, 0, st>>>(z, a, scale, shift, N, H, W, C);
  else
    bn_apply_kernel<false><<<grid_1d(total), 256, 0, st>>>(z, a, scale, shift, N, H, W, C);
  return (int)hipGetLastError();
}

// g: grad of the layer output (pooled shape if pool).  Writes dz [N,H,W,C] and dgamma/dbeta/dbias.
int dpa_bn_bwd(const float* g, const float* z, const float* scale, const float* shift, const float* mean,
               const float* invstd, const float* gamma, float* part, float* coef, float* dgamma, float* dbeta,
               float* dbias, float* dz, int N, int H, int W, int C, int pool, hipStream_t st) {
  if (C % 4 || (256 % (C / 4)) != 0) return -2;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const int Mo = N * Ho * Wo;
  const int nchunks = (Mo + CHUNK - 1) / CHUNK;
  const int per_block = 256 / (C / 4);
  if (pool)
    bn_bwd_reduce_kernel<true><<<cdiv(nchunks, per_block), 256, 0, st>>>(g, z, scale, shift, mean, invstd, part, N, H,
                                                                        W, C);
  else
    bn_bwd_reduce_kernel<false><<<cdiv(nchunks, per_block), 256, 0, st>>>(g, z, scale, shift, mean, invstd, part, N,
                                                                         H, W, C);
  bn_bwd_finalize_kernel<<<C, 256, 0, st>>>(part, nchunks, C, (float)N * H * W, gamma, mean, invstd, dgamma, dbeta,
                                            dbias, coef);
  const long total = (long)Mo * (C / 4);
  if (pool)
    bn_bwd_apply_kernel<true><<<grid_1d(total), 256, 0, st>>>(g, z, scale, shift, coef, dz, N, H, W, C);
  else
    bn_bwd_apply_kernel<false><<<grid_1d(total), 256, 0, st>>>(g, z, scale, shift, coef, dz, N, H, W, C);
  return (int)hipGetLastError();
}

}  // extern "C"
