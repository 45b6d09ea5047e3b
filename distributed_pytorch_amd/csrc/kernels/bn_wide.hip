// K5/K6 for bf16 activations, 16 bytes per lane: the BatchNorm apply passes of the generic bf16
// path (ResNet-50, BASELINE.json stress config; BN + ReLU / + residual + ReLU, and the backward
// apply dz = k1*dy + k2*z + k3 with dy through the ReLU mask), one 8-channel group (one uint4 of
// bf16) per lane and row instead of bn.hip's 4-channel ushort4 groups.  bn.hip's kernels move 8
// bytes per lane per tensor and stream the ResNet-50 tensors at 3.2-3.8 TB/s
// (profiles/r3_resnet50_pmc_traffic.txt); the same passes with 16-byte lanes issue half the memory
// instructions for the same bytes.  Arithmetic per element is bn.hip's (bn_apply_kernel /
// bn_bwd_apply_kernel, same fma order), so results are bitwise identical (GPU test).
//
// Grid: a grid stride that is a multiple of C/8 keeps each thread on one channel group (its
// coefficients loaded once); four (forward) or two (backward) rows' loads in flight per thread.
#include "common.h"

namespace {

__device__ __forceinline__ void unpack8(uint4 v, float (&f)[8]) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = __uint_as_float(w[q] << 16);
    f[2 * q + 1] = __uint_as_float(w[q] & 0xFFFF0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  unsigned w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = (unsigned)bf16_rne(f[2 * q]) | ((unsigned)bf16_rne(f[2 * q + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void coef8(const float* p, int c8, float (&f)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[2 * c8], b = reinterpret_cast<const float4*>(p)[2 * c8 + 1];
  f[0] = a.x, f[1] = a.y, f[2] = a.z, f[3] = a.w, f[4] = b.x, f[5] = b.y, f[6] = b.z, f[7] = b.w;
}

constexpr int UNR = 4;

// forward: ACT 0 relu(fma(z, sc, sh)); 1 fma(z, sc, sh); 2 relu(fma(z, sc, sh) + res) (+ ReLU mask,
// one byte per 4 channels: bit k = channel 4*i + k of that group passed the ReLU)
// RBN (ACT 2): res is itself a BatchNorm input (the downsample branch's conv output); it is mapped
// to fma(res, rscale, rshift) rounded to bf16 -- the value that BN's own apply pass (ACT 1) would
// have stored -- so that pass and its output tensor go.
template <int ACT, bool RBN = false>
__global__ __launch_bounds__(256) void bn_apply_wide_kernel(const uint4* __restrict__ z, const uint4* __restrict__ res,
                                                            uint4* __restrict__ out, unsigned short* __restrict__ mask,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, long total8, int C8,
                                                            const float* __restrict__ rscale = nullptr,
                                                            const float* __restrict__ rshift = nullptr) {
  const long stride = (long)gridDim.x * blockDim.x;
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = (int)(i0 % C8);
  float sc[8], sh[8], rsc[8], rsh[8];
  coef8(scale, c8, sc);
  coef8(shift, c8, sh);
  if constexpr (RBN) {
    coef8(rscale, c8, rsc);
    coef8(rshift, c8, rsh);
  }
  auto body = [&](uint4 zv, uint4 rv, long i) {
    float zf[8], rf[8], o[8];
    unpack8(zv, zf);
    if constexpr (ACT == 2) unpack8(rv, rf);
    if constexpr (RBN) {
#pragma unroll
      for (int e = 0; e < 8; ++e) rf[e] = __uint_as_float((unsigned)bf16_rne(fmaf(rf[e], rsc[e], rsh[e])) << 16);
    }
    unsigned m = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float u = fmaf(zf[e], sc[e], sh[e]);
      if constexpr (ACT == 0) {
        o[e] = fmaxf(u, 0.f);
      } else if constexpr (ACT == 1) {
        o[e] = u;
      } else {
        const float t = u + rf[e];
        m |= (t > 0.f ? 1u : 0u) << e;
        o[e] = fmaxf(t, 0.f);
      }
    }
    out[i] = pack8(o);
    // bytes 2i, 2i+1 = bn.hip's mask bytes of channel groups 2i, 2i+1 (bit k: channel k of the group)
    if (ACT == 2 && mask) mask[i] = (unsigned short)((m & 0xFu) | ((m >> 4) << 8));
  };
  long i = i0;
  for (; i + (UNR - 1) * stride < total8; i += UNR * stride) {
    uint4 zv[UNR], rv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      zv[u] = z[i + u * stride];
      rv[u] = ACT == 2 ? res[i + u * stride] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) body(zv[u], rv[u], i + u * stride);
  }
  for (; i < total8; i += stride) body(z[i], ACT == 2 ? res[i] : make_uint4(0u, 0u, 0u, 0u), i);
}

// backward apply: dy = g (+ g2) through the ReLU mask recomputed from z (ACT 0) or as is (ACT 1);
// dz = fma(k1, dy, fma(k2, z - mu, k3)) (the centred coefficients of bn.hip bwd_coef)
template <int ACT>
__global__ __launch_bounds__(256) void bn_bwd_apply_wide_kernel(const uint4* __restrict__ g, const uint4* __restrict__ g2,
                                                                const uint4* __restrict__ z, uint4* __restrict__ dz,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift,
                                                                const float* __restrict__ coef, long total8, int C8) {
  const long stride = (long)gridDim.x * blockDim.x;
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = (int)(i0 % C8);
  const int C = 8 * C8;
  float sc[8], sh[8], k1[8], k2[8], k3[8], mu[8];
  coef8(scale, c8, sc);
  coef8(shift, c8, sh);
  coef8(coef, c8, k1);
  coef8(coef + C, c8, k2);
  coef8(coef + 2 * C, c8, k3);
  coef8(coef + 3 * C, c8, mu);
  auto body = [&](uint4 gv, uint4 g2v, uint4 zv, long i) {
    float gf[8], zf[8], o[8];
    unpack8(gv, gf);
    unpack8(zv, zf);
    if (g2) {
      float hf[8];
      unpack8(g2v, hf);
#pragma unroll
      for (int e = 0; e < 8; ++e) gf[e] += hf[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dy = ACT == 0 ? (fmaf(zf[e], sc[e], sh[e]) > 0.f ? gf[e] : 0.f) : gf[e];
      o[e] = fmaf(k1[e], dy, fmaf(k2[e], zf[e] - mu[e], k3[e]));
    }
    dz[i] = pack8(o);
  };
  // two rows in flight per thread (40 coefficient registers: four rows' operands would spill)
  constexpr int U = 2;
  long i = i0;
  for (; i + (U - 1) * stride < total8; i += U * stride) {
    uint4 gv[U], hv[U], zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      gv[u] = g[i + u * stride];
      hv[u] = g2 ? g2[i + u * stride] : make_uint4(0u, 0u, 0u, 0u);
      zv[u] = z[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(gv[u], hv[u], zv[u], i + u * stride);
  }
  for (; i < total8; i += stride) body(g[i], g2 ? g2[i] : make_uint4(0u, 0u, 0u, 0u), z[i], i);
}

// Backward reduce (bn.hip bn_bwd_reduce_kernel's 1024-thread geometry, bf16, unpooled, unsplit):
// per (row block, channel) sums of dy, dy*xhat and xhat, with dy = g (+ g2) through the ReLU of
// ACT 0, as is (ACT 1), or through the add+ReLU of ACT 2 (mask from the forward, or the residual),
// dy stored to dyout for ACT 2 (the residual's gradient).  C/8 threads per row, 1024/(C/8) rows per
// iteration, U = 2 rows' loads in flight (4 measured no faster); rows summed in order, then the
// fixed-order LDS tree (the row partition differs from bn.hip's, so sums agree to rounding, not
// bitwise).  part: [block][3][C] as bn.hip's, finalized by the same kernel.
constexpr int RTW = 1024;

__device__ __forceinline__ float4 f4sum(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int ACT, bool MK, int U = 2>
__global__ __launch_bounds__(RTW) void bn_bwd_reduce_wide_kernel(
    const uint4* __restrict__ g, const uint4* __restrict__ g2, const uint4* __restrict__ z,
    const uint4* __restrict__ res, const unsigned short* __restrict__ mask, uint4* __restrict__ dyout,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, float* __restrict__ part, int Mo, int C8, int rpb, int* sig, int sig_val) {
  start_signal(sig, sig_val);
  const int t = threadIdx.x;
  const int RPI = RTW / C8;
  const int lane_c = t % C8, lane_r = t / C8;
  const bool active = lane_r < RPI;
  const int r0 = blockIdx.x * rpb, r1 = min(Mo, r0 + rpb);
  float sdy[8] = {}, sdx[8] = {}, sx[8] = {};
  if (active) {
    float sc[8], sh[8], mu[8], is[8];
    coef8(scale, lane_c, sc);
    coef8(shift, lane_c, sh);
    coef8(mean, lane_c, mu);
    coef8(invstd, lane_c, is);
    constexpr bool mk = ACT == 2 && MK;  // ReLU mask of the forward (else the residual)
    auto row = [&](uint4 gv, uint4 hv, uint4 zv, uint4 rv, unsigned m, long gi) {
      float gf[8], zf[8], rf[8], dyv[8];
      unpack8(gv, gf);
      unpack8(zv, zf);
      if (g2) {
        float hf[8];
        unpack8(hv, hf);
#pragma unroll
        for (int e = 0; e < 8; ++e) gf[e] += hf[e];
      }
      if (ACT == 2 && !mk) unpack8(rv, rf);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float dy;
        if (ACT == 2 && mk) {
          dy = ((m >> (e < 4 ? e : e + 4)) & 1u) ? gf[e] : 0.f;
        } else {
          const float u = fmaf(zf[e], sc[e], sh[e]);
          dy = ACT == 0 ? (u > 0.f ? gf[e] : 0.f) : ACT == 1 ? gf[e] : ((u + rf[e]) > 0.f ? gf[e] : 0.f);
        }
        const float xh = (zf[e] - mu[e]) * is[e];
        sdy[e] += dy;
        sdx[e] = fmaf(dy, xh, sdx[e]);
        sx[e] += xh;
        dyv[e] = dy;
      }
      if (ACT == 2 && dyout) dyout[gi] = pack8(dyv);
    };
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    int r = r0 + lane_r;
    // U rows' loads in flight per thread (rows still summed in ascending order: any U, same sums)
    for (; r + (U - 1) * RPI < r1; r += U * RPI) {
      uint4 gv[U], hv[U], zv[U], rv[U];
      unsigned mv[U];
      long iv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        iv[u] = (long)(r + u * RPI) * C8 + lane_c;
        gv[u] = g[iv[u]];
        hv[u] = g2 ? g2[iv[u]] : zero;
        zv[u] = z[iv[u]];
        rv[u] = ACT == 2 && !mk ? res[iv[u]] : zero;
        mv[u] = mk ? mask[iv[u]] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) row(gv[u], hv[u], zv[u], rv[u], mv[u], iv[u]);
    }
    for (; r < r1; r += RPI) {
      const long i0 = (long)r * C8 + lane_c;
      row(g[i0], g2 ? g2[i0] : zero, z[i0], ACT == 2 && !mk ? res[i0] : zero, mk ? mask[i0] : 0u, i0);
    }
  }
  __shared__ float4 shb[RTW];
  float* o = part + (long)blockIdx.x * 3 * (8 * C8) + lane_c * 8;
  const int C = 8 * C8;
  int p2 = 1;
  while (p2 < RPI) p2 <<= 1;
#pragma unroll
  for (int q = 0; q < 6; ++q) {  // (sum dy, sum dy*xhat, sum xhat) x (channels 0-3, 4-7 of the group)
    const float* v = q < 2 ? sdy : q < 4 ? sdx : sx;
    const int h = (q & 1) * 4;
    shb[t] = make_float4(v[h], v[h + 1], v[h + 2], v[h + 3]);
    __syncthreads();
    for (int off = p2 >> 1; off >= 1; off >>= 1) {
      if (active && lane_r < off && lane_r + off < RPI) shb[t] = f4sum(shb[t], shb[t + off * C8]);
      __syncthreads();
    }
    if (active && lane_r == 0) *reinterpret_cast<float4*>(o + (q >> 1) * C + h) = shb[t];
    __syncthreads();
  }
}

// grid: <= 8192 blocks of 256 threads, the stride a multiple of C8 (one channel group per thread)
int grid_wide(long total8, int C8) {
  long g = (total8 + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (g * 256 < total8) {
    // round the thread count to a multiple of C8
    const long threads = g * 256 / C8 * C8;
    g = threads / 256;
    while (g > 1 && (g * 256) % C8) --g;
    if ((g * 256) % C8) return -1;
  }
  return (int)g;
}

bool wide_on() {
  const char* e = getenv("DPA_BN_WIDE");  // read per call: tests switch it in-process
  return !(e && e[0] == '0');
}

bool wide_red_on() {
  const char* e = getenv("DPA_BN_WIDE_RED");  // read per call: tests switch it in-process
  return wide_on() && !(e && e[0] == '0');
}

}  // namespace

extern "C" {
// Backward reduce for bf16, unpooled, unsplit tensors in bn.hip's 1024-thread geometry: rpb is
// bn.hip's rows per block (rounded up here to whole iterations, so the grid never exceeds its and
// the partial workspace fits).  Returns the number of blocks launched (the finalize's partial
// rows), 0 when not applicable (the caller runs bn.hip's kernel), or -(HIP error).
int dpa_bn_bwd_reduce_wide(const unsigned short* g, const unsigned short* g2, const unsigned short* z,
                           const unsigned short* res, const unsigned char* mask, unsigned short* dyout,
                           const float* scale, const float* shift, const float* mean, const float* invstd,
                           float* part, int Mo, int C, int act, int rpb, int* sig, int sig_val, hipStream_t st) {
  if (!wide_red_on() || C % 8 || C / 8 > RTW || act < 0 || act > 2 || (act == 2 && !mask && !res)) return 0;
  if ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(g2) | reinterpret_cast<uintptr_t>(z) |
       reinterpret_cast<uintptr_t>(res) | reinterpret_cast<uintptr_t>(dyout)) & 15 ||
      reinterpret_cast<uintptr_t>(mask) & 1)
    return 0;
  const int C8 = C / 8, RPI = RTW / C8;
  const int rw = (rpb + RPI - 1) / RPI * RPI;
  const int nblk = (Mo + rw - 1) / rw;
  const uint4 *gg = reinterpret_cast<const uint4*>(g), *hh = reinterpret_cast<const uint4*>(g2),
              *zz = reinterpret_cast<const uint4*>(z), *rr = reinterpret_cast<const uint4*>(res);
  const unsigned short* mm = reinterpret_cast<const unsigned short*>(mask);
  uint4* dd = reinterpret_cast<uint4*>(dyout);
#define LAUNCH(A, M)                                                                                               \
  bn_bwd_reduce_wide_kernel<A, M><<<nblk, RTW, 0, st>>>(gg, hh, zz, rr, mm, dd, scale, shift, mean, invstd, part, Mo, \
                                                     C8, rw, sig, sig_val)
  if (act == 0) LAUNCH(0, false);
  else if (act == 1) LAUNCH(1, false);
  else if (mask) LAUNCH(2, true);
  else LAUNCH(2, false);
#undef LAUNCH
  const int e = (int)hipGetLastError();
  return e ? -e : nblk;
}

// bf16 [M][C] -> bf16 [M][C] (+ mask [M*C/4] bytes for act 2); returns 1 when not applicable (the
// caller runs bn.hip's kernel), else a HIP error code.  rscale / rshift (act 2 only): the residual is a
// BatchNorm input, added as bf16(fma(res, rscale, rshift)) (bn_apply_wide_kernel RBN).
int dpa_bn_apply_wide(const unsigned short* z, const unsigned short* res, unsigned short* out, unsigned char* mask,
                      const float* scale, const float* shift, long M, int C, int act, hipStream_t st,
                      const float* rscale, const float* rshift) {
  if ((rscale != nullptr) != (rshift != nullptr) || (rscale && act != 2)) return -2;
  if (!wide_on() || C % 8 || act < 0 || act > 2 || (act == 2 && !res)) return 1;
  if ((reinterpret_cast<uintptr_t>(z) | reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(res)) & 15 ||
      reinterpret_cast<uintptr_t>(mask) & 1)  // the mask is stored as 2-byte words
    return 1;
  const long total8 = M * (C / 8);
  const int grid = grid_wide(total8, C / 8);
  if (grid < 0) return 1;
  const uint4 *zz = reinterpret_cast<const uint4*>(z), *rr = reinterpret_cast<const uint4*>(res);
  uint4* oo = reinterpret_cast<uint4*>(out);
  unsigned short* mm = reinterpret_cast<unsigned short*>(mask);
  if (act == 0)
    bn_apply_wide_kernel<0><<<grid, 256, 0, st>>>(zz, rr, oo, mm, scale, shift, total8, C / 8);
  else if (act == 1)
    bn_apply_wide_kernel<1><<<grid, 256, 0, st>>>(zz, rr, oo, mm, scale, shift, total8, C / 8);
  else if (rscale)
    bn_apply_wide_kernel<2, true><<<grid, 256, 0, st>>>(zz, rr, oo, mm, scale, shift, total8, C / 8, rscale, rshift);
  else
    bn_apply_wide_kernel<2><<<grid, 256, 0, st>>>(zz, rr, oo, mm, scale, shift, total8, C / 8);
  return (int)hipGetLastError();
}

// backward apply, bf16: g (+ g2) and z [M][C] -> dz [M][C]; act 0 (ReLU) or 1 (identity); returns 1
// when not applicable
int dpa_bn_bwd_apply_wide(const unsigned short* g, const unsigned short* g2, const unsigned short* z,
                          unsigned short* dz, const float* scale, const float* shift, const float* coef, long M, int C,
                          int act, hipStream_t st) {
  if (!wide_on() || C % 8 || (act != 0 && act != 1)) return 1;
  if ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(g2) | reinterpret_cast<uintptr_t>(z) |
       reinterpret_cast<uintptr_t>(dz)) & 15)
    return 1;
  const long total8 = M * (C / 8);
  const int grid = grid_wide(total8, C / 8);
  if (grid < 0) return 1;
  const uint4 *gg = reinterpret_cast<const uint4*>(g), *hh = reinterpret_cast<const uint4*>(g2),
              *zz = reinterpret_cast<const uint4*>(z);
  uint4* oo = reinterpret_cast<uint4*>(dz);
  if (act == 0)
    bn_bwd_apply_wide_kernel<0><<<grid, 256, 0, st>>>(gg, hh, zz, oo, scale, shift, coef, total8, C / 8);
  else
    bn_bwd_apply_wide_kernel<1><<<grid, 256, 0, st>>>(gg, hh, zz, oo, scale, shift, coef, total8, C / 8);
  return (int)hipGetLastError();
}
}  // extern "C"
