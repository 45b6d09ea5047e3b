// NHWC max-pool (k x k, stride s, pad p) forward / backward for the generic path (ResNet stem
// 3x3/s2/p1 on [N,112,112,64] bf16).  Replaces max_pool2d_with_indices and its backward, which in
// the ResNet-50 step cost 130 + 310 us as torch's channels_last kernels.
//
// Forward: one thread per (output pixel, 8 channels): 16-B bf16 (or 2x16-B fp32) loads per window
// tap, running max and the first-max window position (scan order kh, kw; strict '>' keeps the
// first, as torch does) stored as one byte per element.
// Backward: a GATHER over the input, one thread per (input pixel, 8 channels): every output window
// containing the pixel is visited and its gradient added when the stored position points back at
// this pixel.  Each input element is written exactly once: no atomics, no zero-fill pass, and the
// summation order is fixed (deterministic).
#include "common.h"

namespace {

template <typename T>
struct V8 {};
template <>
struct V8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};
template <>
struct V8<u16> {
  static __device__ __forceinline__ void load(const u16* p, float (&v)[8]) {
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = bf16_f((u16)(w[k] & 0xFFFFu));
      v[2 * k + 1] = bf16_f((u16)(w[k] >> 16));
    }
  }
  static __device__ __forceinline__ void store(u16* p, const float (&v)[8]) {
    uint4 q;
    q.x = bf16_rne(v[0]) | ((unsigned)bf16_rne(v[1]) << 16);
    q.y = bf16_rne(v[2]) | ((unsigned)bf16_rne(v[3]) << 16);
    q.z = bf16_rne(v[4]) | ((unsigned)bf16_rne(v[5]) << 16);
    q.w = bf16_rne(v[6]) | ((unsigned)bf16_rne(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = q;
  }
};

struct PoolGeom {
  int N, H, W, C8, P, Q, k, s, p;
};

// BN (BatchNorm + ReLU on load, `bn`): x is the BN input z and every window element is first mapped
// to relu(z * scale + shift), rounded to T as bn_apply stores it -- the same max and positions as
// pooling bn_apply's output, without writing or re-reading that tensor (the ResNet stem).
template <typename T, typename IT, bool BN = false>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          unsigned char* __restrict__ arg, PoolGeom g,
                                                          const float* __restrict__ scale = nullptr,
                                                          const float* __restrict__ shift = nullptr) {
  // IT: 32-bit index arithmetic when the element count allows (64-bit divisions dominated the
  // kernel: 2.5 TB/s on the ResNet-50 stem)
  const IT total = (IT)g.N * g.P * g.Q * g.C8;
  for (IT i = (IT)blockIdx.x * 256u + threadIdx.x; i < total; i += (IT)gridDim.x * 256u) {
    const int c8 = (int)(i % (IT)g.C8);
    IT r = i / (IT)g.C8;
    const int ow = (int)(r % (IT)g.Q);
    r /= (IT)g.Q;
    const int oh = (int)(r % (IT)g.P);
    const int n = (int)(r / (IT)g.P);
    float m[8], sc[8], sh[8];
    unsigned char a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m[k] = -INFINITY;
      a[k] = 0;
    }
    if constexpr (BN) {
      V8<float>::load(scale + c8 * 8, sc);
      V8<float>::load(shift + c8 * 8, sh);
    }
    bool first = true;  // the first in-image tap initialises (pad < k: every window has one)
    for (int kh = 0; kh < g.k; ++kh) {
      const int h = oh * g.s - g.p + kh;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int w = ow * g.s - g.p + kw;
        if ((unsigned)w >= (unsigned)g.W) continue;
        float v[8];
        V8<T>::load(x + (((long)n * g.H + h) * g.W + w) * (g.C8 * 8) + c8 * 8, v);
        if constexpr (BN) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float u = fmaxf(fmaf(v[k], sc[k], sh[k]), 0.f);
            v[k] = sizeof(T) == 2 ? bf16_f(bf16_rne(u)) : u;
          }
        }
        const unsigned char pos = (unsigned char)(kh * g.k + kw);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (first || v[k] > m[k]) {
            m[k] = v[k];
            a[k] = pos;
          }
        first = false;
      }
    }
    V8<T>::store(y + (long)i * 8, m);
    uint2 packed;
    packed.x = a[0] | (a[1] << 8) | (a[2] << 16) | ((unsigned)a[3] << 24);
    packed.y = a[4] | (a[5] << 8) | (a[6] << 16) | ((unsigned)a[7] << 24);
    *reinterpret_cast<uint2*>(arg + (long)i * 8) = packed;
  }
}

template <typename T, typename IT>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                          const unsigned char* __restrict__ arg,
                                                          T* __restrict__ dx, PoolGeom g) {
  const IT total = (IT)g.N * g.H * g.W * g.C8;
  for (IT i = (IT)blockIdx.x * 256u + threadIdx.x; i < total; i += (IT)gridDim.x * 256u) {
    const int c8 = (int)(i % (IT)g.C8);
    IT r = i / (IT)g.C8;
    const int w = (int)(r % (IT)g.W);
    r /= (IT)g.W;
    const int h = (int)(r % (IT)g.H);
    const int n = (int)(r / (IT)g.H);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    // output rows oh with oh*s - p <= h <= oh*s - p + k - 1
    const int hp = h + g.p, wp = w + g.p;
    const int oh0 = hp >= g.k ? (hp - g.k) / g.s + 1 : 0, oh1 = min(g.P - 1, hp / g.s);
    const int ow0 = wp >= g.k ? (wp - g.k) / g.s + 1 : 0, ow1 = min(g.Q - 1, wp / g.s);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = hp - oh * g.s;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = wp - ow * g.s;
        const unsigned char pos = (unsigned char)(kh * g.k + kw);
        const long o = (((long)n * g.P + oh) * g.Q + ow) * g.C8 + c8;
        const uint2 packed = *reinterpret_cast<const uint2*>(arg + o * 8);
        float v[8];
        V8<T>::load(dy + o * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const unsigned char ak = (unsigned char)(((k < 4 ? packed.x : packed.y) >> (8 * (k & 3))) & 0xFFu);
          if (ak == pos) acc[k] += v[k];
        }
      }
    }
    V8<T>::store(dx + (long)i * 8, acc);
  }
}

// 3x3 / stride 2 / pad 1 backward (the ResNet stem), one thread per 2x2 input block x 8 channels: the
// block's pixels are covered by exactly the windows (m..m+1, n..n+1); each window's dy and positions
// are loaded once for the four pixels (the general gather loads them once per covered pixel, 2.25x
// on average).  Per pixel, windows are summed in the general kernel's ascending (oh, ow) order:
// bitwise its result.
template <typename T, typename IT>
__global__ __launch_bounds__(256) void maxpool_bwd_k3s2_kernel(const T* __restrict__ dy,
                                                               const unsigned char* __restrict__ arg,
                                                               T* __restrict__ dx, PoolGeom g) {
  const int Hb = (g.H + 1) / 2, Wb = (g.W + 1) / 2;
  const IT total = (IT)g.N * Hb * Wb * g.C8;
  for (IT i = (IT)blockIdx.x * 256u + threadIdx.x; i < total; i += (IT)gridDim.x * 256u) {
    const int c8 = (int)(i % (IT)g.C8);
    IT r = i / (IT)g.C8;
    const int bn = (int)(r % (IT)Wb);
    r /= (IT)Wb;
    const int bm = (int)(r % (IT)Hb);
    const int n = (int)(r / (IT)Hb);
    float v[2][2][8];
    unsigned char a[2][2][8];
#pragma unroll
    for (int wi = 0; wi < 2; ++wi)
#pragma unroll
      for (int wj = 0; wj < 2; ++wj) {
        const int oh = bm + wi, ow = bn + wj;
        const bool ok = oh < g.P && ow < g.Q;
        const long o = (((long)n * g.P + (ok ? oh : 0)) * g.Q + (ok ? ow : 0)) * g.C8 + c8;
        if (ok) {
          V8<T>::load(dy + o * 8, v[wi][wj]);
          const uint2 packed = *reinterpret_cast<const uint2*>(arg + o * 8);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            a[wi][wj][k] = (unsigned char)(((k < 4 ? packed.x : packed.y) >> (8 * (k & 3))) & 0xFFu);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            v[wi][wj][k] = 0.f;
            a[wi][wj][k] = 0xFF;  // matches no window position
          }
        }
      }
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int h = 2 * bm + dh, w = 2 * bn + dw;
        if (h >= g.H || w >= g.W) continue;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
        for (int wi = 0; wi < 2; ++wi)
#pragma unroll
          for (int wj = 0; wj < 2; ++wj) {
            const int kh = h - 2 * (bm + wi) + 1, kw = w - 2 * (bn + wj) + 1;  // position in window
            if (kh < 0 || kh > 2 || kw < 0 || kw > 2) continue;
            const unsigned char pos = (unsigned char)(kh * 3 + kw);
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if (a[wi][wj][k] == pos) acc[k] += v[wi][wj][k];
          }
        V8<T>::store(dx + (((long)n * g.H + h) * g.W + w) * (g.C8 * 8) + c8 * 8, acc);
      }
  }
}

bool k3s2_on() {
  const char* e = getenv("DPA_POOL_K3S2");  // read per call: tests switch it in-process
  return !(e && e[0] == '0');
}

int grid_for(long n) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

// x [N,H,W,C] (C % 8 == 0) fp32 (bf=0) or bf16 (bf=1) -> y [N,P,Q,C], arg uint8 [N,P,Q,C].
// scale / shift (both or neither, [C] fp32): x is a BatchNorm input, pooled as relu(x*scale + shift).
int dpa_maxpool_fwd(const void* x, void* y, unsigned char* arg, int N, int H, int W, int C, int k, int s, int p,
                    int bf, hipStream_t st, const float* scale, const float* shift) {
  if (C % 8 || k < 1 || k * k > 255 || s < 1 || p < 0 || p >= k || (scale == nullptr) != (shift == nullptr))
    return -2;
  PoolGeom g{N, H, W, C / 8, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  const long total = (long)g.N * g.P * g.Q * g.C8;
  const bool small = total + 8192L * 256 < (1L << 32);  // (the strided index stays below 2^32)
  const int grid = grid_for(total);
#define POOL_FWD(T, IT)                                                                                   \
  do {                                                                                                    \
    if (scale)                                                                                            \
      maxpool_fwd_kernel<T, IT, true><<<grid, 256, 0, st>>>((const T*)x, (T*)y, arg, g, scale, shift);    \
    else                                                                                                  \
      maxpool_fwd_kernel<T, IT><<<grid, 256, 0, st>>>((const T*)x, (T*)y, arg, g);                        \
  } while (0)
  if (bf && small) POOL_FWD(u16, unsigned);
  else if (bf) POOL_FWD(u16, unsigned long);
  else if (small) POOL_FWD(float, unsigned);
  else POOL_FWD(float, unsigned long);
#undef POOL_FWD
  return (int)hipGetLastError();
}

// dy [N,P,Q,C], arg from the forward -> dx [N,H,W,C] (every element written)
int dpa_maxpool_bwd(const void* dy, const unsigned char* arg, void* dx, int N, int H, int W, int C, int k, int s,
                    int p, int bf, hipStream_t st) {
  if (C % 8 || k < 1 || k * k > 255 || s < 1 || p < 0 || p >= k) return -2;
  PoolGeom g{N, H, W, C / 8, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  const long total = (long)g.N * g.H * g.W * g.C8;
  const bool small = total + 8192L * 256 < (1L << 32);
  if (k == 3 && s == 2 && p == 1 && k3s2_on()) {
    const long tb = (long)g.N * ((H + 1) / 2) * ((W + 1) / 2) * g.C8;
    if (bf && small)
      maxpool_bwd_k3s2_kernel<u16, unsigned><<<grid_for(tb), 256, 0, st>>>((const u16*)dy, arg, (u16*)dx, g);
    else if (bf)
      maxpool_bwd_k3s2_kernel<u16, unsigned long><<<grid_for(tb), 256, 0, st>>>((const u16*)dy, arg, (u16*)dx, g);
    else if (small)
      maxpool_bwd_k3s2_kernel<float, unsigned><<<grid_for(tb), 256, 0, st>>>((const float*)dy, arg, (float*)dx, g);
    else
      maxpool_bwd_k3s2_kernel<float, unsigned long><<<grid_for(tb), 256, 0, st>>>((const float*)dy, arg, (float*)dx,
                                                                                   g);
    return (int)hipGetLastError();
  }
  if (bf && small)
    maxpool_bwd_kernel<u16, unsigned><<<grid_for(total), 256, 0, st>>>((const u16*)dy, arg, (u16*)dx, g);
  else if (bf)
    maxpool_bwd_kernel<u16, unsigned long><<<grid_for(total), 256, 0, st>>>((const u16*)dy, arg, (u16*)dx, g);
  else if (small)
    maxpool_bwd_kernel<float, unsigned><<<grid_for(total), 256, 0, st>>>((const float*)dy, arg, (float*)dx, g);
  else
    maxpool_bwd_kernel<float, unsigned long><<<grid_for(total), 256, 0, st>>>((const float*)dy, arg, (float*)dx, g);
  return (int)hipGetLastError();
}
}
