// Shared device-side helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// Every kernel in this directory is written for a 64-lane wavefront and gfx950 MFMA only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#define DPA_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DPA_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) return (int)_e;                                          \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Integer ceil-div usable on host and device.
__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

// Bijective XCD-aware remap of a linear block id: consecutive logical tiles land on the same
// XCD (blocks b and b+8 share an XCD under round-robin dispatch). Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// ---- fp32 -> bf16 operand planes (round-to-nearest-even): x = x0 (+ x1 + x2) ----
// NP = 3 carries the full 24-bit fp32 mantissa (conv_x3.hip header); NP = 1 is plain bf16.
typedef unsigned short u16;
typedef __attribute__((address_space(1))) int gint;  // global-memory int (agent-scope atomics)

// Kernel-start stream signal (engine.py, two-stream backward): one lane of the first workgroup
// stores `val` to `sig` with a relaxed agent-scope atomic store.  When any workgroup of a kernel
// runs, every earlier kernel of its stream has completed and its writes were released at that
// kernel boundary, so a consumer on another stream that sees `val` (signal.hip wait kernel) may
// run the dependent kernels next without a queue marker on the producer stream.
__device__ __forceinline__ void start_signal(int* sig, int val) {
  if (sig != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    __hip_atomic_store((gint*)sig, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u16 bf16_rne(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (u16)(u >> 16);
}
__device__ __forceinline__ float bf16_f(u16 h) { return __uint_as_float(((unsigned)h) << 16); }

// ---- fp16 operand pairs (NP = 2, impl "h2"): x * s = h0 + h1 ----
// h0 = fp16(x s), h1 = fp16(x s - h0), both round-to-nearest-even: 22 significant bits in two
// planes, and a product a * b from THREE plane products a0 b0 + a0 b1 + a1 b0 (the dropped a1 b1
// is below 2^-21 of it) on the fp16 matrix cores -- half the MFMA work of the bf16 triple's six
// products at the same fp32-level error (docs/PERF_NOTES.md, round 5).  fp16's exponent range
// needs a per-tensor power-of-two scale s, undone exactly in the consuming conv's epilogue:
//  * weights and activations (BatchNorm outputs) use fixed scales, H2_SW and H2_SA: their
//    magnitudes are bounded by construction; a split that would leave fp16's range raises the
//    translation unit's overflow word (g_h2_ovf, read by dpa_h2_overflow), which fails the step;
//  * data gradients use a scale from a bound the BatchNorm backward computes for every step
//    (bn.hip): |dz s| < 2^14 always.
// Values below 2^-14 / s keep an absolute error under 2^-25 / s: negligible against the
// fp32-rounding error of the sums they enter.
constexpr float H2_SW = 256.f;  // weight planes: |w| < 255
constexpr float H2_SA = 16.f;   // activation planes: |a| < 4093
constexpr float H2_FP16_MAX = 65504.f;
static __device__ int g_h2_ovf;  // per translation unit
__device__ __forceinline__ u16 f16_bits(float f) { return __builtin_bit_cast(u16, (_Float16)f); }
__device__ __forceinline__ float f16_f(u16 h) { return (float)__builtin_bit_cast(_Float16, h); }
// the scale of a tensor bounded by B: the power of two s with B s < 2^14 (1 for B = 0 / non-finite)
__device__ __forceinline__ float h2_scale_of_bound(float B) {
  if (!(B > 0.f) || !(B < 3.0e38f)) return 1.f;
  int e;
  frexpf(B, &e);  // B = m 2^e, m in [0.5, 1): B < 2^e
  return ldexpf(1.f, min(126, 14 - e));
}
// the conv epilogue's factor 1 / (s_a s_b): a constant part and, for a data-gradient operand, the
// scale of its bound (a device word written by the BatchNorm backward)
__device__ __forceinline__ float h2_out_scale(float c, const unsigned* bound) {
  return bound != nullptr ? c / h2_scale_of_bound(__uint_as_float(*bound)) : c;
}

// NP 1 / 3: bf16 planes of v (s unused); NP 2: the fp16 pair of v * s
template <int NP>
__device__ __forceinline__ void split_val(float v, u16* o, float s = 1.f) {
  if constexpr (NP == 2) {
    const float xs = v * s;
    if (fabsf(xs) > H2_FP16_MAX) g_h2_ovf = 1;
    const u16 h0 = f16_bits(xs);
    o[0] = h0;
    o[1] = f16_bits(xs - f16_f(h0));
  } else {
    const u16 h0 = bf16_rne(v);
    o[0] = h0;
    if (NP == 3) {
      const float r1 = v - bf16_f(h0);
      const u16 h1 = bf16_rne(r1);
      o[1] = h1;
      o[2] = bf16_rne(r1 - bf16_f(h1));
    }
  }
}

// host accessor of a translation unit's overflow word (read, optionally clear)
#define DPA_H2_OVF_ACCESSOR(fn)                                                    \
  extern "C" int fn(int clear) {                                                   \
    int v = 0;                                                                     \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_h2_ovf), sizeof(int)) != hipSuccess) \
      return -1;                                                                   \
    if (clear && v) {                                                              \
      const int z = 0;                                                             \
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_h2_ovf), &z, sizeof(int));              \
    }                                                                              \
    return v;                                                                      \
  }                                                                                \
  extern "C" int* fn##_addr() {                                                    \
    void* p = nullptr;                                                             \
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_h2_ovf)) != hipSuccess) return nullptr; \
    return static_cast<int*>(p);                                                   \
  }

// ---- deterministic split-K reduction: out[i] = sum_k slabs[k * n4 + i] over float4 elements ----
// Block = 64 float4 columns x G split lanes: lane g sums splits g, g+G, ... and the G partials are
// combined in LDS in a fixed order.  G > 1 gives small outputs with many splits (e.g. first-layer
// weight gradients: 1152 float4 x 512 splits) enough parallel loads to stream at HBM rate.
__device__ __forceinline__ void st_out4(float4* o, long i, float4 v) { o[i] = v; }
__device__ __forceinline__ void st_out4(ushort4* o, long i, float4 v) {
  o[i] = make_ushort4(bf16_rne(v.x), bf16_rne(v.y), bf16_rne(v.z), bf16_rne(v.w));
}
__device__ __forceinline__ float4 ld_add4(const float4* a, long i) { return a[i]; }
__device__ __forceinline__ float4 ld_add4(const ushort4* a, long i) {
  const ushort4 h = a[i];
  return make_float4(bf16_f(h.x), bf16_f(h.y), bf16_f(h.z), bf16_f(h.w));
}
// add (optional, out's type): out = sum of the slabs + add -- a second gradient contribution to the
// same tensor folded into the reduction instead of a separate elementwise pass
template <int G, typename TO>
__global__ __launch_bounds__(64 * G) void splitk_reduce_kernel(const float4* __restrict__ slabs,
                                                               TO* __restrict__ out, long n4, int splits,
                                                               const TO* __restrict__ add) {
  __shared__ float4 part[G > 1 ? G : 1][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  // grid-stride over 64-column groups (a capped grid leaves CUs to the other stream's kernels)
  for (long i0 = (long)blockIdx.x * 64; i0 < n4; i0 += (long)gridDim.x * 64) {
    const long i = i0 + c;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n4) {
#pragma unroll 4
      for (int k = g; k < splits; k += G) {
        const float4 v = slabs[(long)k * n4 + i];
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
    }
    if constexpr (G > 1) {
      part[g][c] = s;
      __syncthreads();
      if (g == 0) {
#pragma unroll
        for (int j = 1; j < G; ++j) {
          s.x += part[j][c].x;
          s.y += part[j][c].y;
          s.z += part[j][c].z;
          s.w += part[j][c].w;
        }
      }
      __syncthreads();  // part is rewritten by the next group
    }
    if (g == 0 && i < n4) {
      if (add) {
        const float4 a = ld_add4(add, i);
        s.x += a.x;
        s.y += a.y;
        s.z += a.z;
        s.w += a.w;
      }
      st_out4(out, i, s);
    }
  }
}

// out: float4 (fp32) or ushort4 (bf16, round-to-nearest-even); add: optional addend of out's type
template <typename TO>
inline int launch_splitk_reduce_t(const float* slabs, TO* o4, long n4, int splits, hipStream_t st,
                                  const TO* add = nullptr) {
  const long blocks = (n4 + 63) / 64;
  const long full = blocks;
  const float4* in4 = reinterpret_cast<const float4*>(slabs);
  if (splits >= 16 && full < 4096)
    splitk_reduce_kernel<16, TO><<<blocks, 1024, 0, st>>>(in4, o4, n4, splits, add);
  else if (splits >= 4 && full < 16384)
    splitk_reduce_kernel<4, TO><<<blocks, 256, 0, st>>>(in4, o4, n4, splits, add);
  else
    splitk_reduce_kernel<1, TO><<<blocks, 64, 0, st>>>(in4, o4, n4, splits, add);
  return (int)hipGetLastError();
}
inline int launch_splitk_reduce(const float* slabs, float* out, long n4, int splits, hipStream_t st) {
  return launch_splitk_reduce_t(slabs, reinterpret_cast<float4*>(out), n4, splits, st);
}

