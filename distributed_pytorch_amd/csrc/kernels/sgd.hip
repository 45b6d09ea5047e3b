// K9 — fused multi-tensor SGD (momentum, weight decay, optional grad scale) over ONE flat fp32
// arena.  Replaces the reference's torch.optim.SGD for-loop / foreach path
// (/root/reference/main.py:103-104, per-param add/mul_/add_/add_ — SURVEY §2.3 row "SGD step")
// with a single streaming kernel: 5 × 4 B per parameter (p, g, buf read; p, buf written).
//
// torch semantics (dampening 0, nesterov False):
//   d = g*scale + wd*p ; buf = first ? d : momentum*buf + d ; p -= lr*buf
#include "common.h"

// NP > 0: the updated parameters are also written as NP bf16 operand planes (plane stride ps, same
// element index as the arena): the conv kernels' weight operands are refreshed in the same pass
// instead of a separate split kernel per layer.
template <int NP>
__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ buf, long n4, float lr, float momentum,
                                                       float wd, float gscale, int first, u16* __restrict__ planes,
                                                       long ps) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 bv;
    float d0 = gv.x * gscale + wd * pv.x;
    float d1 = gv.y * gscale + wd * pv.y;
    float d2 = gv.z * gscale + wd * pv.z;
    float d3 = gv.w * gscale + wd * pv.w;
    if (first) {
      bv = make_float4(d0, d1, d2, d3);
    } else {
      bv = reinterpret_cast<float4*>(buf)[i];
      bv.x = momentum * bv.x + d0;
      bv.y = momentum * bv.y + d1;
      bv.z = momentum * bv.z + d2;
      bv.w = momentum * bv.w + d3;
    }
    pv.x -= lr * bv.x;
    pv.y -= lr * bv.y;
    pv.z -= lr * bv.z;
    pv.w -= lr * bv.w;
    reinterpret_cast<float4*>(buf)[i] = bv;
    reinterpret_cast<float4*>(p)[i] = pv;
    if constexpr (NP > 0) {
      u16 o[4][3];
      constexpr float s = NP == 2 ? H2_SW : 1.f;  // fp16 pairs: the weight planes' scale
      split_val<NP>(pv.x, o[0], s);
      split_val<NP>(pv.y, o[1], s);
      split_val<NP>(pv.z, o[2], s);
      split_val<NP>(pv.w, o[3], s);
#pragma unroll
      for (int q = 0; q < NP; ++q)
        reinterpret_cast<ushort4*>(planes + q * ps)[i] = make_ushort4(o[0][q], o[1][q], o[2][q], o[3][q]);
    }
  }
}

// K11 — mean over W stacked copies: out[i] = (sum_w in[w*n + i]) / W   (gather mode, rank 0).
__global__ __launch_bounds__(256) void mean_of_w_kernel(const float* __restrict__ in, float* __restrict__ out, long n,
                                                        int W) {
  const long stride = (long)gridDim.x * blockDim.x;
  const float inv = 1.0f / (float)W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float s = 0.f;
    for (int w = 0; w < W; ++w) s += in[(long)w * n + i];
    out[i] = s * inv;
  }
}

static int grid_for(long n, int block) {
  long g = (n + block - 1) / block;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

// planes: NP operand planes of the same arena slice (plane stride ps; np 2: fp16 pairs of p * H2_SW),
// or nullptr / np = 0
extern "C" int dpa_sgd_flat(float* p, const float* g, float* buf, long n, float lr, float momentum, float wd,
                            float gscale, int first, u16* planes, long ps, int np, hipStream_t s) {
  if (n % 4) return -1;
  const long n4 = n / 4;
  const int grid = grid_for(n4, 256);
  if (planes && np == 3)
    sgd_flat_kernel<3><<<grid, 256, 0, s>>>(p, g, buf, n4, lr, momentum, wd, gscale, first, planes, ps);
  else if (planes && np == 2)
    sgd_flat_kernel<2><<<grid, 256, 0, s>>>(p, g, buf, n4, lr, momentum, wd, gscale, first, planes, ps);
  else if (planes && np == 1)
    sgd_flat_kernel<1><<<grid, 256, 0, s>>>(p, g, buf, n4, lr, momentum, wd, gscale, first, planes, ps);
  else
    sgd_flat_kernel<0><<<grid, 256, 0, s>>>(p, g, buf, n4, lr, momentum, wd, gscale, first, nullptr, 0);
  return (int)hipGetLastError();
}

extern "C" int dpa_mean_of_w(const float* in, float* out, long n, int W, hipStream_t s) {
  mean_of_w_kernel<<<grid_for(n, 256), 256, 0, s>>>(in, out, n, W);
  return (int)hipGetLastError();
}

// out += add over float4 / bf16x4 groups (a gradient contribution joined where it cannot be folded
// into a producing kernel, ops/functional.GradJoin)
template <typename T>
__global__ __launch_bounds__(256) void add_inplace_kernel(T* __restrict__ out, const T* __restrict__ add, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = ld_add4(add, i), o = ld_add4(out, i);
    st_out4(out, i, make_float4(o.x + a.x, o.y + a.y, o.z + a.z, o.w + a.w));
  }
}

extern "C" int dpa_add_inplace(void* out, const void* add, long n, int bf, hipStream_t s) {
  if (n % 4) return -1;
  const long n4 = n / 4;
  if (bf)
    add_inplace_kernel<ushort4><<<grid_for(n4, 256), 256, 0, s>>>((ushort4*)out, (const ushort4*)add, n4);
  else
    add_inplace_kernel<float4><<<grid_for(n4, 256), 256, 0, s>>>((float4*)out, (const float4*)add, n4);
  return (int)hipGetLastError();
}

DPA_H2_OVF_ACCESSOR(dpa_h2_ovf_sgd)
