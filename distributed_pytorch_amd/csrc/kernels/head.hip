// Classifier head of the generic (ResNet) path: global average pool + Linear + softmax
// cross-entropy (mean), forward and backward.  The GEMMs (logits = feat @ W^T + b, and the
// backward's dfeat / dW) run on gemm_f32.hip; everything around them is here, so no GEMM,
// elementwise or reduction pass of the step runs outside the framework's kernels:
//
//   gap        feat[n][c] = mean_hw x[n][hw][c]            (x bf16 or fp32 NHWC, feat fp32)
//   ce_rows    per row: log-sum-exp, loss_row, dlogits = (softmax - onehot(target)) / N
//   ce_finish  loss = sum_n loss_row[n]  (fixed order)     ; optional running accumulator
//   bwd_prep   dl = dlogits * dloss ; db[j] = sum_n dl[n][j]   (fixed order)
//   gap_bwd    dx[n][hw][c] = dfeat[n][c] / HW               (x's dtype)
//
// Every reduction has a fixed order: results are bitwise reproducible.
#include "common.h"

namespace {

__device__ __forceinline__ float4 ld4(const float* p, long i) { return reinterpret_cast<const float4*>(p)[i]; }
__device__ __forceinline__ float4 ld4(const u16* p, long i) {
  const ushort4 h = reinterpret_cast<const ushort4*>(p)[i];
  return make_float4(bf16_f(h.x), bf16_f(h.y), bf16_f(h.z), bf16_f(h.w));
}
__device__ __forceinline__ void st4(float* p, long i, float4 v) { reinterpret_cast<float4*>(p)[i] = v; }
__device__ __forceinline__ void st4(u16* p, long i, float4 v) {
  reinterpret_cast<ushort4*>(p)[i] = make_ushort4(bf16_rne(v.x), bf16_rne(v.y), bf16_rne(v.z), bf16_rne(v.w));
}

// one thread per (n, c4); the HW loop has 4 loads in flight
template <typename T>
__global__ __launch_bounds__(256) void gap_kernel(const T* __restrict__ x, float* __restrict__ feat, int N, int HW,
                                                  int C4) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * C4) return;
  const int n = (int)(i / C4), c4 = (int)(i % C4);
  const long base = (long)n * HW * C4 + c4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int p = 0;
  for (; p + 3 < HW; p += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld4(x, base + (long)(p + u) * C4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s.x += v[u].x;
      s.y += v[u].y;
      s.z += v[u].z;
      s.w += v[u].w;
    }
  }
  for (; p < HW; ++p) {
    const float4 v = ld4(x, base + (long)p * C4);
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  const float inv = 1.f / (float)HW;
  reinterpret_cast<float4*>(feat)[i] = make_float4(s.x * inv, s.y * inv, s.z * inv, s.w * inv);
}

// one 256-thread block per row; J up to any size (strided), block reductions in LDS (fixed order)
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ logits,
                                                      const long long* __restrict__ target,
                                                      float* __restrict__ loss_row, float* __restrict__ dlogits,
                                                      int* __restrict__ correct_row, int N, int J) {
  __shared__ float red[256];
  __shared__ int redi[256];
  const int n = blockIdx.x, t = threadIdx.x;
  const float* lr = logits + (long)n * J;
  float mx = -INFINITY;
  int arg = J;
  for (int j = t; j < J; j += 256) {
    const float v = lr[j];
    if (v > mx) {
      mx = v;
      arg = j;
    }
  }
  red[t] = mx;
  redi[t] = arg;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      const float a = red[t], b = red[t + o];
      const int ia = redi[t], ib = redi[t + o];
      if (b > a || (b == a && ib < ia)) {  // first maximum (torch argmax)
        red[t] = b;
        redi[t] = ib;
      }
    }
    __syncthreads();
  }
  const float m = red[0];
  const int amax = redi[0];
  __syncthreads();
  float se = 0.f;
  for (int j = t; j < J; j += 256) se += __expf(lr[j] - m);
  red[t] = se;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  const float sum = red[0];
  const long long tg = target[n];
  const float lse = m + __logf(sum);
  if (t == 0) {
    loss_row[n] = lse - lr[tg];
    if (correct_row) correct_row[n] = amax == (int)tg ? 1 : 0;
  }
  if (dlogits) {
    const float invN = 1.f / (float)N, inv = 1.f / sum;
    for (int j = t; j < J; j += 256) {
      const float p = __expf(lr[j] - m) * inv;
      dlogits[(long)n * J + j] = (p - (j == tg ? 1.f : 0.f)) * invN;
    }
  }
}

// loss = mean of the rows (one block, fixed order); acc (optional) += loss; correct_sum (optional)
__global__ __launch_bounds__(256) void ce_finish_kernel(const float* __restrict__ loss_row,
                                                        const int* __restrict__ correct_row, int N,
                                                        float* __restrict__ loss, float* __restrict__ acc) {
  __shared__ float red[256];
  __shared__ float redc[256];
  const int t = threadIdx.x;
  float s = 0.f, c = 0.f;
  for (int n = t; n < N; n += 256) {
    s += loss_row[n];
    if (correct_row) c += (float)correct_row[n];
  }
  red[t] = s;
  redc[t] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      red[t] += red[t + o];
      redc[t] += redc[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const float l = red[0] / (float)N;
    if (loss) loss[0] = l;
    if (acc) {  // eval accumulator: [sum of batch-mean losses, correct]
      acc[0] += l;
      if (correct_row) acc[1] += redc[0];
    }
  }
}

// dl = dlogits * g[0]; db[j] = sum_n dl[n][j]: one thread per column j, rows in order
__global__ __launch_bounds__(256) void head_bwd_prep_kernel(const float* __restrict__ dlogits,
                                                            const float* __restrict__ gout, float* __restrict__ dl,
                                                            float* __restrict__ db, int N, int J) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= J) return;
  const float g = gout[0];
  float s = 0.f;
  int n = 0;
  // 16 rows' loads in flight (the rolled loop paid one memory latency per row: 33 us for N = 128 on
  // the ResNet-50 step); rows still summed in order
  for (; n + 16 <= N; n += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = dlogits[(long)(n + u) * J + j] * g;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      dl[(long)(n + u) * J + j] = v[u];
      s += v[u];
    }
  }
  for (; n < N; ++n) {
    const float v = dlogits[(long)n * J + j] * g;
    dl[(long)n * J + j] = v;
    s += v;
  }
  db[j] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void gap_bwd_kernel(const float* __restrict__ dfeat, T* __restrict__ dx, int N,
                                                      int HW, int C4) {
  const long total = (long)N * HW * C4;
  const long stride = (long)gridDim.x * blockDim.x;
  const float inv = 1.f / (float)HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c4 = (int)(i % C4);
    const int n = (int)(i / ((long)HW * C4));
    const float4 f = reinterpret_cast<const float4*>(dfeat)[(long)n * C4 + c4];
    st4(dx, i, make_float4(f.x * inv, f.y * inv, f.z * inv, f.w * inv));
  }
}

int grid1(long n, int block = 256) {
  long g = (n + block - 1) / block;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {
int dpa_gap(const void* x, float* feat, int N, int HW, int C, int xbf, hipStream_t st) {
  if (C % 4) return -2;
  const long n = (long)N * (C / 4);
  const int grid = (int)((n + 255) / 256);
  if (xbf)
    gap_kernel<u16><<<grid, 256, 0, st>>>((const u16*)x, feat, N, HW, C / 4);
  else
    gap_kernel<float><<<grid, 256, 0, st>>>((const float*)x, feat, N, HW, C / 4);
  return (int)hipGetLastError();
}

int dpa_ce(const float* logits, const long long* target, float* loss_row, float* dlogits, int* correct_row,
           float* loss, float* acc, int N, int J, hipStream_t st) {
  ce_rows_kernel<<<N, 256, 0, st>>>(logits, target, loss_row, dlogits, correct_row, N, J);
  ce_finish_kernel<<<1, 256, 0, st>>>(loss_row, correct_row, N, loss, acc);
  return (int)hipGetLastError();
}

int dpa_head_bwd_prep(const float* dlogits, const float* gout, float* dl, float* db, int N, int J, hipStream_t st) {
  head_bwd_prep_kernel<<<(J + 255) / 256, 256, 0, st>>>(dlogits, gout, dl, db, N, J);
  return (int)hipGetLastError();
}

int dpa_gap_bwd(const float* dfeat, void* dx, int N, int HW, int C, int xbf, hipStream_t st) {
  if (C % 4) return -2;
  const long total = (long)N * HW * (C / 4);
  if (xbf)
    gap_bwd_kernel<u16><<<grid1(total), 256, 0, st>>>(dfeat, (u16*)dx, N, HW, C / 4);
  else
    gap_bwd_kernel<float><<<grid1(total), 256, 0, st>>>(dfeat, (float*)dx, N, HW, C / 4);
  return (int)hipGetLastError();
}
}  // extern "C"
