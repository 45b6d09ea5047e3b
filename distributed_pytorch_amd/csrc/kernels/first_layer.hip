// First VGG layer forward: direct fp32 3x3/s1/p1 convolution of the 3-channel network input with
// the BatchNorm statistics computed in the epilogue (model.py:18-24 with in_channels = 3).
//
// With 3 input channels the layer is 27 MACs per output value: 0.9 GFLOP for a 256-image batch,
// ~6 us of vector-ALU work, against 67 MB of fp32 output.  An MFMA implicit GEMM pads the
// reduction to 8 channels x 9 taps and needs the input split into bf16 planes first; here every
// output is an exact fp32 FMA chain (the reference's own precision) and the kernel is bound by its
// output store.  Each block also reduces its pixels' per-channel (mean, M2) — shifted sums per
// thread, Chan merges in a fixed order — which bn_finalize (bn.hip) merges, so no separate
// statistics pass re-reads z.
//
// Geometry: x [N,32,32,4] fp32 (4th channel zero), w [64,3,3,CP] KRSC (CP >= 3 padded input
// channels), z [N,32,32,64].  Block = C0_ROWS image rows of one image (256 pixels); 256 threads =
// 16 channel quads (fastest, so one pixel's 64 channels are one 256-B store) x 16 pixel lanes.
#include "common.h"

namespace {

constexpr int C0_ROWS = 8;
constexpr int C0_W = 32, C0_H = 32, C0_C = 64;
constexpr int C0_PIX = C0_ROWS * C0_W;  // pixels per block (= BN partial rows)

struct Stat {
  float n, mean, m2;
};

__device__ __forceinline__ Stat stat_merge(Stat a, Stat b) {
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float n = a.n + b.n;
  const float d = b.mean - a.mean;
  const float f = b.n / n;
  return Stat{n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}

// One output pixel for K channels: the fixed (row tap, column tap, input channel) fmaf chain every
// kernel of this file uses, so the forward statistics pass, the forward apply pass and the backward
// recompute see bit-identical z.  xs: the staged input with its zero halo; (r, c): the pixel's
// top-left tap in xs.
template <int K, int XC>
__device__ __forceinline__ void conv0_px(const float4 (*xs)[XC], int r, int c, const float (&wr)[K][27],
                                         float (&o)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) o[k] = 0.f;
#pragma unroll
  for (int dr = 0; dr < 3; ++dr)
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) {
      const float4 xv = xs[r + dr][c + dc];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        o[k] = fmaf(wr[k][(dr * 3 + dc) * 3 + 0], xv.x, o[k]);
        o[k] = fmaf(wr[k][(dr * 3 + dc) * 3 + 1], xv.y, o[k]);
        o[k] = fmaf(wr[k][(dr * 3 + dc) * 3 + 2], xv.z, o[k]);
      }
    }
}

// Built without gfx950's packed fp32 instructions (v_pk_fma_f32): see docs/PERF_NOTES.md round 6 --
// under multi-process load, this kernel's packed FMAs produced wrong values for one 16-lane pass
// (one component, one pixel) now and then; the scalar v_fma_f32 form does not (+8.8 us: the doubled
// VALU instruction count only partly hides under the output store).
// (the host compilation pass ignores the attribute: -Wignored-attributes is silenced there)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wignored-attributes"
template <bool STATS>
__global__ __launch_bounds__(256) __attribute__((target("no-packed-fp32-ops"))) void conv0_fwd_kernel(const float4* __restrict__ x, const float* __restrict__ w,
                                                        int CP, float4* __restrict__ z, float2* __restrict__ part) {
  __shared__ float4 xs[C0_ROWS + 2][C0_W + 2];
  __shared__ float4 ws[16][27];   // [channel quad][tap * 3 + ci] -> the quad's 4 output channels
  __shared__ Stat red[4][4][16];  // [wave][channel k][c4] per-wave partials
  const int t = threadIdx.x;
  const int c4 = t & 15, pl = t >> 4;  // channel quad, pixel lane (0..15)
  const int bands = C0_H / C0_ROWS;
  const int n = blockIdx.x / bands, h0 = (blockIdx.x % bands) * C0_ROWS;
  for (int e = t; e < (C0_ROWS + 2) * (C0_W + 2); e += 256) {
    const int rr = e / (C0_W + 2), cc = e % (C0_W + 2);
    const int h = h0 + rr - 1, ww = cc - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h >= 0 && h < C0_H && ww >= 0 && ww < C0_W) v = x[((long)n * C0_H + h) * C0_W + ww];
    xs[rr][cc] = v;
  }
  // weights staged once per block, regrouped so a thread's 4 output channels of one (tap, ci) are
  // one float4; then held in registers
  for (int e = t; e < 16 * 27; e += 256) {
    const int q = e / 27, j = e % 27, rs = j / 3, ci = j % 3;
    const float* src = w + (long)(4 * q) * 9 * CP + rs * CP + ci;
    ws[q][j] = make_float4(src[0], src[9 * CP], src[18 * CP], src[27 * CP]);
  }
  __syncthreads();
  float wr[4][27];
#pragma unroll
  for (int j = 0; j < 27; ++j) {
    const float4 v = ws[c4][j];
    wr[0][j] = v.x;
    wr[1][j] = v.y;
    wr[2][j] = v.z;
    wr[3][j] = v.w;
  }
  float sh[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f}, a2[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int PER = C0_PIX / 16;  // pixels per thread
#pragma unroll 2
  for (int j = 0; j < PER; ++j) {
    const int p = pl + 16 * j;  // pixel within the block: row p / 32, column p % 32
    const int r = p / C0_W, c = p % C0_W;
    float o[4];
    conv0_px<4, C0_W + 2>(xs, r, c, wr, o);
    z[(((long)n * C0_H + h0 + r) * C0_W + c) * 16 + c4] = make_float4(o[0], o[1], o[2], o[3]);
    if constexpr (STATS) {
      if (j == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) sh[k] = o[k];  // per-thread shift: its first value
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = o[k] - sh[k];
        a1[k] += d;
        a2[k] = fmaf(d, d, a2[k]);
      }
    }
  }
  if constexpr (STATS) {
    // per thread: PER values per channel -> (mean, M2); merge the 4 pixel lanes of each wave
    // (lane bits 4, 5) by shuffles, then the 4 waves in LDS, all in a fixed order
    Stat st[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float inv = 1.f / (float)PER;
      st[k] = Stat{(float)PER, sh[k] + a1[k] * inv, fmaxf(a2[k] - a1[k] * a1[k] * inv, 0.f)};
#pragma unroll
      for (int m = 16; m <= 32; m <<= 1) {
        const Stat o{__shfl_xor(st[k].n, m), __shfl_xor(st[k].mean, m), __shfl_xor(st[k].m2, m)};
        st[k] = (t & m) ? stat_merge(o, st[k]) : stat_merge(st[k], o);
      }
    }
    const int lane = t & 63, wv = t >> 6;
    if (lane < 16) {
#pragma unroll
      for (int k = 0; k < 4; ++k) red[wv][k][c4] = st[k];
    }
    __syncthreads();
    if (t < 64) {  // thread t: channel quad t & 15, channel k = t >> 4
      const int q = t & 15, k = t >> 4;
      Stat m = red[0][k][q];
#pragma unroll
      for (int v = 1; v < 4; ++v) m = stat_merge(m, red[v][k][q]);
      part[(long)blockIdx.x * C0_C + 4 * q + k] = make_float2(m.mean, m.m2);
    }
  }
}
#pragma clang diagnostic pop

}  // namespace

extern "C" {
int dpa_bn_finalize(const float* part, int nblk, int rpb, int M, int C, const float* gamma, const float* beta,
                    const float* bias, float* rmean, float* rvar, long long* nbt, float* mean, float* invstd,
                    float* scale, float* shift, float momentum, float eps, hipStream_t st);

long dpa_conv0_part_floats(int N) { return 2L * N * (C0_H / C0_ROWS) * C0_C; }

// Training (part != nullptr): conv + per-block statistics, then the BN finalize (batch statistics,
// running-stat update, scale/shift).  Eval (part == nullptr): conv only.
int dpa_conv0_fwd(const float* x, const float* w, int CP, float* z, float* part, int N, const float* gamma,
                  const float* beta, const float* bias, float* rmean, float* rvar, long long* nbt, float* mean,
                  float* invstd, float* scale, float* shift, float momentum, float eps, hipStream_t st) {
  if (CP < 3) return -2;
  const int nblk = N * (C0_H / C0_ROWS);
  if (part) {
    conv0_fwd_kernel<true><<<nblk, 256, 0, st>>>(reinterpret_cast<const float4*>(x), w, CP,
                                                 reinterpret_cast<float4*>(z), reinterpret_cast<float2*>(part));
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
    return dpa_bn_finalize(part, nblk, C0_PIX, N * C0_H * C0_W, C0_C, gamma, beta, bias, rmean, rvar, nbt, mean,
                           invstd, scale, shift, momentum, eps, st);
  }
  conv0_fwd_kernel<false><<<nblk, 256, 0, st>>>(reinterpret_cast<const float4*>(x), w, CP,
                                                reinterpret_cast<float4*>(z), nullptr);
  return (int)hipGetLastError();
}
}  // extern "C"
