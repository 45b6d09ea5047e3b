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

// STORE = false: statistics only (the recompute path: z is never written, every consumer
// recomputes it from x, see conv0_bn_pool_kernel / bn_bwd_l0_kernel)
template <bool STATS, bool STORE = true>
__global__ __launch_bounds__(256) void conv0_fwd_kernel(const float4* __restrict__ x, const float* __restrict__ w,
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
    if constexpr (STORE) z[(((long)n * C0_H + h0 + r) * C0_W + c) * 16 + c4] = make_float4(o[0], o[1], o[2], o[3]);
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

// ---- forward apply with the conv recomputed: a = maxpool2x2(relu(conv0(x) * scale + shift)) ----
// Geometry as conv0_fwd_kernel (a block = 8 image rows of one image; thread = channel quad x
// column lane); each thread computes the 2x2 window of 4 pooled positions and writes the pooled
// value as fp32 (NP 0) or bf16 operand planes (NP 1/3) [NP][N,16,16,64].  No z is read or written:
// the 27-MAC conv costs less than the 67 MB round trip of z it replaces.
template <int NP>
__global__ __launch_bounds__(256) void conv0_bn_pool_kernel(const float4* __restrict__ x, const float* __restrict__ w,
                                                            int CP, const float* __restrict__ scale,
                                                            const float* __restrict__ shift, float* __restrict__ a,
                                                            u16* __restrict__ a3, long ps) {
  __shared__ float4 xs[C0_ROWS + 2][C0_W + 2];
  __shared__ float4 ws[16][27];
  const int t = threadIdx.x;
  const int c4 = t & 15, pl = t >> 4;  // channel quad, pooled column (0..15)
  const int bands = C0_H / C0_ROWS;
  const int n = blockIdx.x / bands, h0 = (blockIdx.x % bands) * C0_ROWS;
  for (int e = t; e < (C0_ROWS + 2) * (C0_W + 2); e += 256) {
    const int rr = e / (C0_W + 2), cc = e % (C0_W + 2);
    const int h = h0 + rr - 1, ww = cc - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h >= 0 && h < C0_H && ww >= 0 && ww < C0_W) v = x[((long)n * C0_H + h) * C0_W + ww];
    xs[rr][cc] = v;
  }
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
  const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
  const float4 sf = reinterpret_cast<const float4*>(shift)[c4];
  const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, sfv[4] = {sf.x, sf.y, sf.z, sf.w};
#pragma unroll 1
  for (int pr = 0; pr < C0_ROWS / 2; ++pr) {
    float m[4] = {0.f, 0.f, 0.f, 0.f};  // relu output >= 0: 0 is the neutral element of the max
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float o[4];
      conv0_px<4, C0_W + 2>(xs, 2 * pr + (q >> 1), 2 * pl + (q & 1), wr, o);
#pragma unroll
      for (int k = 0; k < 4; ++k) m[k] = fmaxf(m[k], fmaxf(fmaf(o[k], scv[k], sfv[k]), 0.f));
    }
    const long i4 = (((long)n * (C0_H / 2) + h0 / 2 + pr) * (C0_W / 2) + pl) * 16 + c4;
    if constexpr (NP == 0) {
      reinterpret_cast<float4*>(a)[i4] = make_float4(m[0], m[1], m[2], m[3]);
    } else {
      u16 o[4][3];
#pragma unroll
      for (int k = 0; k < 4; ++k) split_val<NP>(m[k], o[k]);
#pragma unroll
      for (int p = 0; p < NP; ++p)
        reinterpret_cast<ushort4*>(a3 + p * ps)[i4] = make_ushort4(o[0][p], o[1][p], o[2][p], o[3][p]);
    }
  }
}

// ---- backward of layer 0 in ONE pass over (g, x), z recomputed ----
// With dz = k1*dy + k2*xhat + k3 (per-channel BN-backward coefficients, bn.hip
// bn_bwd_finalize_kernel; xhat = (z - mean) * invstd), the 3x3 weight gradient splits into sums that
// need no coefficient:
//     dW[co][tap][ci] = k1[co] * S1 + k2[co] * S2 + k3[co] * S3,
//     S1 = sum_p dy[p][co] x_tap[p][ci],  S2 = sum_p xhat[p][co] x_tap[p][ci],  S3 = sum_p x_tap[p][ci]
// so one pass accumulates S1, S2, S3 and the BN reduce sums (sum dy, sum dy*xhat, sum xhat) per
// block, and a small merge kernel forms the coefficients and dW.  This replaces the reduce pass,
// the finalize, the apply+wgrad pass and their reads of the 67 MB z.
// Geometry: block = one image band of L0B_RPB pooled rows x all 16 pooled columns; thread = one
// output channel (lane) of one pooled column per wave (wave w: columns w, w+4, w+8, w+12), so the
// 64 lanes of a wave read the same input pixels from LDS (broadcast) and one 256-B row of g.
constexpr int L0B_RPB = 8;
constexpr int L0B_XR = 2 * L0B_RPB + 2, L0B_XC = C0_W + 2;
constexpr int L0B_PF = 64 * 27 * 2 + 3 * 64 + 27;  // floats per block partial: S1, S2, BN sums, S3

__global__ __launch_bounds__(256) void bn_bwd_l0_kernel(const float* __restrict__ gsrc, int nsplit, long slab,
                                                        const float4* __restrict__ x, const float* __restrict__ w,
                                                        int CP, const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, float* __restrict__ wpart,
                                                        int* sig, int sig_val) {
  start_signal(sig, sig_val);
  constexpr int Ho = C0_H / 2, Wo = C0_W / 2, bands = Ho / L0B_RPB;
  __shared__ float4 xs[L0B_XR][L0B_XC];
  __shared__ float red[4][64][57];  // per wave: S1[27], S2[27], sdy, sdx, sx of each channel
  __shared__ float red3[4][27];
  const int t = threadIdx.x, c = t & 63, wv = t >> 6;
  const int n = blockIdx.x / bands, band = blockIdx.x % bands;
  const int oh0 = band * L0B_RPB, h_lo = 2 * oh0 - 1;
  for (int e = t; e < L0B_XR * L0B_XC; e += 256) {
    const int rr = e / L0B_XC, cc = e % L0B_XC;
    const int h = h_lo + rr, ww = cc - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h >= 0 && h < C0_H && ww >= 0 && ww < C0_W) v = x[((long)n * C0_H + h) * C0_W + ww];
    xs[rr][cc] = v;
  }
  float wr[1][27];
#pragma unroll
  for (int j = 0; j < 27; ++j) wr[0][j] = w[(long)c * 9 * CP + (j / 3) * CP + (j % 3)];
  const float sc = scale[c], sf = shift[c], mu = mean[c], iv = invstd[c];
  __syncthreads();
  float s1[27], s2[27], s3 = 0.f, sdy = 0.f, sdx = 0.f, sx = 0.f;
#pragma unroll
  for (int j = 0; j < 27; ++j) s1[j] = s2[j] = 0.f;
  const int j3 = c < 27 ? c : 0;  // S3 tap of this lane (lanes >= 27 idle for S3)
  const int r3 = (j3 / 3) / 3, s3c = (j3 / 3) % 3, ci3 = j3 % 3;
#pragma unroll 1
  for (int rr = 0; rr < L0B_RPB; ++rr) {
#pragma unroll 1
    for (int cq = 0; cq < 4; ++cq) {
      const int oh = oh0 + rr, ow = wv + 4 * cq;
      const long gi = (((long)n * Ho + oh) * Wo + ow) * 64 + c;
      float g = gsrc[gi];
      for (int sp = 1; sp < nsplit; ++sp) g += gsrc[sp * slab + gi];
      const int xr = 2 * rr, xc = 2 * ow;  // xs coordinates of the window's top-left tap
      float z[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float o[1];
        conv0_px<1, L0B_XC>(xs, xr + (q >> 1), xc + (q & 1), wr, o);
        z[q] = o[0];
      }
      // route the pooled gradient to the first max of relu(BN(z)) in scan order, relu mask
      float y[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = fmaxf(fmaf(z[q], sc, sf), 0.f);
      int arg = 0;
      float mx = y[0];
      if (y[1] > mx) { mx = y[1]; arg = 1; }
      if (y[2] > mx) { mx = y[2]; arg = 2; }
      if (y[3] > mx) { mx = y[3]; arg = 3; }
      float dy[4], xh[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dy[q] = (arg == q && y[q] > 0.f) ? g : 0.f;
        xh[q] = (z[q] - mu) * iv;
        sdy += dy[q];
        sdx = fmaf(dy[q], xh[q], sdx);
        sx += xh[q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int pr = xr + (q >> 1), pc = xc + (q & 1);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const float4 xv = xs[pr + tp / 3][pc + tp % 3];
          s1[tp * 3 + 0] = fmaf(dy[q], xv.x, s1[tp * 3 + 0]);
          s1[tp * 3 + 1] = fmaf(dy[q], xv.y, s1[tp * 3 + 1]);
          s1[tp * 3 + 2] = fmaf(dy[q], xv.z, s1[tp * 3 + 2]);
          s2[tp * 3 + 0] = fmaf(xh[q], xv.x, s2[tp * 3 + 0]);
          s2[tp * 3 + 1] = fmaf(xh[q], xv.y, s2[tp * 3 + 1]);
          s2[tp * 3 + 2] = fmaf(xh[q], xv.z, s2[tp * 3 + 2]);
        }
        s3 += reinterpret_cast<const float*>(&xs[pr + r3][pc + s3c])[ci3];
      }
    }
  }
  // block partial: the 4 waves' sums in wave order
#pragma unroll
  for (int j = 0; j < 27; ++j) {
    red[wv][c][j] = s1[j];
    red[wv][c][27 + j] = s2[j];
  }
  red[wv][c][54] = sdy;
  red[wv][c][55] = sdx;
  red[wv][c][56] = sx;
  if (c < 27) red3[wv][c] = s3;
  __syncthreads();
  float* o = wpart + (long)blockIdx.x * L0B_PF;
  for (int e = t; e < 64 * 57; e += 256) {
    const int ch = e / 57, j = e % 57;
    const float v = (red[0][ch][j] + red[1][ch][j]) + (red[2][ch][j] + red[3][ch][j]);
    // layout: S1 [64][27], S2 [64][27], BN sums [3][64], S3 [27]
    if (j < 27) o[ch * 27 + j] = v;
    else if (j < 54) o[64 * 27 + ch * 27 + (j - 27)] = v;
    else o[2 * 64 * 27 + (j - 54) * 64 + ch] = v;
  }
  if (t < 27) o[2 * 64 * 27 + 3 * 64 + t] = (red3[0][t] + red3[1][t]) + (red3[2][t] + red3[3][t]);
}

// Fixed-order merge of the block partials; per output channel: dgamma, dbeta, dbias and the weight
// gradient dW [co][3][3][CP] (KRSC, channels >= 3 zero).  One 1024-thread block per channel:
// 96 value lanes (3 BN sums, 27 S1, 27 S2, 27 S3) x 10 block groups.
__global__ __launch_bounds__(1024) void bn_bwd_l0_merge_kernel(const float* __restrict__ wpart, int nblk,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ invstd, float Mfull,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                               float* __restrict__ dbias, float* __restrict__ dw,
                                                               int CP) {
  constexpr int VL = 96, GR = 10;
  __shared__ float sh[GR][VL];
  const int co = blockIdx.x, t = threadIdx.x, v = t % VL, gr = t / VL;
  float a = 0.f;
  if (gr < GR && v < 84) {
    long off;
    if (v < 3) off = 2 * 64 * 27 + v * 64 + co;             // sdy, sdx, sx
    else if (v < 30) off = co * 27 + (v - 3);               // S1
    else if (v < 57) off = 64 * 27 + co * 27 + (v - 30);    // S2
    else off = 2 * 64 * 27 + 3 * 64 + (v - 57);             // S3
    int b = gr;
    for (; b + 3 * GR < nblk; b += 4 * GR) {
      float p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) p[u] = wpart[(long)(b + GR * u) * L0B_PF + off];
#pragma unroll
      for (int u = 0; u < 4; ++u) a += p[u];
    }
    for (; b < nblk; b += GR) a += wpart[(long)b * L0B_PF + off];
  }
  if (gr < GR) sh[gr][v] = a;
  __syncthreads();
  if (t < VL) {
    float s = 0.f;
#pragma unroll
    for (int g2 = 0; g2 < GR; ++g2) s += sh[g2][t];
    sh[0][t] = s;
  }
  __syncthreads();
  const float sdy = sh[0][0], sdx = sh[0][1], sx = sh[0][2];
  const float iv = invstd[co];
  const float k1 = gamma[co] * iv;
  const float k2 = -k1 * sdx / Mfull;  // coefficient of xhat
  const float k3 = -k1 * sdy / Mfull;
  if (t == 0) {
    dgamma[co] = sdx;
    dbeta[co] = sdy;
    if (dbias) dbias[co] = k2 * sx;
  }
  for (int e = t; e < 9 * CP; e += 1024) {
    const int rs = e / CP, ci = e % CP;
    float r = 0.f;
    if (ci < 3) {
      const int j = rs * 3 + ci;
      r = k1 * sh[0][3 + j] + k2 * sh[0][30 + j] + k3 * sh[0][57 + j];
    }
    dw[(long)co * 9 * CP + e] = r;
  }
}

}  // namespace

extern "C" {
int dpa_bn_finalize(const float* part, int nblk, int rpb, int M, int C, const float* gamma, const float* beta,
                    const float* bias, float* rmean, float* rvar, long long* nbt, float* mean, float* invstd,
                    float* scale, float* shift, float momentum, float eps, hipStream_t st);

long dpa_conv0_part_floats(int N) { return 2L * N * (C0_H / C0_ROWS) * C0_C; }

// Statistics-only forward (z not stored): conv + per-block partials, then the finalize.
int dpa_conv0_stats(const float* x, const float* w, int CP, float* part, int N, const float* gamma, const float* beta,
                    const float* bias, float* rmean, float* rvar, long long* nbt, float* mean, float* invstd,
                    float* scale, float* shift, float momentum, float eps, hipStream_t st) {
  if (CP < 3) return -2;
  const int nblk = N * (C0_H / C0_ROWS);
  conv0_fwd_kernel<true, false><<<nblk, 256, 0, st>>>(reinterpret_cast<const float4*>(x), w, CP, nullptr,
                                                      reinterpret_cast<float2*>(part));
  const int rc = (int)hipGetLastError();
  if (rc) return rc;
  return dpa_bn_finalize(part, nblk, C0_PIX, N * C0_H * C0_W, C0_C, gamma, beta, bias, rmean, rvar, nbt, mean, invstd,
                         scale, shift, momentum, eps, st);
}

// a = maxpool(relu(conv0(x) * scale + shift)): fp32 a [N,16,16,64] (np 0) or planes a3 [np][...]
int dpa_conv0_bn_pool(const float* x, const float* w, int CP, const float* scale, const float* shift, float* a,
                      unsigned short* a3, int np, long ps, int N, hipStream_t st) {
  if (CP < 3) return -2;
  const int nblk = N * (C0_H / C0_ROWS);
  const float4* x4 = reinterpret_cast<const float4*>(x);
  if (np == 0) conv0_bn_pool_kernel<0><<<nblk, 256, 0, st>>>(x4, w, CP, scale, shift, a, nullptr, ps);
  else if (np == 1) conv0_bn_pool_kernel<1><<<nblk, 256, 0, st>>>(x4, w, CP, scale, shift, nullptr, a3, ps);
  else if (np == 3) conv0_bn_pool_kernel<3><<<nblk, 256, 0, st>>>(x4, w, CP, scale, shift, nullptr, a3, ps);
  else return -2;
  return (int)hipGetLastError();
}

long dpa_bn_bwd_l0_part_floats(int N) { return (long)N * (C0_H / 2 / L0B_RPB) * L0B_PF; }

// Layer-0 backward from (g, x) alone: gsrc = dL/da0 [N,16,16,64] or nsplit slabs (stride slab);
// writes dgamma, dbeta, dbias and dw [64,3,3,CP].  sig/sig_val: kernel-start signal.
int dpa_bn_bwd_l0(const float* gsrc, int nsplit, long slab, const float* x, const float* w, int CP,
                  const float* scale, const float* shift, const float* mean, const float* invstd, const float* gamma,
                  float* wpart, float* dgamma, float* dbeta, float* dbias, float* dw, int N, hipStream_t st, int* sig,
                  int sig_val) {
  if (CP < 3) return -2;
  const int nblk = N * (C0_H / 2 / L0B_RPB);
  bn_bwd_l0_kernel<<<nblk, 256, 0, st>>>(gsrc, nsplit < 1 ? 1 : nsplit, slab, reinterpret_cast<const float4*>(x), w,
                                         CP, scale, shift, mean, invstd, wpart, sig, sig_val);
  bn_bwd_l0_merge_kernel<<<C0_C, 1024, 0, st>>>(wpart, nblk, gamma, invstd, (float)N * C0_H * C0_W, dgamma, dbeta,
                                                dbias, dw, CP);
  return (int)hipGetLastError();
}

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
