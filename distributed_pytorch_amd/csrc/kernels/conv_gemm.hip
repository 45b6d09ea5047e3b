// K1/K2/K3 — convolution as an implicit GEMM on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the reference's mkldnn conv2d forward and convolution_backward
// (SURVEY §2.3 rows "conv2d" and "convolution_backward"; model.py:18-23).
// Layout is NHWC activations and KRSC weights, so every GEMM operand row is a contiguous
// channel run:
//   FPROP  out[m][n]  = sum_k  Xcol[m][k] * W[n][k]          m=(img,oh,ow) n=kout  k=(r,s,c)
//   DGRAD  (stride 1, "same" pad) = FPROP of dZ with Wd[c][r][s][k] = W[k][R-1-r][S-1-s][c]; the B
//          loader reads W with the flipped tap index directly (no transposed weight copy)
//   WGRAD  dW[n][k]   = sum_m  dZ[m][n] * Xcol[m][k]          (split-K over m = N*P*Q)
//
// Tiling: BM x BN block tile, BK = 32 k per LDS stage, double-buffered LDS with register-staged
// prefetch (global loads for tile t+1 are issued before the MFMAs of tile t), one barrier per
// k-tile.  Waves tile the block WAVES_M x WAVES_N; each wave owns (BM/WAVES_M) x (BN/WAVES_N)
// as 32x32 MFMA sub-tiles.  The f32 MFMA consumes k=2 per instruction with lane half h=l>>5
// holding k=h; we permute k inside each 8-wide chunk (MFMA t of chunk q uses k = 8q+4h+t for lane
// half h) so that one ds_read_b128 feeds 4 MFMAs.  The permutation is applied identically to A
// and B, so the sum over k is unchanged (and each MFMA is still an exact f32 fma chain).
//
// Position-major rows + tap skipping (posmajor=1).  The GEMM row index m is ordered
// (oh, ow, img) instead of (img, oh, ow), so a BM-row tile holds ONE output pixel position of BM
// images.  Every row of the tile then has the same set of in-bounds filter taps, and k-tiles of
// taps that fall entirely into the zero padding are skipped instead of multiplied by zeros: on
// 2x2 feature maps only 4 of 9 taps are real (2.25x less MFMA work), 4x4 → 0.69, 8x8 → 0.84.
// WGRAD skips the (position, tap) pairs the same way over its m reduction.  Results are written
// in NHWC memory order whatever the row order, so consumers never see the permutation.
//
// LDS images: a k-contiguous operand is stored [row][BK+4] (16-row b128 lane groups hit 16
// distinct 16-B slots: conflict-free), a row-contiguous operand (WGRAD A/B, DGRAD B) [BK][rows+4].
#include "common.h"

namespace {

constexpr int BK = 32;
constexpr int KPAD = 4;

struct FastDiv {  // unsigned division by a runtime constant d (d >= 1), exact for n < 2^31
  unsigned d, mul, shift;
};

__host__ FastDiv make_fastdiv(unsigned d) {
  FastDiv f;
  f.d = d;
  if (d == 1) {
    f.mul = 0;
    f.shift = 0;
    return f;
  }
  unsigned s = 0;
  while ((1u << s) < d) ++s;
  f.shift = s;
  f.mul = (unsigned)((((unsigned long long)1 << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

__device__ __forceinline__ unsigned fdiv(unsigned n, FastDiv f) {
  if (f.d == 1) return n;
  unsigned t = __umulhi(n, f.mul);
  return (t + n) >> f.shift;
}

struct ConvArgs {
  const float* x;   // FPROP/DGRAD: GEMM input NHWC [N,H,W,C]     WGRAD: input NHWC (B operand)
  const float* w;   // FPROP: weights [Nout][Ktot]; DGRAD: orig weights [C][R][S][Nout]; WGRAD: dZ [N,P,Q,Kout]
  float* out;       // FPROP/DGRAD: out NHWC [N,P,Q,Nout] or slabs    WGRAD: dW [Kout][Ktot] or slabs
  int N, H, W, C;   // input dims
  int P, Q;         // output spatial dims
  int R, S, stride, pad;
  int M;            // N*P*Q
  int Nout;         // FPROP/DGRAD: output channels; WGRAD: Kout
  int Ktot;         // R*S*C
  int gm, gn;       // tile grid
  int splits;       // split-K factor (tiles of the reduction are partitioned over blockIdx.y)
  int posmajor;     // row order (oh,ow,img) + tap skipping (see header)
  long slab;        // elements per split slab (0 when splits==1)
  unsigned xbytes, wbytes;  // buffer-descriptor ranges of x and w (< 2 GiB)
  FastDiv fd_C, fd_S, fd_Q, fd_PQ, fd_N;
};

template <int ROWS, int THREADS>
struct KContigSlots {  // a k-contiguous operand tile ROWS x BK, loaded as float4
  static constexpr int F4_PER_ROW = BK / 4;
  static constexpr int NSLOT = ROWS * F4_PER_ROW / THREADS;
  static constexpr int ROW_STEP = THREADS / F4_PER_ROW;
  static_assert(ROWS * F4_PER_ROW % THREADS == 0, "tile/threads mismatch");
};

template <int ROWS, int THREADS>
struct RowContigSlots {  // a row-contiguous operand tile BK x ROWS, loaded as float4
  static constexpr int F4_PER_K = ROWS / 4;
  static constexpr int NSLOT = BK * F4_PER_K / THREADS;
  static constexpr int K_STEP = THREADS / F4_PER_K;
  static_assert(BK * F4_PER_K % THREADS == 0, "tile/threads mismatch");
  static_assert(THREADS % F4_PER_K == 0, "threads must cover whole k rows");
};

__device__ __forceinline__ float4 ldg4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Branch-free masked load: always issue the load (from the tensor base when masked off) and select
// afterwards — a per-slot "valid ? load : 0" makes hipcc branch around each load and drain vmcnt.
// 16-byte operand load through a buffer descriptor: a masked-off lane reads past the range and
// gets zeros (unconditional load, no select: see conv_x3.hip)
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const float* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 ldg4m(__amdgpu_buffer_rsrc_t r, long off, bool valid) {
  const unsigned vo = valid ? (unsigned)(off * 4) : 0x80000000u;
  const f32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)vo, 0, 0);
  return make_float4(v.x, v.y, v.z, v.w);
}

// logical GEMM row m -> (img, oh, ow)
__device__ __forceinline__ void decode_row(const ConvArgs& a, unsigned m, unsigned& img, unsigned& oh,
                                           unsigned& ow) {
  unsigned pos;
  if (a.posmajor) {
    pos = fdiv(m, a.fd_N);
    img = m - pos * (unsigned)a.N;
  } else {
    img = fdiv(m, a.fd_PQ);
    pos = m - img * (unsigned)(a.P * a.Q);
  }
  oh = fdiv(pos, a.fd_Q);
  ow = pos - oh * (unsigned)a.Q;
}

enum { MODE_FPROP = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_gemm_kernel(ConvArgs a) {
  const __amdgpu_buffer_rsrc_t rx = rsrc_of(a.x, a.xbytes), rw = rsrc_of(a.w, a.wbytes);
  constexpr bool WGRAD = MODE == MODE_WGRAD;
  constexpr bool B_ROWC = MODE != MODE_FPROP;  // B operand row-contiguous in global memory
  constexpr int THREADS = WAVES_M * WAVES_N * 64;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  // LDS sizes (floats) per stage
  constexpr int A_STAGE = WGRAD ? BK * (BM + KPAD) : BM * (BK + KPAD);
  constexpr int B_STAGE = B_ROWC ? BK * (BN + KPAD) : BN * (BK + KPAD);
  __shared__ __attribute__((aligned(16))) float lds[2 * (A_STAGE + B_STAGE)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid / WAVES_N, wc = wid % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;

  const int nwg = a.gm * a.gn;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int bm = tile / a.gn, bn = tile % a.gn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int split = blockIdx.y;

  // ---------------- reduction tile iterator (virtual tile v -> reduction offset) ----------------
  // FPROP/DGRAD reduce over k=(r,s,c); WGRAD over m.  With tap skipping the virtual tiles
  // enumerate only the (tap x c-chunk) [FPROP/DGRAD] or (position x img-chunk) [WGRAD]
  // combinations that can be non-zero for this block.
  bool skip = false;
  int lo0 = 0, lo1 = 0, span1 = 1, per = 1;  // rectangle origin, inner span, tiles per cell
  int ntot;
  if constexpr (!WGRAD) {
    ntot = (a.Ktot + BK - 1) / BK;
    if (a.posmajor && a.C % BK == 0 && a.N % BM == 0) {
      const int pos = m0 / a.N;
      const int oh = pos / a.Q, ow = pos - (pos / a.Q) * a.Q;
      const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
      const int r_lo = max(0, -ih0), r_hi = min(a.R, a.H - ih0);
      const int s_lo = max(0, -iw0), s_hi = min(a.S, a.W - iw0);
      skip = true;
      lo0 = r_lo;
      lo1 = s_lo;
      span1 = max(0, s_hi - s_lo);
      per = a.C / BK;
      ntot = max(0, r_hi - r_lo) * span1 * per;
    }
  } else {
    ntot = (a.M + BK - 1) / BK;
    if (a.posmajor && a.C % BN == 0 && a.N % BK == 0) {
      const int tap = n0 / a.C;  // the block's rsc columns share one tap
      const int r = tap / a.S, s = tap - (tap / a.S) * a.S;
      // positions with ih = oh*st - pad + r in [0, H)
      const int oh_lo = max(0, (a.pad - r + a.stride - 1) / a.stride);
      const int oh_hi = min(a.P, (a.H - 1 + a.pad - r) / a.stride + 1);
      const int ow_lo = max(0, (a.pad - s + a.stride - 1) / a.stride);
      const int ow_hi = min(a.Q, (a.W - 1 + a.pad - s) / a.stride + 1);
      skip = true;
      lo0 = oh_lo;
      lo1 = ow_lo;
      span1 = max(0, ow_hi - ow_lo);
      per = a.N / BK;
      ntot = max(0, oh_hi - oh_lo) * span1 * per;
    }
  }
  const int tchunk = (ntot + a.splits - 1) / a.splits;
  const int vbeg = split * tchunk;
  const int vend = min(ntot, vbeg + tchunk);
  const int ntiles = max(0, vend - vbeg);
  auto tile_off = [&](int v) -> int {  // reduction offset (k for FPROP/DGRAD, m for WGRAD)
    if (!skip) return v * BK;
    const int cell = v / per, sub = v - (v / per) * per;
    const int i0 = lo0 + cell / span1, i1 = lo1 + cell % span1;
    if constexpr (!WGRAD)
      return (i0 * a.S + i1) * a.C + sub * BK;  // (r, s, c-chunk)
    else
      return (i0 * a.Q + i1) * a.N + sub * BK;  // (oh, ow, img-chunk), posmajor m order
  };
  const int KMAX = WGRAD ? a.M : a.Ktot;

  // ---------------- per-thread load-slot precomputation ----------------
  using ASl = typename std::conditional<WGRAD, RowContigSlots<BM, THREADS>, KContigSlots<BM, THREADS>>::type;
  using BSl = typename std::conditional<B_ROWC, RowContigSlots<BN, THREADS>, KContigSlots<BN, THREADS>>::type;
  constexpr int NA = ASl::NSLOT, NB = BSl::NSLOT;

  float4 ra[NA], rb[NB];

  // FPROP/DGRAD A slots: rows m, fixed k4
  int a_img[WGRAD ? 1 : NA], a_ih0[WGRAD ? 1 : NA], a_iw0[WGRAD ? 1 : NA];
  int a_k4 = 0;
  // WGRAD A slots: fixed kout column group, k rows vary
  int a_col = 0, a_krow = 0;
  // FPROP B slots: rows n (weights), fixed k4
  int b_k4 = 0, b_row0 = 0;
  // WGRAD/DGRAD B slots: fixed column group
  int b_rr = 0, b_ss = 0, b_c = 0, b_colvalid = 0, b_krow = 0;

  if constexpr (!WGRAD) {
    a_k4 = tid % (BK / 4);
    const int r0 = tid / (BK / 4);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int m = m0 + r0 + j * ASl::ROW_STEP;
      if (m < a.M) {
        unsigned img, oh, ow;
        decode_row(a, (unsigned)m, img, oh, ow);
        a_img[j] = (int)img;
        a_ih0[j] = (int)oh * a.stride - a.pad;
        a_iw0[j] = (int)ow * a.stride - a.pad;
      } else {
        a_img[j] = -1;
        a_ih0[j] = 0;
        a_iw0[j] = 0;
      }
    }
    if constexpr (MODE == MODE_FPROP) {
      b_k4 = tid % (BK / 4);
      b_row0 = tid / (BK / 4);
    } else {
      b_c = n0 + (tid % BSl::F4_PER_K) * 4;  // output channel of the dgrad GEMM = input channel of W
      b_colvalid = b_c < a.Nout;
      b_krow = tid / BSl::F4_PER_K;
    }
  } else {
    a_col = m0 + (tid % ASl::F4_PER_K) * 4;  // kout index (A rows = kout, tile origin m0)
    a_krow = tid / ASl::F4_PER_K;
    const int rsc = n0 + (tid % BSl::F4_PER_K) * 4;  // B rows = rsc
    b_colvalid = rsc < a.Ktot;
    const unsigned tap = fdiv((unsigned)rsc, a.fd_C);
    b_c = rsc - (int)tap * a.C;
    const unsigned rr = fdiv(tap, a.fd_S);
    b_rr = (int)rr - a.pad;
    b_ss = (int)(tap - rr * a.S) - a.pad;
    b_krow = tid / BSl::F4_PER_K;
  }

  auto load_tile = [&](int v) {
    const int kb = tile_off(vbeg + v);
    if constexpr (!WGRAD) {
      const int k = kb + a_k4 * 4;
      const bool kval = k < KMAX;
      const unsigned tap = fdiv((unsigned)k, a.fd_C);
      const int c = k - (int)tap * a.C;
      const unsigned r = fdiv(tap, a.fd_S);
      const int s = (int)(tap - r * a.S);
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int ih = a_ih0[j] + (int)r, iw = a_iw0[j] + s;
        const bool v = kval && a_img[j] >= 0 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        ra[j] = ldg4m(rx, (((long)a_img[j] * a.H + ih) * a.W + iw) * a.C + c, v);
      }
      if constexpr (MODE == MODE_FPROP) {
        const int kb4 = kb + b_k4 * 4;
        const bool kbv = kb4 < KMAX;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int n = n0 + b_row0 + j * BSl::ROW_STEP;
          const bool v = kbv && n < a.Nout;
          rb[j] = ldg4m(rw, (long)n * a.Ktot + kb4, v);
        }
      } else {
        // DGRAD: B[n=c][k=(r',s',kk)] = W[kk][R-1-r'][S-1-s'][c], W stored [Kout=a.C][R][S][Nout]
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int k = kb + b_krow + j * BSl::K_STEP;
          const unsigned tp = fdiv((unsigned)k, a.fd_C);
          const int kk = k - (int)tp * a.C;
          const unsigned rr = fdiv(tp, a.fd_S);
          const int ss = (int)(tp - rr * a.S);
          const bool v = k < KMAX && b_colvalid;
          rb[j] = ldg4m(rw, (((long)kk * a.R + (a.R - 1 - (int)rr)) * a.S + (a.S - 1 - ss)) * a.Nout + b_c, v);
        }
      }
    } else {
      // A = dZ^T : element (kout, m) = dZ[row(m)][kout];  B = Xcol^T : (rsc, m) = X[img, ih, iw, c]
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int m = kb + a_krow + j * ASl::K_STEP;
        bool v = m < KMAX && a_col < a.Nout;
        unsigned img = 0, oh = 0, ow = 0;
        decode_row(a, (unsigned)m, img, oh, ow);  // unconditional: masked lanes read out of range
        const long row = ((long)img * a.P + oh) * a.Q + ow;
        ra[j] = ldg4m(rw, row * a.Nout + a_col, v);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int m = kb + b_krow + j * BSl::K_STEP;
        bool v = m < KMAX && b_colvalid;
        unsigned img = 0, oh = 0, ow = 0;
        decode_row(a, (unsigned)m, img, oh, ow);  // unconditional: masked lanes read out of range
        const int ih = (int)oh * a.stride + b_rr, iw = (int)ow * a.stride + b_ss;
        v = v && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        rb[j] = ldg4m(rx, (((long)img * a.H + ih) * a.W + iw) * a.C + b_c, v);
      }
    }
  };

  auto store_tile = [&](int stage) {
    float* As = lds + stage * (A_STAGE + B_STAGE);
    float* Bs = As + A_STAGE;
    if constexpr (!WGRAD) {
      const int r0 = tid / (BK / 4);
#pragma unroll
      for (int j = 0; j < NA; ++j)
        *reinterpret_cast<float4*>(As + (r0 + j * ASl::ROW_STEP) * (BK + KPAD) + a_k4 * 4) = ra[j];
      if constexpr (MODE == MODE_FPROP) {
#pragma unroll
        for (int j = 0; j < NB; ++j)
          *reinterpret_cast<float4*>(Bs + (b_row0 + j * BSl::ROW_STEP) * (BK + KPAD) + b_k4 * 4) = rb[j];
      } else {
        const int cb = (tid % BSl::F4_PER_K) * 4;
#pragma unroll
        for (int j = 0; j < NB; ++j)
          *reinterpret_cast<float4*>(Bs + (b_krow + j * BSl::K_STEP) * (BN + KPAD) + cb) = rb[j];
      }
    } else {
      const int ca = (tid % ASl::F4_PER_K) * 4;
#pragma unroll
      for (int j = 0; j < NA; ++j)
        *reinterpret_cast<float4*>(As + (a_krow + j * ASl::K_STEP) * (BM + KPAD) + ca) = ra[j];
      const int cb = (tid % BSl::F4_PER_K) * 4;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        *reinterpret_cast<float4*>(Bs + (b_krow + j * BSl::K_STEP) * (BN + KPAD) + cb) = rb[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute_tile = [&](int stage) {
    const float* As = lds + stage * (A_STAGE + B_STAGE);
    const float* Bs = As + A_STAGE;
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      float4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wr * WTM + i * 32 + li;
        if constexpr (!WGRAD) {
          fa[i] = *reinterpret_cast<const float4*>(As + row * (BK + KPAD) + 8 * q + 4 * lh);
        } else {
          const float* p = As + (8 * q + 4 * lh) * (BM + KPAD) + row;
          fa[i] = make_float4(p[0], p[BM + KPAD], p[2 * (BM + KPAD)], p[3 * (BM + KPAD)]);
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wc * WTN + j * 32 + li;
        if constexpr (!B_ROWC) {
          fb[j] = *reinterpret_cast<const float4*>(Bs + row * (BK + KPAD) + 8 * q + 4 * lh);
        } else {
          const float* p = Bs + (8 * q + 4 * lh) * (BN + KPAD) + row;
          fb[j] = make_float4(p[0], p[BN + KPAD], p[2 * (BN + KPAD)], p[3 * (BN + KPAD)]);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][t], fb[j][t], acc[i][j], 0, 0, 0);
    }
  };

  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < ntiles) load_tile(kt + 1);
      compute_tile(cur);
      if (kt + 1 < ntiles) store_tile(cur ^ 1);
      __syncthreads();
    }
  }

  // ---------------- epilogue: C[row][col], row over BM (A rows), col over BN (B rows) ----------
  // FPROP/DGRAD rows are logical GEMM rows, stored at their NHWC memory row.
  float* out = a.out + (long)split * a.slab;
  const int ldc = WGRAD ? a.Ktot : a.Nout;
  const int nrows = WGRAD ? a.Nout : a.M;
  const int ncols = WGRAD ? a.Ktot : a.Nout;
  const bool remap = !WGRAD && a.posmajor;
  const int PQ = a.P * a.Q;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wc * WTN + j * 32 + li;
      if (col < ncols) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wr * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < nrows) {
            long mrow = row;
            if (remap) {
              const unsigned pos = fdiv((unsigned)row, a.fd_N);
              mrow = (long)(row - (int)pos * a.N) * PQ + pos;
            }
            out[mrow * ldc + col] = acc[i][j][r];
          }
        }
      }
    }
}

// Sum split-K slabs: out[i] = sum_s slab[s*n + i]  (float4 vectorised; n % 4 == 0)

// Dgrad weight transform for stride-1 "same" convs: Wd[c][r][s][k] = W[k][R-1-r][S-1-s][c].
__global__ __launch_bounds__(256) void wflip_kernel(const float* __restrict__ w, float* __restrict__ wd, int K,
                                                    int R, int S, int C) {
  const long total = (long)K * R * S * C;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    // i indexes the OUTPUT wd[c][r][s][k] (k fastest -> coalesced writes)
    const int k = (int)(i % K);
    long t = i / K;
    const int s = (int)(t % S);
    t /= S;
    const int r = (int)(t % R);
    const int c = (int)(t / R);
    wd[i] = w[(((long)k * R + (R - 1 - r)) * S + (S - 1 - s)) * C + c];
  }
}

template <int BM, int BN, int WM, int WN, int MODE>
int launch_cfg(const ConvArgs& a, hipStream_t st) {
  dim3 grid(a.gm * a.gn, a.splits);
  conv_gemm_kernel<BM, BN, WM, WN, MODE><<<grid, WM * WN * 64, 0, st>>>(a);
  return (int)hipGetLastError();
}

int grid_1d(long n) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

static void fill_geom(ConvArgs& a, int N, int H, int W, int C, int R, int S, int stride, int pad) {
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.R = R;
  a.S = S;
  a.stride = stride;
  a.pad = pad;
  a.P = (H + 2 * pad - R) / stride + 1;
  a.Q = (W + 2 * pad - S) / stride + 1;
  a.M = N * a.P * a.Q;
  a.Ktot = R * S * C;
  a.fd_C = make_fastdiv(C);
  a.fd_S = make_fastdiv(S);
  a.fd_Q = make_fastdiv(a.Q);
  a.fd_PQ = make_fastdiv(a.P * a.Q);
  a.fd_N = make_fastdiv(N);
}

namespace {
int set_ranges(ConvArgs& a, long xelems, long welems) {
  if (xelems * 4 >= (1L << 31) || welems * 4 >= (1L << 31)) return 1;
  a.xbytes = (unsigned)(xelems * 4);
  a.wbytes = (unsigned)(welems * 4);
  return 0;
}
}  // namespace

extern "C" {

// effective split count the launcher will use for a reduction of `ntiles_k` BK-tiles
int dpa_conv_splits(int Kred, int splits) {
  const int nt = cdiv(Kred, BK);
  if (splits < 1) splits = 1;
  if (splits > nt) splits = nt;
  return splits < 1 ? 1 : splits;
}

// Forward conv (and, with dgrad=1, the stride-1 "same" data-gradient conv reading the ORIGINAL
// weights with flipped taps).  x: NHWC [N,H,W,C]; w: fprop [Kout][R][S][C], dgrad [C][R][S][Kout]
// (the original conv's weights, whose input channels Kout are this GEMM's outputs); out
// [N,P,Q,Kout].  splits > 1: partial sums go to slab[splits][N,P,Q,Kout]; reduce=1 sums them into
// out here, reduce=0 leaves them for a consumer that sums on the fly (bn_fwd_stats / bn_bwd).
// tile: 0 -> 128x128 (4 waves, 64x64 each), 1 -> 64x64 (4 waves, 32x32 each)
// posmajor: position-major row order + tap skipping (any value is correct; 1 is faster on small maps)
int dpa_conv_fprop(const float* x, const float* w, float* out, float* slab, int N, int H, int W, int C, int Kout,
                   int R, int S, int stride, int pad, int splits, int tile, int dgrad, int reduce, int posmajor,
                   hipStream_t st) {
  ConvArgs a{};
  a.x = x;
  a.w = w;
  fill_geom(a, N, H, W, C, R, S, stride, pad);
  a.Nout = Kout;
  if (C % 4 || Kout % 4) return -2;
  if (dgrad && (stride != 1 || a.P != H || a.Q != W)) return -3;
  if (set_ranges(a, (long)N * H * W * C, (long)Kout * a.Ktot)) return -5;
  const int BMv = tile == 0 ? 128 : 64, BNv = tile == 0 ? 128 : 64;
  a.gm = cdiv(a.M, BMv);
  a.gn = cdiv(Kout, BNv);
  a.splits = dpa_conv_splits(a.Ktot, splits);
  a.posmajor = posmajor ? 1 : 0;
  a.out = a.splits > 1 ? slab : out;
  a.slab = a.splits > 1 ? (long)a.M * Kout : 0;
  int rc;
  if (dgrad)
    rc = tile == 0 ? launch_cfg<128, 128, 2, 2, MODE_DGRAD>(a, st) : launch_cfg<64, 64, 2, 2, MODE_DGRAD>(a, st);
  else
    rc = tile == 0 ? launch_cfg<128, 128, 2, 2, MODE_FPROP>(a, st) : launch_cfg<64, 64, 2, 2, MODE_FPROP>(a, st);
  if (rc) return rc;
  if (a.splits > 1 && reduce) {
    const long n4 = (long)a.M * Kout / 4;
    rc = launch_splitk_reduce(slab, out, n4, a.splits, st);
  }
  return rc;
}

// dW[Kout][R*S*C] = sum_m dZ[m][kout] * Xcol[m][rsc]
int dpa_conv_wgrad(const float* x, const float* dz, float* dw, float* slab, int N, int H, int W, int C, int Kout,
                   int R, int S, int stride, int pad, int splits, int tile, int posmajor, hipStream_t st) {
  ConvArgs a{};
  a.x = x;
  a.w = dz;
  fill_geom(a, N, H, W, C, R, S, stride, pad);
  a.Nout = Kout;
  if (C % 4 || Kout % 4) return -2;
  if (set_ranges(a, (long)N * H * W * C, (long)a.M * Kout)) return -5;
  const int BMv = tile == 0 ? 128 : 64, BNv = tile == 0 ? 128 : 64;
  a.gm = cdiv(Kout, BMv);
  a.gn = cdiv(a.Ktot, BNv);
  a.splits = dpa_conv_splits(a.M, splits);
  a.posmajor = posmajor ? 1 : 0;
  a.out = a.splits > 1 ? slab : dw;
  a.slab = a.splits > 1 ? (long)Kout * a.Ktot : 0;
  int rc = tile == 0 ? launch_cfg<128, 128, 2, 2, MODE_WGRAD>(a, st) : launch_cfg<64, 64, 2, 2, MODE_WGRAD>(a, st);
  if (rc) return rc;
  if (a.splits > 1) {
    const long n4 = (long)Kout * a.Ktot / 4;
    rc = launch_splitk_reduce(slab, dw, n4, a.splits, st);
  }
  return rc;
}

int dpa_wflip(const float* w, float* wd, int K, int R, int S, int C, hipStream_t st) {
  wflip_kernel<<<grid_1d((long)K * R * S * C), 256, 0, st>>>(w, wd, K, R, S, C);
  return (int)hipGetLastError();
}

}  // extern "C"
