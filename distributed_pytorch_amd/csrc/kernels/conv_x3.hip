// K1/K2/K3 (fast path) — implicit-GEMM convolution on gfx950 bf16 MFMA with fp32-grade accuracy.
//
// gfx950's bf16 matrix rate is 16x its fp32 matrix rate (v_mfma_f32_32x32x16_bf16 does 32x32x16
// in 32 cycles; v_mfma_f32_32x32x2_f32 does 32x32x2 in 64).  Every fp32 operand x is stored as
// three bf16 planes x = x0 + x1 + x2 (x0 = rne(x), x1 = rne(x - x0), x2 = rne(x - x0 - x1): 24
// significant bits, i.e. the full fp32 mantissa), and a product is formed from the six plane
// products whose magnitude can reach 2^-24 of a*b:
//        a*b ~= a2*b0 + a1*b1 + a0*b2 + a1*b0 + a0*b1 + a0*b0
// Each bf16 x bf16 product is exact in the fp32 MFMA accumulator, the three dropped products are
// below 2^-24 relative, so results carry fp32 rounding-level error (tests compare against fp64),
// at 6/16 of the fp32-MFMA matrix time.  NP=1 gives the plain bf16 path (one plane, one product).
//
// The operand planes are written by their producers (conv_split / bn_apply / bn_bwd_apply / the
// per-step weight split), so this kernel never converts: it streams bf16 planes global -> LDS
// (register-staged, double-buffered, one barrier per 16-deep k step) and feeds MFMAs.
//
// Modes (same GEMM formulations and position-major tap skipping as conv_gemm.hip):
//   FPROP  out[m][n] = sum_k Xcol[m][k] W[n][k]
//   DGRAD  dX[m][c]  = sum_{(r,s,k)} dZcol[m][(r,s,k)] W[k][R-1-r][S-1-s][c]: the FPROP gather of
//          dZ (padding R-1-pad; a forward stride st becomes an input dilation: tap (r,s) of
//          output row (h,w) reads dZ[(h-pad'+r)/st] only when divisible) against the weight
//          planes read in place, row-contiguous ([(r,s,k)][c]) -- no flipped weight copy
//   WGRAD  dW[n][k]  = sum_m dZ[m][n] Xcol[m][k]
// Row-contiguous operands (WGRAD A and B, DGRAD B) keep the loaded [k][col] order in LDS and the
// MFMA fragments are fetched with the gfx950 transpose read ds_read_b64_tr_b16.
// Tiles: T128 = 128x128 block, 2x2 waves of 64x64 (2x2 32x32 sub-tiles); T64 = 64x64 block, 1x2
// waves of 64x32.  Each thread stages one 16-byte chunk per plane per operand per k step.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

extern "C" int dpa_add_inplace(void* out, const void* add, long n, int bf, hipStream_t s);  // sgd.hip

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// one 16-bit MFMA step: bf16 planes (NP 1 / 3) or fp16 pairs (NP 2; fragments carry fp16 bits)
template <int NP>
__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (NP == 2)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
typedef short s16x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int BKMIN = 16;  // smallest stage depth (split-K granularity)

struct FastDiv {
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

struct Args {
  const u16* x;     // FPROP: GEMM input planes NHWC [N,H,W,C]; WGRAD: conv input planes (B operand)
  long xps;         // plane stride (elements)
  unsigned xbytes;  // bytes of ONE plane of x (buffer-descriptor range; < 2^31)
  const u16* w;     // FPROP: weight planes [Nout][R][S][C]; WGRAD: dZ planes [N,P,Q,Kout]
  long wps;
  unsigned wbytes;  // bytes of one plane of w
  float* out;       // FPROP: NHWC [N,P,Q,Nout] or slabs; WGRAD: dW [Kout][R*S*C] or slabs
  u16* outb;        // bf16 output (OB kernels, single split): FPROP/DGRAD NHWC
  long slab;
  int N, H, W, C, P, Q, R, S, stride, pad;
  int M, Nout, Ktot;
  int gm, gn, splits, posmajor;
  int nmajor;         // block -> tile order: 0 = row tiles outer (an XCD's consecutive tiles share a
                      // row tile), 1 = column tiles outer (they share a column tile: the weight slice)
  int imask, ishift;  // input dilation (DGRAD of a strided conv): 2^ishift, imask = 2^ishift - 1
  FastDiv fd_C, fd_S, fd_Q, fd_PQ, fd_N;
  int* sig;  // optional kernel-start stream signal (common.h start_signal)
  int sig_val;
  float2* stats;  // FPROP, one split: per (row tile, output channel) BN (mean, M2) of the outputs
  // DGRAD of a stride-2 conv, phase-decomposed (nph = 4, blockIdx.z = phase): output rows of one
  // phase (h % 2, w % 2) see only the filter taps r = r0 + 2 r', s = s0 + 2 s' that land on a dZ
  // pixel, so each phase is a stride-1 gather over dZ with an R' x S' sub-filter (1x1/s2: one phase
  // of 1 tap, three of 0; 3x3/s2: 1 + 2 + 2 + 4 taps) instead of the dilated form's 4x MFMA work
  // on zeros.  Rows m of a phase are (img, i, j) of the H/2 x W/2 phase grid (P, Q, M), stored at
  // dx pixel (img, 2i + ph, 2j + pw) of the outH x outW output.
  int sepi;  // OB outputs: 1 = stores staged through LDS as 16-byte row pieces (DPA_OB_EPI)
  int nph, outH, outW;
  float oscale;            // NP 2: 1 / (s_a s_b) of the operands' constant scales ...
  const unsigned* obound;  // ... times 1 / s of a data-gradient operand's bound word (or nullptr)
  struct Phase {
    int Ktot, S, r0, s0, padh, padw;
    FastDiv fd_S;
  } phase[4];
};

__device__ __forceinline__ void decode_row(const Args& a, unsigned m, unsigned& img, unsigned& oh, unsigned& ow) {
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

// 16-byte operand-plane loads through buffer descriptors: a masked-off lane gets an offset beyond
// the descriptor's range and the hardware returns zeros.  The load is unconditional and there is no
// select on its result, so hipcc cannot turn the mask into an exec branch around each load (a
// pointer-select + value-select formulation compiled to s_and_saveexec/s_cbranch per load).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const u16* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, long elem_off, bool valid) {
  const unsigned vo = valid ? (unsigned)(elem_off * 2) : OOB;
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)vo, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}

enum { XM_FPROP = 0, XM_DGRAD = 1, XM_WGRAD = 2 };

// The plane products of one k-slice over a TM x TN register tile, product-major: the TM*TN
// accumulators are independent, so back-to-back MFMAs never wait on each other's result (an
// accumulator-major order gives chains of six dependent MFMAs).  Each accumulator still sees its
// products smallest-first, so results are unchanged bit for bit.  NP 3: the six bf16 products
// a2b0 a1b1 a0b2 a1b0 a0b1 a0b0; NP 2: the three fp16 products a1b0 a0b1 a0b0; NP 1: a0b0.
template <int NP>
struct PlaneProducts {
  static constexpr int Q0 = NP == 3 ? 0 : (NP == 2 ? 3 : 5);  // first product of the list below
  static constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};  // (A plane, B plane)
};
template <int TM, int TN, int NP>
__device__ __forceinline__ void mfma_tile(f32x16 (&acc)[TM][TN], const bf16x8 (&fa)[TM][NP],
                                          const bf16x8 (&fb)[TN][NP]) {
  using PP = PlaneProducts<NP>;
#pragma unroll
  for (int q = PP::Q0; q < 6; ++q)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<NP>(fa[i][PP::PA[q]], fb[j][PP::PB[q]], acc[i][j]);
}

// fp16 pairs (NP 2): the accumulators hold (a s_a)(b s_b); one exact power-of-two multiply returns
// them to the product's own scale before anything is stored or reduced
template <int NP, int TM, int TN>
__device__ __forceinline__ void unscale_acc(f32x16 (&acc)[TM][TN], float oscale, const unsigned* obound) {
  if constexpr (NP == 2) {
    const float f = h2_out_scale(oscale, obound);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] *= f;
  }
}

// ---- BatchNorm statistics in the forward conv's epilogue ----
// The BN that follows a conv needs per-channel (mean, M2) of its output; computing them here, from
// the accumulators, saves the statistics pass's full read of z.  Per output column: each lane
// over its TM x 16 rows in one pass of sums shifted by its first row (as bn_stats_kernel), the two
// half-waves (lane, lane ^ 32), then the WAVES_M row waves through LDS, all merged in a fixed order
// (deterministic).  The block writes (mean, M2) of its rows CHANNEL-MAJOR, part[col][row tile]
// (bn_finalize_cm reads a channel's partials contiguously: a conv has up to thousands of row
// tiles).  The statistics are those of the fp32 accumulators also when the output is stored as
// bf16 (ROUND would take the rounded values: two more VALU operations per element in an epilogue
// of memory-bound convs, for a difference far below bf16 resolution -- round-to-nearest-even
// errors average out of a mean over thousands of rows).  Rows >= M are excluded.
struct EWelford {
  float n, mean, m2;
};
__device__ __forceinline__ EWelford ew_merge(EWelford a, EWelford b) {
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float n = a.n + b.n, d = b.mean - a.mean, f = b.n / n;
  return EWelford{n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}

template <int TM, int TN, int WAVES_M, int WAVES_N, bool ROUND>
__device__ __forceinline__ void epi_col_stats(const f32x16 (&acc)[TM][TN], int rows_left, int wr, int wc, int lane,
                                              float* sh, float2* part, int nblk, int bm, int ncols) {
  constexpr int WTN = TN * 32, BNC = WAVES_N * WTN;
  const int li = lane & 31, lh = lane >> 5;
  __syncthreads();  // every wave is done with the main loop's LDS
  const bool full = rows_left >= TM * 32;  // wave-uniform: no row of this wave tile is past M
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    float k0 = acc[0][j][0];
    if (ROUND) k0 = bf16_f(bf16_rne(k0));
    float n = 0.f, s1 = 0.f, s2 = 0.f;
    if (full) {
      n = TM * 16;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r];
          if (ROUND) v = bf16_f(bf16_rne(v));
          const float d = v - k0;
          s1 += d;
          s2 = fmaf(d, d, s2);
        }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r];
          if (ROUND) v = bf16_f(bf16_rne(v));
          const float d = v - k0;
          if (i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh < rows_left) {
            n += 1.f;
            s1 += d;
            s2 = fmaf(d, d, s2);
          }
        }
    }
    const float inv = n > 0.f ? 1.f / n : 0.f;
    const EWelford mine{n, k0 + s1 * inv, fmaxf(s2 - s1 * s1 * inv, 0.f)};
    const EWelford other{__shfl_xor(mine.n, 32), __shfl_xor(mine.mean, 32), __shfl_xor(mine.m2, 32)};
    const EWelford w = lh == 0 ? ew_merge(mine, other) : ew_merge(other, mine);
    if (lh == 0) {
      float* o = sh + (wr * BNC + wc * WTN + j * 32 + li) * 3;
      o[0] = w.n;
      o[1] = w.mean;
      o[2] = w.m2;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < BNC; c += WAVES_M * WAVES_N * 64) {
    EWelford w{0.f, 0.f, 0.f};
    for (int r = 0; r < WAVES_M; ++r) {
      const float* o = sh + (r * BNC + c) * 3;
      w = ew_merge(w, EWelford{o[0], o[1], o[2]});
    }
    if (c < ncols) part[c * nblk + bm] = make_float2(w.mean, w.m2);  // < BNC * nblk: 32-bit index
  }
}

// Epilogue stores staged through LDS: a wave writes SR rows x WTN columns of its accumulators (as T:
// bf16 bits or fp32) into its own LDS region `ws`, reads them back as 16-byte row pieces and hands each
// piece to store(row_in_wave_tile, col_in_wave_tile, piece).  Slices of SR rows (8 or 16) of every
// 32-row sub-tile, in order.  Wave-local: the caller barriers once before (main-loop LDS reuse).
template <int TM, int TN, int WTN, int SR, typename T, typename Store>
__device__ __forceinline__ void staged_store(const f32x16 (&acc)[TM][TN], T* ws, int lane, Store store) {
  constexpr int EPC = 16 / sizeof(T);  // elements per 16-byte piece
  constexpr int PPR = WTN / EPC;       // pieces per row
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int s = 0; s < 32 / SR; ++s) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if ((r >> 2) / (SR / 8) == s) {  // compile-time: accumulator r holds a row of slice s
            const int lrow = (r & 3) + 8 * ((r >> 2) - s * (SR / 8)) + 4 * lh;
            if constexpr (sizeof(T) == 2)
              ws[lrow * WTN + j * 32 + li] = bf16_rne(acc[i][j][r]);
            else
              ws[lrow * WTN + j * 32 + li] = acc[i][j][r];
          }
        }
#pragma unroll
      for (int c = 0; c < (SR * PPR + 63) / 64; ++c) {
        const int q = lane + 64 * c;
        if (SR * PPR % 64 == 0 || q < SR * PPR) {
          const int rr = q / PPR, pc = q - rr * PPR;
          store(i * 32 + s * SR + rr, pc * EPC, *reinterpret_cast<const uint4*>(ws + rr * WTN + pc * EPC));
        }
      }
    }
}

// BK: reduction depth per LDS stage (16/32/64 = 1/2/4 MFMA k-steps).  LDS image layouts: see the
// APITCH/BPITCH comment in the kernel (XOR swizzles, conflict-free fragment reads).
// NSTAGE: 2 = double-buffered LDS (one barrier per k step); 1 = single LDS stage + register
// prefetch (two barriers per step, half the LDS -> more resident blocks to hide load latency);
// 3 = single LDS stage, two register tiles in flight; 4 = double-buffered LDS AND two register
// tiles in flight: the ds_writes of tile t+1 and the global loads of tile t+3 are issued before
// the MFMAs of tile t, one barrier per step (for grids too small to put 2 blocks on a CU).
// OB: epilogue stores bf16 (round-to-nearest-even) to a.outb instead of fp32 (bf16 activations).
template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE, int NP, int BK, int NSTAGE, bool OB = false>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_x3_kernel(Args a) {
  start_signal(a.sig, a.sig_val);
  constexpr bool WG = MODE == XM_WGRAD;
  constexpr bool DG = MODE == XM_DGRAD;
  constexpr bool ARC = WG, BRC = WG || DG;  // operand images row-contiguous ([k][col]) in LDS
  constexpr int THREADS = WAVES_M * WAVES_N * 64;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  constexpr int CPR = BK / 8;  // 16-B chunks per k-contiguous row
  // staging: every thread owns NCA / NCB 16-byte chunks per plane of A / B per stage
  constexpr int NCA = ARC ? BK * BM / 8 / THREADS : BM * CPR / THREADS;
  constexpr int NCB = BRC ? BK * BN / 8 / THREADS : BN * CPR / THREADS;
  static_assert(NCA >= 1 && NCB >= 1, "tile/threads mismatch");
  static_assert(ARC ? (BK * BM / 8) % THREADS == 0 && THREADS % (BM / 8) == 0
                    : (BM * CPR) % THREADS == 0 && THREADS % CPR == 0, "A slot mapping");
  static_assert(BRC ? (BK * BN / 8) % THREADS == 0 && THREADS % (BN / 8) == 0
                    : (BN * CPR) % THREADS == 0 && THREADS % CPR == 0, "B slot mapping");
  // k-contiguous images are unpadded (BK bf16 per row) with the 16-B chunk index XOR-swizzled by
  // the row's position in the 256-B bank row (conflict-free ds_read_b128 fragment reads, 20 % less
  // LDS than the old +8 padding -> more resident blocks).  Row-contiguous images >= 128 columns are
  // unpadded too, with the 64-B column segment XOR-swizzled by (row & 3): the 4 rows x 64 B that a
  // ds_read_b64_tr_b16 lane group reads land in 4 distinct bank quarters.  64-column images keep
  // +32 bf16 of padding (rows 64 B apart modulo the bank row).
  constexpr bool ASWZ = ARC && BM >= 128, BSWZ = BRC && BN >= 128;
  constexpr int APITCH = ARC ? (ASWZ ? BM : BM + 32) : BK;  // bf16 per LDS row
  constexpr int BPITCH = BRC ? (BSWZ ? BN : BN + 32) : BK;
  constexpr int RPB = 16 / CPR;  // k-contiguous rows per 256-B bank row
  auto swz = [](int row) { return (row / RPB) & (CPR - 1); };
  auto rswz = [](int row, int col, bool on) { return on ? col ^ ((row & 3) << 5) : col; };
  constexpr int AROWS = ARC ? BK : BM, BROWS = BRC ? BK : BN;
  constexpr int A_PLANE = AROWS * APITCH, B_PLANE = BROWS * BPITCH;
  constexpr int STAGE = NP * (A_PLANE + B_PLANE);
  __shared__ __attribute__((aligned(16))) u16 lds[(NSTAGE == 2 || NSTAGE == 4 ? 2 : 1) * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid / WAVES_N, wc = wid % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;

  const int nwg = a.gm * a.gn;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int bm = a.nmajor ? tile % a.gm : tile / a.gn, bn = a.nmajor ? tile / a.gm : tile % a.gn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int split = blockIdx.y;

  // reduction geometry of this block (a phase of a phase-decomposed DGRAD has its own sub-filter)
  int ktot = a.Ktot, sub_s = a.S, padh = a.pad, padw = a.pad, tap_r0 = 0, tap_s0 = 0, tap_st = 1, ph = 0, pw = 0;
  FastDiv fd_sub = a.fd_S;
  if constexpr (DG) {
    if (a.nph > 1) {
      const Args::Phase& q = a.phase[blockIdx.z];
      ph = blockIdx.z >> 1;
      pw = blockIdx.z & 1;
      ktot = q.Ktot;
      sub_s = q.S;
      fd_sub = q.fd_S;
      padh = q.padh;
      padw = q.padw;
      tap_r0 = q.r0;
      tap_s0 = q.s0;
      tap_st = 2;
      if (ktot == 0) {  // a phase no tap reaches (1x1/s2: three of four): its rows of dx are zero;
                        // 16-byte stores of the tile instead of the MFMA epilogue's 2/4-byte ones
        constexpr int EPC = OB ? 8 : 4, CPRW = BN / EPC;
        float* outz = a.out + (long)split * a.slab;
        for (int q = tid; q < BM * CPRW; q += THREADS) {
          const int rl = q / CPRW, col = n0 + (q - rl * CPRW) * EPC, row = m0 + rl;
          if (row < a.M && col < a.Nout) {
            const unsigned img = fdiv((unsigned)row, a.fd_PQ), pos = (unsigned)row - img * (unsigned)(a.P * a.Q);
            const unsigned i = fdiv(pos, a.fd_Q), j = pos - i * (unsigned)a.Q;
            const long mrow = ((long)img * a.outH + 2 * (int)i + ph) * a.outW + 2 * (int)j + pw;
            if constexpr (OB)
              *reinterpret_cast<uint4*>(a.outb + mrow * a.Nout + col) = make_uint4(0u, 0u, 0u, 0u);
            else
              *reinterpret_cast<float4*>(outz + mrow * a.Nout + col) = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
        return;
      }
    }
  }

  // ---------------- reduction tile iterator with padding-tap skipping ----------------
  bool skip = false;
  int lo0 = 0, lo1 = 0, span1 = 1, per = 1, ntot;
  if constexpr (!WG) {
    ntot = (ktot + BK - 1) / BK;
    if (a.posmajor && a.imask == 0 && a.C % BK == 0 && a.N % BM == 0) {
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
      const int tap = n0 / a.C;
      const int r = tap / a.S, s = tap - (tap / a.S) * a.S;
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
  const int ntiles = max(0, min(ntot, vbeg + tchunk) - vbeg);
  auto tile_off = [&](int v) -> int {
    if (!skip) return v * BK;
    const int cell = v / per, sub = v - (v / per) * per;
    const int i0 = lo0 + cell / span1, i1 = lo1 + cell % span1;
    if constexpr (!WG)
      return (i0 * a.S + i1) * a.C + sub * BK;
    else
      return (i0 * a.Q + i1) * a.N + sub * BK;
  };
  const int KMAX = WG ? a.M : ktot;

  // ---------------- per-thread staging slots ----------------
  // FPROP: chunk (row, kc) with kc = tid % CPR fixed, rows tid/CPR + j*(THREADS/CPR).
  // WGRAD: chunk (m-row, col) with col = tid % (cols/8) fixed, m-rows tid/(cols/8) + j*step.
  constexpr int AROWSTEP = ARC ? THREADS / (BM / 8) : THREADS / CPR;
  constexpr int BROWSTEP = BRC ? THREADS / (BN / 8) : THREADS / CPR;
  const int a_r0 = ARC ? tid / (BM / 8) : tid / CPR;
  const int b_r0 = BRC ? tid / (BN / 8) : tid / CPR;
  const int a_c8 = ARC ? (tid % (BM / 8)) * 8 : (tid % CPR) * 8;  // column (row-contig) / k offset (k-contig)
  const int b_c8 = BRC ? (tid % (BN / 8)) * 8 : (tid % CPR) * 8;
  int a_img[WG ? 1 : NCA], a_ih0[WG ? 1 : NCA], a_iw0[WG ? 1 : NCA];  // FPROP A rows
  int wb_rr = 0, wb_ss = 0, wb_c = 0;                                  // WGRAD B column (rsc chunk)
  bool wb_valid = false;
  if constexpr (!WG) {
#pragma unroll
    for (int j = 0; j < NCA; ++j) {
      const int m = m0 + a_r0 + j * AROWSTEP;
      a_img[j] = -1;
      a_ih0[j] = 0;
      a_iw0[j] = 0;
      if (m < a.M) {
        unsigned img, oh, ow;
        decode_row(a, (unsigned)m, img, oh, ow);
        a_img[j] = (int)img;
        a_ih0[j] = (int)oh * a.stride - padh;
        a_iw0[j] = (int)ow * a.stride - padw;
      }
    }
  } else {
    const int rsc = n0 + b_c8;
    wb_valid = rsc < a.Ktot;
    const unsigned tap = fdiv((unsigned)rsc, a.fd_C);
    wb_c = rsc - (int)tap * a.C;
    const unsigned rr = fdiv(tap, a.fd_S);
    wb_rr = (int)rr - a.pad;
    wb_ss = (int)(tap - rr * a.S) - a.pad;
  }

  __amdgpu_buffer_rsrc_t rx[NP], rw[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    rx[p] = plane_rsrc(a.x + p * a.xps, a.xbytes);
    rw[p] = plane_rsrc(a.w + p * a.wps, a.wbytes);
  }

  // staging registers: one set (NSTAGE 1/2) or two alternating sets (NSTAGE 3: two tiles in flight)
  uint4 ra0[NCA][NP], rb0[NCB][NP];
  constexpr bool TWO = NSTAGE >= 3;
  uint4 ra1[TWO ? NCA : 1][NP], rb1[TWO ? NCB : 1][NP];

  auto load_into = [&](int v, auto& ra, auto& rb) {
    const int kb = tile_off(vbeg + v);
    if constexpr (!WG) {
      const int k = kb + a_c8;
      const unsigned tap = fdiv((unsigned)k, a.fd_C);
      const int c = k - (int)tap * a.C;
      const unsigned r = fdiv(tap, fd_sub);
      const int s = (int)(tap - r * sub_s);
      const bool kv = k < KMAX;
#pragma unroll
      for (int j = 0; j < NCA; ++j) {
        int ih = a_ih0[j] + (int)r, iw = a_iw0[j] + s;
        bool va = kv && a_img[j] >= 0;
        if constexpr (DG) {  // dilated input: only taps landing on a stride multiple exist
          va = va && ((ih | iw) & a.imask) == 0;
          ih >>= a.ishift;
          iw >>= a.ishift;
        }
        va = va && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const long aoff = (((long)a_img[j] * a.H + ih) * a.W + iw) * a.C + c;
#pragma unroll
        for (int p = 0; p < NP; ++p) ra[j][p] = bload(rx[p], aoff, va);
      }
      if constexpr (DG) {  // weight rows (r,s,k) of the flipped filter, c-contiguous
#pragma unroll
        for (int j = 0; j < NCB; ++j) {
          const int kr = kb + b_r0 + j * BROWSTEP;
          const int col = n0 + b_c8;
          const bool vb = kr < KMAX && col < a.Nout;
          const unsigned tp = fdiv((unsigned)kr, a.fd_C);
          const int ko = kr - (int)tp * a.C;
          const unsigned rr = fdiv(tp, fd_sub);
          const int ss = (int)(tp - rr * sub_s);
          const int fr = tap_r0 + tap_st * (int)rr, fs = tap_s0 + tap_st * ss;  // filter tap
          const long boff = (((long)ko * a.R + (a.R - 1 - fr)) * a.S + (a.S - 1 - fs)) * a.Nout + col;
#pragma unroll
          for (int p = 0; p < NP; ++p) rb[j][p] = bload(rw[p], boff, vb);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NCB; ++j) {
          const int n = n0 + b_r0 + j * BROWSTEP;
          const bool vb = kv && n < a.Nout;
          const long boff = (long)n * a.Ktot + k;
#pragma unroll
          for (int p = 0; p < NP; ++p) rb[j][p] = bload(rw[p], boff, vb);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NCA; ++j) {
        const int m = kb + a_r0 + j * AROWSTEP;
        const int col = m0 + a_c8;
        const bool v = m < KMAX && col < a.Nout;
        unsigned img = 0, oh = 0, ow = 0;
        decode_row(a, (unsigned)m, img, oh, ow);  // unconditional: no branch (masked lanes read OOB)
        const long off = (((long)img * a.P + oh) * a.Q + ow) * a.Nout + col;
#pragma unroll
        for (int p = 0; p < NP; ++p) ra[j][p] = bload(rw[p], off, v);
      }
#pragma unroll
      for (int j = 0; j < NCB; ++j) {
        const int m = kb + b_r0 + j * BROWSTEP;
        bool v = m < KMAX && wb_valid;
        unsigned img = 0, oh = 0, ow = 0;
        decode_row(a, (unsigned)m, img, oh, ow);  // unconditional: no branch (masked lanes read OOB)
        const int ih = (int)oh * a.stride + wb_rr, iw = (int)ow * a.stride + wb_ss;
        v = v && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const long off = (((long)img * a.H + ih) * a.W + iw) * a.C + wb_c;
#pragma unroll
        for (int p = 0; p < NP; ++p) rb[j][p] = bload(rx[p], off, v);
      }
    }
  };

  auto store_from = [&](int stage, auto& ra, auto& rb) {
    u16* As = lds + stage * STAGE;
    u16* Bs = As + NP * A_PLANE;
#pragma unroll
    for (int j = 0; j < NCA; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        *reinterpret_cast<uint4*>(As + p * A_PLANE + (a_r0 + j * AROWSTEP) * APITCH +
                                  (ARC ? rswz(a_r0 + j * AROWSTEP, a_c8, ASWZ)
                                       : ((a_c8 >> 3) ^ swz(a_r0 + j * AROWSTEP)) << 3)) = ra[j][p];
#pragma unroll
    for (int j = 0; j < NCB; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        *reinterpret_cast<uint4*>(Bs + p * B_PLANE + (b_r0 + j * BROWSTEP) * BPITCH +
                                  (BRC ? rswz(b_r0 + j * BROWSTEP, b_c8, BSWZ)
                                       : ((b_c8 >> 3) ^ swz(b_r0 + j * BROWSTEP)) << 3)) = rb[j][p];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Fragment fetch.  k-contiguous image: lane reads 16 B at [row][8*lh].  Row-contiguous image
  // ([m][col]): two ds_read_b64_tr_b16; lane 4q+p of each 16-lane group addresses row q of its
  // 4-row block, columns 4p..4p+3, and receives its own column (kout/rsc = l&31) of the block.
  auto frag_k = [&](const u16* base, int pitch, int row0, int ks) -> bf16x8 {
    const int row = row0 + li;
    const uint4 v = *reinterpret_cast<const uint4*>(base + row * pitch + (((2 * ks + lh) ^ swz(row)) << 3));
    return __builtin_bit_cast(bf16x8, v);
  };
  auto frag_r = [&](const u16* base, int pitch, int row0, int ks, bool sw) -> bf16x8 {
    {
      const int g = lane >> 4, idx = lane & 15;
      const int q = idx >> 2, p4 = idx & 3;
      const int col = row0 + 16 * (g & 1) + 4 * p4;
      const int mrow = 16 * ks + 8 * (g >> 1) + q;
      typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
      const int scol = rswz(mrow, col, sw);  // rows mrow and mrow + 4 share (row & 3)
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + mrow * pitch + scol));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (mrow + 4) * pitch + scol));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  };

  auto compute_tile = [&](int stage) {
    const u16* As = lds + stage * STAGE;
    const u16* Bs = As + NP * A_PLANE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
    bf16x8 fa[TM][NP], fb[TN][NP];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        if constexpr (ARC)
          fa[i][p] = frag_r(As + p * A_PLANE, APITCH, wr * WTM + i * 32, ks, ASWZ);
        else
          fa[i][p] = frag_k(As + p * A_PLANE, APITCH, wr * WTM + i * 32, ks);
      }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        if constexpr (BRC)
          fb[j][p] = frag_r(Bs + p * B_PLANE, BPITCH, wc * WTN + j * 32, ks, BSWZ);
        else
          fb[j][p] = frag_k(Bs + p * B_PLANE, BPITCH, wc * WTN + j * 32, ks);
      }
    mfma_tile<TM, TN, NP>(acc, fa, fb);  // smallest products first
    }
  };

  auto load_tile = [&](int v) { load_into(v, ra0, rb0); };
  auto store_tile = [&](int stage) { store_from(stage, ra0, rb0); };

  if (NSTAGE == 4 && ntiles > 0) {
    // LDS stage t & 1 holds tile t; ra0/rb0 carry the even tiles, ra1/rb1 the odd ones
    load_into(0, ra0, rb0);
    if (1 < ntiles) load_into(1, ra1, rb1);
    store_from(0, ra0, rb0);
    if (2 < ntiles) load_into(2, ra0, rb0);
    __syncthreads();
    for (int kt = 0; kt < ntiles; kt += 2) {
      if (kt + 1 < ntiles) {
        store_from(1, ra1, rb1);
        if (kt + 3 < ntiles) load_into(kt + 3, ra1, rb1);
      }
      compute_tile(0);
      __syncthreads();
      if (kt + 1 < ntiles) {
        if (kt + 2 < ntiles) {
          store_from(0, ra0, rb0);
          if (kt + 4 < ntiles) load_into(kt + 4, ra0, rb0);
        }
        compute_tile(1);
        __syncthreads();
      }
    }
  } else if (NSTAGE == 3 && ntiles > 0) {
    // single LDS stage, two register tiles in flight: while tile t is consumed from LDS, tiles
    // t+1 and t+2 are loading (uses the VGPR headroom left by the LDS-limited occupancy)
    load_into(0, ra0, rb0);
    store_from(0, ra0, rb0);
    __syncthreads();
    if (1 < ntiles) load_into(1, ra1, rb1);
    if (2 < ntiles) load_into(2, ra0, rb0);
    for (int kt = 0; kt < ntiles; kt += 2) {
      compute_tile(0);
      if (kt + 1 < ntiles) {
        __syncthreads();
        store_from(0, ra1, rb1);
        __syncthreads();
        if (kt + 3 < ntiles) load_into(kt + 3, ra1, rb1);
        compute_tile(0);
        if (kt + 2 < ntiles) {
          __syncthreads();
          store_from(0, ra0, rb0);
          __syncthreads();
          if (kt + 4 < ntiles) load_into(kt + 4, ra0, rb0);
        }
      }
    }
  } else if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
      if constexpr (NSTAGE == 2) {
        const int cur = kt & 1;
        if (kt + 1 < ntiles) load_tile(kt + 1);
        compute_tile(cur);
        if (kt + 1 < ntiles) store_tile(cur ^ 1);
        __syncthreads();
      } else {
        if (kt + 1 < ntiles) load_tile(kt + 1);
        compute_tile(0);
        if (kt + 1 < ntiles) {
          __syncthreads();
          store_tile(0);
          __syncthreads();
        }
      }
    }
  }

  // ---------------- epilogue (fp32; FPROP rows stored at their NHWC memory row) ----------------
  unscale_acc<NP>(acc, a.oscale, a.obound);
  float* out = a.out + (long)split * a.slab;
  const int ldc = WG ? a.Ktot : a.Nout;
  const int nrows = WG ? a.Nout : a.M;
  const int ncols = WG ? a.Ktot : a.Nout;
  const bool remap = !WG && a.posmajor;
  const int PQ = a.P * a.Q;
  auto mrow_of = [&](int row) -> long {
    long mrow = row;
    if (remap) {
      const unsigned pos = fdiv((unsigned)row, a.fd_N);
      mrow = (long)(row - (int)pos * a.N) * PQ + pos;
    }
    if (DG && a.nph > 1) {  // phase grid row -> dx pixel
      const unsigned img = fdiv((unsigned)row, a.fd_PQ), pos = (unsigned)row - img * (unsigned)PQ;
      const unsigned i = fdiv(pos, a.fd_Q), j = pos - i * (unsigned)a.Q;
      mrow = ((long)img * a.outH + 2 * (int)i + ph) * a.outW + 2 * (int)j + pw;
    }
    return mrow;
  };
  bool staged = false;
  {
    // outputs through LDS as 16-byte row pieces (as gemm_stream_kernel): bf16 (OB) or fp32, slices
    // of 16 rows when the main loop's LDS holds them for every wave, else 8 (DPA_OB_EPI=0: direct)
    typedef typename std::conditional<OB, u16, float>::type TO;
    constexpr int LDSE = (int)(sizeof(lds) / sizeof(TO));
    // (not the fp32-output data gradient: its phase / dilation epilogue would spill)
    constexpr int SR = (DG && !OB) ? 0
                       : (WAVES_M * WAVES_N * 16 * WTN <= LDSE ? 16 : (WAVES_M * WAVES_N * 8 * WTN <= LDSE ? 8 : 0));
    if constexpr (SR > 0) {
      if (a.sepi) {
        staged = true;
        __syncthreads();  // every wave is done with the main loop's LDS
        TO* ws = reinterpret_cast<TO*>(lds) + wid * SR * WTN;
        const int rb = m0 + wr * WTM, cb = n0 + wc * WTN;
        staged_store<TM, TN, WTN, SR, TO>(acc, ws, lane, [&](int r, int c, uint4 v) {
          const int row = rb + r, col = cb + c;
          if (row < nrows && col < ncols) {
            if constexpr (OB)
              *reinterpret_cast<uint4*>(a.outb + mrow_of(row) * ldc + col) = v;
            else
              *reinterpret_cast<uint4*>(out + mrow_of(row) * ldc + col) = v;
          }
        });
      }
    }
  }
  if (!staged) {
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
              const long mrow = mrow_of(row);
              if constexpr (OB)
                a.outb[mrow * ldc + col] = bf16_rne(acc[i][j][r]);
              else
                out[mrow * ldc + col] = acc[i][j][r];
            }
          }
        }
      }
  }
  if constexpr (MODE == XM_FPROP) {
    if (a.stats != nullptr)
      epi_col_stats<TM, TN, WAVES_M, WAVES_N, false>(acc, a.M - (m0 + wr * WTM), wr, wc, lane,
                                                  reinterpret_cast<float*>(lds), a.stats + (long)n0 * a.gm, a.gm, bm,
                                                  a.Nout - n0);
  }
}

// ---------------- persistent streaming GEMM: 1x1 / stride-1 forward convolution, bf16 ----------------
// A 1x1 conv is the GEMM Z[m][n] = sum_k X[m][k] W[n][k] (NHWC rows).  On ResNet-50 its reduction is
// short (K = 64..2048, 2..64 steps of 32) and its bf16 output large, so conv_x3_kernel's
// one-tile-per-block schedule runs each block as load -> few MFMA steps -> store with nothing in
// flight across the phases: 1.7 TB/s and 13 % MFMA busy on the tile-7 calls
// (profiles/r3_resnet50_pmc_traffic.txt).  Here a grid of at most 2 blocks per CU walks its tiles
// (b, b + G, ...) as ONE flattened sequence of (tile, k-step) units through a double-buffered LDS
// pipeline: the next unit's operand loads -- the next tile's first k-step at a tile boundary -- are
// issued before the current unit's MFMAs and the tile's epilogue stores, so the output stream of one
// tile overlaps the input stream of the next.  Tile 256x128, 8 waves of 64x64, operand staging, the
// XOR-swizzled k-contiguous LDS images, fragment reads and the epilogue (with optional BN
// statistics, epi_col_stats) are conv_x3_kernel's, so results are bitwise those of its tile 7.
struct SArgs {
  const u16* x;  // A [M][K] bf16
  unsigned xbytes;
  const u16* w;  // B [N][K] bf16 (weights [Nout][1][1][K])
  unsigned wbytes;
  u16* out;      // [M][N] bf16
  int M, N, K;
  int gm, gn;
  float2* stats;  // optional: BN (mean, M2) partials, channel-major [N][gm] (epi_col_stats)
};

// TB (the data gradient of a 1x1 / stride-1 conv, dX[m][c] = sum_k dZ[m][k] W[k][c]): B is read
// row-contiguous, rows k of W [K][N], kept [k][col] in LDS (64-B segments XOR-swizzled by row & 3)
// and fetched with ds_read_b64_tr_b16, as conv_x3_kernel's DGRAD B operand.
template <int BM, int BN, int WAVES_M, int WAVES_N, int BK, bool TB, bool SEPI = true>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) __attribute__((amdgpu_waves_per_eu(4)))
void gemm_stream_kernel(SArgs a) {  // <= 128 VGPRs: two 8-wave blocks per CU
  constexpr int THREADS = WAVES_M * WAVES_N * 64;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int CPR = BK / 8, ROWSTEP = THREADS / CPR;
  constexpr int NCA = BM / ROWSTEP;
  constexpr int NCB = TB ? BK * BN / 8 / THREADS : (BN + ROWSTEP - 1) / ROWSTEP;
  constexpr int BROWSTEP = THREADS / (BN / 8);  // TB: k rows per chunk pass
  static_assert(BM % ROWSTEP == 0 && THREADS % CPR == 0, "A slot mapping");
  static_assert(!TB || (BK * BN / 8) % THREADS == 0, "B slot mapping");
  constexpr int RPB = 16 / CPR;
  constexpr int A_PLANE = BM * BK, B_PLANE = BN * BK, STAGE = A_PLANE + B_PLANE;
  auto rswz = [](int row, int col) { return col ^ ((row & 3) << 5); };
  __shared__ __attribute__((aligned(16))) u16 lds[2 * STAGE];
  __shared__ float esh[WAVES_M * BN * 3];  // epilogue statistics scratch
  auto swz = [](int row) { return (row / RPB) & (CPR - 1); };

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WAVES_N, wc = wid % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;
  const int ntile = a.gm * a.gn, G = gridDim.x;
  const int b = xcd_remap(blockIdx.x, G);  // an XCD's blocks take neighbouring tiles (shared A rows)
  const int KS = (a.K + BK - 1) / BK;
  const int U = (b < ntile ? (ntile - 1 - b) / G + 1 : 0) * KS;
  const __amdgpu_buffer_rsrc_t rx = plane_rsrc(a.x, a.xbytes), rw = plane_rsrc(a.w, a.wbytes);
  const int r0 = tid / CPR, c8 = (tid % CPR) * 8;

  uint4 ra[NCA], rb[NCB];
  auto load = [&](int u) {
    const int t = b + (u / KS) * G, ks = u - (u / KS) * KS;
    const int m0 = (t / a.gn) * BM, n0 = (t - (t / a.gn) * a.gn) * BN;
    const int k = ks * BK + c8;
    const bool kv = k < a.K;
#pragma unroll
    for (int j = 0; j < NCA; ++j) {
      const int m = m0 + r0 + j * ROWSTEP;
      ra[j] = bload(rx, (long)m * a.K + k, kv && m < a.M);
    }
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
      if constexpr (TB) {  // W [K][N]: row kr, 8 columns from n0 + bc8
        const int kr = ks * BK + tid / (BN / 8) + j * BROWSTEP, col = n0 + (tid % (BN / 8)) * 8;
        rb[j] = bload(rw, (long)kr * a.N + col, kr < a.K && col < a.N);
      } else {
        const int n = n0 + r0 + j * ROWSTEP;
        rb[j] = bload(rw, (long)n * a.K + k, kv && n < a.N && r0 + j * ROWSTEP < BN);
      }
    }
  };
  auto store = [&](int st) {
    u16* As = lds + st * STAGE;
    u16* Bs = As + A_PLANE;
#pragma unroll
    for (int j = 0; j < NCA; ++j) {
      const int row = r0 + j * ROWSTEP;
      *reinterpret_cast<uint4*>(As + row * BK + (((c8 >> 3) ^ swz(row)) << 3)) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
      if constexpr (TB) {
        const int kr = tid / (BN / 8) + j * BROWSTEP, col = (tid % (BN / 8)) * 8;
        *reinterpret_cast<uint4*>(Bs + kr * BN + rswz(kr, col)) = rb[j];
      } else {
        const int row = r0 + j * ROWSTEP;
        if (row < BN) *reinterpret_cast<uint4*>(Bs + row * BK + (((c8 >> 3) ^ swz(row)) << 3)) = rb[j];
      }
    }
  };
  auto frag = [&](const u16* base, int row, int ks) -> bf16x8 {
    const uint4 v = *reinterpret_cast<const uint4*>(base + row * BK + (((2 * ks + lh) ^ swz(row)) << 3));
    return __builtin_bit_cast(bf16x8, v);
  };
  auto frag_t = [&](const u16* base, int col0, int ks) -> bf16x8 {  // [k][col] image, transposed read
    const int g = lane >> 4, idx = lane & 15;
    const int q = idx >> 2, p4 = idx & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p4;
    const int krow = 16 * ks + 8 * (g >> 1) + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const int scol = rswz(krow, col);  // rows krow and krow + 4 share (row & 3)
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + krow * BN + scol));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (krow + 4) * BN + scol));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  f32x16 acc[TM][TN];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };
  auto compute = [&](int st) {
    const u16* As = lds + st * STAGE;
    const u16* Bs = As + A_PLANE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[TM][1], fb[TN][1];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i][0] = frag(As, wr * WTM + i * 32 + li, ks);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (TB)
          fb[j][0] = frag_t(Bs, wc * WTN + j * 32, ks);
        else
          fb[j][0] = frag(Bs, wc * WTN + j * 32 + li, ks);
      }
      mfma_tile<TM, TN, 1>(acc, fa, fb);
    }
  };
  // Tile stores through LDS: per 32-row slice of its 64x64 wave tile, a wave writes its bf16 values
  // into its own 4 KB region and reads them back as 16-byte row pieces, so each global store moves
  // 16 B per lane (128-B row segments) instead of 2 B.  Called after a block barrier: both operand
  // stages are free (the next unit's operands are still in registers).
  static_assert(WTN == 64 && WAVES_M * WAVES_N * 32 * WTN * 2 <= 2 * STAGE * 2, "epilogue staging");
  auto epilogue = [&](int t) {
    const int bm = t / a.gn, bn = t - (t / a.gn) * a.gn;
    const int m0 = bm * BM, n0 = bn * BN;
    if constexpr (!SEPI) {  // direct 2-byte stores (A/B: DPA_STREAM_EPI=0)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + wc * WTN + j * 32 + li;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = m0 + wr * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (row < a.M && col < a.N) a.out[(long)row * a.N + col] = bf16_rne(acc[i][j][r]);
          }
        }
    }
    u16* ws = lds + wid * 32 * WTN;
#pragma unroll
    for (int i = 0; i < (SEPI ? TM : 0); ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ws[((r & 3) + 8 * (r >> 2) + 4 * lh) * WTN + j * 32 + li] = bf16_rne(acc[i][j][r]);
#pragma unroll
      for (int c = 0; c < 32 * WTN / 8 / 64; ++c) {
        const int q = lane + 64 * c, rr = q / (WTN / 8), cc = q - rr * (WTN / 8);
        const uint4 v = *reinterpret_cast<const uint4*>(ws + rr * WTN + cc * 8);
        const int row = m0 + wr * WTM + i * 32 + rr, col = n0 + wc * WTN + cc * 8;
        if (row < a.M && col < a.N) *reinterpret_cast<uint4*>(a.out + (long)row * a.N + col) = v;
      }
    }
    if (a.stats != nullptr)
      epi_col_stats<TM, TN, WAVES_M, WAVES_N, false>(acc, a.M - (m0 + wr * WTM), wr, wc, lane, esh,
                                                    a.stats + (long)n0 * a.gm, a.gm, bm, a.N - n0);
  };

  if (U == 0) return;
  zero();
  load(0);
  store(0);
  __syncthreads();
  for (int u = 0; u < U; ++u) {
    if (u + 1 < U) load(u + 1);  // the next unit's operands (the next tile's at a tile boundary)
    compute(u & 1);
    if (u % KS == KS - 1) {
      __syncthreads();  // both LDS stages free for the epilogue's staging
      epilogue(b + (u / KS) * G);
      zero();
      __syncthreads();
    }
    if (u + 1 < U) store((u + 1) & 1);
    __syncthreads();
  }
}

// ---------------- halo-staged direct 3x3 convolution (stride 1, pad 1) ----------------
// conv_x3_kernel gathers its A operand afresh for every filter tap: each input pixel crosses the
// L2 -> CU path once per tap and per column tile, and that gather traffic -- not the matrix cores
// -- bounds it (the one-plane bf16 build streams operand bytes at the same rate as x3).  Here a
// block owns BM consecutive output pixels (NHWC order).  Per chunk of BC reduction channels it
// stages the pixel range [m0 - W - 1, m0 + BM + W + 1) ONCE into LDS -- the block's pixels plus
// one image row and one pixel of halo on each side -- and one zero slot, then runs the 9 taps
// against shifted views of that image: tap (r, s) of local pixel m reads slot m + r*W + s, or the
// zero slot when (y + r - 1, x + s - 1) leaves the image.  Only the per-tap weight tile streams
// (double-buffered LDS, one barrier per tap).  A is loaded once per chunk instead of 9 times.
//   FPROP  out[p][n] = sum_{tap,c} x[p + d(tap)][c] * W[n][tap][c]
//   DGRAD  dx[p][c]  = sum_{tap,k} dz[p + d(tap)][k] * W[k][8 - tap][c]   (stride 1: the flipped
//          weights are read in place, row-contiguous, fragments through ds_read_b64_tr_b16)
// Operand planes, plane products, split-K slabs (a split without chunks writes zeros) and the
// epilogue are those of conv_x3_kernel; output rows are NHWC pixel indices.
struct HArgs {
  const u16* x;  // A planes [NP][N,H,W,C] (DGRAD: dz)
  long xps;
  unsigned xbytes;
  const u16* w;  // weight planes [Kf][3][3][Cf]
  long wps;
  unsigned wbytes;
  float* out;  // [N,H,W,Nout] fp32, or split-K slabs
  u16* outb;   // bf16 output (OB)
  long slab;
  int N, H, W, C, Nout, M;  // C: reduction channels
  int gm, gn, cps;          // row / column tiles, reduction chunks per split
  int* sig;                 // optional kernel-start stream signal (common.h start_signal)
  int sig_val;
  float2* stats;            // FPROP, one split: per (row tile, output channel) BN (mean, M2)
  int sepi;                 // OB: stores staged through LDS
  float oscale;             // NP 2: output scale (Args::oscale / obound)
  const unsigned* obound;
};

// staged slots per block: BM + 2W + 2 pixels and the zero slot (the last one), sized for rows of up
// to BM/4 - 1 pixels -- except fp16-pair planes of 64-channel chunks (tiles 22, 23: twice the
// reduction per barrier), whose image is sized for rows of at most 16 pixels so that it (74.5 KB)
// and the double-buffered weight tiles (64 KB) fit the 160 KB of LDS.
__host__ __device__ constexpr int halo_slots(int BM, int BC, int NP) {
  return BC >= 64 && NP >= 2 ? BM + 2 * 16 + 3 : BM + BM / 2 + 1;
}

template <int BM, int BN, int WAVES_M, int WAVES_N, bool DG, int NP, int BC, bool OB>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_halo_kernel(HArgs a) {
  start_signal(a.sig, a.sig_val);
  constexpr int THREADS = WAVES_M * WAVES_N * 64;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  constexpr int CPR = BC / 8;    // 16-B chunks per staged row
  constexpr int RPB = 16 / CPR;  // staged rows per 256-B bank row
  constexpr int SLOTS = halo_slots(BM, BC, NP), ZS = SLOTS - 1;
  constexpr int A_PLANE = SLOTS * BC;
  constexpr bool BSWZ = DG && BN >= 128;
  constexpr int BPITCH = DG ? (BSWZ ? BN : BN + 32) : BC;
  constexpr int B_PLANE = (DG ? BC : BN) * BPITCH;
  constexpr int ACH = (SLOTS - 1) * CPR;            // 16-B chunks per plane of the staged image (the zero
                                                    // slot ZS is written once, before the main loop)
  constexpr int BCH = DG ? BC * BN / 8 : BN * CPR;  // ... of one tap's weight tile
  constexpr int NCA = (ACH + THREADS - 1) / THREADS;
  constexpr int NCB = (BCH + THREADS - 1) / THREADS;
  __shared__ __attribute__((aligned(16))) u16 lds[NP * A_PLANE + 2 * NP * B_PLANE];
  u16* const As = lds;
  u16* const Bs = lds + NP * A_PLANE;
  auto swz = [](int row) { return (row / RPB) & (CPR - 1); };
  auto rswz = [](int row, int col) { return BSWZ ? col ^ ((row & 3) << 5) : col; };

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WAVES_N, wc = wid % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;
  if (tid < CPR) {  // the zero slot: every out-of-image tap reads it
#pragma unroll
    for (int p = 0; p < NP; ++p)
      *reinterpret_cast<uint4*>(lds + p * A_PLANE + ZS * BC + ((tid ^ ((ZS / RPB) & (CPR - 1))) << 3)) =
          make_uint4(0u, 0u, 0u, 0u);
  }
  const int tile = xcd_remap(blockIdx.x, a.gm * a.gn);
  const int bm = tile / a.gn, bn = tile % a.gn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int HW = a.H * a.W;
  const int nst = BM + 2 * a.W + 2;  // staged pixels: slot j holds pixel m0 - W - 1 + j

  __amdgpu_buffer_rsrc_t rx[NP], rw[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    rx[p] = plane_rsrc(a.x + p * a.xps, a.xbytes);
    rw[p] = plane_rsrc(a.w + p * a.wps, a.wbytes);
  }

  // staging slots: chunk q = tid + j * THREADS is 16-B piece q % CPR of slot q / CPR
  long a_off[NCA];
  bool a_ok[NCA];
#pragma unroll
  for (int j = 0; j < NCA; ++j) {
    const int q = tid + j * THREADS;
    const int slot = q / CPR, cc = q - slot * CPR;
    const int gp = m0 - a.W - 1 + slot;
    a_ok[j] = slot < nst && gp >= 0 && gp < a.M;
    a_off[j] = (long)gp * a.C + cc * 8;
  }
  // weight staging (one tap tile): FPROP rows n with pieces along c; DGRAD rows k of the chunk
  // with pieces along the output channel
  long b_off[NCB];
  bool b_ok[NCB];
#pragma unroll
  for (int j = 0; j < NCB; ++j) {
    const int q = tid + j * THREADS;
    if constexpr (DG) {
      const int k = q / (BN / 8), col = (q - k * (BN / 8)) * 8;
      b_ok[j] = q < BCH && n0 + col < a.Nout;
      b_off[j] = (long)k * 9 * a.Nout + n0 + col;
    } else {
      const int n = q / CPR, cc = q - n * CPR;
      b_ok[j] = q < BCH && n0 + n < a.Nout;
      b_off[j] = (long)(n0 + n) * 9 * a.C + cc * 8;
    }
  }

  uint4 ra[NCA][NP], rb[NCB][NP];
  auto load_a = [&](int c0) {
#pragma unroll
    for (int j = 0; j < NCA; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) ra[j][p] = bload(rx[p], a_off[j] + c0, a_ok[j]);
  };
  auto store_a = [&]() {
#pragma unroll
    for (int j = 0; j < NCA; ++j) {
      const int q = tid + j * THREADS;
      const int slot = q / CPR, cc = q - slot * CPR;
      if ((ACH % THREADS == 0 || q < ACH) && slot < nst) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
          *reinterpret_cast<uint4*>(As + p * A_PLANE + slot * BC + ((cc ^ swz(slot)) << 3)) = ra[j][p];
      }
    }
  };
  auto load_b = [&](int tap, int c0) {
    const long d = DG ? ((long)c0 * 9 + 8 - tap) * a.Nout : (long)tap * a.C + c0;
#pragma unroll
    for (int j = 0; j < NCB; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) rb[j][p] = bload(rw[p], b_off[j] + d, b_ok[j]);
  };
  auto store_b = [&](int stage) {
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
      const int q = tid + j * THREADS;
      if (BCH % THREADS == 0 || q < BCH) {
        int idx;
        if constexpr (DG) {
          const int k = q / (BN / 8), col = (q - k * (BN / 8)) * 8;
          idx = k * BPITCH + rswz(k, col);
        } else {
          const int n = q / CPR, cc = q - n * CPR;
          idx = n * BC + ((cc ^ swz(n)) << 3);
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<uint4*>(Bs + (stage * NP + p) * B_PLANE + idx) = rb[j][p];
      }
    }
  };

  // A fragment rows: local pixel m at image position (y, x)
  int fr_m[TM], fr_y[TM], fr_x[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wr * WTM + i * 32 + li;
    const int pix = (m0 + m) % HW;
    fr_m[i] = m;
    fr_y[i] = pix / a.W;
    fr_x[i] = pix - fr_y[i] * a.W;
  }

  auto frag_k = [&](const u16* base, int row, int ks) -> bf16x8 {
    const uint4 v = *reinterpret_cast<const uint4*>(base + row * BC + (((2 * ks + lh) ^ swz(row)) << 3));
    return __builtin_bit_cast(bf16x8, v);
  };
  auto frag_r = [&](const u16* base, int col0, int ks) -> bf16x8 {
    const int g = lane >> 4, idx = lane & 15;
    const int q = idx >> 2, p4 = idx & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p4;
    const int krow = 16 * ks + 8 * (g >> 1) + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const int scol = rswz(krow, col);  // rows krow and krow + 4 share (row & 3)
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + krow * BPITCH + scol));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (krow + 4) * BPITCH + scol));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int tap, int stage) {
    const int r = tap / 3, s = tap - 3 * (tap / 3);
    int sl[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bool v = (unsigned)(fr_y[i] + r - 1) < (unsigned)a.H && (unsigned)(fr_x[i] + s - 1) < (unsigned)a.W;
      sl[i] = v ? fr_m[i] + r * a.W + s : ZS;
    }
    const u16* Bst = Bs + stage * NP * B_PLANE;
#pragma unroll
    for (int ks = 0; ks < BC / 16; ++ks) {
      bf16x8 fa[TM][NP], fb[TN][NP];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) fa[i][p] = frag_k(As + p * A_PLANE, sl[i], ks);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          if constexpr (DG)
            fb[j][p] = frag_r(Bst + p * B_PLANE, wc * WTN + j * 32, ks);
          else
            fb[j][p] = frag_k(Bst + p * B_PLANE, wc * WTN + j * 32 + li, ks);
        }
      mfma_tile<TM, TN, NP>(acc, fa, fb);
    }
  };

  // ---- main loop: step = (chunk, tap).  The weight tile of step st+1 is written to the other
  // buffer after step st's MFMAs (its loads were issued a step earlier); the next chunk's pixels
  // sit in registers during the 9 taps and replace the staged image at the chunk boundary.
  // fp16-pair 64-channel chunks: each chunk's 9 x 64 products per output go to a fresh accumulator
  // that is then added to the running total -- the fp32 rounding of a long reduction grows with
  // the chain, and this cuts the chain to one chunk plus one add per chunk (64 adds per wave)
  constexpr bool CACC = BC >= 64 && NP == 2;
  f32x16 tot[CACC ? TM : 1][CACC ? TN : 1];
  if constexpr (CACC) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) tot[i][j][r] = 0.f;
  }
  const int nch = a.C / BC;
  const int cb = blockIdx.y * a.cps, ce = min(nch, cb + a.cps);
  const int nsteps = max(0, ce - cb) * 9;
  if (nsteps > 0) {
    load_a(cb * BC);
    load_b(0, cb * BC);
    store_a();
    store_b(0);
    if (nsteps > 1) load_b(1, cb * BC);
    if (cb + 1 < ce) load_a((cb + 1) * BC);
    __syncthreads();
    int tap = 0, ch = cb;
    for (int st = 0; st < nsteps; ++st) {
      compute(tap, st & 1);
      const bool last_tap = tap == 8;
      if constexpr (CACC) {
        if (last_tap) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                tot[i][j][r] += acc[i][j][r];
                acc[i][j][r] = 0.f;
              }
        }
      }
      const int tap1 = last_tap ? 0 : tap + 1, ch1 = last_tap ? ch + 1 : ch;  // step st + 1
      if (st + 1 < nsteps) {
        store_b((st + 1) & 1);
        if (st + 2 < nsteps) load_b(tap1 == 8 ? 0 : tap1 + 1, (tap1 == 8 ? ch1 + 1 : ch1) * BC);
        if (last_tap) {  // every wave is done with this chunk's image before it is replaced
          __syncthreads();
          store_a();
          if (ch + 2 < ce) load_a((ch + 2) * BC);
        }
      }
      __syncthreads();
      tap = tap1;
      ch = ch1;
    }
  }
  if constexpr (CACC) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = tot[i][j][r];
  }

  // ---------------- epilogue (rows are NHWC pixels) ----------------
  unscale_acc<NP>(acc, a.oscale, a.obound);
  float* out = a.out + (long)blockIdx.y * a.slab;
  bool staged = false;
  {  // outputs through LDS as 16-byte row pieces (conv_x3_kernel's epilogue)
    typedef typename std::conditional<OB, u16, float>::type TO;
    constexpr int LDSE = (int)(sizeof(lds) / sizeof(TO));
    constexpr int SR = WAVES_M * WAVES_N * 16 * WTN <= LDSE ? 16 : (WAVES_M * WAVES_N * 8 * WTN <= LDSE ? 8 : 0);
    if constexpr (SR > 0) {
      if (a.sepi) {
        staged = true;
        __syncthreads();  // every wave is done with the main loop's LDS
        TO* ws = reinterpret_cast<TO*>(lds) + wid * SR * WTN;
        const int rb = m0 + wr * WTM, cb = n0 + wc * WTN;
        staged_store<TM, TN, WTN, SR, TO>(acc, ws, lane, [&](int r, int c, uint4 v) {
          const int row = rb + r, col = cb + c;
          if (row < a.M && col < a.Nout) {
            if constexpr (OB)
              *reinterpret_cast<uint4*>(a.outb + (long)row * a.Nout + col) = v;
            else
              *reinterpret_cast<uint4*>(out + (long)row * a.Nout + col) = v;
          }
        });
      }
    }
  }
  if (!staged) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wc * WTN + j * 32 + li;
        if (col < a.Nout) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = m0 + wr * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (row < a.M) {
              if constexpr (OB)
                a.outb[(long)row * a.Nout + col] = bf16_rne(acc[i][j][r]);
              else
                out[(long)row * a.Nout + col] = acc[i][j][r];
            }
          }
        }
      }
  }
  if constexpr (!DG) {
    if (a.stats != nullptr)
      epi_col_stats<TM, TN, WAVES_M, WAVES_N, false>(acc, a.M - (m0 + wr * WTM), wr, wc, lane,
                                                  reinterpret_cast<float*>(lds), a.stats + (long)n0 * a.gm, a.gm, bm,
                                                  a.Nout - n0);
  }
}

// ---------------- halo-staged 3x3 weight gradient (stride 1, pad 1) ----------------
// dW[k][tap][c] = sum_p dZ[p][k] * X[p + d(tap)][c].  A block owns a 128 (k) x 32 (c) tile of all
// 9 taps -- four waves, each a 32-row k slice with nine accumulators -- and reduces over chunks of
// P consecutive pixels.  Per chunk it stages dZ [P][128] and the X halo image (pixels
// [pb - W - 1, pb + P + W + 1) and a zero slot) once, double-buffered, fetches each dZ^T fragment
// once per k-step and reuses it for all 9 taps.  Both images are row-contiguous and read with
// ds_read_b64_tr_b16; the X rows are per-lane slot addresses (the tap shift, or the zero slot),
// so the 9-fold im2col re-gather of conv_x3_kernel's WGRAD is gone.
struct WHArgs {
  const u16* x;  // X planes [NP][N,H,W,C]
  long xps;
  unsigned xbytes;
  const u16* dz;  // dZ planes [NP][N,H,W,K]
  long dzps;
  unsigned dzbytes;
  float* out;  // dW [K][3][3][C] fp32, or split-K slabs
  long slab;
  int N, H, W, C, K, M;
  int gk, gc, nchunks, cps;
  FastDiv fd_HW, fd_W;
  float oscale;  // NP 2: output scale (Args::oscale / obound)
  const unsigned* obound;
};

__host__ __device__ constexpr int halo_wslots(int P) { return 2 * P + 4; }  // P + 2W + 2 (W <= P/2) + zero slot

template <int NP, int P>
__global__ __launch_bounds__(256) void conv_halo_wgrad_kernel(WHArgs a) {
  constexpr int THREADS = 256, BKO = 128, BCW = 32;
  constexpr int SLOTS = halo_wslots(P), ZS = SLOTS - 1;
  constexpr int Z_PLANE = P * BKO, X_PLANE = SLOTS * BCW;
  constexpr int STAGE = NP * (Z_PLANE + X_PLANE);
  constexpr int ZCH = P * BKO / 8, XCH = SLOTS * BCW / 8;  // 16-B pieces per plane
  constexpr int NZ = (ZCH + THREADS - 1) / THREADS, NX = (XCH + THREADS - 1) / THREADS;
  constexpr int KS = P / 16;
  __shared__ __attribute__((aligned(16))) u16 lds[2 * STAGE];
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef short s16x8 __attribute__((ext_vector_type(8)));

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  const int tile = xcd_remap(blockIdx.x, a.gk * a.gc);
  const int bk = tile / a.gc, bcol = tile - bk * a.gc;
  const int k0 = bk * BKO, c0 = bcol * BCW;
  const int cb = blockIdx.y * a.cps, ce = min(a.nchunks, cb + a.cps);
  const int nst = P + 2 * a.W + 2;

  __amdgpu_buffer_rsrc_t rx[NP], rz[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    rx[p] = plane_rsrc(a.x + p * a.xps, a.xbytes);
    rz[p] = plane_rsrc(a.dz + p * a.dzps, a.dzbytes);
  }

  uint4 rzr[NZ][NP], rxr[NX][NP];
  auto load_chunk = [&](int ch) {
    const int pb = ch * P;
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int qq = tid + j * THREADS;
      const int prow = qq / (BKO / 8), col = (qq % (BKO / 8)) * 8;
      const bool v = (ZCH % THREADS == 0 || qq < ZCH) && pb + prow < a.M && k0 + col < a.K;
      const long off = (long)(pb + prow) * a.K + k0 + col;
#pragma unroll
      for (int p = 0; p < NP; ++p) rzr[j][p] = bload(rz[p], off, v);
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int qq = tid + j * THREADS;
      const int slot = qq >> 2, cc = qq & 3;
      const int gp = pb - a.W - 1 + slot;
      const bool v = slot < nst && gp >= 0 && gp < a.M && c0 + cc * 8 < a.C;
      const long off = (long)gp * a.C + c0 + cc * 8;
#pragma unroll
      for (int p = 0; p < NP; ++p) rxr[j][p] = bload(rx[p], off, v);
    }
  };
  auto store_chunk = [&](int stage) {
    u16* Zs = lds + stage * STAGE;
    u16* Xs = Zs + NP * Z_PLANE;
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int qq = tid + j * THREADS;
      if (ZCH % THREADS == 0 || qq < ZCH) {
        const int prow = qq / (BKO / 8), col = (qq % (BKO / 8)) * 8;
#pragma unroll
        for (int p = 0; p < NP; ++p)
          *reinterpret_cast<uint4*>(Zs + p * Z_PLANE + prow * BKO + (col ^ ((prow & 3) << 5))) = rzr[j][p];
      }
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int qq = tid + j * THREADS;
      const int slot = qq >> 2;
      if ((XCH % THREADS == 0 || qq < XCH) && (slot < nst || slot == ZS)) {
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<uint4*>(Xs + p * X_PLANE + qq * 8) = rxr[j][p];
      }
    }
  };

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  const int zc = wid * 32 + 16 * (g & 1) + 4 * p4;  // dZ column (k) this lane addresses
  const int xc = 16 * (g & 1) + 4 * p4;             // X column (c)
  auto compute = [&](int stage, int pb) {
    const u16* Zs = lds + stage * STAGE;
    const u16* Xs = Zs + NP * Z_PLANE;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int zr = 16 * ks + 8 * (g >> 1) + q;  // reduction rows zr (lo) and zr + 4 (hi)
      bf16x8 fa[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const u16* zb = Zs + p * Z_PLANE + (zc ^ ((zr & 3) << 5));
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(zb + zr * BKO));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(zb + (zr + 4) * BKO));
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        fa[p] = __builtin_bit_cast(bf16x8, v);
      }
      // image positions of the two pixels this lane addresses
      int py[2], px[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const unsigned gp = (unsigned)(pb + zr + 4 * h2);
        const unsigned img = fdiv(gp, a.fd_HW);
        const unsigned pix = gp - img * (unsigned)(a.H * a.W);
        const unsigned y = fdiv(pix, a.fd_W);
        py[h2] = (int)y;
        px[h2] = (int)(pix - y * (unsigned)a.W);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int r = tap / 3, s = tap % 3;
        int sl[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const bool v = (unsigned)(py[h2] + r - 1) < (unsigned)a.H && (unsigned)(px[h2] + s - 1) < (unsigned)a.W;
          sl[h2] = v ? zr + 4 * h2 + r * a.W + s : ZS;
        }
        bf16x8 fb[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const u16* xb = Xs + p * X_PLANE + xc;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb + sl[0] * BCW));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb + sl[1] * BCW));
          const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          fb[p] = __builtin_bit_cast(bf16x8, v);
        }
        using PP = PlaneProducts<NP>;
#pragma unroll
        for (int q = PP::Q0; q < 6; ++q) acc[tap] = mfma16<NP>(fa[PP::PA[q]], fb[PP::PB[q]], acc[tap]);
      }
    }
  };

  if (ce > cb) {
    load_chunk(cb);
    store_chunk(0);
    if (cb + 1 < ce) load_chunk(cb + 1);
    __syncthreads();
    for (int ch = cb; ch < ce; ++ch) {
      const int st = (ch - cb) & 1;
      compute(st, ch * P);
      if (ch + 1 < ce) {
        store_chunk(st ^ 1);
        if (ch + 2 < ce) load_chunk(ch + 2);
      }
      __syncthreads();
    }
  }

  if constexpr (NP == 2) {
    const float f = h2_out_scale(a.oscale, a.obound);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] *= f;
  }
  float* out = a.out + (long)blockIdx.y * a.slab;
  const int col = c0 + li;
  if (col < a.C) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = k0 + wid * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < a.K) out[((long)row * 9 + t) * a.C + col] = acc[t][r];
      }
  }
}

// ---------------- position-major direct 3x3 convolution for small images (H*W <= 16) ----------------
// The 4x4 and 2x2 layers (VGG-11 on 32x32 input) have 25-56 % of their 3x3 taps in the zero padding:
// a corner output of a 2x2 image sees 4 of its 9 taps.  conv_halo_kernel's rows are NHWC pixels, so
// a 32-row MFMA sub-tile mixes positions and every tap runs (padding taps read the zero slot), and
// conv_x3_kernel skips padding taps only by re-gathering its A operand per tap.  Here a block owns
// NI images x PPT output positions with the rows POSITION-MAJOR (row = position slot * NI + image):
// every 32-row sub-tile is 32 images at ONE output position, so a tap is either entirely inside the
// image for that sub-tile or entirely padding, and padding taps are skipped outright (no MFMAs, no
// fragment reads).  Per chunk of BC reduction channels the block stages the input pixels its
// positions can reach -- rows y0-1 .. y1+1 of its NI images, slot = pixel * NI + image -- ONCE into
// LDS; the 9 per-tap weight tiles stream through a double-buffered LDS stage with PD tiles in flight
// in registers, with conv_halo_kernel's B layouts and (chunk, tap, k-step, plane product) order
// per accumulator, so the fp32 results are bit-identical to conv_halo_kernel with the same channel
// chunk and split count: a skipped tap only ever added exact zeros there.  `perm` orders a tile's
// positions so that the row waves carry near-equal numbers of in-image taps.  (A variant holding
// the chunk's nine weight tiles in LDS at once, with no per-tap barrier, measured slower: its
// 80-150 KB chunk loads left the prologue and the per-CU load rate exposed, docs/PERF_NOTES.md.)
//   FPROP  out[p][n] = sum_{tap,c} x[p + d(tap)][c] * W[n][tap][c]
//   DGRAD  dx[p][c]  = sum_{tap,k} dz[p + d(tap)][k] * W[k][8 - tap][c]
struct PArgs {
  const u16* x;  // A planes [NP][N,H,W,C] (DGRAD: dz)
  long xps;
  unsigned xbytes;
  const u16* w;  // weight planes [Kf][3][3][Cf]
  long wps;
  unsigned wbytes;
  float* out;  // [N,H,W,Nout] fp32, or split-K slabs
  long slab;
  int N, H, W, C, Nout;  // C: reduction channels
  int gm, gn, cps;       // row tiles (image groups x position blocks), column tiles, chunks per split
  int npb;               // position blocks per image group (H*W / PPT)
  unsigned perm;         // position slot k -> local position, 4 bits per slot
  int* sig;              // optional kernel-start stream signal (common.h start_signal)
  int sig_val;
  float oscale;          // NP 2: output scale (Args::oscale / obound)
  const unsigned* obound;
};

template <int BM, int BN, int WAVES_M, int WAVES_N, bool DG, int NP, int BC, int NI, int NSPX, int PD>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_pos_kernel(PArgs a) {
  start_signal(a.sig, a.sig_val);
  constexpr int THREADS = WAVES_M * WAVES_N * 64;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && NI % 32 == 0 && BM % NI == 0, "tile shape");
  constexpr int SPP = NI / 32;   // 32-row sub-tiles per position
  constexpr int PPT = BM / NI;   // positions per tile
  static_assert(PPT <= 8, "perm holds 8 position slots");
  constexpr int CPR = BC / 8;    // 16-B chunks per staged row
  constexpr int RPB = 16 / CPR;  // staged rows per 256-B bank row
  constexpr int SLOTS = NSPX * NI;
  constexpr int A_PLANE = SLOTS * BC;
  constexpr bool BSWZ = DG && BN >= 128;
  constexpr int BPITCH = DG ? (BSWZ ? BN : BN + 32) : BC;
  constexpr int B_PLANE = (DG ? BC : BN) * BPITCH;
  constexpr int ACH = SLOTS * CPR;
  constexpr int BCH = DG ? BC * BN / 8 : BN * CPR;
  constexpr int NCA = (ACH + THREADS - 1) / THREADS;
  constexpr int NCB = (BCH + THREADS - 1) / THREADS;
  __shared__ __attribute__((aligned(16))) u16 lds[NP * A_PLANE + 2 * NP * B_PLANE];
  u16* const As = lds;
  u16* const Bs = lds + NP * A_PLANE;
  auto swz = [](int row) { return (row / RPB) & (CPR - 1); };
  auto rswz = [](int row, int col) { return BSWZ ? col ^ ((row & 3) << 5) : col; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: the tap tests below branch on it
  const int wr = wid / WAVES_N, wc = wid % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;
  const int tile = xcd_remap(blockIdx.x, a.gm * a.gn);
  const int bm = tile / a.gn, bn = tile % a.gn;
  const int grp = bm / a.npb, pb = bm - grp * a.npb;
  const int img0 = grp * NI, p0 = pb * PPT, n0 = bn * BN;
  const int HW = a.H * a.W;
  const int ylo = max(0, p0 / a.W - 1), yhi = min(a.H, (p0 + PPT - 1) / a.W + 2);
  const int q0 = ylo * a.W, nq = (yhi - ylo) * a.W;  // staged pixels [q0, q0 + nq), nq <= NSPX (host check)

  __amdgpu_buffer_rsrc_t rx[NP], rw[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    rx[p] = plane_rsrc(a.x + p * a.xps, a.xbytes);
    rw[p] = plane_rsrc(a.w + p * a.wps, a.wbytes);
  }

  // A staging: chunk q = tid + j * THREADS is 16-B piece q % CPR of slot q / CPR = pixel * NI + image
  long a_off[NCA];
  bool a_ok[NCA];
#pragma unroll
  for (int j = 0; j < NCA; ++j) {
    const int q = tid + j * THREADS;
    const int slot = q / CPR, cc = q - slot * CPR;
    const int pix = slot / NI, im = img0 + slot - pix * NI;
    a_ok[j] = q < ACH && pix < nq && im < a.N;
    a_off[j] = ((long)im * HW + q0 + pix) * a.C + cc * 8;
  }
  long b_off[NCB];
  bool b_ok[NCB];
#pragma unroll
  for (int j = 0; j < NCB; ++j) {
    const int q = tid + j * THREADS;
    if constexpr (DG) {
      const int k = q / (BN / 8), col = (q - k * (BN / 8)) * 8;
      b_ok[j] = q < BCH && n0 + col < a.Nout;
      b_off[j] = (long)k * 9 * a.Nout + n0 + col;
    } else {
      const int n = q / CPR, cc = q - n * CPR;
      b_ok[j] = q < BCH && n0 + n < a.Nout;
      b_off[j] = (long)(n0 + n) * 9 * a.C + cc * 8;
    }
  }

  // B register ring: the weight tiles of the next PD steps are in flight
  uint4 ra[NCA][NP], rb[PD][NCB][NP];
  auto load_a = [&](int c0) {
#pragma unroll
    for (int j = 0; j < NCA; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) ra[j][p] = bload(rx[p], a_off[j] + c0, a_ok[j]);
  };
  auto store_a = [&]() {
#pragma unroll
    for (int j = 0; j < NCA; ++j) {
      const int q = tid + j * THREADS;
      const int slot = q / CPR, cc = q - slot * CPR;
      if (ACH % THREADS == 0 || q < ACH) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
          *reinterpret_cast<uint4*>(As + p * A_PLANE + slot * BC + ((cc ^ swz(slot)) << 3)) = ra[j][p];
      }
    }
  };
  auto load_b = [&](int rs, int step, int cb0) {  // weight tile of step `step` (chunk cb0 + step / 9)
    const int tap = step % 9, c0 = (cb0 + step / 9) * BC;
    const long d = DG ? ((long)c0 * 9 + 8 - tap) * a.Nout : (long)tap * a.C + c0;
#pragma unroll
    for (int j = 0; j < NCB; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) rb[rs][j][p] = bload(rw[p], b_off[j] + d, b_ok[j]);
  };
  auto store_b = [&](int stage, int rs) {
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
      const int q = tid + j * THREADS;
      if (BCH % THREADS == 0 || q < BCH) {
        int idx;
        if constexpr (DG) {
          const int k = q / (BN / 8), col = (q - k * (BN / 8)) * 8;
          idx = k * BPITCH + rswz(k, col);
        } else {
          const int n = q / CPR, cc = q - n * CPR;
          idx = n * BC + ((cc ^ swz(n)) << 3);
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<uint4*>(Bs + (stage * NP + p) * B_PLANE + idx) = rb[rs][j][p];
      }
    }
  };

  // sub-tile i of this wave: position slot kp -> output position (py, px), image block ib
  int fr_py[TM], fr_px[TM], fr_ib[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int k = wr * TM + i, kp = k / SPP;
    const int pos = p0 + (int)((a.perm >> (4 * kp)) & 15u);
    fr_py[i] = pos / a.W;
    fr_px[i] = pos - fr_py[i] * a.W;
    fr_ib[i] = (k - kp * SPP) * 32;
  }

  auto frag_k = [&](const u16* base, int row, int ks) -> bf16x8 {
    const uint4 v = *reinterpret_cast<const uint4*>(base + row * BC + (((2 * ks + lh) ^ swz(row)) << 3));
    return __builtin_bit_cast(bf16x8, v);
  };
  auto frag_r = [&](const u16* base, int col0, int ks) -> bf16x8 {
    const int g = lane >> 4, idx = lane & 15;
    const int q = idx >> 2, p4 = idx & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p4;
    const int krow = 16 * ks + 8 * (g >> 1) + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const int scol = rswz(krow, col);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + krow * BPITCH + scol));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (krow + 4) * BPITCH + scol));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int tap, int stage) {
    const int r = tap / 3, s = tap - 3 * (tap / 3);
    bool v[TM];
    int sl[TM];
    bool any = false;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int iy = fr_py[i] + r - 1, ix = fr_px[i] + s - 1;
      v[i] = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;  // wave-uniform
      sl[i] = (iy * a.W + ix - q0) * NI + fr_ib[i] + li;
      any = any || v[i];
    }
    if (!any) return;
    const u16* Bst = Bs + stage * NP * B_PLANE;
#pragma unroll
    for (int ks = 0; ks < BC / 16; ++ks) {
      bf16x8 fb[TN][NP];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          if constexpr (DG)
            fb[j][p] = frag_r(Bst + p * B_PLANE, wc * WTN + j * 32, ks);
          else
            fb[j][p] = frag_k(Bst + p * B_PLANE, wc * WTN + j * 32 + li, ks);
        }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (!v[i]) continue;
        bf16x8 fa[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) fa[p] = frag_k(As + p * A_PLANE, sl[i], ks);
        using PP = PlaneProducts<NP>;
#pragma unroll
        for (int q = PP::Q0; q < 6; ++q)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<NP>(fa[PP::PA[q]], fb[j][PP::PB[q]], acc[i][j]);
      }
    }
  };

  // ---- main loop: step = (chunk, tap) as in conv_halo_kernel; the weight tile of step s sits in
  // register slot s % PD from PD steps ahead until it is written to LDS stage s & 1 ----
  const int nch = a.C / BC;
  const int cb = blockIdx.y * a.cps, ce = min(nch, cb + a.cps);
  const int nsteps = max(0, ce - cb) * 9;
  if (nsteps > 0) {
    load_a(cb * BC);
#pragma unroll
    for (int j = 0; j < PD; ++j)
      if (j < nsteps) load_b(j, j, cb);
    store_a();
    store_b(0, 0);
    if (PD < nsteps) load_b(0, PD, cb);
    if (cb + 1 < ce) load_a((cb + 1) * BC);
    __syncthreads();
    for (int s0 = 0; s0 < nsteps; s0 += PD) {
#pragma unroll
      for (int j = 0; j < PD; ++j) {
        const int st = s0 + j;
        if (st < nsteps) {
          const int tap = st % 9, ch = cb + st / 9;
          compute(tap, st & 1);
          if (st + 1 < nsteps) {
            store_b((st + 1) & 1, (j + 1) % PD);
            if (st + 1 + PD < nsteps) load_b((j + 1) % PD, st + 1 + PD, cb);
            if (tap == 8) {  // every wave is done with this chunk's image before it is replaced
              __syncthreads();
              store_a();
              if (ch + 2 < ce) load_a((ch + 2) * BC);
            }
          }
          __syncthreads();
        }
      }
    }
  }

  // ---------------- epilogue: sub-tile rows are (image, position) -> NHWC row image * HW + position
  unscale_acc<NP>(acc, a.oscale, a.obound);
  float* out = a.out + (long)blockIdx.y * a.slab;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int pos = fr_py[i] * a.W + fr_px[i];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wc * WTN + j * 32 + li;
      if (col < a.Nout) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int im = img0 + fr_ib[i] + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (im < a.N) out[((long)im * HW + pos) * a.Nout + col] = acc[i][j][r];
        }
      }
    }
  }
}

// ---------------- fp32 -> operand planes ----------------
// x [n] fp32 -> planes [NP][n] (n % 4 == 0); NP 2: the fp16 pairs of x * s
template <int NP>
__global__ __launch_bounds__(256) void split_kernel(const float* __restrict__ x, u16* __restrict__ out, long n4,
                                                    long ps, float s) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    u16 o[4][3];
    split_val<NP>(v.x, o[0], s);
    split_val<NP>(v.y, o[1], s);
    split_val<NP>(v.z, o[2], s);
    split_val<NP>(v.w, o[3], s);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      ushort4 w = make_ushort4(o[0][p], o[1][p], o[2][p], o[3][p]);
      reinterpret_cast<ushort4*>(out + p * ps)[i] = w;
    }
  }
}

// x fp32 [npix][cin] -> planes [NP][npix][cout] (channels >= cin zero): the network input, padded
// to the 8-channel operand granularity, one 16-byte chunk per pixel per plane.
template <int NP>
__global__ __launch_bounds__(256) void pad_split_kernel(const float* __restrict__ x, u16* __restrict__ out, long npix,
                                                        int cin, long ps, float s) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += stride) {
    u16 o[8][3];
#pragma unroll
    for (int c = 0; c < 8; ++c) split_val<NP>(c < cin ? x[i * cin + c] : 0.f, o[c], s);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      uint4 v;
      v.x = o[0][p] | ((unsigned)o[1][p] << 16);
      v.y = o[2][p] | ((unsigned)o[3][p] << 16);
      v.z = o[4][p] | ((unsigned)o[5][p] << 16);
      v.w = o[6][p] | ((unsigned)o[7][p] << 16);
      reinterpret_cast<uint4*>(out + p * ps)[i] = v;
    }
  }
}

template <int BM, int BN, int WM, int WN, int MODE, int NP, int BK, int NS, bool OB>
int launch_x3(const Args& a, hipStream_t st) {
  dim3 grid(a.gm * a.gn, a.splits, a.nph > 1 ? a.nph : 1);
  conv_x3_kernel<BM, BN, WM, WN, MODE, NP, BK, NS, OB><<<grid, WM * WN * 64, 0, st>>>(a);
  return (int)hipGetLastError();
}

// tile id -> (block tile, stage depth, LDS stages):
//   0: 128x128/k32/2  1: 64x64/k32/2  2: 128x128/k16/2  3: 64x64/k64/2
//   4: 128x128/k16/1  5: 128x128/k32/1  6: 64x64/k32/1  7: 256x128/k32/1 (8 waves)
//   8-11: the 128x128/k32, 128x128/k16, 256x128/k32, 64x64/k32 single-stage tiles with two register
//   tiles in flight (NSTAGE 3)
//   12-15: 128x128/k32, 128x128/k16, 256x128/k32, 64x64/k32 double-buffered with two register
//   tiles in flight (NSTAGE 4)
template <int MODE, int NP, bool OB = false>
int launch_tile(const Args& a, int tile, hipStream_t st) {
  switch (tile) {
    case 7: return launch_x3<256, 128, 4, 2, MODE, NP, 32, 1, OB>(a, st);
    case 8: return launch_x3<128, 128, 2, 2, MODE, NP, 32, 3, OB>(a, st);
    case 9: return launch_x3<128, 128, 2, 2, MODE, NP, 16, 3, OB>(a, st);
    case 10: return launch_x3<256, 128, 4, 2, MODE, NP, 32, 3, OB>(a, st);
    case 11: return launch_x3<64, 64, 1, 2, MODE, NP, 32, 3, OB>(a, st);
    case 12: return launch_x3<128, 128, 2, 2, MODE, NP, 32, 4, OB>(a, st);
    case 13: return launch_x3<128, 128, 2, 2, MODE, NP, 16, 4, OB>(a, st);
    case 14: return launch_x3<256, 128, 4, 2, MODE, NP, 32, 4, OB>(a, st);
    case 15: return launch_x3<64, 64, 1, 2, MODE, NP, 32, 4, OB>(a, st);
    case 0: return launch_x3<128, 128, 2, 2, MODE, NP, 32, 2, OB>(a, st);
    case 1: return launch_x3<64, 64, 1, 2, MODE, NP, 32, 2, OB>(a, st);
    case 2: return launch_x3<128, 128, 2, 2, MODE, NP, 16, 2, OB>(a, st);
    case 3: return launch_x3<64, 64, 1, 2, MODE, NP, 64, 2, OB>(a, st);
    case 4: return launch_x3<128, 128, 2, 2, MODE, NP, 16, 1, OB>(a, st);
    case 5: return launch_x3<128, 128, 2, 2, MODE, NP, 32, 1, OB>(a, st);
    default: return launch_x3<64, 64, 1, 2, MODE, NP, 32, 1, OB>(a, st);
  }
}

// fp32 output, or bf16 output (np == 1 only) for the generic bf16-activation path
template <int MODE>
int launch_any(const Args& a, int tile, int np, int obf, hipStream_t st) {
  if (obf) return launch_tile<MODE, 1, true>(a, tile, st);
  if (np == 2) return launch_tile<MODE, 2>(a, tile, st);
  return np == 3 ? launch_tile<MODE, 3>(a, tile, st) : launch_tile<MODE, 1>(a, tile, st);
}
// epilogue stores staged through LDS as 16-byte row pieces (conv_x3_kernel / conv_halo_kernel): measured
// faster than direct 2-/4-byte stores on every conv of the VGG and ResNet steps (docs/PERF_NOTES.md)
constexpr int ob_epi() { return 1; }
bool small_tile(int tile) { return tile == 1 || tile == 3 || tile == 6 || tile == 11 || tile == 15; }
int tile_rows(int tile) { return small_tile(tile) ? 64 : ((tile == 7 || tile == 10 || tile == 14) ? 256 : 128); }
int tile_cols(int tile) { return small_tile(tile) ? 64 : 128; }

int grid_1d(long n) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

void fill(Args& a, int N, int H, int W, int C, int R, int S, int stride, int pad) {
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

// descriptor ranges (bytes of one plane); the 32-bit buffer offsets need planes < 2 GiB
int set_bytes(Args& a, long xelems, long welems) {
  if (xelems * 2 >= (1L << 31) || welems * 2 >= (1L << 31)) return 1;
  a.xbytes = (unsigned)(xelems * 2);
  a.wbytes = (unsigned)(welems * 2);
  return 0;
}

int xsplits(int Kred, int splits) {
  const int nt = cdiv(Kred, BKMIN);
  if (splits < 1) splits = 1;
  if (splits > nt) splits = nt;
  return splits < 1 ? 1 : splits;
}

// ---- halo tiles: ids 16-21 follow the 16 implicit-GEMM tiles (3x3, stride 1, pad 1 only) ----
//   FPROP / DGRAD: 16 = 256x128 with 16-channel chunks (8 waves), 17 = 256x128 / 32,
//                  18 = 128x128 / 16 (4 waves), 19 = 128x128 / 32,
//                  20 = 256x64 / 32 (8 waves of 64x32), 21 = 128x64 / 32 (4 waves of 64x32) for
//                  64-channel outputs (e.g. the data gradient into a 64-channel layer),
//                  22 = 256x128 / 64, 23 = 256x64 / 64 (8 waves; NP 1, or NP 2 with rows <= 16 px):
//                  four k-steps of MFMAs per barrier instead of two,
//   WGRAD:         16 = 64-pixel chunks, 17 = 32-pixel chunks
bool is_halo(int tile) { return tile >= 16 && tile <= 23; }
int halo_bm(int tile) { return (tile <= 17 || tile == 20 || tile >= 22) ? 256 : 128; }
int halo_bn(int tile) { return tile == 20 || tile == 21 || tile == 23 ? 64 : 128; }
int halo_bc(int tile) { return tile >= 22 ? 64 : ((tile & 1) || tile == 20 ? 32 : 16); }

template <int BM, int BN, int WM, int WN, bool DG, int NP, int BC, bool OB>
int launch_halo(const HArgs& a, int splits, hipStream_t st) {
  dim3 grid(a.gm * a.gn, splits);
  conv_halo_kernel<BM, BN, WM, WN, DG, NP, BC, OB><<<grid, WM * WN * 64, 0, st>>>(a);
  return (int)hipGetLastError();
}

template <bool DG, int NP, bool OB>
int launch_halo_tile(const HArgs& a, int tile, int splits, hipStream_t st) {
  switch (tile) {
    case 16: return launch_halo<256, 128, 4, 2, DG, NP, 16, OB>(a, splits, st);
    case 17: return launch_halo<256, 128, 4, 2, DG, NP, 32, OB>(a, splits, st);
    case 18: return launch_halo<128, 128, 2, 2, DG, NP, 16, OB>(a, splits, st);
    case 20: return launch_halo<256, 64, 4, 2, DG, NP, 32, OB>(a, splits, st);
    case 21: return launch_halo<128, 64, 2, 2, DG, NP, 32, OB>(a, splits, st);
    case 22:
    case 23:
      if constexpr (NP == 3) {  // three planes of a 64-channel chunk do not fit the LDS
        return -6;
      } else {
        return tile == 22 ? launch_halo<256, 128, 4, 2, DG, NP, 64, OB>(a, splits, st)
                          : launch_halo<256, 64, 4, 2, DG, NP, 64, OB>(a, splits, st);
      }
    default: return launch_halo<128, 128, 2, 2, DG, NP, 32, OB>(a, splits, st);
  }
}

// -6: the conv does not fit the halo tile (channels, rows wider than the staged image allows, or
// three planes of a 64-channel chunk)
template <bool DG>
int run_halo(HArgs& a, int tile, int splits, int np, int obf, float* slab, void* out, int reduce, hipStream_t st,
             const void* add = nullptr) {
  const int BM = halo_bm(tile), BC = halo_bc(tile);
  if (a.C % BC || a.Nout % 8 || BM + 2 * a.W + 2 > halo_slots(BM, BC, np) - 1) return -6;
  if (BC >= 64 && np == 3) return -6;
  if (obf && np != 1) return -4;  // bf16 output from one-plane operands (unreduced slabs stay fp32)
  a.M = a.N * a.H * a.W;
  a.gm = cdiv(a.M, BM);
  a.gn = cdiv(a.Nout, halo_bn(tile));
  a.sepi = ob_epi();
  a.cps = cdiv(a.C / BC, splits);
  a.out = splits > 1 ? slab : (float*)out;
  a.outb = (u16*)out;
  if (add && splits > 1 && !reduce) return -4;
  a.slab = splits > 1 ? (long)a.M * a.Nout : 0;
  int rc;
  if (obf && splits == 1)
    rc = launch_halo_tile<DG, 1, true>(a, tile, splits, st);
  else if (np == 3)
    rc = launch_halo_tile<DG, 3, false>(a, tile, splits, st);
  else if (np == 2)
    rc = launch_halo_tile<DG, 2, false>(a, tile, splits, st);
  else
    rc = launch_halo_tile<DG, 1, false>(a, tile, splits, st);
  if (rc) return rc;
  if (splits == 1) return add ? dpa_add_inplace(out, add, (long)a.M * a.Nout, obf, st) : 0;
  if (!reduce) return 0;
  const long n4 = (long)a.M * a.Nout / 4;
  if (obf) return launch_splitk_reduce_t(slab, (ushort4*)out, n4, splits, st, (const ushort4*)add);
  return launch_splitk_reduce_t(slab, (float4*)out, n4, splits, st, (const float4*)add);
}

int halo_bytes(unsigned& xb, long xel, unsigned& wb, long wel) {
  if (xel * 2 >= (1L << 31) || wel * 2 >= (1L << 31)) return -5;
  xb = (unsigned)(xel * 2);
  wb = (unsigned)(wel * 2);
  return 0;
}

template <int NP, int P>
int launch_halo_wgrad(const WHArgs& a, int splits, hipStream_t st) {
  dim3 grid(a.gk * a.gc, splits);
  conv_halo_wgrad_kernel<NP, P><<<grid, 256, 0, st>>>(a);
  return (int)hipGetLastError();
}

int run_halo_wgrad(WHArgs& a, int tile, int splits, int np, float* dw, float* slab, hipStream_t st) {
  if (tile != 16 && tile != 17) return -6;
  const int P = tile == 16 ? 64 : 32;
  if (a.C % 8 || a.K % 8 || P + 2 * a.W + 2 > halo_wslots(P) - 1) return -6;
  a.M = a.N * a.H * a.W;
  if (halo_bytes(a.xbytes, (long)a.M * a.C, a.dzbytes, (long)a.M * a.K)) return -5;
  a.nchunks = cdiv(a.M, P);
  a.gk = cdiv(a.K, 128);
  a.gc = cdiv(a.C, 32);
  a.cps = cdiv(a.nchunks, splits);
  a.fd_HW = make_fastdiv(a.H * a.W);
  a.fd_W = make_fastdiv(a.W);
  a.out = splits > 1 ? slab : dw;
  a.slab = splits > 1 ? (long)a.K * 9 * a.C : 0;
  int rc;
  if (np == 3)
    rc = P == 64 ? launch_halo_wgrad<3, 64>(a, splits, st) : launch_halo_wgrad<3, 32>(a, splits, st);
  else if (np == 2)
    rc = P == 64 ? launch_halo_wgrad<2, 64>(a, splits, st) : launch_halo_wgrad<2, 32>(a, splits, st);
  else
    rc = P == 64 ? launch_halo_wgrad<1, 64>(a, splits, st) : launch_halo_wgrad<1, 32>(a, splits, st);
  if (rc || splits == 1) return rc;
  return launch_splitk_reduce(slab, dw, (long)a.K * 9 * a.C / 4, splits, st);
}


// ---- streaming GEMM tile (1x1 / stride 1 / pad 0 forward, bf16 in and out, one split): id 30 ----
bool is_stream(int tile) { return tile == 30; }

// -6: the call does not fit the streaming kernel (it is tuned as a candidate alongside the others)
int run_stream(const u16* x, const u16* w, void* out, int M, int N, int K, int np, int obf, int splits,
               float* stats, hipStream_t st, bool dgrad = false) {
  if (np != 1 || !obf || splits != 1 || K % 8 || N % 8) return -6;
  SArgs s{};
  s.x = x;
  s.w = w;
  if ((long)M * K * 2 >= (1L << 31) || (long)N * K * 2 >= (1L << 31)) return -5;
  s.xbytes = (unsigned)((long)M * K * 2);
  s.wbytes = (unsigned)((long)N * K * 2);
  s.out = (u16*)out;
  s.M = M;
  s.N = N;
  s.K = K;
  s.gm = cdiv(M, 256);
  s.gn = cdiv(N, 128);
  s.stats = reinterpret_cast<float2*>(stats);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = std::min(s.gm * s.gn, 2 * cus);
  if (dgrad) {
    gemm_stream_kernel<256, 128, 4, 2, 32, true><<<grid, 512, 0, st>>>(s);
  } else {
    gemm_stream_kernel<256, 128, 4, 2, 32, false><<<grid, 512, 0, st>>>(s);
  }
  return (int)hipGetLastError();
}

// ---- position-major tiles (small images): ids 24-29 ----
//   24 / 25: 256 rows (32 images x 8 positions) x 128, 4x2 waves, 32-channel chunks, <= 12 staged
//            pixels (4x4 images), weight tiles 1 / 4 steps ahead
//   26:      256 rows (64 images x 4 positions) x 128, 4x2 waves, 32-channel chunks, <= 4 staged pixels
//   27 / 28: 256 rows (64 images x 4 positions) x 64, 4x2 waves of 64x32, 32-channel chunks, <= 4
//            staged pixels (2x2 images), weight tiles 1 / 4 steps ahead
//   29:      as 24 with 16-channel chunks
bool is_pos(int tile) { return tile >= 24 && tile <= 29; }
int pos_bm(int) { return 256; }
int pos_ni(int tile) { return (tile >= 26 && tile <= 28) ? 64 : 32; }
int pos_bn(int tile) { return (tile == 27 || tile == 28) ? 64 : 128; }
int pos_bc(int tile) { return tile == 29 ? 16 : 32; }
int pos_nspx(int tile) { return (tile >= 26 && tile <= 28) ? 4 : 12; }
int pos_waves_m(int) { return 4; }

// staged pixels of the worst position block, or -1 when the positions do not tile the image
int pos_staged(int H, int W, int ppt) {
  if (H < 2 || W < 2 || (H * W) % ppt) return -1;
  int worst = 0;
  for (int p0 = 0; p0 < H * W; p0 += ppt) {
    const int ylo = std::max(0, p0 / W - 1), yhi = std::min(H, (p0 + ppt - 1) / W + 2);
    worst = std::max(worst, (yhi - ylo) * W);
  }
  return worst;
}

// Position order of a tile (4 bits per slot): longest-processing-time assignment of the positions of
// the first position block to the row waves (PPT / waves_m positions each), by in-image tap count.
unsigned pos_perm(int H, int W, int ppt, int waves_m) {
  const int per = std::max(1, ppt / waves_m), groups = ppt / per;
  int cnt[8], order[8], gsum[8] = {0}, gn[8] = {0}, slot[8][8];
  for (int l = 0; l < ppt; ++l) {
    const int y = l / W, x = l % W;
    const int ry = 3 - (y == 0) - (y == H - 1), rx = 3 - (x == 0) - (x == W - 1);
    cnt[l] = ry * rx;
    order[l] = l;
  }
  std::stable_sort(order, order + ppt, [&](int u, int v) { return cnt[u] > cnt[v]; });
  for (int t = 0; t < ppt; ++t) {
    int best = -1;
    for (int g = 0; g < groups; ++g)
      if (gn[g] < per && (best < 0 || gsum[g] < gsum[best])) best = g;
    slot[best][gn[best]++] = order[t];
    gsum[best] += cnt[order[t]];
  }
  unsigned perm = 0;
  int k = 0;
  for (int g = 0; g < groups; ++g)
    for (int e = 0; e < per; ++e) perm |= (unsigned)slot[g][e] << (4 * k++);
  return perm;
}

template <int BM, int BN, int WM, int WN, bool DG, int NP, int BC, int NI, int NSPX, int PD>
int launch_pos(const PArgs& a, int splits, hipStream_t st) {
  dim3 grid(a.gm * a.gn, splits);
  conv_pos_kernel<BM, BN, WM, WN, DG, NP, BC, NI, NSPX, PD><<<grid, WM * WN * 64, 0, st>>>(a);
  return (int)hipGetLastError();
}

template <bool DG, int NP>
int launch_pos_tile(const PArgs& a, int tile, int splits, hipStream_t st) {
  switch (tile) {
    case 24: return launch_pos<256, 128, 4, 2, DG, NP, 32, 32, 12, 1>(a, splits, st);
    case 25: return launch_pos<256, 128, 4, 2, DG, NP, 32, 32, 12, 4>(a, splits, st);
    case 26: return launch_pos<256, 128, 4, 2, DG, NP, 32, 64, 4, 1>(a, splits, st);
    case 27: return launch_pos<256, 64, 4, 2, DG, NP, 32, 64, 4, 1>(a, splits, st);
    case 28: return launch_pos<256, 64, 4, 2, DG, NP, 32, 64, 4, 4>(a, splits, st);
    default: return launch_pos<256, 128, 4, 2, DG, NP, 16, 32, 12, 1>(a, splits, st);
  }
}

// -6: the conv does not fit the tile (channels, or more staged pixels than the tile holds)
template <bool DG>
int run_pos(PArgs& a, int tile, int splits, int np, int obf, float* slab, void* out, int reduce, hipStream_t st,
            const void* add = nullptr) {
  const int BM = pos_bm(tile), NI = pos_ni(tile), BC = pos_bc(tile), ppt = BM / NI;
  const int ns = pos_staged(a.H, a.W, ppt);
  if (obf || a.C % BC || a.Nout % 8 || ns < 0 || ns > pos_nspx(tile)) return -6;
  if (add && splits > 1 && !reduce) return -4;
  const long M = (long)a.N * a.H * a.W;
  a.npb = a.H * a.W / ppt;
  a.perm = pos_perm(a.H, a.W, ppt, pos_waves_m(tile));
  a.gm = cdiv(a.N, NI) * a.npb;
  a.gn = cdiv(a.Nout, pos_bn(tile));
  a.cps = cdiv(a.C / BC, splits);
  a.out = splits > 1 ? slab : (float*)out;
  a.slab = splits > 1 ? M * a.Nout : 0;
  const int rc = np == 3   ? launch_pos_tile<DG, 3>(a, tile, splits, st)
                 : np == 2 ? launch_pos_tile<DG, 2>(a, tile, splits, st)
                           : launch_pos_tile<DG, 1>(a, tile, splits, st);
  if (rc) return rc;
  if (splits == 1) return add ? dpa_add_inplace(out, add, M * a.Nout, 0, st) : 0;
  if (!reduce) return 0;
  return launch_splitk_reduce_t(slab, (float4*)out, M * a.Nout / 4, splits, st, (const float4*)add);
}

}  // namespace

extern "C" {

int dpa_x3_splits(int Kred, int splits) { return xsplits(Kred, splits); }

// rows per row tile of fprop tile `tile` (the stats partial row block), 0 if it cannot emit stats
int dpa_conv_stats_rows(int tile) {
  return is_pos(tile) ? 0 : (is_stream(tile) ? 256 : (is_halo(tile) ? halo_bm(tile) : tile_rows(tile)));
}

// x planes [NP][N,H,W,C] (plane stride xps), w planes [NP][Kout][R][S][C] (stride wps; for a data
// gradient pass the flipped/transposed Wd planes), out fp32 [N,P,Q,Kout] (or slabs, see
// conv_gemm.hip).  np: 1 (bf16), 3 (fp32 via bf16x6) or 2 (fp32 via fp16 pairs; outputs times
// h2_out_scale(oscale, obound)).  tile: 0 = 128x128, 1 = 64x64.
// posmajor: bit 0 = position-major GEMM rows, bit 1 = column-tile-outer block order (Args.nmajor;
// implicit-GEMM tiles only, the halo kernels ignore it).
// stats (optional, one split, implicit-GEMM or halo tiles): float2 [Kout][row tiles of conv_stats_rows]
// BN (mean, M2) partials of the output, channel-major (epi_col_stats), for dpa_bn_finalize_cm.
int dpa_conv_x3_fprop(const u16* x, long xps, const u16* w, long wps, void* out, float* slab, int N, int H, int W,
                      int C, int Kout, int R, int S, int stride, int pad, int splits, int tile, int reduce,
                      int posmajor, int np, int obf, hipStream_t st, float* stats, float oscale,
                      const unsigned* obound) {
  if (stats && (is_pos(tile) || (is_halo(tile) ? xsplits(9 * C, splits) : xsplits(R * S * C, splits)) > 1)) return -7;
  if (is_stream(tile)) {
    if (R != 1 || S != 1 || stride != 1 || pad != 0) return -6;
    return run_stream(x, w, out, N * H * W, Kout, C, np, obf, xsplits(C, splits), stats, st);
  }
  if (is_halo(tile)) {
    if (stride != 1 || pad != 1 || R != 3 || S != 3) return -6;
    HArgs h{};
    h.oscale = oscale;
    h.obound = obound;
    h.x = x;
    h.xps = xps;
    h.w = w;
    h.wps = wps;
    h.N = N;
    h.H = H;
    h.W = W;
    h.C = C;
    h.Nout = Kout;
    h.stats = reinterpret_cast<float2*>(stats);
    if (halo_bytes(h.xbytes, (long)N * H * W * C, h.wbytes, (long)Kout * 9 * C)) return -5;
    return run_halo<false>(h, tile, xsplits(9 * C, splits), np, obf, slab, out, reduce, st);
  }
  if (is_pos(tile)) {
    if (stride != 1 || pad != 1 || R != 3 || S != 3) return -6;
    PArgs q{};
    q.oscale = oscale;
    q.obound = obound;
    q.x = x;
    q.xps = xps;
    q.w = w;
    q.wps = wps;
    q.N = N;
    q.H = H;
    q.W = W;
    q.C = C;
    q.Nout = Kout;
    if (halo_bytes(q.xbytes, (long)N * H * W * C, q.wbytes, (long)Kout * 9 * C)) return -5;
    return run_pos<false>(q, tile, xsplits(9 * C, splits), np, obf, slab, out, reduce, st);
  }
  Args a{};
  a.oscale = oscale;
  a.obound = obound;
  a.x = x;
  a.xps = xps;
  a.w = w;
  a.wps = wps;
  fill(a, N, H, W, C, R, S, stride, pad);
  a.Nout = Kout;
  if (C % 8 || Kout % 8) return -2;
  if (set_bytes(a, (long)N * H * W * C, (long)Kout * a.Ktot)) return -5;
  a.gm = cdiv(a.M, tile_rows(tile));
  a.gn = cdiv(Kout, tile_cols(tile));
  a.splits = xsplits(a.Ktot, splits);
  a.posmajor = posmajor & 1;
  a.nmajor = (posmajor >> 1) & 1;
  a.stats = reinterpret_cast<float2*>(stats);
  a.sepi = ob_epi();
  if (obf && np != 1) return -4;
  a.out = a.splits > 1 ? slab : (float*)out;
  a.outb = (u16*)out;
  a.slab = a.splits > 1 ? (long)a.M * Kout : 0;
  const int rc = launch_any<XM_FPROP>(a, tile, np, obf && a.splits == 1, st);
  if (rc) return rc;
  if (a.splits > 1 && reduce) {
    const long n4 = (long)a.M * Kout / 4;
    if (obf) return launch_splitk_reduce_t(slab, (ushort4*)out, n4, a.splits, st);
    return launch_splitk_reduce(slab, (float*)out, n4, a.splits, st);
  }
  return 0;
}

// Data gradient of conv(x [N,H,W,C], w [K,R,S,C], stride, pad) -> dZ [N,Hd,Wd,K]:
// dx [N,H,W,C] fp32 (or slabs) from dz planes [NP][N,Hd,Wd,K] and the forward weight planes.
// stride must be a power of two.
// add (optional, dx's type): dx = dgrad + add -- a second gradient contribution to the same tensor.
// With split-K it is folded into the reduction (no extra pass); with one split an in-place add
// follows (an epilogue read of the addend made the bf16 dgrad kernels ~1.7x slower: the loads sit
// in front of the stores).
int dpa_conv_x3_dgrad(const u16* dz, long dzps, const u16* w, long wps, void* dx, float* slab, int N, int Hd, int Wd,
                      int K, int C, int R, int S, int stride, int pad, int H, int W, int splits, int tile, int reduce,
                      int posmajor, int np, int obf, hipStream_t st, const void* add, int* sig, int sig_val,
                      float oscale, const unsigned* obound) {
  if (is_stream(tile)) {  // dX = dZ W for a 1x1 / stride-1 conv (W [K][C] read row-contiguous)
    if (R != 1 || S != 1 || stride != 1 || pad != 0 || sig) return -6;
    const int rc = run_stream(dz, w, dx, N * H * W, C, K, np, obf, xsplits(K, splits), nullptr, st, true);
    if (rc || !add) return rc;
    return dpa_add_inplace(dx, add, (long)N * H * W * C, obf, st);
  }
  if (is_halo(tile)) {
    if (stride != 1 || pad != 1 || R != 3 || S != 3 || Hd != H || Wd != W) return -6;
    HArgs h{};
    h.oscale = oscale;
    h.obound = obound;
    h.sig = sig;
    h.sig_val = sig_val;
    h.x = dz;
    h.xps = dzps;
    h.w = w;
    h.wps = wps;
    h.N = N;
    h.H = H;
    h.W = W;
    h.C = K;
    h.Nout = C;
    if (halo_bytes(h.xbytes, (long)N * H * W * K, h.wbytes, (long)K * 9 * C)) return -5;
    return run_halo<true>(h, tile, xsplits(9 * K, splits), np, obf, slab, dx, reduce, st, add);
  }
  if (is_pos(tile)) {
    if (stride != 1 || pad != 1 || R != 3 || S != 3 || Hd != H || Wd != W) return -6;
    PArgs q{};
    q.oscale = oscale;
    q.obound = obound;
    q.sig = sig;
    q.sig_val = sig_val;
    q.x = dz;
    q.xps = dzps;
    q.w = w;
    q.wps = wps;
    q.N = N;
    q.H = H;
    q.W = W;
    q.C = K;
    q.Nout = C;
    if (halo_bytes(q.xbytes, (long)N * H * W * K, q.wbytes, (long)K * 9 * C)) return -5;
    return run_pos<true>(q, tile, xsplits(9 * K, splits), np, obf, slab, dx, reduce, st, add);
  }
  Args a{};
  a.oscale = oscale;
  a.obound = obound;
  a.sig = sig;
  a.sig_val = sig_val;
  a.x = dz;
  a.xps = dzps;
  a.w = w;
  a.wps = wps;
  if (stride < 1 || (stride & (stride - 1)) || R - 1 - pad < 0) return -3;
  const int padd = R - 1 - pad;  // padding of the dilated-dZ gather
  fill(a, N, Hd, Wd, K, R, S, 1, padd);
  if (set_bytes(a, (long)N * Hd * Wd * K, (long)K * R * S * C)) return -5;
  const long Mfull = (long)N * H * W;
  // stride 2 with even output sides: phase-decomposed (Args.phase); DPA_DGRAD_PHASE=0 keeps the
  // dilated form (A/B)
  const char* phase_env = getenv("DPA_DGRAD_PHASE");  // read per call: tests switch it in-process
  const bool phase_on = !(phase_env && phase_env[0] == '0');
  const bool phased = phase_on && stride == 2 && H % 2 == 0 && W % 2 == 0 && (posmajor & 1) == 0;
  a.nph = 1;
  if (phased) {
    a.nph = 4;
    a.outH = H;
    a.outW = W;
    a.P = H / 2;
    a.Q = W / 2;
    int kmax = 0;
    for (int z = 0; z < 4; ++z) {
      Args::Phase& q = a.phase[z];
      const int zh = z >> 1, zw = z & 1;
      q.r0 = (padd - zh) & 1;  // first tap with (h - padd + r) even for h = 2i + zh
      q.s0 = (padd - zw) & 1;
      const int Rp = q.r0 < R ? (R - q.r0 + 1) / 2 : 0, Sp = q.s0 < S ? (S - q.s0 + 1) / 2 : 0;
      q.S = Sp > 0 ? Sp : 1;
      q.fd_S = make_fastdiv(q.S);
      q.Ktot = Rp * Sp * K;
      // tap r0 + 2r' of phase row i reads dZ row i + r' + (zh - padd + r0) / 2
      q.padh = -((zh - padd + q.r0) / 2);
      q.padw = -((zw - padd + q.s0) / 2);
      kmax = std::max(kmax, q.Ktot);
    }
    a.Ktot = kmax;
  } else {
    a.P = H;
    a.Q = W;
    a.imask = stride - 1;
    while ((1 << a.ishift) < stride) ++a.ishift;
  }
  a.M = N * a.P * a.Q;
  a.fd_Q = make_fastdiv(a.Q);
  a.fd_PQ = make_fastdiv(a.P * a.Q);
  a.Nout = C;
  if (C % 8 || K % 8) return -2;
  a.gm = cdiv(a.M, tile_rows(tile));
  a.gn = cdiv(C, tile_cols(tile));
  a.splits = xsplits(a.Ktot, splits);
  a.posmajor = posmajor & 1;
  a.nmajor = (posmajor >> 1) & 1;
  a.sepi = ob_epi();
  if (obf && np != 1) return -4;
  a.out = a.splits > 1 ? slab : (float*)dx;
  a.outb = (u16*)dx;
  if (add && a.splits > 1 && !reduce) return -4;
  a.slab = a.splits > 1 ? Mfull * C : 0;
  const int rc = launch_any<XM_DGRAD>(a, tile, np, obf && a.splits == 1, st);
  if (rc) return rc;
  if (a.splits == 1 && add) return dpa_add_inplace(dx, add, Mfull * C, obf, st);
  if (a.splits > 1 && reduce) {
    const long n4 = Mfull * C / 4;
    if (obf) return launch_splitk_reduce_t(slab, (ushort4*)dx, n4, a.splits, st, (const ushort4*)add);
    return launch_splitk_reduce_t(slab, (float4*)dx, n4, a.splits, st, (const float4*)add);
  }
  return 0;
}

// dW[Kout][R*S*C] = sum_m dZ[m][kout] Xcol[m][rsc]; x planes [NP][N,H,W,C], dz planes [NP][N,P,Q,Kout]
int dpa_conv_x3_wgrad(const u16* x, long xps, const u16* dz, long dzps, float* dw, float* slab, int N, int H, int W,
                      int C, int Kout, int R, int S, int stride, int pad, int splits, int tile, int posmajor, int np,
                      hipStream_t st, float oscale, const unsigned* obound) {
  if (is_halo(tile)) {
    if (stride != 1 || pad != 1 || R != 3 || S != 3) return -6;
    WHArgs h{};
    h.oscale = oscale;
    h.obound = obound;
    h.x = x;
    h.xps = xps;
    h.dz = dz;
    h.dzps = dzps;
    h.N = N;
    h.H = H;
    h.W = W;
    h.C = C;
    h.K = Kout;
    return run_halo_wgrad(h, tile, xsplits(N * H * W, splits), np, dw, slab, st);
  }
  Args a{};
  a.oscale = oscale;
  a.obound = obound;
  a.x = x;
  a.xps = xps;
  a.w = dz;
  a.wps = dzps;
  fill(a, N, H, W, C, R, S, stride, pad);
  if (set_bytes(a, (long)N * H * W * C, (long)a.M * Kout)) return -5;
  a.Nout = Kout;
  if (C % 8 || Kout % 8) return -2;
  a.gm = cdiv(Kout, tile_rows(tile));
  a.gn = cdiv(a.Ktot, tile_cols(tile));
  a.splits = xsplits(a.M, splits);
  a.posmajor = posmajor & 1;
  a.nmajor = (posmajor >> 1) & 1;
  a.out = a.splits > 1 ? slab : dw;
  a.slab = a.splits > 1 ? (long)Kout * a.Ktot : 0;
  a.sepi = ob_epi();
  const int rc = np == 3   ? launch_tile<XM_WGRAD, 3>(a, tile, st)
                 : np == 2 ? launch_tile<XM_WGRAD, 2>(a, tile, st)
                           : launch_tile<XM_WGRAD, 1>(a, tile, st);
  if (rc) return rc;
  if (a.splits > 1) {
    const long n4 = (long)Kout * a.Ktot / 4;
    return launch_splitk_reduce(slab, dw, n4, a.splits, st);
  }
  return 0;
}

// np 2: the fp16 pairs of x * scale (scale a power of two; conv outputs divide it out)
int dpa_split_planes(const float* x, u16* out, long n, long ps, int np, float scale, hipStream_t st) {
  if (n % 4) return -2;
  if (np == 3)
    split_kernel<3><<<grid_1d(n / 4), 256, 0, st>>>(x, out, n / 4, ps, 1.f);
  else if (np == 2)
    split_kernel<2><<<grid_1d(n / 4), 256, 0, st>>>(x, out, n / 4, ps, scale);
  else
    split_kernel<1><<<grid_1d(n / 4), 256, 0, st>>>(x, out, n / 4, ps, 1.f);
  return (int)hipGetLastError();
}

// np 2: activation planes (scale H2_SA)
int dpa_pad_split8(const float* x, u16* out, long npix, int cin, long ps, int np, hipStream_t st) {
  if (cin > 8) return -2;
  if (np == 3)
    pad_split_kernel<3><<<grid_1d(npix), 256, 0, st>>>(x, out, npix, cin, ps, 1.f);
  else if (np == 2)
    pad_split_kernel<2><<<grid_1d(npix), 256, 0, st>>>(x, out, npix, cin, ps, H2_SA);
  else
    pad_split_kernel<1><<<grid_1d(npix), 256, 0, st>>>(x, out, npix, cin, ps, 1.f);
  return (int)hipGetLastError();
}

DPA_H2_OVF_ACCESSOR(dpa_h2_ovf_conv)

}  // extern "C"
