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

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
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
  int imask, ishift;  // input dilation (DGRAD of a strided conv): 2^ishift, imask = 2^ishift - 1
  FastDiv fd_C, fd_S, fd_Q, fd_PQ, fd_N;
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
  const int bm = tile / a.gn, bn = tile % a.gn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int split = blockIdx.y;

  // ---------------- reduction tile iterator with padding-tap skipping ----------------
  bool skip = false;
  int lo0 = 0, lo1 = 0, span1 = 1, per = 1, ntot;
  if constexpr (!WG) {
    ntot = (a.Ktot + BK - 1) / BK;
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
  const int KMAX = WG ? a.M : a.Ktot;

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
        a_ih0[j] = (int)oh * a.stride - a.pad;
        a_iw0[j] = (int)ow * a.stride - a.pad;
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
      const unsigned r = fdiv(tap, a.fd_S);
      const int s = (int)(tap - r * a.S);
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
          const unsigned rr = fdiv(tp, a.fd_S);
          const int ss = (int)(tp - rr * a.S);
          const long boff = (((long)ko * a.R + (a.R - 1 - (int)rr)) * a.S + (a.S - 1 - ss)) * a.Nout + col;
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
    // smallest products first
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (NP == 3) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], acc[i][j], 0, 0, 0);
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0);
      }
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
  float* out = a.out + (long)split * a.slab;
  const int ldc = WG ? a.Ktot : a.Nout;
  const int nrows = WG ? a.Nout : a.M;
  const int ncols = WG ? a.Ktot : a.Nout;
  const bool remap = !WG && a.posmajor;
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
            if constexpr (OB)
              a.outb[mrow * ldc + col] = bf16_rne(acc[i][j][r]);
            else
              out[mrow * ldc + col] = acc[i][j][r];
          }
        }
      }
    }
}


// ---------------- fp32 -> bf16 planes ----------------
// x [n] fp32 -> planes [NP][n] (n % 4 == 0)
template <int NP>
__global__ __launch_bounds__(256) void split_kernel(const float* __restrict__ x, u16* __restrict__ out, long n4,
                                                    long ps) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    u16 o[4][3];
    split_val<NP>(v.x, o[0]);
    split_val<NP>(v.y, o[1]);
    split_val<NP>(v.z, o[2]);
    split_val<NP>(v.w, o[3]);
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
                                                        int cin, long ps) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += stride) {
    u16 o[8][3];
#pragma unroll
    for (int c = 0; c < 8; ++c) split_val<NP>(c < cin ? x[i * cin + c] : 0.f, o[c]);
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
  dim3 grid(a.gm * a.gn, a.splits);
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
  return np == 3 ? launch_tile<MODE, 3>(a, tile, st) : launch_tile<MODE, 1>(a, tile, st);
}
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

}  // namespace

extern "C" {

int dpa_x3_splits(int Kred, int splits) { return xsplits(Kred, splits); }

// x planes [NP][N,H,W,C] (plane stride xps), w planes [NP][Kout][R][S][C] (stride wps; for a data
// gradient pass the flipped/transposed Wd planes), out fp32 [N,P,Q,Kout] (or slabs, see
// conv_gemm.hip).  np: 1 (bf16) or 3 (fp32 via bf16x6).  tile: 0 = 128x128, 1 = 64x64.
int dpa_conv_x3_fprop(const u16* x, long xps, const u16* w, long wps, void* out, float* slab, int N, int H, int W,
                      int C, int Kout, int R, int S, int stride, int pad, int splits, int tile, int reduce,
                      int posmajor, int np, int obf, hipStream_t st) {
  Args a{};
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
  a.posmajor = posmajor ? 1 : 0;
  if (obf && (np != 1 || (a.splits > 1 && !reduce))) return -4;
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
int dpa_conv_x3_dgrad(const u16* dz, long dzps, const u16* w, long wps, void* dx, float* slab, int N, int Hd, int Wd,
                      int K, int C, int R, int S, int stride, int pad, int H, int W, int splits, int tile, int reduce,
                      int posmajor, int np, int obf, hipStream_t st) {
  Args a{};
  a.x = dz;
  a.xps = dzps;
  a.w = w;
  a.wps = wps;
  if (stride < 1 || (stride & (stride - 1)) || R - 1 - pad < 0) return -3;
  fill(a, N, Hd, Wd, K, R, S, 1, R - 1 - pad);
  if (set_bytes(a, (long)N * Hd * Wd * K, (long)K * R * S * C)) return -5;
  a.P = H;
  a.Q = W;
  a.M = N * H * W;
  a.fd_Q = make_fastdiv(W);
  a.fd_PQ = make_fastdiv(H * W);
  a.imask = stride - 1;
  while ((1 << a.ishift) < stride) ++a.ishift;
  a.Nout = C;
  if (C % 8 || K % 8) return -2;
  a.gm = cdiv(a.M, tile_rows(tile));
  a.gn = cdiv(C, tile_cols(tile));
  a.splits = xsplits(a.Ktot, splits);
  a.posmajor = posmajor ? 1 : 0;
  if (obf && (np != 1 || (a.splits > 1 && !reduce))) return -4;
  a.out = a.splits > 1 ? slab : (float*)dx;
  a.outb = (u16*)dx;
  a.slab = a.splits > 1 ? (long)a.M * C : 0;
  const int rc = launch_any<XM_DGRAD>(a, tile, np, obf && a.splits == 1, st);
  if (rc) return rc;
  if (a.splits > 1 && reduce) {
    const long n4 = (long)a.M * C / 4;
    if (obf) return launch_splitk_reduce_t(slab, (ushort4*)dx, n4, a.splits, st);
    return launch_splitk_reduce(slab, (float*)dx, n4, a.splits, st);
  }
  return 0;
}

// dW[Kout][R*S*C] = sum_m dZ[m][kout] Xcol[m][rsc]; x planes [NP][N,H,W,C], dz planes [NP][N,P,Q,Kout]
int dpa_conv_x3_wgrad(const u16* x, long xps, const u16* dz, long dzps, float* dw, float* slab, int N, int H, int W,
                      int C, int Kout, int R, int S, int stride, int pad, int splits, int tile, int posmajor, int np,
                      hipStream_t st) {
  Args a{};
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
  a.posmajor = posmajor ? 1 : 0;
  a.out = a.splits > 1 ? slab : dw;
  a.slab = a.splits > 1 ? (long)Kout * a.Ktot : 0;
  const int rc = np == 3 ? launch_tile<XM_WGRAD, 3>(a, tile, st) : launch_tile<XM_WGRAD, 1>(a, tile, st);
  if (rc) return rc;
  if (a.splits > 1) {
    const long n4 = (long)Kout * a.Ktot / 4;
    return launch_splitk_reduce(slab, dw, n4, a.splits, st);
  }
  return 0;
}

int dpa_split_planes(const float* x, u16* out, long n, long ps, int np, hipStream_t st) {
  if (n % 4) return -2;
  if (np == 3)
    split_kernel<3><<<grid_1d(n / 4), 256, 0, st>>>(x, out, n / 4, ps);
  else
    split_kernel<1><<<grid_1d(n / 4), 256, 0, st>>>(x, out, n / 4, ps);
  return (int)hipGetLastError();
}

int dpa_pad_split8(const float* x, u16* out, long npix, int cin, long ps, int np, hipStream_t st) {
  if (cin > 8) return -2;
  if (np == 3)
    pad_split_kernel<3><<<grid_1d(npix), 256, 0, st>>>(x, out, npix, cin, ps);
  else
    pad_split_kernel<1><<<grid_1d(npix), 256, 0, st>>>(x, out, npix, cin, ps);
  return (int)hipGetLastError();
}

}  // extern "C"
