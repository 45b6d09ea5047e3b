// K4-K6 in ONE launch per layer: training BatchNorm2d (+ReLU, +2x2/s2 max-pool), forward and
// backward, for the small activations of the VGG tail (model.py:16,24,25).
//
// bn.hip runs a BN layer as three kernels (statistics -> finalize -> apply).  On the 2x2..8x8
// layers every one of them moves only 2-16 MB, so each costs a kernel boundary plus a
// latency-bound ramp (profiles/r2_s3_final_x3_step_timeline.txt: 5-11 us apiece, 16-20 us per
// layer and direction).  Here one launch does all three:
//
//   * the grid is (channel slices of CS = 4*CL channels) x (R row blocks); a 256-thread block owns
//     RB = RL*U row units (RL = 256/CL row lanes, U units per thread) of its slice and KEEPS ITS
//     WHOLE TILE IN REGISTERS (a row unit is one pixel, or one 2x2 pool window = 4 pixels);
//   * it reduces its tile to per-channel partials (forward: exact two-pass (mean, M2) of the tile;
//     backward: sum dy, sum dy*xhat, sum xhat), publishes them, and takes a ticket on its slice's
//     arrival counter;
//   * every block of the slice waits until the slice's R partials are in (bounded spin), then
//     merges them in ONE fixed order — every block computes bit-identical coefficients, no
//     atomics on data, deterministic — and applies them to the tile it still holds:
//     forward writes relu(BN(z)) (max-pooled) as fp32 or bf16 operand planes, backward writes dz.
//
// Cross-workgroup hand-off (cdna_hip_programming.md §6 Guideline 16): plain partial stores ->
// every storing wave s_waitcnt vmcnt(0) -> barrier -> one lane: agent-scope release fence, asm
// vmcnt(0), relaxed agent fetch_add on the slice counter; the consumer: one lane polls the counter
// relaxed (s_sleep between polls), one agent-scope acquire, vmcnt(0), barrier, then plain loads.
// The counters are self-resetting: after the merge every block adds to the slice's departure
// counter and the last departer zeroes both (no block of this launch polls any more by then; the
// next launch is stream-ordered behind this one).  The workspace is zeroed once at allocation.
//
// Residency: a slice's R blocks must run concurrently.  Blocks are numbered slice-major and the
// dispatcher places them in order, so the rendezvous can only stall while other kernels (the
// weight-gradient stream, RCCL) hold the CUs it needs -- they never wait for this kernel, so the
// stall ends when they do.  The geometry query refuses (the engine then runs the three-kernel BN)
// any grid above 512 blocks and any slice of R blocks above half of the chip's co-resident capacity
// for this kernel (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs, or DPA_BN_FUSED_CAP blocks
// when set: tests force the fallback with it) -- half, so a slice still fits while the other
// stream's kernels hold the rest of the chip.  A block that waits longer than `ticks` of the wall clock (the
// engine's own short bound, DPA_BN_FUSED_TIMEOUT_US, 2 s by default) sets tmo[0] = 1 and continues
// (garbage, never a hang; the engine raises on the word after the step).
#include "common.h"

namespace {

constexpr int FT = 256;  // threads per block

struct FArgs {
  const float* src;  // forward: z or nsplit slabs of it; backward: g (pooled shape) or slabs of it
  long slab;         // elements per slab
  int nsplit;
  float* zw;         // forward: z written when nsplit > 1
  const float* z;    // backward: the forward conv output z [N,H,W,C]
  int N, H, W, C;
  int R;             // row blocks per slice
  float* part;       // [slices * R][PF][CS]
  unsigned* cnt;     // [slices][32]: word 0 arrivals, word 16 departures
  const float* gamma;
  const float* beta;
  const float* bias;
  float* rmean;
  float* rvar;
  long long* nbt;
  float* mean;    // forward out / backward in
  float* invstd;  // forward out / backward in
  float* scale;   // forward out / backward in (the ReLU / pool routing)
  float* shift;
  float* dgamma;  // backward outputs
  float* dbeta;
  float* dbias;
  float* out;     // fp32 output (NP == 0): forward a, backward dz
  u16* out3;      // bf16 planes (NP > 0)
  long ps;        // plane stride
  int apply;      // forward: 0 = statistics and coefficients only (the consumer applies them)
  float momentum, eps;
  int* tmo;
  unsigned long long ticks;
  int phantom;  // tests only (DPA_BN_FUSED_TEST_PHANTOM): wait for R + phantom arrivals, i.e. time out
  int* sig;  // optional kernel-start stream signal (common.h start_signal)
  int sig_val;
};

__device__ __forceinline__ float4 ld4g(const float* p, long i4) { return reinterpret_cast<const float4*>(p)[i4]; }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float gk(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

template <int NP>
__device__ __forceinline__ void store_out(const FArgs& a, long i4, float4 v) {
  if constexpr (NP == 0) {
    reinterpret_cast<float4*>(a.out)[i4] = v;
  } else {
    u16 o[4][3];
    constexpr float s = NP == 2 ? H2_SA : 1.f;  // (fp16 pairs: activation planes only, forward)
    split_val<NP>(v.x, o[0], s);
    split_val<NP>(v.y, o[1], s);
    split_val<NP>(v.z, o[2], s);
    split_val<NP>(v.w, o[3], s);
#pragma unroll
    for (int p = 0; p < NP; ++p)
      reinterpret_cast<ushort4*>(a.out3 + p * a.ps)[i4] = make_ushort4(o[0][p], o[1][p], o[2][p], o[3][p]);
  }
}

// Sum a float4 over the RL row lanes of a block (lanes that share a channel lane): xor-shuffles
// over the row bits of the wave, then the 4 waves' sums in LDS in wave order.  Every thread gets
// the block total of its channel lane.  sh: [4][CL] float4 scratch.  Fixed order: deterministic.
template <int CL>
__device__ __forceinline__ float4 block_rows_sum(float4 v, float4 (*sh)[CL]) {
#pragma unroll
  for (int o = CL; o < 64; o <<= 1) {
    v.x += __shfl_xor(v.x, o, 64);
    v.y += __shfl_xor(v.y, o, 64);
    v.z += __shfl_xor(v.z, o, 64);
    v.w += __shfl_xor(v.w, o, 64);
  }
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (lane < CL) sh[w][lane] = v;
  __syncthreads();
  const int cl = lane % CL;
  const float4 r = add4(add4(sh[0][cl], sh[1][cl]), add4(sh[2][cl], sh[3][cl]));
  __syncthreads();
  return r;
}

// Publish this block's partials (already stored by some of its lanes) and wait for the slice's
// R arrivals.  Returns with every thread allowed to read every partial of the slice (plain loads).
__device__ __forceinline__ void slice_rendezvous(const FArgs& a, unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its partial stores
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    typedef __attribute__((address_space(1))) unsigned gu32;
    __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(a.R + a.phantom)) {
      if (wall_clock64() - t0 > a.ticks) {
        __hip_atomic_store((gint*)a.tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// After every read of the slice's partials: the last of the R blocks to get here zeroes both
// counters for the next launch.
__device__ __forceinline__ void slice_depart(const FArgs& a, unsigned* cnt) {
  __syncthreads();
  if (threadIdx.x == 0) {
    typedef __attribute__((address_space(1))) unsigned gu32;
    const unsigned d = __hip_atomic_fetch_add((gu32*)(cnt + 16), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned)a.R - 1) {
      __hip_atomic_store((gu32*)cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu32*)(cnt + 16), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------- forward
// Row unit r: pixel r of [M][C] (!POOL) or pooled position r = (n, oh, ow) of [N,H/2,W/2] whose
// window is the 4 pixels (2oh + i, 2ow + j).  Partials: (mean, M2) of the block's RB*(POOL?4:1)
// values per channel, PF = 2.
template <bool POOL, int NP, int U, int CL>
__global__ __launch_bounds__(FT) void bn_fused_fwd_kernel(FArgs a) {
  constexpr int RL = FT / CL, CS = 4 * CL, Q = POOL ? 4 : 1, RB = RL * U;
  const int t = threadIdx.x, cl = t % CL, rl = t / CL;
  const int slice = blockIdx.x / a.R, rb = blockIdx.x - slice * a.R;
  const int C4 = a.C >> 2;
  const int c4 = slice * CL + cl;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  __shared__ float4 sh[4][CL];
  __shared__ float2 mrg[FT / CS][CS];
  __shared__ float4 coef[2][CL];

  // float4 index of pixel q of row unit u (activations < 2^31 float4)
  auto idx_of = [&](int u, int q) -> int {
    const int r = rb * RB + rl + u * RL;
    if constexpr (POOL) {
      const int ow = r % Wo, tt = r / Wo, oh = tt % Ho, n = tt / Ho;
      return ((n * a.H + 2 * oh + (q >> 1)) * a.W + 2 * ow + (q & 1)) * C4 + c4;
    } else {
      return r * C4 + c4;
    }
  };
  float4 v[U][Q];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < Q; ++q) v[u][q] = ld4g(a.src, idx_of(u, q));
  if (a.nsplit > 1) {
    const long slab4 = a.slab >> 2;
    for (int s = 1; s < a.nsplit; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < Q; ++q) v[u][q] = add4(v[u][q], ld4g(a.src, s * slab4 + idx_of(u, q)));
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < Q; ++q) reinterpret_cast<float4*>(a.zw)[idx_of(u, q)] = v[u][q];
  }

  // exact two-pass statistics of the block's tile
  constexpr float inv_nb = 1.f / (float)(RB * Q);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < Q; ++q) s = add4(s, v[u][q]);
  s = block_rows_sum<CL>(s, sh);
  const float4 mb = make_float4(s.x * inv_nb, s.y * inv_nb, s.z * inv_nb, s.w * inv_nb);
  float4 m2 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float4 d = make_float4(v[u][q].x - mb.x, v[u][q].y - mb.y, v[u][q].z - mb.z, v[u][q].w - mb.w);
      m2.x = fmaf(d.x, d.x, m2.x);
      m2.y = fmaf(d.y, d.y, m2.y);
      m2.z = fmaf(d.z, d.z, m2.z);
      m2.w = fmaf(d.w, d.w, m2.w);
    }
  m2 = block_rows_sum<CL>(m2, sh);
  unsigned* cnt = a.cnt + slice * 32;
  float* pb = a.part + (long)blockIdx.x * 2 * CS;  // [2][CS]: means, then M2s
  if (t < CL) {
    reinterpret_cast<float4*>(pb)[cl] = mb;
    reinterpret_cast<float4*>(pb + CS)[cl] = m2;
  }
  slice_rendezvous(a, cnt);

  // fixed-order Chan merge of the slice's R partials: channel ch, group grp merges partials
  // grp, grp + G, ...; then the G group results in order (every block: the same sums)
  {
    constexpr int G = FT / CS;
    const int ch = t % CS, grp = t / CS;
    const float* ps0 = a.part + (long)slice * a.R * 2 * CS;
    float n = 0.f, mu = 0.f, M2 = 0.f;
    const float nb = (float)(RB * Q);
    // MB partials' loads in flight at once, then their merges (a dependent L2 round trip per
    // partial would dominate the kernel)
    constexpr int MB = 8;
    for (int k0 = grp; k0 < a.R; k0 += MB * G) {
      float pm[MB], pq[MB];
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        const int k = k0 + u * G;
        pm[u] = k < a.R ? ps0[(long)k * 2 * CS + ch] : 0.f;
        pq[u] = k < a.R ? ps0[(long)k * 2 * CS + CS + ch] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        if (k0 + u * G < a.R) {
          const float nn = n + nb, d = pm[u] - mu, f = nb / nn;
          mu += d * f;
          M2 += pq[u] + d * d * n * f;
          n = nn;
        }
      }
    }
    mrg[grp][ch] = make_float2(mu, M2);
    __syncthreads();
    if (grp == 0) {
      float nt = n;
#pragma unroll
      for (int g2 = 1; g2 < G; ++g2) {
        const float2 o = mrg[g2][ch];
        const float no = (float)((a.R - g2 + G - 1) / G) * nb;
        if (no > 0.f) {
          const float nn = nt + no, d = o.x - mu, f = no / nn;
          mu += d * f;
          M2 += o.y + d * d * nt * f;
          nt = nn;
        }
      }
      const int c = slice * CS + ch;
      const float var = M2 / nt;
      const float inv = rsqrtf(var + a.eps);
      const float gm = a.gamma[c];
      const float sc = gm * inv, sf = a.beta[c] - mu * gm * inv;
      reinterpret_cast<float*>(&coef[0][0])[ch] = sc;
      reinterpret_cast<float*>(&coef[1][0])[ch] = sf;
      if (rb == 0) {
        a.mean[c] = mu;
        a.invstd[c] = inv;
        a.scale[c] = sc;
        a.shift[c] = sf;
        if (a.rmean) {
          const float b = a.bias ? a.bias[c] : 0.f;
          const float unb = nt > 1.f ? M2 / (nt - 1.f) : var;
          a.rmean[c] = (1.f - a.momentum) * a.rmean[c] + a.momentum * (mu + b);
          a.rvar[c] = (1.f - a.momentum) * a.rvar[c] + a.momentum * unb;
        }
        if (c == 0 && a.nbt) a.nbt[0] += 1;
      }
    }
  }
  slice_depart(a, cnt);  // (its barrier also publishes coef to the block)
  if (!a.apply) return;
  const float4 sc = coef[0][cl], sf = coef[1][cl];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float4 y[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q)
      y[q] = make_float4(fmaxf(fmaf(v[u][q].x, sc.x, sf.x), 0.f), fmaxf(fmaf(v[u][q].y, sc.y, sf.y), 0.f),
                         fmaxf(fmaf(v[u][q].z, sc.z, sf.z), 0.f), fmaxf(fmaf(v[u][q].w, sc.w, sf.w), 0.f));
    float4 o = y[0];
    if constexpr (POOL)
      o = make_float4(fmaxf(fmaxf(y[0].x, y[1].x), fmaxf(y[2].x, y[3].x)),
                      fmaxf(fmaxf(y[0].y, y[1].y), fmaxf(y[2].y, y[3].y)),
                      fmaxf(fmaxf(y[0].z, y[1].z), fmaxf(y[2].z, y[3].z)),
                      fmaxf(fmaxf(y[0].w, y[1].w), fmaxf(y[2].w, y[3].w)));
    store_out<NP>(a, (rb * RB + rl + u * RL) * C4 + c4, o);
  }
}

// ---------------------------------------------------------------- backward
// dy at the unit's pixels from the pooled / unpooled gradient g: the ReLU mask and the 2x2 argmax
// (first max in window scan order, as torch) recomputed from z with the forward scale/shift.
// Partials: sum dy, sum dy*xhat, sum xhat (PF = 3).  dz = k1*dy + k2*z + k3 (bn.hip
// bn_bwd_finalize_kernel's coefficients).
template <bool POOL, int NP, int U, int CL>
__global__ __launch_bounds__(FT) void bn_fused_bwd_kernel(FArgs a) {
  start_signal(a.sig, a.sig_val);
  constexpr int RL = FT / CL, CS = 4 * CL, Q = POOL ? 4 : 1, RB = RL * U;
  const int t = threadIdx.x, cl = t % CL, rl = t / CL;
  const int slice = blockIdx.x / a.R, rb = blockIdx.x - slice * a.R;
  const int C4 = a.C >> 2;
  const int c4 = slice * CL + cl;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  __shared__ float4 sh[4][CL];
  __shared__ float mrg[FT / CS][3][CS];
  __shared__ float4 coef[3][CL];

  auto gi_of = [&](int u) -> int { return (rb * RB + rl + u * RL) * C4 + c4; };
  auto idx_of = [&](int u, int q) -> int {
    const int r = rb * RB + rl + u * RL;
    if constexpr (POOL) {
      const int ow = r % Wo, tt = r / Wo, oh = tt % Ho, n = tt / Ho;
      return ((n * a.H + 2 * oh + (q >> 1)) * a.W + 2 * ow + (q & 1)) * C4 + c4;
    } else {
      return r * C4 + c4;
    }
  };
  float4 g[U], zv[U][Q];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    g[u] = ld4g(a.src, gi_of(u));
#pragma unroll
    for (int q = 0; q < Q; ++q) zv[u][q] = ld4g(a.z, idx_of(u, q));
  }
  if (a.nsplit > 1) {
    const long slab4 = a.slab >> 2;
    for (int s = 1; s < a.nsplit; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u) g[u] = add4(g[u], ld4g(a.src, s * slab4 + gi_of(u)));
  }
  const float4 fsc = ld4g(a.scale, c4), fsh = ld4g(a.shift, c4);
  const float4 mu = ld4g(a.mean, c4), is = ld4g(a.invstd, c4);
  // dy in place of g's routing: d[u][q] (4 channels each)
  float4 dy[U][Q];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float dd[Q][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float sck = gk(fsc, k), shk = gk(fsh, k), gg = gk(g[u], k);
      if constexpr (POOL) {
        const float y0 = fmaxf(fmaf(gk(zv[u][0], k), sck, shk), 0.f), y1 = fmaxf(fmaf(gk(zv[u][1], k), sck, shk), 0.f);
        const float y2 = fmaxf(fmaf(gk(zv[u][2], k), sck, shk), 0.f), y3 = fmaxf(fmaf(gk(zv[u][3], k), sck, shk), 0.f);
        int arg = 0;
        float mx = y0;
        if (y1 > mx) { mx = y1; arg = 1; }
        if (y2 > mx) { mx = y2; arg = 2; }
        if (y3 > mx) { mx = y3; arg = 3; }
        dd[0][k] = (arg == 0 && y0 > 0.f) ? gg : 0.f;
        dd[Q > 1 ? 1 : 0][k] = (arg == 1 && y1 > 0.f) ? gg : 0.f;
        dd[Q > 2 ? 2 : 0][k] = (arg == 2 && y2 > 0.f) ? gg : 0.f;
        dd[Q > 3 ? 3 : 0][k] = (arg == 3 && y3 > 0.f) ? gg : 0.f;
      } else {
        dd[0][k] = fmaf(gk(zv[u][0], k), sck, shk) > 0.f ? gg : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) dy[u][q] = make_float4(dd[q][0], dd[q][1], dd[q][2], dd[q][3]);
  }
  float4 sdy = make_float4(0.f, 0.f, 0.f, 0.f), sdx = sdy, sx = sdy;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float4 xh = make_float4((zv[u][q].x - mu.x) * is.x, (zv[u][q].y - mu.y) * is.y,
                                    (zv[u][q].z - mu.z) * is.z, (zv[u][q].w - mu.w) * is.w);
      sdy = add4(sdy, dy[u][q]);
      sdx = make_float4(fmaf(dy[u][q].x, xh.x, sdx.x), fmaf(dy[u][q].y, xh.y, sdx.y), fmaf(dy[u][q].z, xh.z, sdx.z),
                        fmaf(dy[u][q].w, xh.w, sdx.w));
      sx = add4(sx, xh);
    }
  sdy = block_rows_sum<CL>(sdy, sh);
  sdx = block_rows_sum<CL>(sdx, sh);
  sx = block_rows_sum<CL>(sx, sh);
  unsigned* cnt = a.cnt + slice * 32;
  float* pb = a.part + (long)blockIdx.x * 3 * CS;  // [3][CS]
  if (t < CL) {
    reinterpret_cast<float4*>(pb)[cl] = sdy;
    reinterpret_cast<float4*>(pb + CS)[cl] = sdx;
    reinterpret_cast<float4*>(pb + 2 * CS)[cl] = sx;
  }
  slice_rendezvous(a, cnt);
  {
    constexpr int G = FT / CS;
    const int ch = t % CS, grp = t / CS;
    const float* ps0 = a.part + (long)slice * a.R * 3 * CS;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    constexpr int MB = 8;
    for (int k0 = grp; k0 < a.R; k0 += MB * G) {
      float p0[MB], p1[MB], p2[MB];
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        const int k = k0 + u * G;
        const float* p = ps0 + (long)k * 3 * CS + ch;
        const bool ok = k < a.R;
        p0[u] = ok ? p[0] : 0.f;
        p1[u] = ok ? p[CS] : 0.f;
        p2[u] = ok ? p[2 * CS] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        s0 += p0[u];
        s1 += p1[u];
        s2 += p2[u];
      }
    }
    mrg[grp][0][ch] = s0;
    mrg[grp][1][ch] = s1;
    mrg[grp][2][ch] = s2;
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int g2 = 1; g2 < G; ++g2) {
        s0 += mrg[g2][0][ch];
        s1 += mrg[g2][1][ch];
        s2 += mrg[g2][2][ch];
      }
      const int c = slice * CS + ch;
      const float Mfull = (float)a.N * a.H * a.W;
      const float iv = a.invstd[c], gm = a.gamma[c];
      const float k1 = gm * iv;
      const float k2x = -k1 * s1 / Mfull;
      const float k3 = -k1 * s0 / Mfull;
      reinterpret_cast<float*>(&coef[0][0])[ch] = k1;
      reinterpret_cast<float*>(&coef[1][0])[ch] = k2x * iv;
      reinterpret_cast<float*>(&coef[2][0])[ch] = k3 - k2x * iv * a.mean[c];
      if (rb == 0) {
        a.dgamma[c] = s1;
        a.dbeta[c] = s0;
        if (a.dbias) a.dbias[c] = k2x * s2;
      }
    }
  }
  slice_depart(a, cnt);
  const float4 k1 = coef[0][cl], k2 = coef[1][cl], k3 = coef[2][cl];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float4 o = make_float4(fmaf(k1.x, dy[u][q].x, fmaf(k2.x, zv[u][q].x, k3.x)),
                                   fmaf(k1.y, dy[u][q].y, fmaf(k2.y, zv[u][q].y, k3.y)),
                                   fmaf(k1.z, dy[u][q].z, fmaf(k2.z, zv[u][q].z, k3.z)),
                                   fmaf(k1.w, dy[u][q].w, fmaf(k2.w, zv[u][q].w, k3.w)));
      store_out<NP>(a, idx_of(u, q), o);
    }
}

// ---------------------------------------------------------------- host
// instantiated tiles: the per-unit register budget, <= ~170 VGPRs and no scratch in every variant
constexpr int UMAX_FWD_POOL = 4, UMAX_FWD = 16, UMAX_BWD_POOL = 2, UMAX_BWD = 8;

struct Geo {
  int CL, U, R, slices;
};

// Largest tile per thread (U units) whose grid is <= rmax row blocks per slice; units of 4 pixels
// (pool) hold 4x the registers, and the backward holds g too.
// Row blocks per slice: as few as possible (every block merges all R partials of its slice, and
// all R must be resident together) but at least RMIN while a smaller tile allows it (bandwidth
// of the load / store phases); at most rmax.
constexpr int RMIN = 16;
bool pick_geo(int Mo, int C, bool pool, bool bwd, int rmax, Geo& g) {
  g.CL = (C % 64 == 0) ? 16 : (C % 32 == 0 ? 8 : 0);
  if (!g.CL) return false;
  g.slices = C / (4 * g.CL);
  const int RL = FT / g.CL;
  const int umax = pool ? (bwd ? UMAX_BWD_POOL : UMAX_FWD_POOL) : (bwd ? UMAX_BWD : UMAX_FWD);
  bool found = false;
  for (int u = 1; u <= umax; u *= 2) {
    if (Mo % (RL * u)) break;
    const int R = Mo / (RL * u);
    if (R > rmax) continue;
    if (found && R < RMIN) break;
    g.U = u;
    g.R = R;
    found = true;
  }
  return found;
}

template <int U, int CL>
void launch_fwd(bool pool, int np, int grid, const FArgs& a, hipStream_t st) {
#define LF(P, NPT) bn_fused_fwd_kernel<P, NPT, U, CL><<<grid, FT, 0, st>>>(a)
  if (pool) {
    if constexpr (U <= UMAX_FWD_POOL) {
      if (np == 0) LF(true, 0);
      else if (np == 1) LF(true, 1);
      else if (np == 2) LF(true, 2);
      else LF(true, 3);
    }
  } else {
    if (np == 0) LF(false, 0);
    else if (np == 1) LF(false, 1);
    else if (np == 2) LF(false, 2);
    else LF(false, 3);
  }
#undef LF
}

template <int U, int CL>
void launch_bwd(bool pool, int np, int grid, const FArgs& a, hipStream_t st) {
#define LB(P, NPT) bn_fused_bwd_kernel<P, NPT, U, CL><<<grid, FT, 0, st>>>(a)
  if (pool) {
    if constexpr (U <= UMAX_BWD_POOL) {
      if (np == 0) LB(true, 0);
      else if (np == 1) LB(true, 1);
      else LB(true, 3);
    }
  } else {
    if constexpr (U <= UMAX_BWD) {
      if (np == 0) LB(false, 0);
      else if (np == 1) LB(false, 1);
      else LB(false, 3);
    }
  }
#undef LB
}

// Co-resident blocks per CU of the kernel a geometry runs, minimum over the output plane counts.
template <int U, int CL>
int occupancy(bool bwd, bool pool) {
  int lo = 1 << 30;
  auto take = [&](const void* fn) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, FT, 0) != hipSuccess) n = 0;
    lo = n < lo ? n : lo;
  };
#define OCC(B, P)                                                            \
  do {                                                                       \
    take(reinterpret_cast<const void*>(&B##_kernel<P, 0, U, CL>));           \
    take(reinterpret_cast<const void*>(&B##_kernel<P, 1, U, CL>));           \
    take(reinterpret_cast<const void*>(&B##_kernel<P, 3, U, CL>));           \
  } while (0)
  if (bwd) {
    if (pool) {
      if constexpr (U <= UMAX_BWD_POOL) OCC(bn_fused_bwd, true);
    } else {
      if constexpr (U <= UMAX_BWD) OCC(bn_fused_bwd, false);
    }
  } else {
    if (pool) {
      if constexpr (U <= UMAX_FWD_POOL) OCC(bn_fused_fwd, true);
    } else {
      OCC(bn_fused_fwd, false);
    }
  }
#undef OCC
  return lo == (1 << 30) ? 0 : lo;
}

// Blocks of this geometry's kernel that the idle chip holds at once (DPA_BN_FUSED_CAP overrides).
long resident_capacity(bool bwd, bool pool, const Geo& g) {
  if (const char* e = getenv("DPA_BN_FUSED_CAP")) return atol(e);
  // occupancy per (direction, pool, U, CL), queried once per process (host calls on every launch
  // would add to the enqueue time of the step)
  static int cache[2][2][5][2] = {};
  const int ui = g.U == 1 ? 0 : g.U == 2 ? 1 : g.U == 4 ? 2 : g.U == 8 ? 3 : 4;
  int& slot = cache[bwd][pool][ui][g.CL == 16];
  if (slot) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return (long)(slot - 1) * cus;
  }
  int occ = 0;
#define CASE(UU) \
  case UU: occ = g.CL == 16 ? occupancy<UU, 16>(bwd, pool) : occupancy<UU, 8>(bwd, pool); break;
  switch (g.U) {
    CASE(1)
    CASE(2)
    CASE(4)
    CASE(8)
    CASE(16)
    default: break;
  }
#undef CASE
  slot = occ + 1;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return (long)occ * cus;
}

constexpr int GRID_MAX = 512;

// pick_geo plus the residency guard (see the header comment)
bool pick_geo_resident(int Mo, int C, bool pool, bool bwd, int rmax, Geo& g) {
  if (!pick_geo(Mo, C, pool, bwd, rmax, g)) return false;
  const long grid = (long)g.slices * g.R;
  return grid <= GRID_MAX && 2L * g.R <= resident_capacity(bwd, pool, g);
}

template <int CL>
int dispatch(bool bwd, bool pool, int np, const Geo& g, const FArgs& a, hipStream_t st) {
  // fp16-pair data-gradient planes need the bound of the whole tensor before the apply phase, which
  // this kernel's per-slice rendezvous cannot give: the three-kernel BN backward carries them
  if (bwd && np == 2) return -2;
  const int grid = g.slices * g.R;
  switch (g.U) {
#define CASE(UU)                                   \
  case UU:                                         \
    if (bwd) launch_bwd<UU, CL>(pool, np, grid, a, st); \
    else launch_fwd<UU, CL>(pool, np, grid, a, st);     \
    break;
    CASE(1)
    CASE(2)
    CASE(4)
    CASE(8)
    CASE(16)
#undef CASE
    default:
      return -6;
  }
  return (int)hipGetLastError();
}

unsigned long long ticks_of(long long us) {
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (khz <= 0) khz = 100000;
  return (unsigned long long)us * (unsigned long long)khz / 1000ull;
}

int test_phantom() {
  const char* e = getenv("DPA_BN_FUSED_TEST_PHANTOM");
  return e ? atoi(e) : 0;
}

}  // namespace

extern "C" {
// Geometry query: 0 when the one-launch BN runs this layer (Mo row units of C channels) with at most
// rmax row blocks per channel slice; writes the workspace floats and counter words it needs.
int dpa_bn_fused_geo(int Mo, int C, int pool, int bwd, int rmax, long* part_floats, long* cnt_words, int* blocks) {
  Geo g;
  if (!pick_geo_resident(Mo, C, pool != 0, bwd != 0, rmax, g)) return -6;
  if (part_floats) *part_floats = (long)g.slices * g.R * (bwd ? 3 : 2) * 4 * g.CL;
  if (cnt_words) *cnt_words = (long)g.slices * 32;
  if (blocks) *blocks = g.slices * g.R;
  return 0;
}

// Forward: src = z [N,H,W,C] fp32 or nsplit slabs of it (z is then written to zw); writes mean,
// invstd, scale, shift, the running statistics and nbt, and (apply != 0) relu(BN(z)) [2x2 pooled]
// as fp32 out or bf16 planes out3 [np][...] (plane stride ps).
int dpa_bn_fused_fwd(const float* src, int nsplit, float* zw, int N, int H, int W, int C, int pool, int rmax,
                     float* part, unsigned* cnt, const float* gamma, const float* beta, const float* bias,
                     float* rmean, float* rvar, long long* nbt, float* mean, float* invstd, float* scale,
                     float* shift, int apply, float* out, u16* out3, int np, long ps, float momentum, float eps,
                     int* tmo, long long timeout_us, hipStream_t st) {
  const int Mo = N * (pool ? (H / 2) * (W / 2) : H * W);
  Geo g;
  if (C % 4 || !pick_geo_resident(Mo, C, pool != 0, false, rmax, g)) return -6;
  FArgs a{};
  a.src = src;
  a.nsplit = nsplit < 1 ? 1 : nsplit;
  a.slab = (long)N * H * W * C;
  a.zw = zw;
  a.N = N, a.H = H, a.W = W, a.C = C, a.R = g.R;
  a.part = part;
  a.cnt = cnt;
  a.gamma = gamma, a.beta = beta, a.bias = bias, a.rmean = rmean, a.rvar = rvar, a.nbt = nbt;
  a.mean = mean, a.invstd = invstd, a.scale = scale, a.shift = shift;
  a.out = out, a.out3 = out3, a.ps = ps, a.apply = apply;
  a.momentum = momentum, a.eps = eps;
  a.tmo = tmo;
  a.ticks = ticks_of(timeout_us);
  a.phantom = test_phantom();
  return g.CL == 16 ? dispatch<16>(false, pool != 0, np, g, a, st) : dispatch<8>(false, pool != 0, np, g, a, st);
}

// Backward: gsrc = dL/d(layer output) [N,Ho,Wo,C] fp32 or nsplit slabs of it; z, scale, shift, mean,
// invstd from the forward; writes dgamma, dbeta, dbias and dz (fp32 out or bf16 planes out3).
int dpa_bn_fused_bwd(const float* gsrc, int nsplit, const float* z, int N, int H, int W, int C, int pool, int rmax,
                     float* part, unsigned* cnt, const float* scale, const float* shift, const float* mean,
                     const float* invstd, const float* gamma, float* dgamma, float* dbeta, float* dbias, float* out,
                     u16* out3, int np, long ps, int* tmo, long long timeout_us, hipStream_t st, int* sig,
                     int sig_val) {
  const int Mo = N * (pool ? (H / 2) * (W / 2) : H * W);
  Geo g;
  if (C % 4 || !pick_geo_resident(Mo, C, pool != 0, true, rmax, g)) return -6;
  FArgs a{};
  a.src = gsrc;
  a.nsplit = nsplit < 1 ? 1 : nsplit;
  a.slab = (long)Mo * C;
  a.z = z;
  a.N = N, a.H = H, a.W = W, a.C = C, a.R = g.R;
  a.part = part;
  a.cnt = cnt;
  a.gamma = gamma;
  a.mean = const_cast<float*>(mean), a.invstd = const_cast<float*>(invstd);
  a.scale = const_cast<float*>(scale), a.shift = const_cast<float*>(shift);
  a.dgamma = dgamma, a.dbeta = dbeta, a.dbias = dbias;
  a.out = out, a.out3 = out3, a.ps = ps;
  a.tmo = tmo;
  a.ticks = ticks_of(timeout_us);
  a.phantom = test_phantom();
  a.sig = sig;
  a.sig_val = sig_val;
  return g.CL == 16 ? dispatch<16>(true, pool != 0, np, g, a, st) : dispatch<8>(true, pool != 0, np, g, a, st);
}
}  // extern "C"

DPA_H2_OVF_ACCESSOR(dpa_h2_ovf_fused)
