// K7/K8 — classifier head: Linear(Cin -> J) + softmax cross-entropy (mean reduction), forward
// and backward fused.  Replaces addmm / _log_softmax / nll_loss and their backwards
// (model.py:40,45 and main.py:34,99).
//
// fc_ce_rows: one wavefront per sample row: logits (wave reductions over Cin), log-sum-exp,
//   per-row loss, dlogits = (softmax - onehot)/B, and dx = dlogits @ W  — all in registers.
// fc_ce_wgrad: dW[j][c] = sum_b dlogits[b][j] * x[b][c], db[j] = sum_b dlogits[b][j], and the
//   batch-mean loss (fixed summation order -> bitwise reproducible).
#include "common.h"

namespace {
// Compile-time bounds: MAXJ classes, MAXCL = Cin / 64 values per lane kept in registers.  The VGG
// head (J = 10, Cin = 512) runs the <10, 8> instance, anything else up to J = 16, Cin = 1024 the
// generic one (every loop over MAXJ / MAXCL is fully unrolled, so tight bounds mean no dead lanes).
constexpr int GEN_J = 16, GEN_CL = 16;

// W [J][Cin] is staged once per block into LDS (one round of independent 16-B loads), the row
// (Cin/64 values per lane) is held in registers, and the J wave reductions are interleaved: the
// kernel pays ~two global-memory latencies instead of a chain of dependent L2 round trips.
//
// Bn: the last conv layer's BatchNorm + ReLU + 2x2 max-pool folded into the row load (VGG on 32x32:
// the pool leaves one pixel, so a feature row is the max over the 4 pixels of z [B][4][Cin] of
// relu(z*scale + shift), the same operations in the same order as bn_apply).  The features are
// also stored to x (the weight-gradient kernel reads them), and the separate bn_apply launch goes.
struct BnIn {
  const float* z;
  const float* scale;
  const float* shift;
};

template <bool TRAIN, int MAXJ, int MAXCL, bool BNIN = false>
__global__ __launch_bounds__(256) void fc_ce_rows_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         const long long* __restrict__ target,
                                                         float* __restrict__ loss_row, float* __restrict__ dlogits,
                                                         float* __restrict__ dx, int* __restrict__ correct_row,
                                                         float* __restrict__ logits_out, int B, int Cin, int J,
                                                         BnIn bn = BnIn{nullptr, nullptr, nullptr}) {
  extern __shared__ float w_s[];  // [J][Cin]
  // All of the block's W loads are issued together, then the row's loads, and only then is the LDS
  // image written: one memory latency for both instead of one per 4 KB of W plus one for the row
  // (the rolled copy loop cost ~5 dependent round trips on the VGG step's critical path).
  constexpr int WIT = (MAXJ * 64 * MAXCL + 1023) / 1024;  // float4 per thread (256 threads)
  float4 wt[WIT];
#pragma unroll
  for (int u = 0; u < WIT; ++u) {
    const int i = threadIdx.x * 4 + u * 1024;
    wt[u] = i < J * Cin ? *reinterpret_cast<const float4*>(w + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int lane = threadIdx.x & 63;
  const int row = min(blockIdx.x * 4 + (threadIdx.x >> 6), B - 1);  // tail waves load a valid row
  const bool rv = blockIdx.x * 4 + (threadIdx.x >> 6) < B;
  const float* xr = x + (long)row * Cin;
  float xv[MAXCL];
  if constexpr (BNIN) {
    const float* zr = bn.z + (long)row * 4 * Cin;
    float* xo = const_cast<float*>(xr);
#pragma unroll
    for (int k = 0; k < MAXCL; ++k) {
      const int c = lane + 64 * k;
      float v = 0.f;
      if (c < Cin) {
        const float sc = bn.scale[c], sh = bn.shift[c];
        const float v00 = fmaxf(fmaf(zr[c], sc, sh), 0.f), v01 = fmaxf(fmaf(zr[Cin + c], sc, sh), 0.f);
        const float v10 = fmaxf(fmaf(zr[2 * Cin + c], sc, sh), 0.f), v11 = fmaxf(fmaf(zr[3 * Cin + c], sc, sh), 0.f);
        v = fmaxf(fmaxf(v00, v01), fmaxf(v10, v11));
        if (rv) xo[c] = v;
      }
      xv[k] = v;
    }
  } else {
#pragma unroll
    for (int k = 0; k < MAXCL; ++k) {
      const int c = lane + 64 * k;
      xv[k] = c < Cin ? xr[c] : 0.f;
    }
  }
#pragma unroll
  for (int u = 0; u < WIT; ++u) {
    const int i = threadIdx.x * 4 + u * 1024;
    if (i < J * Cin) *reinterpret_cast<float4*>(w_s + i) = wt[u];
  }
  __syncthreads();
  if (!rv) return;
  float logit[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    float s = 0.f;
    if (j < J) {
#pragma unroll
      for (int k = 0; k < MAXCL; ++k) {
        const int c = lane + 64 * k;
        if (c < Cin) s = fmaf(xv[k], w_s[j * Cin + c], s);
      }
    }
    logit[j] = s;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) logit[j] += __shfl_xor(logit[j], o, 64);
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) logit[j] = j < J ? logit[j] + bias[j] : -INFINITY;
  float mx = logit[0];
  int arg = 0;
#pragma unroll
  for (int j = 1; j < MAXJ; ++j)
    if (j < J && logit[j] > mx) {
      mx = logit[j];
      arg = j;
    }
  float se = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
    if (j < J) se += expf(logit[j] - mx);
  const float lse = mx + logf(se);
  const int t = (int)target[row];
  float lt = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
    if (j == t) lt = logit[j];
  if (lane == 0) {
    loss_row[row] = lse - lt;
    if (correct_row) correct_row[row] = (arg == t) ? 1 : 0;
  }
  if (logits_out && lane < J) {
#pragma unroll
    for (int j = 0; j < MAXJ; ++j)
      if (j == lane) logits_out[(long)row * J + j] = logit[j];
  }
  if (TRAIN) {
    const float invB = 1.f / (float)B;
    float dl[MAXJ];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) dl[j] = j < J ? (expf(logit[j] - lse) - (j == t ? 1.f : 0.f)) * invB : 0.f;
    if (lane < J) {
#pragma unroll
      for (int j = 0; j < MAXJ; ++j)
        if (j == lane) dlogits[(long)row * J + j] = dl[j];
    }
#pragma unroll
    for (int k = 0; k < MAXCL; ++k) {
      const int c = lane + 64 * k;
      if (c < Cin) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < MAXJ; ++j)
          if (j < J) s = fmaf(dl[j], w_s[j * Cin + c], s);
        dx[(long)row * Cin + c] = s;
      }
    }
  }
}

// grid: cdiv(Cin,8) + 1 blocks of 256 threads = 8 columns x 32 row-groups.  dlogits [B][J] is
// staged in LDS; each thread issues its rows' x loads together, the row-groups are combined
// through LDS in a fixed order (deterministic).  The last block reduces db and the batch-mean loss.
template <int MAXJ>
__global__ __launch_bounds__(256) void fc_ce_wgrad_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ dlogits,
                                                          const float* __restrict__ loss_row, float* __restrict__ dw,
                                                          float* __restrict__ db, float* __restrict__ loss_out,
                                                          float* __restrict__ loss_accum, int B, int Cin, int J) {
  const int ncb = (Cin + 7) / 8;
  const int t = threadIdx.x;
  if ((int)blockIdx.x < ncb) {
    extern __shared__ float dl_s[];  // [B][J]
    __shared__ float red[32][8][MAXJ + 1];
    for (int i = t; i < B * J; i += 256) dl_s[i] = dlogits[i];
    __syncthreads();
    const int cl = t & 7, rg = t >> 3;
    const int c = blockIdx.x * 8 + cl;
    float acc[MAXJ];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) acc[j] = 0.f;
    if (c < Cin) {
      int b = rg;
      for (; b + 96 < B; b += 128) {
        float xv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) xv[u] = x[(long)(b + 32 * u) * Cin + c];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < MAXJ; ++j)
            if (j < J) acc[j] = fmaf(dl_s[(b + 32 * u) * J + j], xv[u], acc[j]);
      }
      for (; b < B; b += 32) {
        const float xv = x[(long)b * Cin + c];
#pragma unroll
        for (int j = 0; j < MAXJ; ++j)
          if (j < J) acc[j] = fmaf(dl_s[b * J + j], xv, acc[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) red[rg][cl][j] = acc[j];
    __syncthreads();
    if (t < 8 * J) {
      const int j = t / 8, cc = t % 8;
      float s = 0.f;
      for (int k = 0; k < 32; ++k) s += red[k][cc][j];
      const int col = blockIdx.x * 8 + cc;
      if (col < Cin) dw[(long)j * Cin + col] = s;
    }
  } else {
    __shared__ float sh[256];
    __shared__ float sj[16][17];  // 16 row groups x 16 class lanes (+1 pad), independent of MAXJ
    // db: thread (j = t % 16, g = t / 16) sums rows g, g+16, ...
    const int jj = t % 16, g = t / 16;
    float s = 0.f;
    if (jj < J)
      for (int b = g; b < B; b += 16) s += dlogits[(long)b * J + jj];
    sj[g][jj] = s;
    float l = 0.f;
    for (int b = t; b < B; b += 256) l += loss_row[b];
    sh[t] = l;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) sh[t] += sh[t + o];
      __syncthreads();
    }
    if (t < J) {
      float d = 0.f;
      for (int k = 0; k < 16; ++k) d += sj[k][t];
      db[t] = d;
    }
    if (t == 0) {
      const float lm = sh[0] / (float)B;
      loss_out[0] = lm;
      if (loss_accum) loss_accum[0] += lm;
    }
  }
}

// Eval accumulation: acc[0] += mean loss of this batch, acc[1] += #correct (as float, exact < 2^24)
__global__ __launch_bounds__(256) void eval_accum_kernel(const float* __restrict__ loss_row,
                                                         const int* __restrict__ correct_row, float* __restrict__ acc,
                                                         int B) {
  __shared__ float sl[256];
  __shared__ int sc[256];
  float l = 0.f;
  int c = 0;
  for (int b = threadIdx.x; b < B; b += 256) {
    l += loss_row[b];
    c += correct_row[b];
  }
  sl[threadIdx.x] = l;
  sc[threadIdx.x] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sl[threadIdx.x] += sl[threadIdx.x + o];
      sc[threadIdx.x] += sc[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    acc[0] += sl[0] / (float)B;
    acc[1] += (float)sc[0];
  }
}

}  // namespace

extern "C" {

// bn_z / bn_scale / bn_shift (optional, VGG head): x is then OUTPUT -- the features are computed from
// the last conv layer's z [B][2][2][Cin] (BN + ReLU + 2x2 max-pool, see BnIn) and stored there.
// parts: bit 0 = the row kernel (loss rows, dlogits, dx), bit 1 = the weight-gradient kernel (dW, db,
// batch loss).  The VGG engine issues the row kernel on the critical path and the weight gradient on
// its weight-gradient stream (nothing on the critical path reads dW, db or the loss).
int dpa_fc_ce_train(const float* x, const float* w, const float* b, const long long* target, float* loss_row,
                    float* dlogits, float* dx, float* dw, float* db, float* loss_out, float* loss_accum, int B,
                    int Cin, int J, hipStream_t st, const float* bn_z, const float* bn_scale, const float* bn_shift,
                    int parts) {
  if (J > GEN_J || Cin > 64 * GEN_CL || Cin % 4 || (long)B * J * 4 > 48 * 1024) return -2;
  const bool rows = parts & 1, wg = parts & 2;
  if (bn_z) {
    if (!bn_scale || !bn_shift || J > 10 || Cin > 512) return -2;
    if (rows)
      fc_ce_rows_kernel<true, 10, 8, true><<<cdiv(B, 4), 256, J * Cin * 4, st>>>(
          x, w, b, target, loss_row, dlogits, dx, nullptr, nullptr, B, Cin, J, BnIn{bn_z, bn_scale, bn_shift});
  } else if (J <= 10 && Cin <= 512) {
    if (rows)
      fc_ce_rows_kernel<true, 10, 8><<<cdiv(B, 4), 256, J * Cin * 4, st>>>(x, w, b, target, loss_row, dlogits, dx,
                                                                            nullptr, nullptr, B, Cin, J);
  } else if (rows) {
    fc_ce_rows_kernel<true, GEN_J, GEN_CL><<<cdiv(B, 4), 256, J * Cin * 4, st>>>(x, w, b, target, loss_row, dlogits,
                                                                                dx, nullptr, nullptr, B, Cin, J);
  }
  if (wg) {
    if (J <= 10)
      fc_ce_wgrad_kernel<10><<<cdiv(Cin, 8) + 1, 256, B * J * 4, st>>>(x, dlogits, loss_row, dw, db, loss_out,
                                                                       loss_accum, B, Cin, J);
    else
      fc_ce_wgrad_kernel<GEN_J><<<cdiv(Cin, 8) + 1, 256, B * J * 4, st>>>(x, dlogits, loss_row, dw, db, loss_out,
                                                                          loss_accum, B, Cin, J);
  }
  return (int)hipGetLastError();
}

int dpa_fc_ce_eval(const float* x, const float* w, const float* b, const long long* target, float* loss_row,
                   int* correct_row, float* logits, float* acc, int B, int Cin, int J, hipStream_t st) {
  if (J > GEN_J || Cin > 64 * GEN_CL || Cin % 4) return -2;
  if (J <= 10 && Cin <= 512)
    fc_ce_rows_kernel<false, 10, 8><<<cdiv(B, 4), 256, J * Cin * 4, st>>>(x, w, b, target, loss_row, nullptr, nullptr,
                                                                           correct_row, logits, B, Cin, J);
  else
    fc_ce_rows_kernel<false, GEN_J, GEN_CL><<<cdiv(B, 4), 256, J * Cin * 4, st>>>(x, w, b, target, loss_row, nullptr,
                                                                                 nullptr, correct_row, logits, B,
                                                                                 Cin, J);
  if (acc) eval_accum_kernel<<<1, 256, 0, st>>>(loss_row, correct_row, acc, B);
  return (int)hipGetLastError();
}

}  // extern "C"
