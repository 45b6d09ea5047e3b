// Small exact-fp32 GEMM on the fp32-input matrix cores (v_mfma_f32_32x32x2_f32), for the generic
// path's classifier head (ResNet-50: logits = feat @ W^T + b, dfeat = dl @ W, dW = dl^T @ feat;
// M or N = batch).  These replaced hipBLASLt calls, so the training step runs no library GEMM.
//
//   C[M][N] = sum_k opA[m][k] * opB[k][n]  (+ bias[n])      fp32 in, fp32 out, row-major C
//   A: AK = k-contiguous rows (A[m * lda + k]) or m-contiguous (A[k * lda + m])
//   B: BK = k-contiguous (B[n * ldb + k], i.e. W stored [N][K]) or n-contiguous (B[k * ldb + n])
//
// Tile: 64 x 64 per 256-thread block, 2 x 2 waves of one 32 x 32 accumulator each, KT = 32 deep
// LDS stages ([k][m] / [k][n] images: an operand fragment is 32 consecutive floats of one k row,
// conflict-free).  The fp32 MFMA is a k-ordered fmaf chain (exact fp32 products, one rounding per
// product), so results match an fp32 dot product in that order.  Split-K over blockIdx.y writes
// fp32 slabs that common.h's fixed-order split-K reduction sums (deterministic); the bias is added
// by split 0 only.
#include "common.h"

namespace {

constexpr int GT = 64, KT = 32;

template <bool AK, bool BK>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ B, int ldb,
                                                       float* __restrict__ C, long slab, int M, int N, int K,
                                                       int kchunk, const float* __restrict__ bias) {
  __shared__ float As[KT][GT];
  __shared__ float Bs[KT][GT];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int gn = (N + GT - 1) / GT;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / gn) * GT, n0 = (tile % gn) * GT;
  const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  // stage one operand tile [KT][64] from global (zero outside the matrix)
  auto stage = [&](float (*dst)[GT], const float* src, int ld, bool kcontig, int r0, int R, int k0) {
    if (kcontig) {  // src[row * ld + k]: 64 rows x 8 float4 along k, transposed into [k][row]
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = t + j * 256, row = q >> 3, k4 = (q & 7) * 4;
        const int gr = r0 + row, gk = k0 + k4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (gr < R) {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = (gk + u < ke) ? src[(long)gr * ld + gk + u] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) dst[k4 + u][row] = v[u];
      }
    } else {  // src[k * ld + row]: 32 k rows x 16 float4 along the row index
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = t + j * 256, kk = q >> 4, c4 = (q & 15) * 4;
        const int gk = k0 + kk, gr = r0 + c4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (gk < ke) {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = (gr + u < R) ? src[(long)gk * ld + gr + u] : 0.f;
        }
        *reinterpret_cast<float4*>(&dst[kk][c4]) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };

  for (int k0 = kb; k0 < ke; k0 += KT) {
    stage(As, A, lda, AK, m0, M, k0);
    stage(Bs, B, ldb, BK, n0, N, k0);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KT; kk += 2) {
      const float a = As[kk + (lane >> 5)][wm * 32 + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  float* out = C + (long)blockIdx.y * slab;
  const int col = n0 + wn * 32 + (lane & 31);
  if (col < N) {
    const float bv = (bias != nullptr && blockIdx.y == 0) ? bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) out[(long)row * N + col] = acc[r] + bv;
    }
  }
}

}  // namespace

extern "C" {
// C = opA @ opB (+ bias): ak / bk as in the header; splits > 1 needs slab >= splits * M * N floats
// and M * N % 4 == 0.
int dpa_gemm_f32(const float* A, int lda, int ak, const float* B, int ldb, int bk, float* C, int M, int N, int K,
                 const float* bias, float* slab, int splits, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return -2;
  if (splits < 1) splits = 1;
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + KT - 1) / KT * KT;
  splits = (K + kchunk - 1) / kchunk;
  if (splits > 1 && (!slab || ((long)M * N) % 4)) return -2;
  const int tiles = ((M + GT - 1) / GT) * ((N + GT - 1) / GT);
  dim3 grid(tiles, splits);
  float* out = splits > 1 ? slab : C;
  const long sl = splits > 1 ? (long)M * N : 0;
#define GL(AKV, BKV) gemm_f32_kernel<AKV, BKV><<<grid, 256, 0, st>>>(A, lda, B, ldb, out, sl, M, N, K, kchunk, bias)
  if (ak && bk) GL(true, true);
  else if (ak) GL(true, false);
  else if (bk) GL(false, true);
  else GL(false, false);
#undef GL
  int rc = (int)hipGetLastError();
  if (rc || splits == 1) return rc;
  return launch_splitk_reduce(slab, C, (long)M * N / 4, splits, st);
}
}  // extern "C"
