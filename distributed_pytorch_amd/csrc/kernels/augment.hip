// K10 — on-device CIFAR augmentation + normalisation.  Replaces the reference's DataLoader
// worker pipeline RandomCrop(32, padding=4) -> RandomHorizontalFlip -> ToTensor -> Normalize
// (/root/reference/main.py:71-82) for a device-resident uint8 dataset, so no host->device copy
// and no worker processes sit in the training loop.
//
// images: uint8 [Ntotal][Hs][Ws][3] (HWC), idx: int64 [B] dataset indices for this batch.
// out: fp32 NHWC [B][Hs][Ws][4] (channel 3 zero: the first conv is run with C padded to 4).
// Per-sample crop offsets / flip come from a counter-based hash of (seed, sample index, salt),
// so the stream is reproducible and independent of launch geometry.
#include "common.h"

namespace {

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Norm {
  float m[3], inv_s[3];
};

__global__ __launch_bounds__(256) void augment_kernel(const unsigned char* __restrict__ img,
                                                      const long long* __restrict__ idx,
                                                      const long long* __restrict__ labels,
                                                      float* __restrict__ out, long long* __restrict__ target, int Hs,
                                                      int Ws, int pad, int train, unsigned long long seed,
                                                      unsigned long long salt, Norm nm) {
  const int b = blockIdx.x;
  const long long src = idx[b];
  int dy = pad, dx = pad, flip = 0;
  if (train) {
    const unsigned long long h = mix64(seed ^ mix64(salt * 0x100000001B3ull + (unsigned long long)b));
    const int span = 2 * pad + 1;
    dy = (int)(h % span);
    dx = (int)((h >> 16) % span);
    flip = (int)((h >> 40) & 1);
  }
  if (threadIdx.x == 0 && target) target[b] = labels[src];
  const unsigned char* im = img + (long)src * Hs * Ws * 3;
  float4* o = reinterpret_cast<float4*>(out) + (long)b * Hs * Ws;
  for (int p = threadIdx.x; p < Hs * Ws; p += blockDim.x) {
    const int y = p / Ws, x = p % Ws;
    const int xs = flip ? (Ws - 1 - x) : x;  // flip applied after the crop
    const int sy = y + dy - pad, sx = xs + dx - pad;
    float r = 0.f, g = 0.f, bl = 0.f;
    if ((unsigned)sy < (unsigned)Hs && (unsigned)sx < (unsigned)Ws) {
      const unsigned char* q = im + ((long)sy * Ws + sx) * 3;
      r = q[0] * (1.f / 255.f);
      g = q[1] * (1.f / 255.f);
      bl = q[2] * (1.f / 255.f);
    }
    o[p] = make_float4((r - nm.m[0]) * nm.inv_s[0], (g - nm.m[1]) * nm.inv_s[1], (bl - nm.m[2]) * nm.inv_s[2], 0.f);
  }
}

}  // namespace

extern "C" int dpa_augment(const unsigned char* img, const long long* idx, const long long* labels, float* out,
                           long long* target, int B, int Hs, int Ws, int pad, int train, unsigned long long seed,
                           unsigned long long salt, const float* mean, const float* std, hipStream_t st) {
  Norm nm;
  for (int c = 0; c < 3; ++c) {
    nm.m[c] = mean[c];
    nm.inv_s[c] = 1.f / std[c];
  }
  augment_kernel<<<B, 256, 0, st>>>(img, idx, labels, out, target, Hs, Ws, pad, train, seed, salt, nm);
  return (int)hipGetLastError();
}
