// Sustained bf16 MFMA rate on this GPU: register-only v_mfma_f32_32x32x16_bf16 streams (no memory
// traffic), 4 independent accumulators per wave, 1-4 waves per SIMD.  Calibrates what fraction
// of the datasheet peak a conv kernel's "MFMA busy" can reach under full load.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_peak tools/mfma_peak.hip && tools/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * (threadIdx.x - i));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 12345.678f) out[0] = s;  // keep the chain live
}

int main() {
  float* out;
  hipMalloc(&out, 4);
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int wps = 1; wps <= 4; wps *= 2) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
    const int blocks = cus * wps;
    mfma_loop<<<blocks, 256>>>(out, 100);
    hipEventRecord(e0);
    mfma_loop<<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * blocks * 4;  // 4 waves per block
    printf("{\"waves_per_simd\": %d, \"ms\": %.3f, \"tflops_bf16\": %.1f}\n", wps, ms, flops / (ms * 1e-3) / 1e12);
  }
  return 0;
}
