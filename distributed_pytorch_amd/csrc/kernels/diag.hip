// Diagnostic kernels (tests and tools only; nothing on the training path).
#include "common.h"

// One wave sleeps until `ticks` of the constant-rate wall clock have passed, then writes done[0]=1.
// The loop is also capped at `max_iter` sleeps, so it ends even if the clock were not advancing.
__global__ __launch_bounds__(64) void spin_kernel(unsigned long long ticks, long long max_iter, int* done) {
  const unsigned long long t0 = wall_clock64();
  long long it = 0;
  while (wall_clock64() - t0 < ticks && it < max_iter) {
    __builtin_amdgcn_s_sleep(127);
    ++it;
  }
  if (threadIdx.x == 0) done[0] = 1;
}

extern "C" int dpa_spin(long long usec, int* done, hipStream_t s) {
  int dev = 0, khz = 0;
  DPA_HIP_CHECK(hipGetDevice(&dev));
  DPA_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;  // gfx9 wall clock: 100 MHz
  const unsigned long long ticks = (unsigned long long)usec * (unsigned long long)khz / 1000ull;
  // s_sleep 127 is ~8k cycles (>= 3 us at MI355X clocks): usec sleeps bound the loop at ~3x usec
  spin_kernel<<<1, 64, 0, s>>>(ticks, usec + 1, done);
  return (int)hipGetLastError();
}
