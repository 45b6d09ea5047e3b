// Cross-stream wait on a kernel-start signal (common.h start_signal).
//
// The VGG engine's backward runs weight gradients on a second stream.  A HIP event recorded on the
// critical-path stream between BN backward and the data-gradient conv puts a queue marker there
// that costs ~6.5 us of idle GPU per layer (profiles/r2_final_x3_step_timeline.txt: the gap in
// front of every data-gradient conv).  Instead the data-gradient conv's first workgroup stores the
// step's epoch to a flag word when it starts — by then the BN backward kernels before it have
// completed and been released at the kernel boundary — and the weight-gradient stream runs this
// one-wave kernel, which polls the word (relaxed agent-scope atomic loads, s_sleep between polls)
// until it holds the epoch.  Kernels queued after it on the weight-gradient stream are dispatched
// only once it has ended, with the dispatch's own acquire, so they read the BN backward's output.
//
// The poll is bounded: after `ticks` of the 100 MHz wall clock it gives up, sets tmo[0] = 1 and
// returns, so a missing signal can never hang the device; the engine checks tmo (engine.py
// check_signals) and raises.
#include "common.h"

namespace {

__global__ __launch_bounds__(64) void wait_signal_kernel(const int* __restrict__ sig, int val,
                                                         unsigned long long ticks, int* __restrict__ tmo) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load((const gint*)sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < val) {
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_store((gint*)tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// a kernel that only signals (tests; and a producer stream whose next kernel cannot carry it)
__global__ __launch_bounds__(64) void set_signal_kernel(int* __restrict__ sig, int val) { start_signal(sig, val); }

// Per-step health snapshot (engine.py VGGEngine.health_mark): lane i copies the device word *w[i]
// (an fp16-pair overflow word, a bounded-wait timeout word, a peer-collective timeout word) into
// out[i] -- pinned host memory, read by the host once the step's event has completed, so a step
// that went wrong fails the run one step later without a synchronising read inside the step.
// The words were written by kernels ordered before this one (stream order, or the joins that
// precede the optimizer step), so plain agent-scope loads see them.
__global__ __launch_bounds__(64) void health_kernel(const int* const* __restrict__ w, int n, int* __restrict__ out,
                                                    int tag) {
  const int t = threadIdx.x;
  if (t < n) {
    const int* p = w[t];
    out[t] = p != nullptr ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  }
  if (t == 63) out[63] = tag;  // which step this slot describes
}

}  // namespace

extern "C" {
int dpa_wait_signal(const int* sig, int val, long long timeout_us, int* tmo, hipStream_t st) {
  int dev = 0, khz = 0;
  DPA_HIP_CHECK(hipGetDevice(&dev));
  DPA_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;
  const unsigned long long ticks = (unsigned long long)timeout_us * (unsigned long long)khz / 1000ull;
  wait_signal_kernel<<<1, 64, 0, st>>>(sig, val, ticks, tmo);
  return (int)hipGetLastError();
}

int dpa_set_signal(int* sig, int val, hipStream_t st) {
  set_signal_kernel<<<1, 64, 0, st>>>(sig, val);
  return (int)hipGetLastError();
}

// w: device array of n (<= 63) word pointers; out: 64 ints of host-pinned (device-mapped) memory
int dpa_health_copy(const int* const* w, int n, int* out, int tag, hipStream_t st) {
  if (n < 0 || n > 63) return -2;
  health_kernel<<<1, 64, 0, st>>>(w, n, out, tag);
  return (int)hipGetLastError();
}
}  // extern "C"
