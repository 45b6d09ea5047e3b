// Peer-memory all-reduce (SUM, fp32) over the ranks of one node: every rank maps its peers'
// gradient arenas, staging buffers and signal words through HIP IPC (runtime/ipc_comm.cpp), and
// one kernel per collective reads them directly -- over xGMI between MI355X GPUs, or through the
// same HBM when several ranks share one GPU (the only multi-rank device path a one-GPU lease can
// run).  Reference semantics: all_reduce(SUM) of the DDP buckets / per-parameter grads
// (/root/reference/main_all_reduce.py:45-48, main_ddp.py:137); SURVEY §5.8 (mesh-aware sync).
//
// Two-shot, B workgroups per rank (a fixed CU budget, like RCCL's channel count):
//   barrier A  block b of every rank has started: the collective's inputs (written by kernels
//              stream-ordered before it on each rank) are complete;
//   phase 1    reduce-scatter: rank r sums slice r of the n elements over all ranks IN RANK ORDER
//              (0, 1, ..., W-1) and stores it in its own staging buffer;
//   barrier B  block b of every rank has stored its part of phase 1 (release / acquire at system
//              scope around the flag);
//   phase 2    all-gather: rank r copies every rank's reduced slice from that rank's staging buffer
//              into its own data.
// Every element is summed once, in one fixed order, so all ranks hold bitwise identical results
// (deterministic, like the RCCL path's replicas).  Data is only read before barrier B and written
// after it; a rank rewrites its staging buffer only in the next collective's phase 1, after that
// collective's barrier A, which every peer reaches only once it has left this one: no end barrier.
// Signal words are monotonic epochs (one per collective) in uncached memory, one per (phase,
// source rank, block); waits are bounded (tmo word + exit, never a hang).
#include "common.h"

namespace {

constexpr int IPC_MAXW = 8;    // ranks
constexpr int IPC_MAXB = 128;  // workgroups per rank
constexpr int IPC_T = 256;

struct IpcArgs {
  float* data[IPC_MAXW];      // each rank's data (already at this collective's first element)
  float* stage[IPC_MAXW];     // each rank's staging buffer (>= slice elements)
  unsigned* sig[IPC_MAXW];    // each rank's signal array [2][IPC_MAXW][IPC_MAXB]
  int rank, world;
  long n, ns;                 // elements; slice length (multiple of 4)
  unsigned epoch;
  int* tmo;
  unsigned long long ticks;
};

typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void ipc_barrier(const IpcArgs& a, int phase) {
  const int t = threadIdx.x, b = blockIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores (phase 1 staging) are done
  __syncthreads();
  if (t < 64) {
    if (t == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: visible to every peer
    if (t < a.world && t != a.rank)
      __hip_atomic_store((gu32*)(a.sig[t] + (phase * IPC_MAXW + a.rank) * IPC_MAXB + b), a.epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < a.world && t != a.rank) {
      const gu32* w = (const gu32*)(a.sig[a.rank] + (phase * IPC_MAXW + t) * IPC_MAXB + b);
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
        if (wall_clock64() - t0 > a.ticks) {
          __hip_atomic_store((gint*)a.tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (t == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

__device__ __forceinline__ float4 f4add(float4 x, float4 y) {
  return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
}

__global__ __launch_bounds__(IPC_T) void ipc_allreduce_kernel(IpcArgs a) {
  const int W = a.world, r = a.rank, t = threadIdx.x;
  const int B = gridDim.x, b = blockIdx.x;
  ipc_barrier(a, 0);
  // phase 1: slice r, this block's part of it (float4 elements of the slice, strided by block)
  const long s0 = (long)r * a.ns;
  const long s1 = s0 + a.ns < a.n ? s0 + a.ns : a.n;
  const long len = s1 > s0 ? s1 - s0 : 0;
  const long len4 = len / 4;
  for (long i = (long)b * IPC_T + t; i < len4; i += (long)B * IPC_T) {
    float4 s = reinterpret_cast<const float4*>(a.data[0] + s0)[i];
    for (int p = 1; p < W; ++p) s = f4add(s, reinterpret_cast<const float4*>(a.data[p] + s0)[i]);
    reinterpret_cast<float4*>(a.stage[r])[i] = s;
  }
  if (b == 0) {  // the slice's tail (< 4 elements: only the last slice has one)
    for (long i = len4 * 4 + t; i < len; i += IPC_T) {
      float s = a.data[0][s0 + i];
      for (int p = 1; p < W; ++p) s += a.data[p][s0 + i];
      a.stage[r][i] = s;
    }
  }
  ipc_barrier(a, 1);
  // phase 2: every slice from its owner's staging buffer, starting at the next rank (spreads the
  // reads over the peers' links)
  for (int k = 0; k < W; ++k) {
    const int p = (r + 1 + k) % W;
    const long q0 = (long)p * a.ns;
    const long q1 = q0 + a.ns < a.n ? q0 + a.ns : a.n;
    const long ql = q1 > q0 ? q1 - q0 : 0;
    const long ql4 = ql / 4;
    const float4* src = reinterpret_cast<const float4*>(a.stage[p]);
    float4* dst = reinterpret_cast<float4*>(a.data[r] + q0);
    for (long i = (long)b * IPC_T + t; i < ql4; i += (long)B * IPC_T) dst[i] = src[i];
    if (b == 0)
      for (long i = ql4 * 4 + t; i < ql; i += IPC_T) a.data[r][q0 + i] = a.stage[p][i];
  }
}

}  // namespace

extern "C" {
// data[w] / stage[w] / sig[w]: device pointers of rank w's buffers as mapped in THIS process (this
// rank's own at index rank); data pointers must be 16-byte aligned.  blocks <= 128 (the same on every
// rank).  Returns a HIP error code, -2 for bad arguments.
int dpa_ipc_allreduce(float* const* data, float* const* stage, unsigned* const* sig, int rank, int world, long n,
                      unsigned epoch, int blocks, int* tmo, long long timeout_us, hipStream_t st) {
  if (world < 1 || world > IPC_MAXW || rank < 0 || rank >= world || blocks < 1 || blocks > IPC_MAXB || n < 0) return -2;
  IpcArgs a{};
  for (int w = 0; w < world; ++w) {
    if ((reinterpret_cast<uintptr_t>(data[w]) & 15) || (reinterpret_cast<uintptr_t>(stage[w]) & 15)) return -2;
    a.data[w] = data[w];
    a.stage[w] = stage[w];
    a.sig[w] = sig[w];
  }
  a.rank = rank;
  a.world = world;
  a.n = n;
  a.ns = ((n + world - 1) / world + 3) / 4 * 4;
  a.epoch = epoch;
  a.tmo = tmo;
  int dev = 0, khz = 0;
  DPA_HIP_CHECK(hipGetDevice(&dev));
  DPA_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;
  a.ticks = (unsigned long long)timeout_us * (unsigned long long)khz / 1000ull;
  ipc_allreduce_kernel<<<blocks, IPC_T, 0, st>>>(a);
  return (int)hipGetLastError();
}

// slice length the kernel uses (the staging buffer must hold it)
long dpa_ipc_slice(long n, int world) { return ((n + world - 1) / world + 3) / 4 * 4; }

// signal words per rank
long dpa_ipc_sig_words() { return 2L * IPC_MAXW * IPC_MAXB; }
}  // extern "C"
