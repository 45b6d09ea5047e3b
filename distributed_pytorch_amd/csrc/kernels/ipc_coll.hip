// Peer-memory collectives over the ranks of one node: every rank maps its peers' registered
// memory (gradient / parameter / momentum / buffer arenas), inboxes, staging buffers and signal
// words through HIP IPC (runtime/ipc_comm.cpp), and one kernel per collective reads them
// directly -- over xGMI between MI355X GPUs, or through the same HBM when several ranks share one
// GPU (the only multi-rank device path a one-GPU lease can run).  Reference semantics:
//   all_reduce(SUM)        main_all_reduce.py:45-48, the DDP buckets of main_ddp.py:137
//   gather -> mean -> scatter (== broadcast of the mean)   main_gather.py:49,59
//   broadcast              DDP's initial state and per-forward BN-buffer sync
//   reduce-scatter / all-gather   the ZeRO-1 mode (new scope)
// mesh-aware, every rank reads all its peers at once, one link each.
//
// B workgroups per rank (a fixed CU budget, like RCCL's channel count).  Every collective is
//   [bounce]   an input that is not registered memory is first copied into this rank's inbox;
//   barrier A  block b of every rank has started: every rank's input (written by kernels
//              stream-ordered before it, or by the bounce) is complete and visible;
//   phase 1    the data movement (all-reduce: reduce-scatter into the staging buffers);
//   barrier B  block b of every rank is done reading its peers (all-reduce: has stored its part of
//              the reduce-scatter);
//   phase 2    all-reduce only: all-gather of the reduced slices from the peers' staging buffers.
// Work partition: a message of len words is split into 4-word groups; group i of a segment belongs
// to block (i / 256) mod B in every phase and on every rank (the same grid-stride loop everywhere),
// so block b only ever reads peer words written by block b of that peer before the barrier that
// separates them -- a per-block barrier is enough, and no grid-wide one is needed.
//
// Why reuse of the inbox / staging buffers needs no trailing barrier: a rank's next collective
// starts only after its previous kernel finished (one stream), i.e. after every block of it passed
// barrier B, i.e. after every block of every peer finished reading this rank's inbox and registered
// memory (phase 1).  The all-reduce's staging buffer is read by peers in phase 2 -- after barrier B
// -- and rewritten only in the next all-reduce's phase 1, after that collective's barrier A, which a
// peer's block b reaches only once its previous kernel (with its phase 2 reads) has completed.
// All ranks issue the same sequence of collectives, so the signal epochs (one per collective,
// monotonic) agree.  Results are bitwise identical on every rank (each element is reduced once, in
// rank order 0..W-1, by its slice owner).
#include "common.h"
#include "ipc_coll.h"

namespace {

constexpr int IPC_T = 256;

typedef __attribute__((address_space(1))) unsigned gu32;

// Cross-process / cross-GPU memory model of the barrier (gfx950 ordering rules):
//  * A producer's data is written by earlier kernels of its stream (ordered before this kernel and
//    released at their end: the end-of-kernel release writes the XCD L2s back to memory), by this
//    kernel's bounce copy, or by phase 1.  Each wave waits for its own stores (vmcnt(0)) and the
//    workgroup syncs; the system-scope RELEASE fence then writes this XCD's L2 back to memory, so
//    everything the block wrote (and the XCD cached dirty) is in HBM before the flag store.
//  * The flag words live in uncached (hipDeviceMallocUncached) memory of the waiting rank: stores
//    from peers (over xGMI or from another process on the same GPU) and the poll meet in memory.
//  * The consumer's system-scope ACQUIRE fence after the poll invalidates its L2 / L1, so the
//    peer reads that follow cannot hit lines cached before the producer's writeback.
// Waits are bounded: after `ticks` of the wall clock the block gives up and raises the tmo word
// (the results of that collective are then invalid; the host reports it, nothing hangs).
__device__ __forceinline__ void ipc_barrier(const DpaIpcArgs& a, int phase) {
  const int t = threadIdx.x, b = blockIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < 64) {
    // every lane that stores a flag or polls one runs the fences itself (system scope: visible to
    // every peer), so the ordering does not depend on a fence in lane 0 acting for the whole wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (t < a.world && t != a.rank)
      __hip_atomic_store((gu32*)(a.sig[t] + (phase * DPA_IPC_MAXW + a.rank) * DPA_IPC_MAXB + b), a.epoch,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < a.world && t != a.rank) {
      const gu32* w = (const gu32*)(a.sig[a.rank] + (phase * DPA_IPC_MAXW + t) * DPA_IPC_MAXB + b);
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
        if (wall_clock64() - t0 > a.ticks) {
          __hip_atomic_store((gint*)a.tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

__device__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// words [4i, 4i + 4) of p, clipped to len (the vector path needs a 16-byte aligned p)
__device__ __forceinline__ uint4 ld4(const unsigned* p, long i, long len) {
  const long w = 4 * i;
  if (w + 4 <= len && al16(p)) return reinterpret_cast<const uint4*>(p)[i];
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (w < len) v.x = p[w];
  if (w + 1 < len) v.y = p[w + 1];
  if (w + 2 < len) v.z = p[w + 2];
  if (w + 3 < len) v.w = p[w + 3];
  return v;
}
__device__ __forceinline__ void st4(unsigned* p, long i, long len, uint4 v) {
  const long w = 4 * i;
  if (w + 4 <= len && al16(p)) {
    reinterpret_cast<uint4*>(p)[i] = v;
    return;
  }
  if (w < len) p[w] = v.x;
  if (w + 1 < len) p[w + 1] = v.y;
  if (w + 2 < len) p[w + 2] = v.z;
  if (w + 3 < len) p[w + 3] = v.w;
}

template <int RED>
__device__ __forceinline__ float red1(float x, float y) {
  if constexpr (RED == DPA_IPC_SUM) return x + y;
  else if constexpr (RED == DPA_IPC_MAX) return fmaxf(x, y);
  else return fminf(x, y);
}
template <int RED>
__device__ __forceinline__ uint4 red4(uint4 x, uint4 y) {
  return make_uint4(__float_as_uint(red1<RED>(__uint_as_float(x.x), __uint_as_float(y.x))),
                    __float_as_uint(red1<RED>(__uint_as_float(x.y), __uint_as_float(y.y))),
                    __float_as_uint(red1<RED>(__uint_as_float(x.z), __uint_as_float(y.z))),
                    __float_as_uint(red1<RED>(__uint_as_float(x.w), __uint_as_float(y.w))));
}

// group i of rank order 0..W-1 reduced: the loads of all W ranks are issued before the adds
template <int RED>
__device__ __forceinline__ uint4 reduce_group(const DpaIpcArgs& a, long seg_off, long i, long len) {
  uint4 v[DPA_IPC_MAXW];
#pragma unroll
  for (int p = 0; p < DPA_IPC_MAXW; ++p)
    if (p < a.world) v[p] = ld4(a.src[p] + seg_off, i, len);
  uint4 s = v[0];
#pragma unroll
  for (int p = 1; p < DPA_IPC_MAXW; ++p)
    if (p < a.world) s = red4<RED>(s, v[p]);
  return s;
}

__device__ __forceinline__ long seg_len(long total, long s0, long len) {
  const long m = total - s0;
  return m < 0 ? 0 : (m < len ? m : len);
}

template <int RED>
__global__ __launch_bounds__(IPC_T) void ipc_coll_kernel(DpaIpcArgs a) {
  const int W = a.world, r = a.rank;
  const long g0 = (long)blockIdx.x * IPC_T + threadIdx.x, gs = (long)gridDim.x * IPC_T;
  if (a.in != nullptr) {  // bounce: this rank's input into its inbox (same partition as the readers)
    for (int q = 0; q < a.pc_nseg; ++q) {
      const long len = seg_len(a.pc_total, q * a.pc_len, a.pc_len);
      const unsigned* s = a.in + q * a.istride;
      unsigned* d = a.inbox + q * a.pc_len;
      for (long i = g0; 4 * i < len; i += gs) st4(d, i, len, ld4(s, i, len));
    }
  }
  ipc_barrier(a, 0);
  if (a.op == DPA_IPC_BARRIER) return;
  if (a.op == DPA_IPC_ALL_REDUCE) {
    // phase 1: slice r reduced over all ranks into this rank's staging buffer
    const long s0 = (long)r * a.ns, len = seg_len(a.n, s0, a.ns);
    for (long i = g0; 4 * i < len; i += gs) st4(a.stage[r], i, len, reduce_group<RED>(a, s0, i, len));
    ipc_barrier(a, 1);
    // phase 2: every slice from its owner's staging buffer, starting at the next rank (spreads the
    // reads over the peers' links)
    for (int k = 0; k < W; ++k) {
      const int p = (r + 1 + k) % W;
      const long q0 = (long)p * a.ns, ql = seg_len(a.n, q0, a.ns);
      for (long i = g0; 4 * i < ql; i += gs) st4(a.dst + q0, i, ql, ld4(a.stage[p], i, ql));
    }
    return;
  }
  const long n = a.n;
  if (a.op == DPA_IPC_BROADCAST) {
    if (r != a.root)
      for (long i = g0; 4 * i < n; i += gs) st4(a.dst, i, n, ld4(a.src[a.root], i, n));
  } else if (a.op == DPA_IPC_GATHER) {
    if (r == a.root)
      for (long i = g0; 4 * i < n; i += gs) {
        uint4 v[DPA_IPC_MAXW];
#pragma unroll
        for (int p = 0; p < DPA_IPC_MAXW; ++p)
          if (p < W) v[p] = ld4(a.src[p], i, n);
#pragma unroll
        for (int p = 0; p < DPA_IPC_MAXW; ++p)
          if (p < W) st4(a.dst + p * a.dstride, i, n, v[p]);
      }
  } else if (a.op == DPA_IPC_REDUCE_SCATTER) {
    // (in place is safe: segment r of this rank is read by this rank only, by the same thread
    // that writes it)
    for (long i = g0; 4 * i < n; i += gs) st4(a.dst, i, n, reduce_group<RED>(a, (long)r * a.sstride, i, n));
  } else if (a.op == DPA_IPC_ALL_GATHER) {
    // this rank's own slot is skipped when the input already is that slot (peers may be reading it)
    const bool self_in_place = a.src[r] == a.dst + r * a.dstride;
    for (long i = g0; 4 * i < n; i += gs) {
      uint4 v[DPA_IPC_MAXW];
#pragma unroll
      for (int p = 0; p < DPA_IPC_MAXW; ++p)
        if (p < W && !(p == r && self_in_place)) v[p] = ld4(a.src[p], i, n);
#pragma unroll
      for (int p = 0; p < DPA_IPC_MAXW; ++p)
        if (p < W && !(p == r && self_in_place)) st4(a.dst + p * a.dstride, i, n, v[p]);
    }
  }
  ipc_barrier(a, 1);  // peers are done reading this rank's memory before it moves on
}

}  // namespace

extern "C" {
int dpa_ipc_coll(DpaIpcArgs* a, int blocks, long long timeout_us, hipStream_t st) {
  if (a->world < 1 || a->world > DPA_IPC_MAXW || a->rank < 0 || a->rank >= a->world || blocks < 1 ||
      blocks > DPA_IPC_MAXB || a->n < 0 || a->op < 0 || a->op > DPA_IPC_BARRIER || a->root < 0 ||
      a->root >= a->world || a->red < 0 || a->red > DPA_IPC_MIN)
    return -2;
  if (a->op == DPA_IPC_ALL_REDUCE && ((a->ns & 3) || (long)a->world * a->ns < a->n)) return -2;
  int dev = 0, khz = 0;
  DPA_HIP_CHECK(hipGetDevice(&dev));
  DPA_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;
  a->ticks = (unsigned long long)timeout_us * (unsigned long long)khz / 1000ull;
  if (a->red == DPA_IPC_MAX)
    ipc_coll_kernel<DPA_IPC_MAX><<<blocks, IPC_T, 0, st>>>(*a);
  else if (a->red == DPA_IPC_MIN)
    ipc_coll_kernel<DPA_IPC_MIN><<<blocks, IPC_T, 0, st>>>(*a);
  else
    ipc_coll_kernel<DPA_IPC_SUM><<<blocks, IPC_T, 0, st>>>(*a);
  return (int)hipGetLastError();
}

long dpa_ipc_slice(long n, int world) { return ((n + world - 1) / world + 3) / 4 * 4; }

long dpa_ipc_sig_words() { return 2L * DPA_IPC_MAXW * DPA_IPC_MAXB; }
}  // extern "C"
