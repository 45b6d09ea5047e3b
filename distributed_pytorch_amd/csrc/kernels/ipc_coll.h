// Launch interface of the peer-memory collectives (kernels/ipc_coll.hip), shared with the host
// communicator (runtime/ipc_comm.cpp).  Plain data only: compiled by hipcc and by the host compiler.
#pragma once
#include <hip/hip_runtime.h>

#define DPA_IPC_MAXW 8    // ranks
#define DPA_IPC_MAXB 128  // workgroups per rank

enum DpaIpcOp {
  DPA_IPC_ALL_REDUCE = 0,      // in place, two-shot through the staging buffers
  DPA_IPC_BROADCAST = 1,       // non-root ranks pull the root's words
  DPA_IPC_GATHER = 2,          // the root pulls every rank's words into dst slot p
  DPA_IPC_REDUCE_SCATTER = 3,  // rank r reduces segment r of every rank's input
  DPA_IPC_ALL_GATHER = 4,      // every rank pulls every rank's words into dst slot p
  DPA_IPC_BARRIER = 5,
};
enum DpaIpcRed { DPA_IPC_SUM = 0, DPA_IPC_MAX = 1, DPA_IPC_MIN = 2 };

// Every length, offset and stride is in 4-byte words (reductions read the words as fp32).
struct DpaIpcArgs {
  const unsigned* src[DPA_IPC_MAXW];  // rank p's input as mapped in this process (its registered
                                      // memory, or its inbox when the input is bounced)
  unsigned* stage[DPA_IPC_MAXW];      // all-reduce: rank p's staging buffer
  unsigned* sig[DPA_IPC_MAXW];        // rank p's signal array [2][MAXW][MAXB]
  // bounce: before the first barrier this rank copies pc_nseg segments of pc_len words (clipped to
  // pc_total words overall) from in + q * istride to inbox + q * pc_len (in == nullptr: none)
  const unsigned* in;
  unsigned* inbox;
  long pc_len, pc_total, istride;
  int pc_nseg;
  unsigned* dst;  // this rank's output
  long n;         // words: all-reduce / broadcast: the whole message; gather / all-gather: one
                  // rank's contribution; reduce-scatter: one rank's segment
  long sstride;   // words between the segments of src[p] (reduce-scatter)
  long dstride;   // words between the rank slots of dst (gather / all-gather)
  long ns;        // all-reduce: slice words (multiple of 4)
  int rank, world, root, op, red;
  unsigned epoch;
  int* tmo;
  unsigned long long ticks;
};

extern "C" {
// blocks: workgroups per rank (1..DPA_IPC_MAXB, the same on every rank); returns a HIP error code,
// -2 for bad arguments
int dpa_ipc_coll(DpaIpcArgs* a, int blocks, long long timeout_us, hipStream_t st);
// all-reduce slice length for n words over `world` ranks (the staging buffer must hold it)
long dpa_ipc_slice(long n, int world);
// signal words per rank
long dpa_ipc_sig_words();
}
