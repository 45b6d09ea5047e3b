// Peer-memory communicator: HIP IPC mappings of every rank's buffers plus the two-shot all-reduce
// kernel (kernels/ipc_allreduce.hip).  One process per GPU over xGMI, or several processes on one
// GPU (the one-GPU lease's only device-side multi-rank path; RCCL refuses two ranks on one device).
//
// Bootstrap (parallel/ipc.py): every rank exports opaque handles (the IPC handle of the allocation
// holding a buffer plus the buffer's offset in it) for its signal array, its staging buffer and any
// data region it registers; the handles go through the rendezvous store; each rank opens its peers'.
// Signal words live in uncached device memory (hipDeviceMallocUncached) so that polls and flag
// stores of different processes and devices meet in memory.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

namespace dpa {

class IpcComm {
 public:
  // stage_floats: the staging buffer's size (>= the largest collective's slice, dpa_ipc_slice)
  IpcComm(int rank, int world, int device, long stage_floats);
  ~IpcComm();
  IpcComm(const IpcComm&) = delete;
  IpcComm& operator=(const IpcComm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  long stage_floats() const { return stage_floats_; }

  // 72-byte handle (hipIpcMemHandle_t + int64 offset) of a device pointer of this process
  static std::string export_handle(const void* p);
  std::string sig_handle() const { return export_handle(sig_); }
  std::string stage_handle() const { return export_handle(stage_); }

  // peers' signal arrays and staging buffers (handles indexed by rank; this rank's entry ignored)
  void set_peers(const std::vector<std::string>& sig, const std::vector<std::string>& stage);
  // a data region of `floats` elements, `local` in this process, peers' through their handles;
  // returns its id
  int add_region(const std::vector<std::string>& handles, float* local, long floats);

  // SUM all-reduce of [off, off + n) of region `id` on `stream` (every rank issues the same
  // sequence of collectives).  blocks: workgroups per rank (same on every rank).
  void all_reduce(int id, long off, long n, int blocks, long long timeout_us, hipStream_t stream);
  // a bounded wait of some collective gave up (results invalid); clears the word
  bool take_timeout();

 private:
  void* open(const std::string& h);

  int rank_, world_, device_;
  long stage_floats_;
  unsigned* sig_ = nullptr;
  float* stage_ = nullptr;
  int* tmo_ = nullptr;
  unsigned epoch_ = 0;
  std::vector<unsigned*> sig_peer_;
  std::vector<float*> stage_peer_;
  struct Region {
    std::vector<float*> base;
    long floats;
  };
  std::vector<Region> regions_;
  std::vector<void*> opened_;  // IPC mappings to close (allocation bases)
};

}  // namespace dpa
