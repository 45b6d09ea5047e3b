// Peer-memory communicator: HIP IPC mappings of every rank's buffers plus the peer-memory
// collective kernel (kernels/ipc_coll.hip): all-reduce (sum/max/min), broadcast, gather,
// reduce-scatter, all-gather and a device barrier.  One process per GPU over xGMI, or several
// processes on one GPU (the one-GPU lease's only device-side multi-rank path; RCCL refuses two
// ranks on one device).
//
// Bootstrap (parallel/ipc.py): every rank exports opaque handles (the IPC handle of the allocation
// holding a buffer plus the buffer's offset in it) for its signal array, staging buffer, inbox and
// every memory region it registers; the handles go through the rendezvous store; each rank opens
// its peers'.  Signal words live in uncached device memory (hipDeviceMallocUncached) so that polls
// and flag stores of different processes and devices meet in memory.
//
// Inputs: a registered region (zero copy -- the peers read it in place; the input's word offset in
// the region must be the same on every rank, as for the engine's arenas, except for the in-place
// all-gather, whose input is each rank's own slot of the output) or any other device
// memory, which the kernel first copies into this rank's inbox ("bounce"; collectives larger than
// the inbox run as several pieces).  Every length is in 4-byte words.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <utility>
#include <vector>

struct DpaIpcArgs;

namespace dpa {

class IpcComm {
 public:
  // stage_words: the all-reduce staging buffer (>= the largest piece's slice); inbox_words: the
  // bounce buffer
  IpcComm(int rank, int world, int device, long stage_words, long inbox_words);
  ~IpcComm();
  IpcComm(const IpcComm&) = delete;
  IpcComm& operator=(const IpcComm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  long stage_words() const { return stage_words_; }
  long inbox_words() const { return inbox_words_; }

  // 72-byte handle (hipIpcMemHandle_t + int64 offset) of a device pointer of this process
  static std::string export_handle(const void* p);
  std::string sig_handle() const { return export_handle(sig_); }
  std::string stage_handle() const { return export_handle(stage_); }
  std::string inbox_handle() const { return export_handle(inbox_); }

  // peers' signal arrays, staging buffers and inboxes (handles indexed by rank; own entry ignored)
  void set_peers(const std::vector<std::string>& sig, const std::vector<std::string>& stage,
                 const std::vector<std::string>& inbox);
  // a region of `words` words, `local` in this process, the peers' through their handles; returns
  // its id
  int add_region(const std::vector<std::string>& handles, void* local, long words);

  // rid >= 0: the input is region rid at word offset off (== buf / in); rid < 0: bounced.
  // All collectives are issued on `st`, every rank the same sequence, `blocks` the same everywhere.
  void all_reduce(int rid, long off, void* buf, long n, int red, int blocks, long long tmo_us, hipStream_t st);
  void broadcast(int rid, long off, void* buf, long n, int root, int blocks, long long tmo_us, hipStream_t st);
  // out: the root's [world][n] words (ignored elsewhere)
  void gather(int rid, long off, const void* in, void* out, long n, int root, int blocks, long long tmo_us,
              hipStream_t st);
  // in: [world][n] words; out: this rank's n words (may be in's segment `rank`)
  void reduce_scatter(int rid, long off, const void* in, void* out, long n, int red, int blocks, long long tmo_us,
                      hipStream_t st);
  // in: this rank's n words (may be out's slot `rank`); out: [world][n] words
  void all_gather(int rid, long off, const void* in, void* out, long n, int blocks, long long tmo_us,
                  hipStream_t st);
  void barrier(int blocks, long long tmo_us, hipStream_t st);
  // the device word a timed-out peer wait raises (per-step health snapshot reads it)
  int* tmo_word() const { return tmo_; }

  // [offset, words) pieces of a collective of n words (one rank's words for gather / reduce-scatter /
  // all-gather): the piece sizes the staging buffer and the inbox allow, multiples of 4 words
  static std::vector<std::pair<long, long>> pieces(int op, long n, int world, long stage_words, long inbox_words,
                                                   bool registered);
  // a bounded wait of some collective gave up (results invalid); clears the word
  bool take_timeout();
  long launches() const { return launches_; }

 private:
  void* open(const std::string& h);
  void base_args(DpaIpcArgs& a, int op) const;
  const unsigned* region_ptr(int rid, long off, long n, int w) const;
  void launch(DpaIpcArgs& a, int blocks, long long tmo_us, hipStream_t st);

  int rank_, world_, device_;
  long stage_words_, inbox_words_;
  unsigned* sig_ = nullptr;
  unsigned* stage_ = nullptr;
  unsigned* inbox_ = nullptr;
  int* tmo_ = nullptr;
  unsigned epoch_ = 0;
  long launches_ = 0;
  std::vector<unsigned*> sig_peer_, stage_peer_, inbox_peer_;
  struct Region {
    std::vector<unsigned*> base;
    long words;
  };
  std::vector<Region> regions_;
  std::vector<void*> opened_;  // IPC mappings to close (allocation bases)
};

}  // namespace dpa
