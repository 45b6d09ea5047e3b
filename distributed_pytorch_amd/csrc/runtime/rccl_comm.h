// Native RCCL communicator: one process per MI355X, collectives issued on a dedicated comm HIP
// stream that is fenced against the caller's compute stream with HIP events (no host sync).
//
// Replaces the reference's c10d ProcessGroupGloo usage:
//   gather/scatter (main_gather.py:49,59)  -> grouped ncclSend/ncclRecv + ncclBroadcast
//   all_reduce     (main_all_reduce.py:47) -> ncclAllReduce
//   DDP Reducer buckets / buffer broadcast (main_ddp.py:137) -> ncclAllReduce / ncclBroadcast
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dpa {

// Failure handling: every issued op is tracked with a completion event; a
// watchdog thread polls ncclCommGetAsyncError and the oldest outstanding op.  On an async RCCL
// error or an op outstanding longer than `timeout_s`, it records the error, aborts the
// communicator (unblocking RCCL kernels stuck on a dead peer) and, if `exit_on_error`, terminates
// the process (exit code 70) so the launcher tears the job down instead of hanging.
// `debug_sync` makes every op host-synchronous and error-checked (race / ordering debugging).
struct WatchdogConfig {
  double timeout_s = 600.0;
  double poll_s = 0.2;
  bool enabled = true;
  bool exit_on_error = true;
  bool debug_sync = false;
};

// Thread-safety contract.  Two threads touch the communicator: the issuing (Python) thread and the
// watchdog.  `comm_` is only read or changed with `comm_mu_` held: every enqueue holds it for the
// duration of the RCCL call(s), and the communicator is aborted / destroyed (and `comm_` cleared)
// under it, so no thread can use a handle another thread is tearing down.  `state_` moves
// kHealthy -> kFailed (watchdog recorded an error) -> kAborted (communicator released) and never
// back; an op issued in any state but kHealthy throws.
class RcclComm {
 public:
  // uid: NCCL_UNIQUE_ID_BYTES bytes created by rank 0 (unique_id()) and shared out of band.
  // max_ctas > 0: the communicator runs its collectives on at most that many workgroups (RCCL
  // channels, ncclConfig_t::maxCTAs) -- the CU footprint beside the overlapped backward.
  RcclComm(int rank, int world, const std::string& uid, int device, hipStream_t comm_stream,
           WatchdogConfig wd = WatchdogConfig(), int max_ctas = 0);
  ~RcclComm();

  static std::string unique_id();
  static int version();

  int rank() const { return rank_; }
  int world() const { return world_; }
  hipStream_t stream() const { return stream_; }
  // ranks RCCL itself reports for this communicator (ncclCommCount); -1 once aborted
  int comm_count();
  // the channel (workgroup) budget the communicator was created with; 0 = RCCL's default
  int max_ctas() const { return max_ctas_; }

  // All ops: comm stream waits for everything already queued on `after` (the compute stream),
  // then runs the collective.  Returns immediately.
  void all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t after);
  // the same collective issued on `stream` itself (no comm-stream hop): the caller orders it after
  // every earlier collective of this communicator (a join with the comm stream) -- the last bucket
  // of a backward, whose update follows on that stream
  void all_reduce_here(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t stream);
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t after);
  // Rank `root` receives world*count elements into recv (its own contribution copied in place).
  void gather(const void* send, void* recv, size_t count, ncclDataType_t dt, int root, hipStream_t after);
  void reduce_scatter(const void* send, void* recv, size_t recvcount, ncclDataType_t dt, ncclRedOp_t op,
                      hipStream_t after);
  void all_gather(const void* send, void* recv, size_t sendcount, ncclDataType_t dt, hipStream_t after);
  void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t after);
  void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t after);

  // `waiter` waits (device-side) for all comm work issued so far.
  void wait(hipStream_t waiter);
  // Host blocks until all comm work issued so far completes.
  void synchronize();
  // Non-blocking: returns "" if healthy, else an error string (async RCCL error or watchdog).
  std::string async_error();
  void abort();
  // ops issued and still outstanding (watchdog view)
  size_t outstanding();
  uint64_t ops_issued() const { return ops_issued_.load(); }

 private:
  enum State : int { kHealthy = 0, kFailed = 1, kAborted = 2 };
  void fence_after(hipStream_t after);
  void check(ncclResult_t r, const char* what);
  // throws if the communicator is not healthy; caller holds comm_mu_
  void require_healthy_locked();
  // track completion (or sync in debug mode) of an op issued on `on` (default: the comm stream);
  // caller does NOT hold comm_mu_
  void end_op(const char* what, hipStream_t on = nullptr);
  void watchdog_loop();
  void fail(const std::string& msg);  // watchdog thread only
  void release_locked(bool abort);    // caller holds comm_mu_
  void warmup_connections();          // constructor only

  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;  // guarded by comm_mu_
  // The handle as created, for the one abort the watchdog may issue WITHOUT comm_mu_: when an
  // issuer has held the lock past the timeout it is stuck inside RCCL (ncclCommAbort is callable
  // from another thread and unblocks it); the handle is then only cleared, never released again.
  ncclComm_t comm_raw_ = nullptr;
  int max_ctas_ = 0;
  std::timed_mutex comm_mu_;
  hipStream_t stream_;
  hipEvent_t ev_in_, ev_out_;
  std::atomic<int> state_{kHealthy};
  WatchdogConfig wd_;
  struct Op {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t;
    const char* what;
  };
  std::mutex mu_;  // guards ops_, free_events_, error_
  std::deque<Op> ops_;
  std::vector<hipEvent_t> free_events_;
  std::string error_;
  std::atomic<uint64_t> ops_issued_{0};
  std::atomic<bool> stop_{false};
  std::mutex wake_mu_;
  std::condition_variable cv_;
  std::thread watchdog_;
};

}  // namespace dpa
