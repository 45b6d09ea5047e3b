#include "rccl_comm.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace dpa {

using Lock = std::unique_lock<std::timed_mutex>;

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

void RcclComm::check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL error in ") + what + ": " + ncclGetErrorString(r));
}

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

int RcclComm::version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

namespace {
// Fence / completion events only order streams of this device (and let the watchdog observe
// completion), so they record with a device-scope release: a system-scope one writes back and
// invalidates L2 under the compute kernels running beside the collective.
unsigned event_flags() { return hipEventDisableTiming | hipEventReleaseToDevice; }
}  // namespace

RcclComm::RcclComm(int rank, int world, const std::string& uid, int device, hipStream_t comm_stream,
                   WatchdogConfig wd, int max_ctas)
    : rank_(rank), world_(world), device_(device), stream_(comm_stream), wd_(wd) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad RCCL unique id size");
  hip_check(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  if (max_ctas > 0) {
    // a bounded channel count: fewer RCCL workgroups share the CUs with the backward kernels
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 1;
    cfg.minCTAs = 1;
    cfg.maxCTAs = max_ctas;
    check(ncclCommInitRankConfig(&comm_, world, id, rank, &cfg), "ncclCommInitRankConfig");
  } else {
    check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  }
  max_ctas_ = max_ctas;
  comm_raw_ = comm_;
  hip_check(hipEventCreateWithFlags(&ev_in_, event_flags()), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&ev_out_, event_flags()), "hipEventCreate");
  const char* w = std::getenv("DPA_RCCL_WARMUP");
  if (world_ > 1 && !(w && std::string(w) == "0")) warmup_connections();
  if (wd_.enabled) watchdog_ = std::thread([this] { watchdog_loop(); });
}

// RCCL connects peers lazily, inside the first collective / send-recv group that needs them, and
// that enqueue call can block on a dead peer while it holds comm_mu_.  One tiny round of every
// pattern the sync modes issue (all-reduce, broadcast, the gather's grouped send/recv to rank 0)
// at start-up makes every later enqueue a pure queue operation.
void RcclComm::warmup_connections() {
  void* buf = nullptr;
  const size_t n = 64;  // floats per rank
  hip_check(hipMalloc(&buf, n * sizeof(float) * (size_t)(world_ + 1)), "hipMalloc");
  hip_check(hipMemsetAsync(buf, 0, n * sizeof(float) * (size_t)(world_ + 1), stream_), "hipMemsetAsync");
  float* b = static_cast<float*>(buf);
  check(ncclAllReduce(b, b, n, ncclFloat32, ncclSum, comm_, stream_), "ncclAllReduce(warmup)");
  check(ncclBroadcast(b, b, n, ncclFloat32, 0, comm_, stream_), "ncclBroadcast(warmup)");
  check(ncclGroupStart(), "ncclGroupStart");
  if (rank_ == 0) {
    for (int p = 1; p < world_; ++p) check(ncclRecv(b + (size_t)p * n, n, ncclFloat32, p, comm_, stream_), "ncclRecv");
  } else {
    check(ncclSend(b + (size_t)world_ * n, n, ncclFloat32, 0, comm_, stream_), "ncclSend");
  }
  check(ncclGroupEnd(), "ncclGroupEnd");
  // Bounded wait: the watchdog thread does not run yet, and a peer that dies between
  // ncclCommInitRank and here would leave an unbounded synchronize hanging.  Only this
  // thread knows the communicator, so aborting it here is safe.
  hipEvent_t ev;
  hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventRecord(ev, stream_), "hipEventRecord");
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) break;
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (q != hipErrorNotReady || waited > wd_.timeout_s) {
      hipEventDestroy(ev);
      std::fprintf(stderr, "[dpa rank %d] RCCL connection warm-up %s after %.1f s\n", rank_,
                   q != hipErrorNotReady ? hipGetErrorString(q) : "timed out", waited);
      std::fflush(stderr);
      if (wd_.exit_on_error) std::_Exit(70);
      ncclCommAbort(comm_);
      comm_ = comm_raw_ = nullptr;
      throw std::runtime_error("RCCL connection warm-up failed (peer dead or hung)");
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  hipEventDestroy(ev);
  hip_check(hipFree(buf), "hipFree");
}

RcclComm::~RcclComm() {
  stop_ = true;
  cv_.notify_all();
  if (watchdog_.joinable()) watchdog_.join();
  {
    Lock g(comm_mu_);
    // a healthy communicator is destroyed in order; one whose peer failed is aborted (destroy
    // could wait forever on collectives that will never complete)
    release_locked(state_.load() != kHealthy);
  }
  for (auto& op : ops_) hipEventDestroy(op.ev);
  for (auto ev : free_events_) hipEventDestroy(ev);
  hipEventDestroy(ev_in_);
  hipEventDestroy(ev_out_);
}

void RcclComm::release_locked(bool abort) {
  if (comm_) {
    if (abort)
      ncclCommAbort(comm_);
    else
      ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  state_ = kAborted;
}

void RcclComm::require_healthy_locked() {
  if (state_.load() != kHealthy || !comm_) {
    std::lock_guard<std::mutex> g(mu_);
    throw std::runtime_error("RCCL communicator is aborted: " + (error_.empty() ? std::string("abort()") : error_));
  }
}

int RcclComm::comm_count() {
  Lock g(comm_mu_);
  if (!comm_ || state_.load() != kHealthy) return -1;
  int n = -1;
  if (ncclCommCount(comm_, &n) != ncclSuccess) return -1;
  return n;
}

void RcclComm::end_op(const char* what, hipStream_t on) {
  ops_issued_++;
  if (on == nullptr) on = stream_;
  if (wd_.debug_sync) {  // host-synchronous op: surfaces ordering bugs and errors at the call site
    hip_check(hipStreamSynchronize(on), what);
    const std::string e = async_error();
    if (!e.empty()) throw std::runtime_error(std::string("RCCL error after ") + what + ": " + e);
    return;
  }
  if (!wd_.enabled) return;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!free_events_.empty()) {
      ev = free_events_.back();
      free_events_.pop_back();
    } else {
      hip_check(hipEventCreateWithFlags(&ev, event_flags()), "hipEventCreate");
    }
  }
  hip_check(hipEventRecord(ev, on), "hipEventRecord");
  std::lock_guard<std::mutex> g(mu_);
  ops_.push_back(Op{ev, std::chrono::steady_clock::now(), what});
}

size_t RcclComm::outstanding() {
  std::lock_guard<std::mutex> g(mu_);
  return ops_.size();
}

void RcclComm::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (error_.empty()) error_ = msg;
  }
  int expect = kHealthy;
  state_.compare_exchange_strong(expect, kFailed);  // from now on every issue throws
  std::fprintf(stderr, "[dpa rank %d] RCCL watchdog: %s\n", rank_, msg.c_str());
  std::fflush(stderr);
  if (wd_.exit_on_error) {
    // the process is about to end: the driver reclaims the context (and with it the RCCL kernels
    // spinning on the dead peer); no abort call that could itself block on the fabric
    std::fprintf(stderr, "[dpa rank %d] terminating the process (exit 70) so the launcher can tear the job down\n",
                 rank_);
    std::fflush(stderr);
    std::_Exit(70);
  }
  // Abort under comm_mu_: an issue that is in flight finishes first (enqueue calls return without
  // waiting on peers), and no issuer can ever see the handle after it is released.  An issuer that
  // holds the lock longer than the timeout is itself stuck inside RCCL on this blocking
  // communicator; aborting it from here would free state that thread still uses, so
  // the process ends as in the default mode.
  const auto t0 = std::chrono::steady_clock::now();
  while (!stop_) {
    Lock g(comm_mu_, std::defer_lock);
    if (g.try_lock_for(std::chrono::milliseconds(500))) {
      release_locked(true);
      return;
    }
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (waited > wd_.timeout_s) {
      std::fprintf(stderr,
                   "[dpa rank %d] RCCL watchdog: an enqueue is stuck inside RCCL; terminating the process (exit 70)\n",
                   rank_);
      std::fflush(stderr);
      std::_Exit(70);
    }
  }
}

void RcclComm::watchdog_loop() {
  hipSetDevice(device_);
  const auto poll = std::chrono::duration<double>(wd_.poll_s);
  while (!stop_) {
    {
      std::unique_lock<std::mutex> lk(wake_mu_);
      cv_.wait_for(lk, poll, [this] { return stop_.load(); });
    }
    if (stop_ || state_.load() != kHealthy) break;
    // retire completed ops in issue order; time out the oldest pending one
    std::string timeout_msg;
    {
      std::lock_guard<std::mutex> g(mu_);
      while (!ops_.empty()) {
        const hipError_t q = hipEventQuery(ops_.front().ev);
        if (q == hipSuccess) {
          free_events_.push_back(ops_.front().ev);
          ops_.pop_front();
          continue;
        }
        const double age = std::chrono::duration<double>(std::chrono::steady_clock::now() - ops_.front().t).count();
        if (q == hipErrorNotReady && age > wd_.timeout_s) {
          char buf[256];
          std::snprintf(buf, sizeof(buf), "%s outstanding for %.1f s (timeout %.1f s): peer dead or hung",
                        ops_.front().what, age, wd_.timeout_s);
          timeout_msg = buf;
        } else if (q != hipErrorNotReady) {
          timeout_msg = std::string("HIP error on the comm stream: ") + hipGetErrorString(q);
        }
        break;
      }
    }
    if (!timeout_msg.empty()) {
      fail(timeout_msg);
      break;
    }
    std::string async_msg;
    {
      Lock g(comm_mu_, std::try_to_lock);  // the issuer holds it only for an enqueue: skip this poll
      if (g.owns_lock() && comm_) {
        ncclResult_t e = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &e) == ncclSuccess && e != ncclSuccess && e != ncclInProgress)
          async_msg = std::string("asynchronous RCCL error: ") + ncclGetErrorString(e);
      }
    }
    if (!async_msg.empty()) {
      fail(async_msg);
      break;
    }
  }
}

void RcclComm::fence_after(hipStream_t after) {
  if (after == stream_) return;
  hip_check(hipEventRecord(ev_in_, after), "hipEventRecord");
  hip_check(hipStreamWaitEvent(stream_, ev_in_, 0), "hipStreamWaitEvent");
}

void RcclComm::all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t after) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    fence_after(after);
    check(ncclAllReduce(buf, buf, count, dt, op, comm_, stream_), "ncclAllReduce");
  }
  end_op("all_reduce");
}

void RcclComm::all_reduce_here(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t stream) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    check(ncclAllReduce(buf, buf, count, dt, op, comm_, stream), "ncclAllReduce");
  }
  end_op("all_reduce", stream);
}

void RcclComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t after) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    fence_after(after);
    check(ncclBroadcast(buf, buf, count, dt, root, comm_, stream_), "ncclBroadcast");
  }
  end_op("broadcast");
}

static size_t dt_size(ncclDataType_t dt) {
  switch (dt) {
    case ncclInt8:
    case ncclUint8:
      return 1;
    case ncclFloat16:
    case ncclBfloat16:
      return 2;
    case ncclInt32:
    case ncclUint32:
    case ncclFloat32:
      return 4;
    default:
      return 8;
  }
}

void RcclComm::gather(const void* send, void* recv, size_t count, ncclDataType_t dt, int root, hipStream_t after) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    fence_after(after);
    const size_t bytes = count * dt_size(dt);
    check(ncclGroupStart(), "ncclGroupStart");
    if (rank_ == root) {
      for (int p = 0; p < world_; ++p) {
        char* dst = static_cast<char*>(recv) + (size_t)p * bytes;
        if (p == root) {
          if (dst != send) hip_check(hipMemcpyAsync(dst, send, bytes, hipMemcpyDeviceToDevice, stream_), "memcpy");
        } else {
          check(ncclRecv(dst, count, dt, p, comm_, stream_), "ncclRecv");
        }
      }
    } else {
      check(ncclSend(send, count, dt, root, comm_, stream_), "ncclSend");
    }
    check(ncclGroupEnd(), "ncclGroupEnd");
  }
  end_op("gather");
}

void RcclComm::reduce_scatter(const void* send, void* recv, size_t recvcount, ncclDataType_t dt, ncclRedOp_t op,
                              hipStream_t after) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    fence_after(after);
    check(ncclReduceScatter(send, recv, recvcount, dt, op, comm_, stream_), "ncclReduceScatter");
  }
  end_op("reduce_scatter");
}

void RcclComm::all_gather(const void* send, void* recv, size_t sendcount, ncclDataType_t dt, hipStream_t after) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    fence_after(after);
    check(ncclAllGather(send, recv, sendcount, dt, comm_, stream_), "ncclAllGather");
  }
  end_op("all_gather");
}

void RcclComm::send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t after) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    fence_after(after);
    check(ncclSend(buf, count, dt, peer, comm_, stream_), "ncclSend");
  }
  end_op("send");
}

void RcclComm::recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t after) {
  {
    Lock g(comm_mu_);
    require_healthy_locked();
    fence_after(after);
    check(ncclRecv(buf, count, dt, peer, comm_, stream_), "ncclRecv");
  }
  end_op("recv");
}

void RcclComm::wait(hipStream_t waiter) {
  if (waiter == stream_) return;
  hip_check(hipEventRecord(ev_out_, stream_), "hipEventRecord");
  hip_check(hipStreamWaitEvent(waiter, ev_out_, 0), "hipStreamWaitEvent");
}

void RcclComm::synchronize() { hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize"); }

std::string RcclComm::async_error() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!error_.empty()) return error_;
  }
  Lock g(comm_mu_);
  if (state_.load() != kHealthy) return "communicator aborted";
  if (!comm_) return "no communicator";
  ncclResult_t e = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError(comm_, &e);
  if (r != ncclSuccess) return ncclGetErrorString(r);
  if (e != ncclSuccess && e != ncclInProgress) return ncclGetErrorString(e);
  return "";
}

void RcclComm::abort() {
  stop_ = true;
  cv_.notify_all();
  if (watchdog_.joinable() && watchdog_.get_id() != std::this_thread::get_id()) watchdog_.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    if (error_.empty()) error_ = "abort()";
  }
  Lock g(comm_mu_);
  release_locked(true);
}

}  // namespace dpa
