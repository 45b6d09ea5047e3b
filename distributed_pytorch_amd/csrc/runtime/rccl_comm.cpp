#include "rccl_comm.h"

#include <cstring>
#include <stdexcept>

namespace dpa {

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

RcclComm::RcclComm(int rank, int world, const std::string& uid, int device, hipStream_t comm_stream)
    : rank_(rank), world_(world), device_(device), stream_(comm_stream) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad RCCL unique id size");
  hip_check(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  hip_check(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming), "hipEventCreate");
}

RcclComm::~RcclComm() {
  if (comm_) {
    if (aborted_)
      ncclCommAbort(comm_);
    else
      ncclCommDestroy(comm_);
  }
  hipEventDestroy(ev_in_);
  hipEventDestroy(ev_out_);
}

void RcclComm::fence_after(hipStream_t after) {
  if (after == stream_) return;
  hip_check(hipEventRecord(ev_in_, after), "hipEventRecord");
  hip_check(hipStreamWaitEvent(stream_, ev_in_, 0), "hipStreamWaitEvent");
}

void RcclComm::all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t after) {
  fence_after(after);
  check(ncclAllReduce(buf, buf, count, dt, op, comm_, stream_), "ncclAllReduce");
}

void RcclComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t after) {
  fence_after(after);
  check(ncclBroadcast(buf, buf, count, dt, root, comm_, stream_), "ncclBroadcast");
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

void RcclComm::reduce_scatter(const void* send, void* recv, size_t recvcount, ncclDataType_t dt, ncclRedOp_t op,
                              hipStream_t after) {
  fence_after(after);
  check(ncclReduceScatter(send, recv, recvcount, dt, op, comm_, stream_), "ncclReduceScatter");
}

void RcclComm::all_gather(const void* send, void* recv, size_t sendcount, ncclDataType_t dt, hipStream_t after) {
  fence_after(after);
  check(ncclAllGather(send, recv, sendcount, dt, comm_, stream_), "ncclAllGather");
}

void RcclComm::send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t after) {
  fence_after(after);
  check(ncclSend(buf, count, dt, peer, comm_, stream_), "ncclSend");
}

void RcclComm::recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t after) {
  fence_after(after);
  check(ncclRecv(buf, count, dt, peer, comm_, stream_), "ncclRecv");
}

void RcclComm::wait(hipStream_t waiter) {
  if (waiter == stream_) return;
  hip_check(hipEventRecord(ev_out_, stream_), "hipEventRecord");
  hip_check(hipStreamWaitEvent(waiter, ev_out_, 0), "hipStreamWaitEvent");
}

void RcclComm::synchronize() { hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize"); }

std::string RcclComm::async_error() {
  if (!comm_) return "no communicator";
  ncclResult_t e = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError(comm_, &e);
  if (r != ncclSuccess) return ncclGetErrorString(r);
  if (e != ncclSuccess && e != ncclInProgress) return ncclGetErrorString(e);
  return "";
}

void RcclComm::abort() {
  if (comm_ && !aborted_.exchange(true)) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

}  // namespace dpa
