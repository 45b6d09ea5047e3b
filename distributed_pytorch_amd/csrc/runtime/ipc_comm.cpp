#include "ipc_comm.h"

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>

#include "kernels/ipc_coll.h"

namespace dpa {

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

constexpr size_t HANDLE_BYTES = sizeof(hipIpcMemHandle_t) + sizeof(int64_t);

static long round4(long v) { return v / 4 * 4; }

IpcComm::IpcComm(int rank, int world, int device, long stage_words, long inbox_words)
    : rank_(rank), world_(world), device_(device), stage_words_(round4(stage_words)),
      inbox_words_(round4(inbox_words)) {
  if (world < 1 || world > DPA_IPC_MAXW || rank < 0 || rank >= world) throw std::runtime_error("IpcComm: 1..8 ranks");
  if (stage_words_ < 4 || inbox_words_ < 4L * world) throw std::runtime_error("IpcComm: buffers too small");
  hip_ok(hipSetDevice(device), "hipSetDevice");
  const size_t sig_bytes = (size_t)dpa_ipc_sig_words() * sizeof(unsigned);
  hip_ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sig_bytes, hipDeviceMallocUncached),
         "hipExtMallocWithFlags(uncached signals)");
  hip_ok(hipMemset(sig_, 0, sig_bytes), "hipMemset");
  hip_ok(hipMalloc(reinterpret_cast<void**>(&stage_), (size_t)stage_words_ * 4), "hipMalloc(stage)");
  hip_ok(hipMalloc(reinterpret_cast<void**>(&inbox_), (size_t)inbox_words_ * 4), "hipMalloc(inbox)");
  hip_ok(hipMalloc(reinterpret_cast<void**>(&tmo_), sizeof(int)), "hipMalloc(tmo)");
  hip_ok(hipMemset(tmo_, 0, sizeof(int)), "hipMemset");
  hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  sig_peer_.assign(world, nullptr);
  stage_peer_.assign(world, nullptr);
  inbox_peer_.assign(world, nullptr);
  sig_peer_[rank] = sig_;
  stage_peer_[rank] = stage_;
  inbox_peer_[rank] = inbox_;
}

IpcComm::~IpcComm() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  hipFree(sig_);
  hipFree(stage_);
  hipFree(inbox_);
  hipFree(tmo_);
}

std::string IpcComm::export_handle(const void* p) {
  void* base = nullptr;
  size_t size = 0;
  hip_ok(hipMemGetAddressRange(&base, &size, const_cast<void*>(p)), "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  hip_ok(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
  const int64_t off = static_cast<const char*>(p) - static_cast<const char*>(base);
  std::string out(HANDLE_BYTES, '\0');
  std::memcpy(&out[0], &h, sizeof(h));
  std::memcpy(&out[sizeof(h)], &off, sizeof(off));
  return out;
}

void* IpcComm::open(const std::string& s) {
  if (s.size() != HANDLE_BYTES) throw std::runtime_error("IpcComm: bad handle size");
  hipIpcMemHandle_t h;
  int64_t off = 0;
  std::memcpy(&h, s.data(), sizeof(h));
  std::memcpy(&off, s.data() + sizeof(h), sizeof(off));
  void* base = nullptr;
  hip_ok(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  opened_.push_back(base);
  return static_cast<char*>(base) + off;
}

void IpcComm::set_peers(const std::vector<std::string>& sig, const std::vector<std::string>& stage,
                        const std::vector<std::string>& inbox) {
  if ((int)sig.size() != world_ || (int)stage.size() != world_ || (int)inbox.size() != world_)
    throw std::runtime_error("IpcComm: handle count");
  hip_ok(hipSetDevice(device_), "hipSetDevice");
  for (int w = 0; w < world_; ++w) {
    if (w == rank_) continue;
    sig_peer_[w] = static_cast<unsigned*>(open(sig[w]));
    stage_peer_[w] = static_cast<unsigned*>(open(stage[w]));
    inbox_peer_[w] = static_cast<unsigned*>(open(inbox[w]));
  }
}

int IpcComm::add_region(const std::vector<std::string>& handles, void* local, long words) {
  if ((int)handles.size() != world_) throw std::runtime_error("IpcComm: handle count");
  hip_ok(hipSetDevice(device_), "hipSetDevice");
  Region r;
  r.base.assign(world_, nullptr);
  r.words = words;
  for (int w = 0; w < world_; ++w)
    r.base[w] = w == rank_ ? static_cast<unsigned*>(local) : static_cast<unsigned*>(open(handles[w]));
  regions_.push_back(r);
  return (int)regions_.size() - 1;
}

void IpcComm::base_args(DpaIpcArgs& a, int op) const {
  std::memset(&a, 0, sizeof(a));
  for (int w = 0; w < world_; ++w) {
    if (!sig_peer_[w] || !stage_peer_[w] || !inbox_peer_[w]) throw std::runtime_error("IpcComm: peers not set");
    a.sig[w] = sig_peer_[w];
    a.stage[w] = stage_peer_[w];
  }
  a.rank = rank_;
  a.world = world_;
  a.op = op;
  a.inbox = inbox_;
  a.tmo = tmo_;
}

const unsigned* IpcComm::region_ptr(int rid, long off, long n, int w) const {
  if (rid < 0 || rid >= (int)regions_.size()) throw std::runtime_error("IpcComm: unknown region");
  const Region& r = regions_[rid];
  if (off < 0 || n < 0 || off + n > r.words) throw std::runtime_error("IpcComm: range outside the region");
  return r.base[w] + off;
}

std::vector<std::pair<long, long>> IpcComm::pieces(int op, long n, int world, long stage_words, long inbox_words,
                                                   bool registered) {
  stage_words = round4(stage_words);
  inbox_words = round4(inbox_words);
  long cap;
  if (op == DPA_IPC_ALL_REDUCE) {  // a piece's slice fits the staging buffer; a bounced piece, the inbox
    cap = stage_words * world;
    if (!registered) cap = std::min(cap, inbox_words / (4L * world) * (4L * world));
  } else if (op == DPA_IPC_REDUCE_SCATTER) {  // bounced: every rank segment's piece in the inbox
    cap = registered ? n : inbox_words / (4L * world) * 4L;
  } else {
    cap = registered ? n : inbox_words;
  }
  if (cap < 1) throw std::runtime_error("IpcComm: buffers too small for a piece");
  std::vector<std::pair<long, long>> out;
  for (long done = 0; done < n; done += cap) out.emplace_back(done, std::min(cap, n - done));
  return out;
}

void IpcComm::launch(DpaIpcArgs& a, int blocks, long long tmo_us, hipStream_t st) {
  a.epoch = ++epoch_;
  const int rc = dpa_ipc_coll(&a, blocks, tmo_us, st);
  if (rc != 0) throw std::runtime_error("dpa_ipc_coll failed: " + std::to_string(rc));
  ++launches_;
}

void IpcComm::all_reduce(int rid, long off, void* buf, long n, int red, int blocks, long long tmo_us,
                         hipStream_t st) {
  unsigned* data = static_cast<unsigned*>(buf);
  if (rid >= 0) {
    if (region_ptr(rid, off, n, rank_) != data) throw std::runtime_error("IpcComm: buffer is not region+off");
  }
  for (const auto& pc : pieces(DPA_IPC_ALL_REDUCE, n, world_, stage_words_, inbox_words_, rid >= 0)) {
    const long done = pc.first, k = pc.second;
    DpaIpcArgs a;
    base_args(a, DPA_IPC_ALL_REDUCE);
    a.red = red;
    a.n = k;
    a.ns = dpa_ipc_slice(k, world_);
    if (a.ns > stage_words_) throw std::runtime_error("IpcComm: staging buffer too small");
    a.dst = data + done;
    for (int w = 0; w < world_; ++w) a.src[w] = rid >= 0 ? region_ptr(rid, off + done, k, w) : inbox_peer_[w];
    if (rid < 0) {
      a.in = data + done;
      a.pc_len = a.ns;
      a.pc_total = k;
      a.istride = a.ns;
      a.pc_nseg = world_;
    }
    launch(a, blocks, tmo_us, st);
  }
}

void IpcComm::broadcast(int rid, long off, void* buf, long n, int root, int blocks, long long tmo_us,
                        hipStream_t st) {
  unsigned* data = static_cast<unsigned*>(buf);
  if (rid >= 0 && region_ptr(rid, off, n, rank_) != data) throw std::runtime_error("IpcComm: buffer is not region+off");
  for (const auto& pc : pieces(DPA_IPC_BROADCAST, n, world_, stage_words_, inbox_words_, rid >= 0)) {
    const long done = pc.first, k = pc.second;
    DpaIpcArgs a;
    base_args(a, DPA_IPC_BROADCAST);
    a.root = root;
    a.n = k;
    a.dst = data + done;
    for (int w = 0; w < world_; ++w) a.src[w] = rid >= 0 ? region_ptr(rid, off + done, k, w) : inbox_peer_[w];
    if (rid < 0 && rank_ == root) {
      a.in = data + done;
      a.pc_len = a.pc_total = a.istride = k;
      a.pc_nseg = 1;
    }
    launch(a, blocks, tmo_us, st);
  }
}

void IpcComm::gather(int rid, long off, const void* in, void* out, long n, int root, int blocks, long long tmo_us,
                     hipStream_t st) {
  const unsigned* src = static_cast<const unsigned*>(in);
  if (rid >= 0 && region_ptr(rid, off, n, rank_) != src) throw std::runtime_error("IpcComm: input is not region+off");
  if (rank_ == root && out == nullptr) throw std::runtime_error("IpcComm: gather needs the root's output");
  for (const auto& pc : pieces(DPA_IPC_GATHER, n, world_, stage_words_, inbox_words_, rid >= 0)) {
    const long done = pc.first, k = pc.second;
    DpaIpcArgs a;
    base_args(a, DPA_IPC_GATHER);
    a.root = root;
    a.n = k;
    a.dstride = n;
    a.dst = out ? static_cast<unsigned*>(out) + done : nullptr;
    for (int w = 0; w < world_; ++w) a.src[w] = rid >= 0 ? region_ptr(rid, off + done, k, w) : inbox_peer_[w];
    if (rid < 0) {
      a.in = src + done;
      a.pc_len = a.pc_total = a.istride = k;
      a.pc_nseg = 1;
    }
    launch(a, blocks, tmo_us, st);
  }
}

void IpcComm::reduce_scatter(int rid, long off, const void* in, void* out, long n, int red, int blocks,
                             long long tmo_us, hipStream_t st) {
  const unsigned* src = static_cast<const unsigned*>(in);
  if (rid >= 0 && region_ptr(rid, off, n * world_, rank_) != src)
    throw std::runtime_error("IpcComm: input is not region+off");
  for (const auto& pc : pieces(DPA_IPC_REDUCE_SCATTER, n, world_, stage_words_, inbox_words_, rid >= 0)) {
    const long done = pc.first, k = pc.second;
    DpaIpcArgs a;
    base_args(a, DPA_IPC_REDUCE_SCATTER);
    a.red = red;
    a.n = k;
    a.dst = static_cast<unsigned*>(out) + done;
    if (rid >= 0) {
      for (int w = 0; w < world_; ++w) a.src[w] = region_ptr(rid, off, n * world_, w) + done;
      a.sstride = n;
    } else {  // the inbox holds this piece of every segment: [world][k]
      for (int w = 0; w < world_; ++w) a.src[w] = inbox_peer_[w];
      a.sstride = k;
      a.in = src + done;
      a.pc_len = k;
      a.pc_total = k * world_;
      a.istride = n;
      a.pc_nseg = world_;
    }
    launch(a, blocks, tmo_us, st);
  }
}

void IpcComm::all_gather(int rid, long off, const void* in, void* out, long n, int blocks, long long tmo_us,
                         hipStream_t st) {
  const unsigned* src = static_cast<const unsigned*>(in);
  if (rid >= 0 && region_ptr(rid, off, n, rank_) != src) throw std::runtime_error("IpcComm: input is not region+off");
  // in place (the input is this rank's slot of the output, as ZeRO-1's parameter all-gather): rank
  // w's input is ITS slot w, i.e. at offset off + (w - rank) * n of the region
  const bool inplace = src == static_cast<const unsigned*>(out) + (long)rank_ * n;
  for (const auto& pc : pieces(DPA_IPC_ALL_GATHER, n, world_, stage_words_, inbox_words_, rid >= 0)) {
    const long done = pc.first, k = pc.second;
    DpaIpcArgs a;
    base_args(a, DPA_IPC_ALL_GATHER);
    a.n = k;
    a.dstride = n;
    a.dst = static_cast<unsigned*>(out) + done;
    for (int w = 0; w < world_; ++w)
      a.src[w] = rid >= 0 ? region_ptr(rid, off + (inplace ? (long)(w - rank_) * n : 0L) + done, k, w) : inbox_peer_[w];
    if (rid < 0) {
      a.in = src + done;
      a.pc_len = a.pc_total = a.istride = k;
      a.pc_nseg = 1;
    }
    launch(a, blocks, tmo_us, st);
  }
}

void IpcComm::barrier(int blocks, long long tmo_us, hipStream_t st) {
  DpaIpcArgs a;
  base_args(a, DPA_IPC_BARRIER);
  launch(a, blocks, tmo_us, st);
}

bool IpcComm::take_timeout() {
  int v = 0;
  hip_ok(hipMemcpy(&v, tmo_, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy(tmo)");
  if (v) hip_ok(hipMemset(tmo_, 0, sizeof(int)), "hipMemset");
  return v != 0;
}

}  // namespace dpa
