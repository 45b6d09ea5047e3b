#include "ipc_comm.h"

#include <cstdint>
#include <cstring>
#include <stdexcept>

extern "C" {
int dpa_ipc_allreduce(float* const* data, float* const* stage, unsigned* const* sig, int rank, int world, long n,
                      unsigned epoch, int blocks, int* tmo, long long timeout_us, hipStream_t st);
long dpa_ipc_slice(long n, int world);
long dpa_ipc_sig_words();
}

namespace dpa {

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

constexpr size_t HANDLE_BYTES = sizeof(hipIpcMemHandle_t) + sizeof(int64_t);

IpcComm::IpcComm(int rank, int world, int device, long stage_floats)
    : rank_(rank), world_(world), device_(device), stage_floats_(stage_floats) {
  if (world < 1 || world > 8 || rank < 0 || rank >= world) throw std::runtime_error("IpcComm: 1..8 ranks");
  hip_ok(hipSetDevice(device), "hipSetDevice");
  const size_t sig_bytes = (size_t)dpa_ipc_sig_words() * sizeof(unsigned);
  hip_ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sig_bytes, hipDeviceMallocUncached),
         "hipExtMallocWithFlags(uncached signals)");
  hip_ok(hipMemset(sig_, 0, sig_bytes), "hipMemset");
  hip_ok(hipMalloc(reinterpret_cast<void**>(&stage_), (size_t)(stage_floats > 0 ? stage_floats : 4) * sizeof(float)),
         "hipMalloc(stage)");
  hip_ok(hipMalloc(reinterpret_cast<void**>(&tmo_), sizeof(int)), "hipMalloc(tmo)");
  hip_ok(hipMemset(tmo_, 0, sizeof(int)), "hipMemset");
  hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  sig_peer_.assign(world, nullptr);
  stage_peer_.assign(world, nullptr);
  sig_peer_[rank] = sig_;
  stage_peer_[rank] = stage_;
}

IpcComm::~IpcComm() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  hipFree(sig_);
  hipFree(stage_);
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

void IpcComm::set_peers(const std::vector<std::string>& sig, const std::vector<std::string>& stage) {
  if ((int)sig.size() != world_ || (int)stage.size() != world_) throw std::runtime_error("IpcComm: handle count");
  hip_ok(hipSetDevice(device_), "hipSetDevice");
  for (int w = 0; w < world_; ++w) {
    if (w == rank_) continue;
    sig_peer_[w] = static_cast<unsigned*>(open(sig[w]));
    stage_peer_[w] = static_cast<float*>(open(stage[w]));
  }
}

int IpcComm::add_region(const std::vector<std::string>& handles, float* local, long floats) {
  if ((int)handles.size() != world_) throw std::runtime_error("IpcComm: handle count");
  hip_ok(hipSetDevice(device_), "hipSetDevice");
  Region r;
  r.base.assign(world_, nullptr);
  r.floats = floats;
  for (int w = 0; w < world_; ++w) r.base[w] = w == rank_ ? local : static_cast<float*>(open(handles[w]));
  regions_.push_back(r);
  return (int)regions_.size() - 1;
}

void IpcComm::all_reduce(int id, long off, long n, int blocks, long long timeout_us, hipStream_t stream) {
  if (id < 0 || id >= (int)regions_.size()) throw std::runtime_error("IpcComm: unknown region");
  const Region& r = regions_[id];
  if (off < 0 || n < 0 || off + n > r.floats) throw std::runtime_error("IpcComm: range outside the region");
  if (dpa_ipc_slice(n, world_) > stage_floats_) throw std::runtime_error("IpcComm: staging buffer too small");
  for (int w = 0; w < world_; ++w)
    if (!sig_peer_[w] || !stage_peer_[w]) throw std::runtime_error("IpcComm: peers not set");
  float* data[8];
  for (int w = 0; w < world_; ++w) data[w] = r.base[w] + off;
  const int rc = dpa_ipc_allreduce(data, stage_peer_.data(), sig_peer_.data(), rank_, world_, n, ++epoch_, blocks,
                                   tmo_, timeout_us, stream);
  if (rc != 0) throw std::runtime_error("dpa_ipc_allreduce failed: " + std::to_string(rc));
}

bool IpcComm::take_timeout() {
  int v = 0;
  hip_ok(hipMemcpy(&v, tmo_, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy(tmo)");
  if (v) hip_ok(hipMemset(tmo_, 0, sizeof(int)), "hipMemset");
  return v != 0;
}

}  // namespace dpa
