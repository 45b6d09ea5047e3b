// Python bindings for the gfx950 kernels and the native RCCL communicator.
// Thin: validate tensors, fetch the caller's current HIP stream, call the extern "C" launchers.
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <torch/extension.h>

#include "runtime/ipc_comm.h"
#include "runtime/rccl_comm.h"
#include "runtime/tcp_store.h"

extern "C" {
int dpa_sgd_flat(float* p, const float* g, float* buf, long n, float lr, float momentum, float wd, float gscale,
                 int first, unsigned short* planes, long ps, int np, hipStream_t s);
int dpa_spin(long long usec, int* done, hipStream_t s);
int dpa_mean_of_w(const float* in, float* out, long n, int W, hipStream_t s);
int dpa_add_inplace(void* out, const void* add, long n, int bf, hipStream_t s);
int dpa_conv_fprop(const float* x, const float* w, float* out, float* slab, int N, int H, int W, int C, int Kout,
                   int R, int S, int stride, int pad, int splits, int tile, int dgrad, int reduce, int posmajor,
                   hipStream_t st);
int dpa_conv_splits(int Kred, int splits);
int dpa_conv_wgrad(const float* x, const float* dz, float* dw, float* slab, int N, int H, int W, int C, int Kout,
                   int R, int S, int stride, int pad, int splits, int tile, int posmajor, hipStream_t st);
int dpa_wflip(const float* w, float* wd, int K, int R, int S, int C, hipStream_t st);
long dpa_bn_part_floats(int M, int C, int bwd);
int dpa_bn_fwd_stats(const void* src, int nsplit, void* z, float* part, int M, int C, const float* gamma,
                     const float* beta, const float* bias, float* rmean, float* rvar, long long* nbt, float* mean,
                     float* invstd, float* scale, float* shift, float momentum, float eps, int zbf, hipStream_t st);
int dpa_bn_eval_params(const float* gamma, const float* beta, const float* bias, const float* rmean,
                       const float* rvar, float* scale, float* shift, int C, float eps, hipStream_t st);
int dpa_bn_apply(const void* z, float* a, unsigned short* a3, int np, const float* scale, const float* shift, int N,
                 int H, int W, int C, int pool, int act, const void* res, int zbf, hipStream_t st,
                 unsigned char* mask);
int dpa_bn_bwd(const void* gsrc, int nsplit, void* g, const void* z, const float* scale, const float* shift,
               const float* mean, const float* invstd, const float* gamma, float* part, float* coef, float* dgamma,
               float* dbeta, float* dbias, float* dz, unsigned short* dz3, int np, int N, int H, int W, int C,
               int pool, int act, const void* res, void* dres, int zbf, hipStream_t st, int* sig, int sig_val,
               const void* g2, const unsigned char* mask, unsigned* bound);
long dpa_wgrad0_part_floats(int N);
int dpa_gap(const void* x, float* feat, int N, int HW, int C, int xbf, hipStream_t st);
int dpa_ce(const float* logits, const long long* target, float* loss_row, float* dlogits, int* correct_row,
           float* loss, float* acc, int N, int J, hipStream_t st);
int dpa_head_bwd_prep(const float* dlogits, const float* gout, float* dl, float* db, int N, int J, hipStream_t st);
int dpa_gap_bwd(const float* dfeat, void* dx, int N, int HW, int C, int xbf, hipStream_t st);
long dpa_conv0_part_floats(int N);
int dpa_gemm_f32(const float* A, int lda, int ak, const float* B, int ldb, int bk, float* C, int M, int N, int K,
                 const float* bias, float* slab, int splits, hipStream_t st);
int dpa_conv0_fwd(const float* x, const float* w, int CP, float* z, float* part, int N, const float* gamma,
                  const float* beta, const float* bias, float* rmean, float* rvar, long long* nbt, float* mean,
                  float* invstd, float* scale, float* shift, float momentum, float eps, hipStream_t st);
int dpa_bn_bwd_wgrad0(const float* gsrc, int nsplit, float* g, const float* z, const float* scale,
                      const float* shift, const float* mean, const float* invstd, const float* gamma, float* part,
                      float* coef, float* dgamma, float* dbeta, float* dbias, const float* x, float* wpart,
                      float* dw, int CP, int N, hipStream_t st, int* sig, int sig_val);
int dpa_fc_ce_train(const float* x, const float* w, const float* b, const long long* target, float* loss_row,
                    float* dlogits, float* dx, float* dw, float* db, float* loss_out, float* loss_accum, int B,
                    int Cin, int J, hipStream_t st, const float* bn_z, const float* bn_scale,
                    const float* bn_shift, int parts);
int dpa_fc_ce_eval(const float* x, const float* w, const float* b, const long long* target, float* loss_row,
                   int* correct_row, float* logits, float* acc, int B, int Cin, int J, hipStream_t st);
int dpa_x3_splits(int Kred, int splits);
int dpa_conv_x3_fprop(const unsigned short* x, long xps, const unsigned short* w, long wps, void* out, float* slab,
                      int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad, int splits, int tile,
                      int reduce, int posmajor, int np, int obf, hipStream_t st, float* stats, float oscale,
                      const unsigned* obound);
int dpa_conv_stats_rows(int tile);
long dpa_ipc_slice(long n, int world);
int dpa_bn_finalize_cm(const float* part, int nblk, int rpb, int M, int C, const float* gamma, const float* beta,
                       const float* bias, float* rmean, float* rvar, long long* nbt, float* mean, float* invstd,
                       float* scale, float* shift, float momentum, float eps, hipStream_t st);
int dpa_conv_x3_wgrad(const unsigned short* x, long xps, const unsigned short* dz, long dzps, float* dw, float* slab,
                      int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad, int splits, int tile,
                      int posmajor, int np, hipStream_t st, float oscale, const unsigned* obound);
int dpa_split_planes(const float* x, unsigned short* out, long n, long ps, int np, float scale, hipStream_t st);
int dpa_h2_ovf_conv(int clear);
int dpa_h2_ovf_bn(int clear);
int dpa_h2_ovf_sgd(int clear);
int dpa_h2_ovf_fused(int clear);
int dpa_pad_split8(const float* x, unsigned short* out, long npix, int cin, long ps, int np, hipStream_t st);
int dpa_conv_x3_dgrad(const unsigned short* dz, long dzps, const unsigned short* w, long wps, void* dx, float* slab,
                      int N, int Hd, int Wd, int K, int C, int R, int S, int stride, int pad, int H, int W, int splits,
                      int tile, int reduce, int posmajor, int np, int obf, hipStream_t st, const void* add, int* sig,
                      int sig_val, float oscale, const unsigned* obound);
int dpa_wait_signal(const int* sig, int val, long long timeout_us, int* tmo, hipStream_t st);
int dpa_bn_fused_geo(int Mo, int C, int pool, int bwd, int rmax, long* part_floats, long* cnt_words, int* blocks);
int dpa_bn_fused_fwd(const float* src, int nsplit, float* zw, int N, int H, int W, int C, int pool, int rmax,
                     float* part, unsigned* cnt, const float* gamma, const float* beta, const float* bias,
                     float* rmean, float* rvar, long long* nbt, float* mean, float* invstd, float* scale,
                     float* shift, int apply, float* out, unsigned short* out3, int np, long ps, float momentum,
                     float eps, int* tmo, long long timeout_us, hipStream_t st);
int dpa_bn_fused_bwd(const float* gsrc, int nsplit, const float* z, int N, int H, int W, int C, int pool, int rmax,
                     float* part, unsigned* cnt, const float* scale, const float* shift, const float* mean,
                     const float* invstd, const float* gamma, float* dgamma, float* dbeta, float* dbias, float* out,
                     unsigned short* out3, int np, long ps, int* tmo, long long timeout_us, hipStream_t st, int* sig,
                     int sig_val);

int dpa_set_signal(int* sig, int val, hipStream_t st);
int dpa_health_copy(const int* const* w, int n, int* out, int tag, hipStream_t st);
int* dpa_h2_ovf_conv_addr();
int* dpa_h2_ovf_bn_addr();
int* dpa_h2_ovf_sgd_addr();
int* dpa_h2_ovf_fused_addr();
int dpa_bn_apply_wide(const unsigned short* z, const unsigned short* res, unsigned short* out, unsigned char* mask,
                      const float* scale, const float* shift, long M, int C, int act, hipStream_t st,
                      const float* rscale, const float* rshift);
int dpa_maxpool_fwd(const void* x, void* y, unsigned char* arg, int N, int H, int W, int C, int k, int s, int p,
                    int bf, hipStream_t st, const float* scale, const float* shift);
int dpa_maxpool_bwd(const void* dy, const unsigned char* arg, void* dx, int N, int H, int W, int C, int k, int s,
                    int p, int bf, hipStream_t st);
int dpa_augment(const unsigned char* img, const long long* idx, const long long* labels, float* out,
                long long* target, int B, int Hs, int Ws, int pad, int train, unsigned long long seed,
                unsigned long long salt, const float* mean, const float* std, hipStream_t st);
}

namespace {

using torch::Tensor;
using OptT = c10::optional<Tensor>;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void chk(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed: rc=", rc, (rc > 0 ? std::string(" ") + hipGetErrorString((hipError_t)rc) : ""));
}

// Cross-stream dependency event with caller-chosen flags.  torch.cuda.Event records with a
// system-scope release (L2 writeback + invalidate at every record); dependencies between streams of
// ONE device only need device scope (hipEventReleaseToDevice), which keeps L2 warm and lets the
// next kernel on the recording stream start sooner.
struct DevEvent {
  hipEvent_t ev{};
  explicit DevEvent(int64_t flags) {
    TORCH_CHECK(hipEventCreateWithFlags(&ev, (unsigned)flags) == hipSuccess, "hipEventCreateWithFlags failed");
  }
  ~DevEvent() {
    if (ev) (void)hipEventDestroy(ev);
  }
  DevEvent(const DevEvent&) = delete;
  DevEvent& operator=(const DevEvent&) = delete;
  void record(int64_t stream) {
    TORCH_CHECK(hipEventRecord(ev, reinterpret_cast<hipStream_t>(stream)) == hipSuccess, "hipEventRecord failed");
  }
  void wait(int64_t stream) {
    TORCH_CHECK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev, 0) == hipSuccess,
                "hipStreamWaitEvent failed");
  }
  void synchronize() { TORCH_CHECK(hipEventSynchronize(ev) == hipSuccess, "hipEventSynchronize failed"); }
  bool query() {
    const hipError_t q = hipEventQuery(ev);
    TORCH_CHECK(q == hipSuccess || q == hipErrorNotReady, "hipEventQuery failed");
    return q == hipSuccess;
  }
};

void need(const Tensor& t, const char* name, at::ScalarType dt = at::kFloat) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == dt, name, " has wrong dtype ", t.scalar_type());
}

float* fp(const Tensor& t) { return t.data_ptr<float>(); }
float* ofp(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }

// ---------------- optimizer / elementwise ----------------
// planes (optional): bf16 [NP, p.numel()] operand planes of the whole arena, refreshed in the same pass
void sgd_flat(Tensor p, Tensor g, Tensor buf, double lr, double momentum, double wd, double gscale, bool first,
              int64_t offset, int64_t count, OptT planes) {
  need(p, "p");
  need(g, "g");
  need(buf, "buf");
  if (count < 0) count = p.numel() - offset;
  TORCH_CHECK(offset % 4 == 0 && count % 4 == 0, "sgd_flat: offset/count must be multiples of 4");
  TORCH_CHECK(offset + count <= p.numel() && p.numel() == g.numel() && p.numel() == buf.numel(), "sgd_flat sizes");
  unsigned short* pl = nullptr;
  long ps = 0;
  int np = 0;
  if (planes.has_value() && planes->defined()) {
    const Tensor& t = *planes;
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 2 && t.size(1) == p.numel() &&
                    ((t.scalar_type() == at::kBFloat16 && (t.size(0) == 1 || t.size(0) == 3)) ||
                     (t.scalar_type() == at::kHalf && t.size(0) == 2)),
                "sgd_flat: planes must be contiguous bfloat16 [1 or 3, p.numel()] or float16 [2, p.numel()]");
    np = t.size(0);
    ps = t.stride(0);
    pl = reinterpret_cast<unsigned short*>(t.data_ptr()) + offset;
  }
  chk(dpa_sgd_flat(fp(p) + offset, fp(g) + offset, fp(buf) + offset, count, (float)lr, (float)momentum, (float)wd,
                   (float)gscale, first ? 1 : 0, pl, ps, np, cur_stream()),
      "sgd_flat");
}

// Diagnostics: occupy the current stream for ~usec microseconds (one wave, bounded loop) and then
// write 1 to done[0].  Used to hold a collective behind a long kernel (watchdog timeout test).
// one int32 word on the GPU (a stream-signal flag or timeout word)
int* signal_ptr(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kInt32 && t.numel() >= 1, what,
              ": signal word must be a CUDA int32 tensor");
  return t.data_ptr<int>();
}

int* opt_signal(const OptT& t, const char* what) {
  return (t.has_value() && t->defined()) ? signal_ptr(*t, what) : nullptr;
}

// the current stream waits (one polling wave) until sig[0] >= val; tmo[0] = 1 after timeout_us
void wait_signal(Tensor sig, int64_t val, int64_t timeout_us, Tensor tmo) {
  chk(dpa_wait_signal(signal_ptr(sig, "wait_signal"), (int)val, timeout_us, signal_ptr(tmo, "wait_signal"),
                      cur_stream()),
      "wait_signal");
}

void set_signal(Tensor sig, int64_t val) {
  chk(dpa_set_signal(signal_ptr(sig, "set_signal"), (int)val, cur_stream()), "set_signal");
}

// device addresses of the fp16-pair overflow words of every kernel file (per-step health snapshot)
std::vector<int64_t> h2_overflow_addrs() {
  std::vector<int64_t> out;
  for (int* (*f)() : {dpa_h2_ovf_conv_addr, dpa_h2_ovf_bn_addr, dpa_h2_ovf_sgd_addr, dpa_h2_ovf_fused_addr}) {
    int* p = f();
    TORCH_CHECK(p != nullptr, "h2_overflow_addrs: hipGetSymbolAddress failed");
    out.push_back(reinterpret_cast<int64_t>(p));
  }
  return out;
}

// ptrs: int64 GPU tensor of n word addresses; out: pinned host int32 tensor of >= 64 words.  One
// one-wave kernel on the current stream copies the words (and `tag` into out[63]).
void health_copy(Tensor ptrs, Tensor out, int64_t tag) {
  TORCH_CHECK(ptrs.is_cuda() && ptrs.scalar_type() == at::kLong && ptrs.is_contiguous() && ptrs.numel() <= 63,
              "health_copy: ptrs must be a contiguous int64 GPU tensor of <= 63 addresses");
  TORCH_CHECK(!out.is_cuda() && out.is_pinned() && out.scalar_type() == at::kInt && out.is_contiguous() &&
                  out.numel() >= 64,
              "health_copy: out must be a pinned host int32 tensor of >= 64 words");
  void* dptr = nullptr;
  chk((int)hipHostGetDevicePointer(&dptr, out.data_ptr(), 0), "health_copy: hipHostGetDevicePointer");
  chk(dpa_health_copy(reinterpret_cast<const int* const*>(ptrs.data_ptr()), (int)ptrs.numel(), static_cast<int*>(dptr),
                      (int)tag, cur_stream()),
      "health_copy");
}

void spin(int64_t usec, Tensor done) {
  need(done, "done", at::kInt);
  TORCH_CHECK(usec >= 0 && usec <= 10000000, "spin: usec out of range");
  chk(dpa_spin(usec, done.data_ptr<int>(), cur_stream()), "spin");
}

// out += add (same shape, fp32 or bf16, contiguous)
void add_inplace(Tensor out, Tensor add) {
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && add.is_contiguous() && out.numel() == add.numel() &&
                  out.scalar_type() == add.scalar_type(),
              "add_inplace: matching contiguous GPU tensors expected");
  const bool bf = out.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || out.scalar_type() == at::kFloat, "add_inplace: fp32 or bf16");
  chk(dpa_add_inplace(out.data_ptr(), add.data_ptr(), out.numel(), bf ? 1 : 0, cur_stream()), "add_inplace");
}

void mean_of_w(Tensor in, Tensor out, int64_t W) {
  need(in, "in");
  need(out, "out");
  TORCH_CHECK(in.numel() == W * out.numel(), "mean_of_w sizes");
  chk(dpa_mean_of_w(fp(in), fp(out), out.numel(), (int)W, cur_stream()), "mean_of_w");
}

// ---------------- convolution ----------------
// x [N,H,W,C], w [K,R,S,C] (dgrad: the original conv's weights [C,R,S,K]), out [N,P,Q,K]
void conv_fprop(Tensor x, Tensor w, Tensor out, OptT slab, int64_t stride, int64_t pad, int64_t splits, int64_t tile,
                bool dgrad, bool reduce, bool posmajor) {
  need(x, "x");
  need(w, "w");
  need(out, "out");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && out.dim() == 4, "conv_fprop: 4-d NHWC/KRSC tensors expected");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  int K, R, S;
  if (dgrad) {
    K = w.size(3), R = w.size(1), S = w.size(2);
    TORCH_CHECK(w.size(0) == C, "conv_fprop(dgrad): weight [C,R,S,K] expected");
  } else {
    K = w.size(0), R = w.size(1), S = w.size(2);
    TORCH_CHECK(w.size(3) == C, "conv_fprop: channel mismatch");
  }
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(out.size(0) == N && out.size(1) == P && out.size(2) == Q && out.size(3) == K, "conv_fprop: out shape");
  float* sl = nullptr;
  const int eff = dpa_conv_splits(R * S * C, (int)splits);
  if (eff > 1) {
    TORCH_CHECK(slab.has_value() && slab->defined(), "conv_fprop: split-K needs a slab workspace");
    need(*slab, "slab");
    TORCH_CHECK(slab->numel() >= (int64_t)eff * N * P * Q * K, "conv_fprop: slab too small");
    sl = fp(*slab);
  }
  chk(dpa_conv_fprop(fp(x), fp(w), fp(out), sl, N, H, W, C, K, R, S, (int)stride, (int)pad, (int)splits, (int)tile,
                     dgrad ? 1 : 0, reduce ? 1 : 0, posmajor ? 1 : 0, cur_stream()),
      "conv_fprop");
}

int64_t conv_splits(int64_t Kred, int64_t splits) { return dpa_conv_splits((int)Kred, (int)splits); }

// x [N,H,W,C], dz [N,P,Q,K], dw [K,R,S,C]
void conv_wgrad(Tensor x, Tensor dz, Tensor dw, OptT slab, int64_t stride, int64_t pad, int64_t splits, int64_t tile,
                bool posmajor) {
  need(x, "x");
  need(dz, "dz");
  need(dw, "dw");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = dw.size(0), R = dw.size(1), S = dw.size(2);
  TORCH_CHECK(dw.size(3) == C && dz.size(3) == K && dz.size(0) == N, "conv_wgrad: shape mismatch");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(dz.size(1) == P && dz.size(2) == Q, "conv_wgrad: dz spatial");
  float* sl = nullptr;
  const int eff = dpa_conv_splits(N * P * Q, (int)splits);
  if (eff > 1) {
    TORCH_CHECK(slab.has_value() && slab->defined(), "conv_wgrad: split-K needs a slab workspace");
    need(*slab, "slab");
    TORCH_CHECK(slab->numel() >= (int64_t)eff * K * R * S * C, "conv_wgrad: slab too small");
    sl = fp(*slab);
  }
  chk(dpa_conv_wgrad(fp(x), fp(dz), fp(dw), sl, N, H, W, C, K, R, S, (int)stride, (int)pad, (int)splits, (int)tile,
                     posmajor ? 1 : 0, cur_stream()),
      "conv_wgrad");
}

void wflip(Tensor w, Tensor wd) {
  need(w, "w");
  need(wd, "wd");
  const int K = w.size(0), R = w.size(1), S = w.size(2), C = w.size(3);
  TORCH_CHECK(wd.size(0) == C && wd.size(1) == R && wd.size(2) == S && wd.size(3) == K, "wflip: wd shape");
  chk(dpa_wflip(fp(w), fp(wd), K, R, S, C, cur_stream()), "wflip");
}

// ---------------- bf16-plane (fp32 via bf16x6, or plain bf16) convolution ----------------
// Plane tensors are bfloat16 [NP, ...] (NP = 1 or 3), contiguous.
using u16 = unsigned short;
u16* up(const Tensor& t) { return reinterpret_cast<u16*>(t.data_ptr()); }

// operand planes: bfloat16 [1 or 3, ...] (bf16 / bf16-triple operands) or float16 [2, ...] (fp16
// pairs, impl "h2"); plane_count of a tensor that is one of them
bool is_plane_dtype(const Tensor& t) { return t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf; }

// a data-gradient bound word (int32 [>= 1], written by bn_bwd) or nullptr
const unsigned* bound_ptr(const OptT& b, const char* what) {
  if (!b.has_value() || !b->defined()) return nullptr;
  TORCH_CHECK(b->is_cuda() && b->scalar_type() == torch::kInt32 && b->numel() >= 1, what,
              ": bound must be an int32 GPU tensor");
  return reinterpret_cast<const unsigned*>(b->data_ptr<int32_t>());
}

// Each plane must be contiguous and 16-byte aligned; planes may be strided views of a larger
// buffer (e.g. the engine's weight-plane arena) as long as the plane stride keeps that alignment.
void need_planes(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(is_plane_dtype(t), name, " must be bfloat16 or float16 planes");
  TORCH_CHECK(t.scalar_type() == at::kHalf ? t.size(0) == 2 : (t.size(0) == 1 || t.size(0) == 3), name,
              ": bfloat16 planes come in 1 or 3, float16 pairs in 2 (dim 0)");
  TORCH_CHECK(t.select(0, 0).is_contiguous(), name, ": each plane must be contiguous");
  TORCH_CHECK(t.size(0) == 1 || t.stride(0) % 8 == 0, name, ": plane stride must be a multiple of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, ": planes must be 16-byte aligned");
}

int64_t x3_splits(int64_t Kred, int64_t splits) { return dpa_x3_splits((int)Kred, (int)splits); }

// fp32 conv output, or bf16 (one-plane convs only: the generic bf16-activation path)
void* conv_out_ptr(const Tensor& out, int np, const char* name, int& obf) {
  TORCH_CHECK(out.is_cuda() && out.is_contiguous(), name, " must be a contiguous GPU tensor");
  if (out.scalar_type() == at::kBFloat16) {
    TORCH_CHECK(np == 1, name, ": bf16 output needs bf16 (1-plane) operands");
    obf = 1;
  } else {
    TORCH_CHECK(out.scalar_type() == at::kFloat, name, " must be float32 or bfloat16");
    obf = 0;
  }
  return out.data_ptr();
}

// x3 [NP,N,H,W,C], w3 [NP,K,R,S,C], out [N,P,Q,K] fp32 (or bf16 when NP == 1)
// np 2 (float16 pairs): the output is multiplied by oscale (1 / (s_x s_w)) and, with obound, by
// 1 / the scale of that data-gradient bound word
void conv_x3_fprop(Tensor x3, Tensor w3, Tensor out, OptT slab, int64_t stride, int64_t pad, int64_t splits,
                   int64_t tile, bool reduce, int64_t posmajor, OptT stats, double oscale, OptT obound) {
  need_planes(x3, "x3");
  need_planes(w3, "w3");
  const int np = x3.size(0);
  TORCH_CHECK(w3.size(0) == np, "plane count mismatch");
  int obf = 0;
  void* op = conv_out_ptr(out, np, "out", obf);
  const int N = x3.size(1), H = x3.size(2), W = x3.size(3), C = x3.size(4);
  const int K = w3.size(1), R = w3.size(2), S = w3.size(3);
  TORCH_CHECK(w3.size(4) == C, "conv_x3_fprop: channel mismatch");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(out.size(0) == N && out.size(1) == P && out.size(2) == Q && out.size(3) == K, "conv_x3_fprop: out shape");
  float* sl = nullptr;
  const int eff = dpa_x3_splits(R * S * C, (int)splits);
  if (eff > 1) {
    TORCH_CHECK(slab.has_value() && slab->defined(), "conv_x3_fprop: split-K needs a slab workspace");
    need(*slab, "slab");
    TORCH_CHECK(slab->numel() >= (int64_t)eff * N * P * Q * K, "conv_x3_fprop: slab too small");
    sl = fp(*slab);
  }
  float* stp = nullptr;
  if (stats.has_value() && stats->defined()) {  // BN partials from the epilogue (one split only)
    need(*stats, "stats");
    const int rows = dpa_conv_stats_rows((int)tile);
    TORCH_CHECK(rows > 0, "conv_x3_fprop: this tile cannot emit BN statistics");
    TORCH_CHECK(stats->numel() >= 2 * (int64_t)((N * P * Q + rows - 1) / rows) * K, "conv_x3_fprop: stats too small");
    stp = fp(*stats);
  }
  chk(dpa_conv_x3_fprop(up(x3), x3.stride(0), up(w3), w3.stride(0), op, sl, N, H, W, C, K, R, S, (int)stride,
                        (int)pad, (int)splits, (int)tile, reduce ? 1 : 0, (int)posmajor, np, obf, cur_stream(), stp,
                        (float)oscale, bound_ptr(obound, "conv_x3_fprop")),
      "conv_x3_fprop");
}

// BN finalize from channel-major (mean, M2) partials [C][nblk] of row blocks of rpb rows (a conv
// epilogue's statistics)
void bn_finalize(Tensor part, int64_t nblk, int64_t rpb, int64_t M, Tensor gamma, Tensor beta, OptT bias, OptT rmean,
                 OptT rvar, OptT nbt, Tensor mean, Tensor invstd, Tensor scale, Tensor shift, double momentum,
                 double eps) {
  need(part, "part");
  const int C = gamma.numel();
  TORCH_CHECK(nblk == (M + rpb - 1) / rpb && part.numel() >= 2 * nblk * C, "bn_finalize: partial layout");
  long long* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    need(*nbt, "nbt", at::kLong);
    nb = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>());
  }
  chk(dpa_bn_finalize_cm(fp(part), (int)nblk, (int)rpb, (int)M, C, fp(gamma), fp(beta), ofp(bias), ofp(rmean),
                         ofp(rvar), nb, fp(mean), fp(invstd), fp(scale), fp(shift), (float)momentum, (float)eps,
                         cur_stream()),
      "bn_finalize");
}

// x3 [NP,N,H,W,C], dz3 [NP,N,P,Q,K], dw [K,R,S,C] fp32
void conv_x3_wgrad(Tensor x3, Tensor dz3, Tensor dw, OptT slab, int64_t stride, int64_t pad, int64_t splits,
                   int64_t tile, int64_t posmajor, double oscale, OptT obound) {
  need_planes(x3, "x3");
  need_planes(dz3, "dz3");
  need(dw, "dw");
  const int np = x3.size(0);
  TORCH_CHECK(dz3.size(0) == np, "plane count mismatch");
  const int N = x3.size(1), H = x3.size(2), W = x3.size(3), C = x3.size(4);
  const int K = dw.size(0), R = dw.size(1), S = dw.size(2);
  TORCH_CHECK(dw.size(3) == C && dz3.size(4) == K && dz3.size(1) == N, "conv_x3_wgrad: shape mismatch");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(dz3.size(2) == P && dz3.size(3) == Q, "conv_x3_wgrad: dz spatial");
  float* sl = nullptr;
  const int eff = dpa_x3_splits(N * P * Q, (int)splits);
  if (eff > 1) {
    TORCH_CHECK(slab.has_value() && slab->defined(), "conv_x3_wgrad: split-K needs a slab workspace");
    need(*slab, "slab");
    TORCH_CHECK(slab->numel() >= (int64_t)eff * K * R * S * C, "conv_x3_wgrad: slab too small");
    sl = fp(*slab);
  }
  chk(dpa_conv_x3_wgrad(up(x3), x3.stride(0), up(dz3), dz3.stride(0), fp(dw), sl, N, H, W, C, K, R, S, (int)stride,
                        (int)pad, (int)splits, (int)tile, (int)posmajor, np, cur_stream(), (float)oscale,
                        bound_ptr(obound, "conv_x3_wgrad")),
      "conv_x3_wgrad");
}

// dz3 [NP,N,Hd,Wd,K], w3 [NP,K,R,S,C] (forward weight planes), dx [N,H,W,C] fp32: data gradient of
// conv(x, w, stride, pad); stride a power of two.
void conv_x3_dgrad(Tensor dz3, Tensor w3, Tensor dx, OptT slab, int64_t stride, int64_t pad, int64_t splits,
                   int64_t tile, bool reduce, int64_t posmajor, OptT add, OptT sig, int64_t sig_val, double oscale,
                   OptT obound) {
  need_planes(dz3, "dz3");
  need_planes(w3, "w3");
  const int np = dz3.size(0);
  TORCH_CHECK(w3.size(0) == np, "plane count mismatch");
  int obf = 0;
  void* op = conv_out_ptr(dx, np, "dx", obf);
  const int N = dz3.size(1), Hd = dz3.size(2), Wd = dz3.size(3), K = dz3.size(4);
  const int R = w3.size(2), S = w3.size(3), C = w3.size(4);
  TORCH_CHECK(w3.size(1) == K, "conv_x3_dgrad: weight K mismatch");
  const int H = dx.size(1), W = dx.size(2);
  TORCH_CHECK(dx.size(0) == N && dx.size(3) == C, "conv_x3_dgrad: dx shape");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 == Hd && (W + 2 * pad - S) / stride + 1 == Wd,
              "conv_x3_dgrad: dz spatial does not match conv(dx)");
  float* sl = nullptr;
  const int eff = dpa_x3_splits(R * S * K, (int)splits);
  if (eff > 1) {
    TORCH_CHECK(slab.has_value() && slab->defined(), "conv_x3_dgrad: split-K needs a slab workspace");
    need(*slab, "slab");
    TORCH_CHECK(slab->numel() >= (int64_t)eff * N * H * W * C, "conv_x3_dgrad: slab too small");
    sl = fp(*slab);
  }
  const void* ap = nullptr;
  if (add.has_value() && add->defined()) {
    TORCH_CHECK(add->is_cuda() && add->is_contiguous() && add->numel() == dx.numel() &&
                    add->scalar_type() == dx.scalar_type(),
                "conv_x3_dgrad: add must match dx (shape, dtype, contiguous)");
    ap = add->data_ptr();
  }
  int* sp = opt_signal(sig, "conv_x3_dgrad");
  chk(dpa_conv_x3_dgrad(up(dz3), dz3.stride(0), up(w3), w3.stride(0), op, sl, N, Hd, Wd, K, C, R, S, (int)stride,
                        (int)pad, H, W, (int)splits, (int)tile, reduce ? 1 : 0, (int)posmajor, np, obf,
                        cur_stream(), ap, sp, (int)sig_val, (float)oscale, bound_ptr(obound, "conv_x3_dgrad")),
      "conv_x3_dgrad");
}

// x fp32 [..., cin] (cin <= 8) -> out [NP, ..., 8] bf16 planes, channels >= cin zero
void pad_split8(Tensor x, Tensor out) {
  need(x, "x");
  need_planes(out, "out");
  TORCH_CHECK(out.size(-1) == 8 && x.size(-1) <= 8, "pad_split8: out [NP, ..., 8]");
  const long npix = x.numel() / x.size(-1);
  TORCH_CHECK(out.numel() == out.size(0) * npix * 8, "pad_split8: pixel count mismatch");
  chk(dpa_pad_split8(fp(x), up(out), npix, x.size(-1), out.stride(0), out.size(0), cur_stream()), "pad_split8");
}

// x fp32 (any shape) -> out [NP, *x.shape] bf16 planes, or float16 pairs of x * scale
void split_planes(Tensor x, Tensor out, double scale) {
  need(x, "x");
  need_planes(out, "out");
  TORCH_CHECK(out.numel() == out.size(0) * x.numel(), "split_planes: out must be [NP, *x.shape]");
  chk(dpa_split_planes(fp(x), up(out), x.numel(), out.stride(0), out.size(0), (float)scale, cur_stream()),
      "split_planes");
}

// the fp16-pair overflow words of every kernel file (a split saw |x s| beyond float16's range);
// clear: reset them
bool h2_overflow(bool clear) {
  int any = 0;
  for (int (*f)(int) : {dpa_h2_ovf_conv, dpa_h2_ovf_bn, dpa_h2_ovf_sgd, dpa_h2_ovf_fused}) {
    const int v = f(clear ? 1 : 0);
    TORCH_CHECK(v >= 0, "h2_overflow: could not read an overflow word");
    any |= v;
  }
  return any != 0;
}


// ---------------- batch norm ----------------
// Activation-like BN operands (z, grads, residuals) are fp32 or bf16; all of one call share a dtype.
void* act_ptr(const Tensor& t, const char* name, bool bf) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.scalar_type() == (bf ? at::kBFloat16 : at::kFloat), name, " must be ",
              bf ? "bfloat16" : "float32", " like z");
  return t.data_ptr();
}
int64_t bn_part_floats(int64_t M, int64_t C, bool bwd) { return dpa_bn_part_floats((int)M, (int)C, bwd ? 1 : 0); }

// src: z [M][C], or nsplit slabs of it (then the summed z is written to z)
void bn_fwd_stats(Tensor src, int64_t nsplit, Tensor z, Tensor part, Tensor gamma, Tensor beta, OptT bias, OptT rmean,
                  OptT rvar, OptT nbt, Tensor mean, Tensor invstd, Tensor scale, Tensor shift, double momentum,
                  double eps) {
  const bool bf = z.scalar_type() == at::kBFloat16;
  void* zp = act_ptr(z, "z", bf);
  const void* sp = act_ptr(src, "src", bf);
  need(part, "part");
  const int C = z.size(-1);
  const int M = z.numel() / C;
  TORCH_CHECK(src.numel() >= nsplit * (int64_t)M * C, "bn_fwd_stats: src too small");
  TORCH_CHECK(part.numel() >= dpa_bn_part_floats(M, C, 0), "bn_fwd_stats: part too small");
  long long* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    need(*nbt, "nbt", at::kLong);
    nb = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>());
  }
  chk(dpa_bn_fwd_stats(sp, (int)nsplit, zp, fp(part), M, C, fp(gamma), fp(beta), ofp(bias), ofp(rmean), ofp(rvar),
                       nb, fp(mean), fp(invstd), fp(scale), fp(shift), (float)momentum, (float)eps, bf ? 1 : 0,
                       cur_stream()),
      "bn_fwd_stats");
}

void bn_eval_params(Tensor gamma, Tensor beta, OptT bias, Tensor rmean, Tensor rvar, Tensor scale, Tensor shift,
                    double eps) {
  chk(dpa_bn_eval_params(fp(gamma), fp(beta), ofp(bias), fp(rmean), fp(rvar), fp(scale), fp(shift), gamma.numel(),
                         (float)eps, cur_stream()),
      "bn_eval_params");
}

// a: fp32 [N,Ho,Wo,C] or bf16 planes [NP,N,Ho,Wo,C].  act: 0 relu, 1 none, 2 relu(. + res)
// z (and res): fp32 or bf16 [N,H,W,C]; a: fp32 [N,Ho,Wo,C], bf16 [N,Ho,Wo,C] (one plane) or bf16
// planes [NP,N,Ho,Wo,C]
// mask (optional, act 2): uint8 [z.numel() / 4] written with the ReLU mask the backward reads
unsigned char* mask_ptr(const OptT& mask, const Tensor& z, const char* what) {
  if (!mask.has_value() || !mask->defined()) return nullptr;
  TORCH_CHECK(mask->is_cuda() && mask->is_contiguous() && mask->scalar_type() == at::kByte &&
                  mask->numel() == z.numel() / 4,
              what, ": mask must be a contiguous uint8 CUDA tensor of z.numel() / 4 bytes");
  return mask->data_ptr<unsigned char>();
}

// BN + add + ReLU whose residual is another BatchNorm's INPUT rz (ResNet downsample branch): out =
// relu(z*scale + shift + bf16(rz*rscale + rshift)), plus the ReLU mask; bf16 [N,H,W,C], C % 8 == 0.
// Returns false when the 16-byte-lane kernel cannot run it (the caller applies the two BNs separately).
bool bn_apply_rbn(Tensor z, Tensor out, Tensor scale, Tensor shift, Tensor rz, Tensor rscale, Tensor rshift,
                  Tensor mask) {
  for (const Tensor* t : {&z, &out, &rz}) need(*t, "bn_apply_rbn: z/out/rz", at::kBFloat16);
  for (const Tensor* t : {&scale, &shift, &rscale, &rshift}) need(*t, "bn_apply_rbn: coefficients");
  need(mask, "bn_apply_rbn: mask", at::kByte);
  const int64_t C = z.size(-1);
  TORCH_CHECK(out.numel() == z.numel() && rz.numel() == z.numel() && mask.numel() == z.numel() / 4 &&
                  scale.numel() == C && shift.numel() == C && rscale.numel() == C && rshift.numel() == C,
              "bn_apply_rbn: shapes");
  const int rc = dpa_bn_apply_wide(reinterpret_cast<const unsigned short*>(z.data_ptr<at::BFloat16>()),
                                   reinterpret_cast<const unsigned short*>(rz.data_ptr<at::BFloat16>()),
                                   reinterpret_cast<unsigned short*>(out.data_ptr<at::BFloat16>()),
                                   mask.data_ptr<uint8_t>(), fp(scale), fp(shift), z.numel() / C, (int)C, 2,
                                   cur_stream(), fp(rscale), fp(rshift));
  if (rc == 1) return false;
  chk(rc, "bn_apply_rbn");
  return true;
}

void bn_apply(Tensor z, Tensor a, Tensor scale, Tensor shift, bool pool, int64_t act, OptT res, OptT mask) {
  const bool bf = z.scalar_type() == at::kBFloat16;
  const void* zp = act_ptr(z, "z", bf);
  unsigned char* mp = mask_ptr(mask, z, "bn_apply");
  const void* rp = nullptr;
  if (act == 2) {
    TORCH_CHECK(res.has_value() && res->defined(), "bn_apply: act=2 needs the residual");
    TORCH_CHECK(res->numel() == z.numel(), "bn_apply: residual shape");
    rp = act_ptr(*res, "res", bf);
  }
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  const int64_t outn = (int64_t)N * (pool ? (H / 2) * (W / 2) : H * W) * C;
  if (is_plane_dtype(a)) {
    int np = 1;
    if (a.numel() != outn || a.scalar_type() == at::kHalf) {
      need_planes(a, "a3");
      TORCH_CHECK(a.numel() == a.size(0) * outn, "bn_apply: a3 shape");
      np = a.size(0);
    } else {
      TORCH_CHECK(a.is_cuda() && a.is_contiguous(), "bn_apply: a must be contiguous");
    }
    chk(dpa_bn_apply(zp, nullptr, up(a), np, fp(scale), fp(shift), N, H, W, C, pool ? 1 : 0, (int)act, rp,
                     bf ? 1 : 0, cur_stream(), mp),
        "bn_apply");
  } else {
    need(a, "a");
    TORCH_CHECK(a.numel() == outn, "bn_apply: a shape");
    chk(dpa_bn_apply(zp, fp(a), nullptr, 0, fp(scale), fp(shift), N, H, W, C, pool ? 1 : 0, (int)act, rp, bf ? 1 : 0,
                     cur_stream(), mp),
        "bn_apply");
  }
}

// gsrc: grad wrt the layer output (pooled shape if pool) or nsplit slabs of it (then the sum is
// written to g).
// First VGG layer's backward: BN backward (ReLU + 2x2 max-pool) fused with the 3x3 weight gradient
// on the fp32 network input (bn.hip, bn_bwd_wgrad0_kernel).  z [N,32,32,64], g [N,16,16,64],
// x [N,32,32,4], dw [64,3,3,CP], wpart >= wgrad0_part_floats(N).
void bn_bwd_wgrad0(Tensor gsrc, int64_t nsplit, Tensor g, Tensor z, Tensor scale, Tensor shift, Tensor mean,
                   Tensor invstd, Tensor gamma, Tensor part, Tensor coef, Tensor dgamma, Tensor dbeta, OptT dbias,
                   Tensor x, Tensor wpart, Tensor dw, OptT sig, int64_t sig_val) {
  for (auto* t : {&gsrc, &g, &z, &scale, &shift, &mean, &invstd, &gamma, &part, &coef, &dgamma, &dbeta, &x, &wpart, &dw})
    need(*t, "bn_bwd_wgrad0 operand");
  const int N = z.size(0);
  TORCH_CHECK(z.dim() == 4 && z.size(1) == 32 && z.size(2) == 32 && z.size(3) == 64, "bn_bwd_wgrad0: z [N,32,32,64]");
  TORCH_CHECK(g.numel() == (int64_t)N * 16 * 16 * 64, "bn_bwd_wgrad0: g [N,16,16,64]");
  TORCH_CHECK(gsrc.numel() >= nsplit * g.numel(), "bn_bwd_wgrad0: gsrc too small");
  TORCH_CHECK(x.dim() == 4 && x.size(0) == N && x.size(1) == 32 && x.size(2) == 32 && x.size(3) == 4,
              "bn_bwd_wgrad0: x [N,32,32,4]");
  TORCH_CHECK(dw.dim() == 4 && dw.size(0) == 64 && dw.size(1) == 3 && dw.size(2) == 3 && dw.size(3) >= 3,
              "bn_bwd_wgrad0: dw [64,3,3,CP]");
  TORCH_CHECK(wpart.numel() >= dpa_wgrad0_part_floats(N), "bn_bwd_wgrad0: wpart too small");
  TORCH_CHECK(part.numel() >= dpa_bn_part_floats(N * 256, 64, 1), "bn_bwd_wgrad0: part too small");
  TORCH_CHECK(coef.numel() >= 4 * 64 && scale.numel() == 64 && gamma.numel() == 64, "bn_bwd_wgrad0: channel vectors");
  chk(dpa_bn_bwd_wgrad0(fp(gsrc), (int)nsplit, fp(g), fp(z), fp(scale), fp(shift), fp(mean), fp(invstd), fp(gamma),
                        fp(part), fp(coef), fp(dgamma), fp(dbeta), ofp(dbias), fp(x), fp(wpart), fp(dw),
                        (int)dw.size(3), N, cur_stream(), opt_signal(sig, "bn_bwd_wgrad0"), (int)sig_val),
      "bn_bwd_wgrad0");
}

// First VGG layer forward (first_layer.hip): direct fp32 3x3 conv of x [N,32,32,4] with w [64,3,3,CP]
// into z [N,32,32,64].  Training (part given): BN batch statistics from the conv epilogue, then the
// finalize (running stats, scale/shift); eval (part None): the conv only.
void conv0_fwd(Tensor x, Tensor w, Tensor z, OptT part, OptT gamma, OptT beta, OptT bias, OptT rmean, OptT rvar,
               OptT nbt, OptT mean, OptT invstd, OptT scale, OptT shift, double momentum, double eps) {
  need(x, "x");
  need(w, "w");
  need(z, "z");
  const int N = x.size(0);
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 32 && x.size(2) == 32 && x.size(3) == 4, "conv0_fwd: x [N,32,32,4]");
  TORCH_CHECK(w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 && w.size(2) == 3 && w.size(3) >= 3,
              "conv0_fwd: w [64,3,3,CP]");
  TORCH_CHECK(z.numel() == (int64_t)N * 32 * 32 * 64, "conv0_fwd: z [N,32,32,64]");
  float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    need(*part, "part");
    TORCH_CHECK(part->numel() >= dpa_conv0_part_floats(N), "conv0_fwd: part too small");
    for (const OptT* o : {&gamma, &beta, &mean, &invstd, &scale, &shift})
      TORCH_CHECK(o->has_value() && (*o)->defined() && (*o)->numel() == 64, "conv0_fwd: channel vectors [64]");
    pp = fp(*part);
  }
  long long* nb = nbt.has_value() && nbt->defined() ? reinterpret_cast<long long*>(nbt->data_ptr<int64_t>()) : nullptr;
  chk(dpa_conv0_fwd(fp(x), fp(w), (int)w.size(3), fp(z), pp, N, ofp(gamma), ofp(beta), ofp(bias), ofp(rmean),
                    ofp(rvar), nb, ofp(mean), ofp(invstd), ofp(scale), ofp(shift), (float)momentum, (float)eps,
                    cur_stream()),
      "conv0_fwd");
}

// C = opA(A) @ opB(B) (+ bias), fp32 on the fp32 matrix cores (gemm_f32.hip).  opA(A) = A [M,K] or,
// trans_a, A^T of A [K,M]; opB(B) = B [K,N] or, trans_b, B^T of B [N,K].  splits > 1: split-K
// through slab (>= splits * M * N floats), fixed-order reduction.
void gemm_f32(Tensor A, Tensor B, Tensor C, bool trans_a, bool trans_b, OptT bias, int64_t splits, OptT slab) {
  need(A, "A");
  need(B, "B");
  need(C, "C");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm_f32: 2-D operands");
  const int M = trans_a ? A.size(1) : A.size(0), K = trans_a ? A.size(0) : A.size(1);
  const int N = trans_b ? B.size(0) : B.size(1), KB = trans_b ? B.size(1) : B.size(0);
  TORCH_CHECK(K == KB && C.size(0) == M && C.size(1) == N, "gemm_f32: shapes");
  float* sp = nullptr;
  if (splits > 1) {
    TORCH_CHECK(slab.has_value() && slab->defined() && slab->numel() >= splits * (int64_t)M * N,
                "gemm_f32: split-K needs a slab of splits * M * N floats");
    need(*slab, "slab");
    sp = fp(*slab);
  }
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->numel() == N, "gemm_f32: bias [N]");
  chk(dpa_gemm_f32(fp(A), A.size(1), trans_a ? 0 : 1, fp(B), B.size(1), trans_b ? 1 : 0, fp(C), M, N, K, ofp(bias), sp,
                   (int)splits, cur_stream()),
      "gemm_f32");
}

// ---------------- generic classifier head (head.hip) ----------------
// x [N,H,W,C] (bf16 or fp32) -> feat [N,C] fp32 (spatial mean)
void gap(Tensor x, Tensor feat) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4, "gap: contiguous NHWC GPU tensor expected");
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || x.scalar_type() == at::kFloat, "gap: x must be bf16 or fp32");
  need(feat, "feat");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  TORCH_CHECK(feat.numel() == (int64_t)N * C, "gap: feat [N,C]");
  chk(dpa_gap(x.data_ptr(), fp(feat), N, HW, C, bf ? 1 : 0, cur_stream()), "gap");
}

// logits [N,J] fp32, target [N] int64 -> loss_row [N], optional dlogits [N,J] = (softmax - onehot)/N,
// optional correct_row [N] int32, loss [1] = batch mean, acc [2] += (loss, #correct)
void softmax_ce(Tensor logits, Tensor target, Tensor loss_row, OptT dlogits, OptT correct_row, OptT loss, OptT acc) {
  need(logits, "logits");
  need(loss_row, "loss_row");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == at::kLong && target.is_contiguous(), "target int64");
  const int N = logits.size(0), J = logits.size(1);
  TORCH_CHECK(target.numel() == N && loss_row.numel() >= N, "softmax_ce: sizes");
  int* cr = nullptr;
  if (correct_row.has_value() && correct_row->defined()) {
    TORCH_CHECK(correct_row->scalar_type() == at::kInt && correct_row->numel() >= N, "correct_row int32 [N]");
    cr = correct_row->data_ptr<int>();
  }
  if (dlogits.has_value() && dlogits->defined()) TORCH_CHECK(dlogits->numel() == (int64_t)N * J, "dlogits [N,J]");
  chk(dpa_ce(fp(logits), reinterpret_cast<const long long*>(target.data_ptr<int64_t>()), fp(loss_row), ofp(dlogits),
             cr, ofp(loss), ofp(acc), N, J, cur_stream()),
      "softmax_ce");
}

void head_bwd_prep(Tensor dlogits, Tensor gout, Tensor dl, Tensor db) {
  need(dlogits, "dlogits");
  need(gout, "gout");
  need(dl, "dl");
  need(db, "db");
  const int N = dlogits.size(0), J = dlogits.size(1);
  TORCH_CHECK(dl.numel() == dlogits.numel() && db.numel() == J && gout.numel() >= 1, "head_bwd_prep: sizes");
  chk(dpa_head_bwd_prep(fp(dlogits), fp(gout), fp(dl), fp(db), N, J, cur_stream()), "head_bwd_prep");
}

void gap_bwd(Tensor dfeat, Tensor dx) {
  need(dfeat, "dfeat");
  TORCH_CHECK(dx.is_cuda() && dx.is_contiguous() && dx.dim() == 4, "gap_bwd: dx NHWC");
  const bool bf = dx.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || dx.scalar_type() == at::kFloat, "gap_bwd: dx bf16 or fp32");
  const int N = dx.size(0), HW = dx.size(1) * dx.size(2), C = dx.size(3);
  TORCH_CHECK(dfeat.numel() == (int64_t)N * C, "gap_bwd: dfeat [N,C]");
  chk(dpa_gap_bwd(fp(dfeat), dx.data_ptr(), N, HW, C, bf ? 1 : 0, cur_stream()), "gap_bwd");
}

void bn_bwd(Tensor gsrc, int64_t nsplit, Tensor g, Tensor z, Tensor scale, Tensor shift, Tensor mean, Tensor invstd,
            Tensor gamma, Tensor part, Tensor coef, Tensor dgamma, Tensor dbeta, OptT dbias, Tensor dz, bool pool,
            int64_t act, OptT res, OptT dres, OptT sig, int64_t sig_val, OptT g2, OptT mask, OptT bound) {
  const bool bf = z.scalar_type() == at::kBFloat16;
  const void* zp = act_ptr(z, "z", bf);
  const void* gsp = act_ptr(gsrc, "gsrc", bf);
  void* gp = act_ptr(g, "g", bf);
  const void* rp = nullptr;
  void* drp = nullptr;
  const unsigned char* mp = mask_ptr(mask, z, "bn_bwd");
  if (act == 2) {
    // the ReLU mask of the forward (bn_apply mask=...) replaces the residual
    TORCH_CHECK((mp || (res.has_value() && res->defined())) && dres.has_value() && dres->defined(),
                "bn_bwd: act=2 needs (res or mask) and dres");
    TORCH_CHECK(dres->numel() == z.numel(), "bn_bwd: residual shape");
    if (!mp) {
      TORCH_CHECK(res->numel() == z.numel(), "bn_bwd: residual shape");
      rp = act_ptr(*res, "res", bf);
    }
    drp = act_ptr(*dres, "dres", bf);
  }
  float* dzf = nullptr;
  u16* dz3 = nullptr;
  int np = 0;
  if (is_plane_dtype(dz)) {
    if (dz.numel() == z.numel() && dz.scalar_type() == at::kBFloat16) {  // one plane, [N,H,W,C]
      TORCH_CHECK(dz.is_cuda() && dz.is_contiguous(), "bn_bwd: dz must be contiguous");
      np = 1;
    } else {
      need_planes(dz, "dz3");
      TORCH_CHECK(dz.numel() == dz.size(0) * z.numel(), "bn_bwd: dz3 shape");
      np = dz.size(0);
    }
    dz3 = up(dz);
  } else {
    need(dz, "dz");
    dzf = fp(dz);
  }
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  const int Mo = N * (pool ? (H / 2) * (W / 2) : H * W);
  TORCH_CHECK(g.numel() == (int64_t)Mo * C, "bn_bwd: g shape");
  TORCH_CHECK(gsrc.numel() >= nsplit * (int64_t)Mo * C, "bn_bwd: gsrc too small");
  TORCH_CHECK(part.numel() >= dpa_bn_part_floats(Mo, C, 1), "bn_bwd: part too small");
  TORCH_CHECK(coef.numel() >= 4L * C, "bn_bwd: coef too small (4 rows: k1, c2, k3, mean)");
  const void* g2p = nullptr;
  if (g2.has_value() && g2->defined()) {
    TORCH_CHECK(g2->numel() == g.numel() && g2->scalar_type() == g.scalar_type() && nsplit == 1,
                "bn_bwd: g2 must match g (type, size) and nsplit must be 1");
    g2p = act_ptr(*g2, "g2", bf);
  }
  chk(dpa_bn_bwd(gsp, (int)nsplit, gp, zp, fp(scale), fp(shift), fp(mean), fp(invstd), fp(gamma), fp(part), fp(coef),
                 fp(dgamma), fp(dbeta), ofp(dbias), dzf, dz3, np, N, H, W, C, pool ? 1 : 0, (int)act, rp, drp,
                 bf ? 1 : 0, cur_stream(), opt_signal(sig, "bn_bwd"), (int)sig_val, g2p, mp,
                 const_cast<unsigned*>(bound_ptr(bound, "bn_bwd"))),
      "bn_bwd");
}

// ---------------- one-launch BatchNorm (bn_fused.hip) ----------------
// (part_floats, cnt_words, blocks) of the fused layer, or None when its geometry does not fit.
py::object bn_fused_geo(int64_t Mo, int64_t C, bool pool, bool bwd, int64_t rmax) {
  long pf = 0, cw = 0;
  int nb = 0;
  if (dpa_bn_fused_geo((int)Mo, (int)C, pool ? 1 : 0, bwd ? 1 : 0, (int)rmax, &pf, &cw, &nb) != 0) return py::none();
  return py::make_tuple((int64_t)pf, (int64_t)cw, (int64_t)nb);
}

// out (optional): fp32 [N,Ho,Wo,C] or bf16 planes [NP,N,Ho,Wo,C]; fp32 only
struct OutPtrs {
  float* f = nullptr;
  u16* b = nullptr;
  int np = 0;
  long ps = 0;
};
OutPtrs out_ptrs(const OptT& out, int64_t n, const char* what) {
  OutPtrs o;
  if (!out.has_value() || !out->defined()) return o;
  const Tensor& t = *out;
  if (is_plane_dtype(t)) {
    if (t.numel() == n && t.scalar_type() == at::kBFloat16) {
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), what, ": out must be contiguous");
      o.np = 1;
    } else {
      need_planes(t, what);
      TORCH_CHECK(t.numel() == t.size(0) * n, what, ": planes shape");
      o.np = t.size(0);
    }
    o.b = up(t);
    o.ps = n;
  } else {
    need(t, what);
    TORCH_CHECK(t.numel() == n, what, ": out shape");
    o.f = fp(t);
  }
  return o;
}

void bn_fused_fwd(Tensor src, int64_t nsplit, Tensor z, bool pool, int64_t rmax, Tensor part, Tensor cnt,
                  Tensor gamma, Tensor beta, OptT bias, OptT rmean, OptT rvar, OptT nbt, Tensor mean, Tensor invstd,
                  Tensor scale, Tensor shift, OptT out, double momentum, double eps, Tensor tmo,
                  int64_t timeout_us) {
  need(src, "src");
  need(z, "z");
  need(part, "part");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == torch::kInt32, "bn_fused_fwd: cnt must be int32");
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  const int Mo = N * (pool ? (H / 2) * (W / 2) : H * W);
  long pf = 0, cw = 0;
  int nb = 0;
  TORCH_CHECK(dpa_bn_fused_geo(Mo, C, pool ? 1 : 0, 0, (int)rmax, &pf, &cw, &nb) == 0, "bn_fused_fwd: no geometry");
  TORCH_CHECK(part.numel() >= pf && cnt.numel() >= cw, "bn_fused_fwd: workspace too small");
  TORCH_CHECK(src.numel() >= nsplit * z.numel(), "bn_fused_fwd: src too small");
  long long* nb_p = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    need(*nbt, "nbt", at::kLong);
    nb_p = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>());
  }
  const OutPtrs o = out_ptrs(out, (int64_t)Mo * C, "bn_fused_fwd");
  chk(dpa_bn_fused_fwd(fp(src), (int)nsplit, fp(z), N, H, W, C, pool ? 1 : 0, (int)rmax, fp(part),
                       reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), fp(gamma), fp(beta), ofp(bias), ofp(rmean),
                       ofp(rvar), nb_p, fp(mean), fp(invstd), fp(scale), fp(shift), (o.f || o.b) ? 1 : 0, o.f, o.b,
                       o.np, o.ps, (float)momentum, (float)eps, signal_ptr(tmo, "bn_fused_fwd"), timeout_us,
                       cur_stream()),
      "bn_fused_fwd");
}



void bn_fused_bwd(Tensor gsrc, int64_t nsplit, Tensor z, bool pool, int64_t rmax, Tensor part, Tensor cnt,
                  Tensor scale, Tensor shift, Tensor mean, Tensor invstd, Tensor gamma, Tensor dgamma, Tensor dbeta,
                  OptT dbias, Tensor dz, Tensor tmo, int64_t timeout_us, OptT sig, int64_t sig_val) {
  need(gsrc, "gsrc");
  need(z, "z");
  need(part, "part");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == torch::kInt32, "bn_fused_bwd: cnt must be int32");
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  const int Mo = N * (pool ? (H / 2) * (W / 2) : H * W);
  long pf = 0, cw = 0;
  int nb = 0;
  TORCH_CHECK(dpa_bn_fused_geo(Mo, C, pool ? 1 : 0, 1, (int)rmax, &pf, &cw, &nb) == 0, "bn_fused_bwd: no geometry");
  TORCH_CHECK(part.numel() >= pf && cnt.numel() >= cw, "bn_fused_bwd: workspace too small");
  TORCH_CHECK(gsrc.numel() >= nsplit * (int64_t)Mo * C, "bn_fused_bwd: gsrc too small");
  const OutPtrs o = out_ptrs(dz, z.numel(), "bn_fused_bwd");
  chk(dpa_bn_fused_bwd(fp(gsrc), (int)nsplit, fp(z), N, H, W, C, pool ? 1 : 0, (int)rmax, fp(part),
                       reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), fp(scale), fp(shift), fp(mean), fp(invstd),
                       fp(gamma), fp(dgamma), fp(dbeta), ofp(dbias), o.f, o.b, o.np, o.ps,
                       signal_ptr(tmo, "bn_fused_bwd"), timeout_us, cur_stream(), opt_signal(sig, "bn_fused_bwd"),
                       (int)sig_val),
      "bn_fused_bwd");
}

// ---------------- classifier head ----------------
// bn_z [B,2,2,Cin] fp32 + bn_scale/bn_shift [Cin] (optional): the features x [B,Cin] are computed
// from the last conv's output (BN + ReLU + 2x2 max-pool) inside the head kernel and written to x
void fc_ce_train(Tensor x, Tensor w, Tensor b, Tensor target, Tensor loss_row, Tensor dlogits, Tensor dx, Tensor dw,
                 Tensor db, Tensor loss_out, OptT loss_accum, OptT bn_z, OptT bn_scale, OptT bn_shift, int64_t parts) {
  TORCH_CHECK(parts >= 1 && parts <= 3, "fc_ce_train: parts must be 1 (rows), 2 (weight gradient) or 3 (both)");
  need(x, "x");
  need(target, "target", at::kLong);
  const int B = x.size(0), Cin = x.size(1), J = w.size(0);
  const float* zp = nullptr;
  if (bn_z.has_value() && bn_z->defined()) {
    need(*bn_z, "bn_z");
    TORCH_CHECK(bn_z->dim() == 4 && bn_z->size(0) == B && bn_z->size(1) == 2 && bn_z->size(2) == 2 &&
                    bn_z->size(3) == Cin,
                "fc_ce_train: bn_z must be [B,2,2,Cin]");
    TORCH_CHECK(bn_scale.has_value() && bn_shift.has_value() && bn_scale->numel() == Cin && bn_shift->numel() == Cin,
                "fc_ce_train: bn_scale / bn_shift [Cin] needed with bn_z");
    need(*bn_scale, "bn_scale");
    need(*bn_shift, "bn_shift");
    zp = fp(*bn_z);
  }
  chk(dpa_fc_ce_train(fp(x), fp(w), fp(b), reinterpret_cast<const long long*>(target.data_ptr<int64_t>()),
                      fp(loss_row), fp(dlogits), fp(dx), fp(dw), fp(db), fp(loss_out), ofp(loss_accum), B, Cin, J,
                      cur_stream(), zp, zp ? fp(*bn_scale) : nullptr, zp ? fp(*bn_shift) : nullptr, (int)parts),
      "fc_ce_train");
}

void fc_ce_eval(Tensor x, Tensor w, Tensor b, Tensor target, Tensor loss_row, Tensor correct_row, OptT logits,
                OptT acc) {
  need(x, "x");
  need(target, "target", at::kLong);
  need(correct_row, "correct_row", at::kInt);
  const int B = x.size(0), Cin = x.size(1), J = w.size(0);
  chk(dpa_fc_ce_eval(fp(x), fp(w), fp(b), reinterpret_cast<const long long*>(target.data_ptr<int64_t>()),
                     fp(loss_row), correct_row.data_ptr<int>(), ofp(logits), ofp(acc), B, Cin, J, cur_stream()),
      "fc_ce_eval");
}

// ---------------- data ----------------
void augment(Tensor images, Tensor idx, Tensor labels, Tensor out, OptT target, int64_t pad, bool train,
             int64_t seed, int64_t salt, std::vector<double> mean, std::vector<double> std_) {
  need(images, "images", at::kByte);
  need(idx, "idx", at::kLong);
  need(labels, "labels", at::kLong);
  need(out, "out");
  TORCH_CHECK(images.dim() == 4 && images.size(3) == 3, "augment: images must be [N,H,W,3] uint8");
  const int B = idx.numel(), Hs = images.size(1), Ws = images.size(2);
  TORCH_CHECK(out.numel() == (int64_t)B * Hs * Ws * 4, "augment: out must be [B,H,W,4]");
  float m[3], s[3];
  for (int c = 0; c < 3; ++c) {
    m[c] = (float)mean.at(c);
    s[c] = (float)std_.at(c);
  }
  long long* tp = nullptr;
  if (target.has_value() && target->defined()) {
    need(*target, "target", at::kLong);
    tp = reinterpret_cast<long long*>(target->data_ptr<int64_t>());
  }
  chk(dpa_augment(images.data_ptr<uint8_t>(), reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()),
                  reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()), fp(out), tp, B, Hs, Ws, (int)pad,
                  train ? 1 : 0, (unsigned long long)seed, (unsigned long long)salt, m, s, cur_stream()),
      "augment");
}

// ---------------- NHWC max-pool (generic path) ----------------
void maxpool_check(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 4, name, " must be a contiguous 4-D GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, name, " must be fp32 or bf16");
}

// scale / shift (optional, fp32 [C]): x is a BatchNorm input, pooled as relu(x*scale + shift)
void maxpool_fwd(Tensor x, Tensor y, Tensor arg, int64_t k, int64_t s, int64_t p, OptT scale, OptT shift) {
  maxpool_check(x, "x");
  maxpool_check(y, "y");
  const bool bn = scale.has_value() && scale->defined();
  TORCH_CHECK(bn == (shift.has_value() && shift->defined()), "maxpool_fwd: scale and shift go together");
  if (bn) {
    need(*scale, "scale");
    need(*shift, "shift");
    TORCH_CHECK(scale->numel() == x.size(3) && shift->numel() == x.size(3), "maxpool_fwd: scale/shift size");
  }
  TORCH_CHECK(y.scalar_type() == x.scalar_type() && arg.scalar_type() == at::kByte && arg.sizes() == y.sizes() &&
                  arg.is_contiguous(), "maxpool_fwd: y/arg shape or dtype");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(y.size(0) == N && y.size(1) == (H + 2 * p - k) / s + 1 && y.size(2) == (W + 2 * p - k) / s + 1 &&
                  y.size(3) == C, "maxpool_fwd: output shape");
  chk(dpa_maxpool_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr<uint8_t>(), N, H, W, C, (int)k, (int)s, (int)p,
                      x.scalar_type() == at::kBFloat16 ? 1 : 0, cur_stream(), ofp(scale), ofp(shift)),
      "maxpool_fwd");
}

void maxpool_bwd(Tensor dy, Tensor arg, Tensor dx, int64_t k, int64_t s, int64_t p) {
  maxpool_check(dy, "dy");
  maxpool_check(dx, "dx");
  TORCH_CHECK(dx.scalar_type() == dy.scalar_type() && arg.scalar_type() == at::kByte && arg.sizes() == dy.sizes() &&
                  arg.is_contiguous(), "maxpool_bwd: dy/arg shape or dtype");
  const int N = dx.size(0), H = dx.size(1), W = dx.size(2), C = dx.size(3);
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == (H + 2 * p - k) / s + 1 && dy.size(2) == (W + 2 * p - k) / s + 1 &&
                  dy.size(3) == C, "maxpool_bwd: gradient shape");
  chk(dpa_maxpool_bwd(dy.data_ptr(), arg.data_ptr<uint8_t>(), dx.data_ptr(), N, H, W, C, (int)k, (int)s, (int)p,
                      dx.scalar_type() == at::kBFloat16 ? 1 : 0, cur_stream()),
      "maxpool_bwd");
}

// ---------------- RCCL communicator ----------------
ncclDataType_t nccl_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat:
      return ncclFloat32;
    case at::kBFloat16:
      return ncclBfloat16;
    case at::kHalf:
      return ncclFloat16;
    case at::kLong:
      return ncclInt64;
    case at::kInt:
      return ncclInt32;
    case at::kByte:
      return ncclUint8;
    case at::kDouble:
      return ncclFloat64;
    default:
      TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "unknown reduce op ", op);
}

class PyRcclComm {
 public:
  PyRcclComm(int rank, int world, py::bytes uid, int device, bool high_priority, double timeout_s, double poll_s,
             bool watchdog, bool exit_on_error, bool debug_sync, int max_ctas)
      : stream_(c10::hip::getStreamFromPool(high_priority, (c10::DeviceIndex)device)),
        comm_(rank, world, std::string(uid), device, stream_.stream(),
              dpa::WatchdogConfig{timeout_s, poll_s, watchdog, exit_on_error, debug_sync}, max_ctas) {}

  void track(const Tensor& t) { c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_); }

  void all_reduce(Tensor t, const std::string& op) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "all_reduce: contiguous GPU tensor expected");
    track(t);
    comm_.all_reduce(t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), cur_stream());
  }
  void all_reduce_here(Tensor t, const std::string& op) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "all_reduce_here: contiguous GPU tensor expected");
    comm_.all_reduce_here(t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), cur_stream());
  }
  void broadcast(Tensor t, int root) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "broadcast: contiguous GPU tensor expected");
    track(t);
    comm_.broadcast(t.data_ptr(), t.numel(), nccl_dtype(t), root, cur_stream());
  }
  void gather(Tensor send, OptT recv, int root) {
    TORCH_CHECK(send.is_cuda() && send.is_contiguous(), "gather: contiguous GPU tensor expected");
    track(send);
    void* rp = nullptr;
    if (comm_.rank() == root) {
      TORCH_CHECK(recv.has_value() && recv->numel() == send.numel() * comm_.world(), "gather: recv must be world*n");
      track(*recv);
      rp = recv->data_ptr();
    }
    comm_.gather(send.data_ptr(), rp, send.numel(), nccl_dtype(send), root, cur_stream());
  }
  void reduce_scatter(Tensor send, Tensor recv, const std::string& op) {
    TORCH_CHECK(send.numel() == recv.numel() * comm_.world(), "reduce_scatter: send must be world*recv");
    track(send);
    track(recv);
    comm_.reduce_scatter(send.data_ptr(), recv.data_ptr(), recv.numel(), nccl_dtype(recv), nccl_op(op), cur_stream());
  }
  void all_gather(Tensor send, Tensor recv) {
    TORCH_CHECK(recv.numel() == send.numel() * comm_.world(), "all_gather: recv must be world*send");
    track(send);
    track(recv);
    comm_.all_gather(send.data_ptr(), recv.data_ptr(), send.numel(), nccl_dtype(send), cur_stream());
  }
  void send(Tensor t, int peer) {
    track(t);
    comm_.send(t.data_ptr(), t.numel(), nccl_dtype(t), peer, cur_stream());
  }
  void recv(Tensor t, int peer) {
    track(t);
    comm_.recv(t.data_ptr(), t.numel(), nccl_dtype(t), peer, cur_stream());
  }
  void wait() { comm_.wait(cur_stream()); }
  void synchronize() { comm_.synchronize(); }
  std::string async_error() { return comm_.async_error(); }
  void abort() { comm_.abort(); }
  int64_t stream_ptr() { return reinterpret_cast<int64_t>(stream_.stream()); }
  int64_t outstanding() { return (int64_t)comm_.outstanding(); }
  int64_t ops_issued() { return (int64_t)comm_.ops_issued(); }
  int comm_count() { return comm_.comm_count(); }
  int max_ctas() const { return comm_.max_ctas(); }
  int rank() const { return comm_.rank(); }
  int world() const { return comm_.world(); }

 private:
  c10::hip::HIPStream stream_;
  dpa::RcclComm comm_;
};

// Peer-memory communicator (runtime/ipc_comm.cpp, kernels/ipc_coll.hip).  Tensors of any dtype
// move as 4-byte words; reductions read them as fp32 (parallel/ipc.py checks the dtype).
static int64_t ipc_words(const Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "ipc: contiguous GPU tensor expected");
  TORCH_CHECK(t.nbytes() % 4 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 4 == 0,
              "ipc: tensor must be a whole number of 4-byte words");
  return (int64_t)(t.nbytes() / 4);
}

class PyIpcComm {
 public:
  PyIpcComm(int rank, int world, int device, int64_t stage_words, int64_t inbox_words)
      : c_(rank, world, device, (long)stage_words, (long)inbox_words) {}
  py::bytes sig_handle() { return py::bytes(c_.sig_handle()); }
  int64_t tmo_ptr() { return reinterpret_cast<int64_t>(c_.tmo_word()); }
  py::bytes stage_handle() { return py::bytes(c_.stage_handle()); }
  py::bytes inbox_handle() { return py::bytes(c_.inbox_handle()); }
  static py::bytes tensor_handle(const Tensor& t) {
    TORCH_CHECK(t.is_cuda(), "ipc: GPU tensor expected");
    return py::bytes(dpa::IpcComm::export_handle(t.data_ptr()));
  }
  void set_peers(const std::vector<std::string>& sig, const std::vector<std::string>& stage,
                 const std::vector<std::string>& inbox) {
    c_.set_peers(sig, stage, inbox);
  }
  int add_region(const std::vector<std::string>& handles, Tensor local) {
    return c_.add_region(handles, local.data_ptr(), (long)ipc_words(local));
  }
  // rid < 0: the input is bounced through the inbox; off: the input's word offset in region rid
  void all_reduce(int rid, int64_t off, Tensor t, int red, int blocks, int64_t tmo_us) {
    c_.all_reduce(rid, (long)off, t.data_ptr(), (long)ipc_words(t), red, blocks, (long long)tmo_us, cur_stream());
  }
  void broadcast(int rid, int64_t off, Tensor t, int root, int blocks, int64_t tmo_us) {
    c_.broadcast(rid, (long)off, t.data_ptr(), (long)ipc_words(t), root, blocks, (long long)tmo_us, cur_stream());
  }
  void gather(int rid, int64_t off, Tensor send, c10::optional<Tensor> recv, int root, int blocks, int64_t tmo_us) {
    const int64_t n = ipc_words(send);
    void* out = nullptr;
    if (recv.has_value()) {
      TORCH_CHECK(ipc_words(*recv) >= n * c_.world(), "ipc gather: recv too small");
      out = recv->data_ptr();
    }
    c_.gather(rid, (long)off, send.data_ptr(), out, (long)n, root, blocks, (long long)tmo_us, cur_stream());
  }
  void reduce_scatter(int rid, int64_t off, Tensor send, Tensor recv, int red, int blocks, int64_t tmo_us) {
    const int64_t n = ipc_words(recv);
    TORCH_CHECK(ipc_words(send) == n * c_.world(), "ipc reduce_scatter: send must be world x recv");
    c_.reduce_scatter(rid, (long)off, send.data_ptr(), recv.data_ptr(), (long)n, red, blocks, (long long)tmo_us,
                      cur_stream());
  }
  void all_gather(int rid, int64_t off, Tensor send, Tensor recv, int blocks, int64_t tmo_us) {
    const int64_t n = ipc_words(send);
    TORCH_CHECK(ipc_words(recv) == n * c_.world(), "ipc all_gather: recv must be world x send");
    c_.all_gather(rid, (long)off, send.data_ptr(), recv.data_ptr(), (long)n, blocks, (long long)tmo_us, cur_stream());
  }
  void barrier(int blocks, int64_t tmo_us) { c_.barrier(blocks, (long long)tmo_us, cur_stream()); }
  bool take_timeout() { return c_.take_timeout(); }
  int64_t launches() const { return (int64_t)c_.launches(); }
  int rank() const { return c_.rank(); }
  int world() const { return c_.world(); }

 private:
  dpa::IpcComm c_;
};

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "distributed_pytorch_amd native extension (gfx950 HIP kernels + RCCL communicator)";
  m.def("sgd_flat", &sgd_flat, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("lr"), py::arg("momentum"),
        py::arg("wd"), py::arg("gscale"), py::arg("first"), py::arg("offset") = 0, py::arg("count") = -1,
        py::arg("planes") = py::none());
  m.def("spin", &spin, py::arg("usec"), py::arg("done"));
  m.def("mean_of_w", &mean_of_w);
  m.def("add_inplace", &add_inplace);
  m.def("conv_fprop", &conv_fprop, py::arg("x"), py::arg("w"), py::arg("out"), py::arg("slab"), py::arg("stride"),
        py::arg("pad"), py::arg("splits") = 1, py::arg("tile") = 0, py::arg("dgrad") = false, py::arg("reduce") = true,
        py::arg("posmajor") = false);
  m.def("conv_splits", &conv_splits);
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dz"), py::arg("dw"), py::arg("slab"), py::arg("stride"),
        py::arg("pad"), py::arg("splits") = 1, py::arg("tile") = 0, py::arg("posmajor") = false);
  m.def("wflip", &wflip);
  m.def("x3_splits", &x3_splits);
  m.def("conv_x3_fprop", &conv_x3_fprop, py::arg("x3"), py::arg("w3"), py::arg("out"), py::arg("slab"),
        py::arg("stride"), py::arg("pad"), py::arg("splits") = 1, py::arg("tile") = 0, py::arg("reduce") = true,
        py::arg("posmajor") = 0, py::arg("stats") = py::none(), py::arg("oscale") = 1.0,
        py::arg("obound") = py::none());
  m.def("conv_stats_rows", [](int64_t tile) { return (int64_t)dpa_conv_stats_rows((int)tile); });
  m.def("bn_finalize", &bn_finalize);
  m.def("conv_x3_wgrad", &conv_x3_wgrad, py::arg("x3"), py::arg("dz3"), py::arg("dw"), py::arg("slab"),
        py::arg("stride"), py::arg("pad"), py::arg("splits") = 1, py::arg("tile") = 0, py::arg("posmajor") = 0,
        py::arg("oscale") = 1.0, py::arg("obound") = py::none());
  m.def("conv_x3_dgrad", &conv_x3_dgrad, py::arg("dz3"), py::arg("w3"), py::arg("dx"), py::arg("slab"),
        py::arg("stride"), py::arg("pad"), py::arg("splits") = 1, py::arg("tile") = 0, py::arg("reduce") = true,
        py::arg("posmajor") = 0, py::arg("add") = py::none(), py::arg("sig") = py::none(),
        py::arg("sig_val") = 0, py::arg("oscale") = 1.0, py::arg("obound") = py::none());
  m.def("wait_signal", &wait_signal, py::arg("sig"), py::arg("val"), py::arg("timeout_us"), py::arg("tmo"));
  m.def("set_signal", &set_signal, py::arg("sig"), py::arg("val"));
  m.def("h2_overflow_addrs", &h2_overflow_addrs);
  m.def("health_copy", &health_copy, py::arg("ptrs"), py::arg("out"), py::arg("tag"));
  m.def("split_planes", &split_planes, py::arg("x"), py::arg("out"), py::arg("scale") = 1.0);
  m.def("h2_overflow", &h2_overflow, py::arg("clear") = false);
  m.attr("H2_SW") = 256.0;  // fp16-pair plane scales (kernels/common.h)
  m.attr("H2_SA") = 16.0;
  m.def("pad_split8", &pad_split8);
  m.def("bn_part_floats", &bn_part_floats);
  m.def("bn_fwd_stats", &bn_fwd_stats);
  m.def("bn_eval_params", &bn_eval_params);
  m.def("bn_apply_rbn", &bn_apply_rbn, py::arg("z"), py::arg("out"), py::arg("scale"), py::arg("shift"),
        py::arg("rz"), py::arg("rscale"), py::arg("rshift"), py::arg("mask"));
  m.def("bn_apply", &bn_apply, py::arg("z"), py::arg("a"), py::arg("scale"), py::arg("shift"), py::arg("pool"),
        py::arg("act") = 0, py::arg("res") = py::none(), py::arg("mask") = py::none());
  m.def("bn_bwd", &bn_bwd, py::arg("gsrc"), py::arg("nsplit"), py::arg("g"), py::arg("z"), py::arg("scale"),
        py::arg("shift"), py::arg("mean"), py::arg("invstd"), py::arg("gamma"), py::arg("part"), py::arg("coef"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("dbias"), py::arg("dz"), py::arg("pool"), py::arg("act") = 0,
        py::arg("res") = py::none(), py::arg("dres") = py::none(), py::arg("sig") = py::none(),
        py::arg("sig_val") = 0, py::arg("g2") = py::none(), py::arg("mask") = py::none(),
        py::arg("bound") = py::none());
  m.def("bn_fused_geo", &bn_fused_geo, py::arg("Mo"), py::arg("C"), py::arg("pool"), py::arg("bwd"),
        py::arg("rmax"));
  m.def("bn_fused_fwd", &bn_fused_fwd, py::arg("src"), py::arg("nsplit"), py::arg("z"), py::arg("pool"),
        py::arg("rmax"), py::arg("part"), py::arg("cnt"), py::arg("gamma"), py::arg("beta"), py::arg("bias"),
        py::arg("rmean"), py::arg("rvar"), py::arg("nbt"), py::arg("mean"), py::arg("invstd"), py::arg("scale"),
        py::arg("shift"), py::arg("out"), py::arg("momentum"), py::arg("eps"), py::arg("tmo"),
        py::arg("timeout_us"));
  m.def("bn_fused_bwd", &bn_fused_bwd, py::arg("gsrc"), py::arg("nsplit"), py::arg("z"), py::arg("pool"),
        py::arg("rmax"), py::arg("part"), py::arg("cnt"), py::arg("scale"), py::arg("shift"), py::arg("mean"),
        py::arg("invstd"), py::arg("gamma"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dbias"), py::arg("dz"),
        py::arg("tmo"), py::arg("timeout_us"), py::arg("sig") = py::none(), py::arg("sig_val") = 0);
  m.def("bn_bwd_wgrad0", &bn_bwd_wgrad0, py::arg("gsrc"), py::arg("nsplit"), py::arg("g"), py::arg("z"),
        py::arg("scale"), py::arg("shift"), py::arg("mean"), py::arg("invstd"), py::arg("gamma"), py::arg("part"),
        py::arg("coef"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dbias"), py::arg("x"), py::arg("wpart"),
        py::arg("dw"), py::arg("sig") = py::none(), py::arg("sig_val") = 0);
  m.def("gap", &gap);
  m.def("gemm_f32", &gemm_f32, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("trans_a") = false,
        py::arg("trans_b") = false, py::arg("bias") = py::none(), py::arg("splits") = 1, py::arg("slab") = py::none());
  m.def("softmax_ce", &softmax_ce, py::arg("logits"), py::arg("target"), py::arg("loss_row"),
        py::arg("dlogits") = py::none(), py::arg("correct_row") = py::none(), py::arg("loss") = py::none(),
        py::arg("acc") = py::none());
  m.def("head_bwd_prep", &head_bwd_prep);
  m.def("gap_bwd", &gap_bwd);
  m.def("conv0_fwd", &conv0_fwd, py::arg("x"), py::arg("w"), py::arg("z"), py::arg("part") = py::none(),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(), py::arg("bias") = py::none(),
        py::arg("rmean") = py::none(), py::arg("rvar") = py::none(), py::arg("nbt") = py::none(),
        py::arg("mean") = py::none(), py::arg("invstd") = py::none(), py::arg("scale") = py::none(),
        py::arg("shift") = py::none(), py::arg("momentum") = 0.1, py::arg("eps") = 1e-5);
  m.def("conv0_part_floats", [](int64_t N) { return dpa_conv0_part_floats((int)N); });
  m.def("wgrad0_part_floats", [](int64_t N) { return dpa_wgrad0_part_floats((int)N); });
  m.def("fc_ce_train", &fc_ce_train, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("target"), py::arg("loss_row"),
        py::arg("dlogits"), py::arg("dx"), py::arg("dw"), py::arg("db"), py::arg("loss_out"), py::arg("loss_accum"),
        py::arg("bn_z") = py::none(), py::arg("bn_scale") = py::none(), py::arg("bn_shift") = py::none(),
        py::arg("parts") = 3);
  m.def("fc_ce_eval", &fc_ce_eval);
  m.def("augment", &augment);
  m.def("maxpool_fwd", &maxpool_fwd, py::arg("x"), py::arg("y"), py::arg("arg"), py::arg("k"), py::arg("s"),
        py::arg("p"), py::arg("scale") = py::none(), py::arg("shift") = py::none());
  m.def("maxpool_bwd", &maxpool_bwd);
  // A HIP stream with an explicit priority (lower number = higher priority; HIP's range is reported
  // by stream_priority_range()).  Owned by the caller; lives until stream_destroy.
  m.def("stream_create", [](int64_t priority) {
    hipStream_t s = nullptr;
    TORCH_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, (int)priority) == hipSuccess,
                "hipStreamCreateWithPriority failed");
    return reinterpret_cast<int64_t>(s);
  });
  m.def("stream_destroy", [](int64_t s) { (void)hipStreamDestroy(reinterpret_cast<hipStream_t>(s)); });
  m.def("stream_priority_range", []() {
    int least = 0, greatest = 0;
    TORCH_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess, "hipDeviceGetStreamPriorityRange");
    return std::make_pair(least, greatest);
  });
  py::class_<DevEvent>(m, "DevEvent")
      .def(py::init<int64_t>(), py::arg("flags"))
      .def("record", &DevEvent::record, py::arg("stream"))
      .def("wait", &DevEvent::wait, py::arg("stream"))
      .def("synchronize", &DevEvent::synchronize)
      .def("query", &DevEvent::query);
  m.attr("EVENT_DISABLE_TIMING") = (int64_t)hipEventDisableTiming;
  m.attr("EVENT_RELEASE_TO_DEVICE") = (int64_t)hipEventReleaseToDevice;
  m.attr("EVENT_DISABLE_SYSTEM_FENCE") = (int64_t)hipEventDisableSystemFence;
  m.def("rccl_unique_id", []() { return py::bytes(dpa::RcclComm::unique_id()); });
  m.def("rccl_version", &dpa::RcclComm::version);
  // native rendezvous store (bootstrap without torch.distributed); blocking calls release the GIL
  py::class_<dpa::TcpStoreServer>(m, "TcpStoreServer")
      .def(py::init<const std::string&, int>(), py::arg("host"), py::arg("port"))
      .def_property_readonly("port", &dpa::TcpStoreServer::port);
  py::class_<dpa::TcpStoreClient>(m, "TcpStoreClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"), py::arg("timeout_s") = 600.0,
           py::call_guard<py::gil_scoped_release>())
      .def("set", [](dpa::TcpStoreClient& c, const std::string& k, py::bytes v) {
        std::string sv(v);
        py::gil_scoped_release nogil;
        c.set(k, sv);
      })
      .def("get", [](dpa::TcpStoreClient& c, const std::string& k, double timeout_s) {
        std::string v;
        {
          py::gil_scoped_release nogil;
          v = c.get(k, timeout_s);
        }
        return py::bytes(v);
      }, py::arg("key"), py::arg("timeout_s") = -1.0)
      .def("add", &dpa::TcpStoreClient::add, py::call_guard<py::gil_scoped_release>())
      .def("delete", &dpa::TcpStoreClient::del, py::call_guard<py::gil_scoped_release>())
      .def("num_keys", &dpa::TcpStoreClient::num_keys, py::call_guard<py::gil_scoped_release>())
      .def("wait", &dpa::TcpStoreClient::wait, py::arg("keys"), py::arg("timeout_s") = -1.0,
           py::call_guard<py::gil_scoped_release>())
      .def("barrier", &dpa::TcpStoreClient::barrier, py::call_guard<py::gil_scoped_release>());
  py::class_<PyIpcComm>(m, "IpcComm")
      .def(py::init<int, int, int, int64_t, int64_t>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("stage_words"), py::arg("inbox_words"))
      .def("sig_handle", &PyIpcComm::sig_handle)
      .def("tmo_ptr", &PyIpcComm::tmo_ptr)
      .def("stage_handle", &PyIpcComm::stage_handle)
      .def("inbox_handle", &PyIpcComm::inbox_handle)
      .def_static("tensor_handle", &PyIpcComm::tensor_handle)
      .def("set_peers", &PyIpcComm::set_peers)
      .def("add_region", &PyIpcComm::add_region)
      .def("all_reduce", &PyIpcComm::all_reduce)
      .def("broadcast", &PyIpcComm::broadcast)
      .def("gather", &PyIpcComm::gather)
      .def("reduce_scatter", &PyIpcComm::reduce_scatter)
      .def("all_gather", &PyIpcComm::all_gather)
      .def("barrier", &PyIpcComm::barrier)
      .def("take_timeout", &PyIpcComm::take_timeout, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("launches", &PyIpcComm::launches)
      .def_property_readonly("rank", &PyIpcComm::rank)
      .def_property_readonly("world", &PyIpcComm::world);
  m.def("ipc_slice", [](int64_t n, int world) { return (int64_t)dpa_ipc_slice((long)n, world); });
  m.def("ipc_pieces", [](int op, int64_t n, int world, int64_t stage_words, int64_t inbox_words, bool registered) {
    std::vector<std::pair<int64_t, int64_t>> out;
    for (const auto& p : dpa::IpcComm::pieces(op, (long)n, world, (long)stage_words, (long)inbox_words, registered))
      out.emplace_back(p.first, p.second);
    return out;
  }, py::arg("op"), py::arg("n"), py::arg("world"), py::arg("stage_words"), py::arg("inbox_words"),
     py::arg("registered"));
  py::class_<PyRcclComm>(m, "RcclComm")
      .def(py::init<int, int, py::bytes, int, bool, double, double, bool, bool, bool, int>(), py::arg("rank"),
           py::arg("world"), py::arg("uid"), py::arg("device"), py::arg("high_priority") = false,
           py::arg("timeout_s") = 600.0, py::arg("poll_s") = 0.2, py::arg("watchdog") = true,
           py::arg("exit_on_error") = true, py::arg("debug_sync") = false, py::arg("max_ctas") = 0)
      .def_property_readonly("max_ctas", &PyRcclComm::max_ctas)
      .def("outstanding", &PyRcclComm::outstanding)
      .def("ops_issued", &PyRcclComm::ops_issued)
      .def("comm_count", &PyRcclComm::comm_count)
      .def("all_reduce", &PyRcclComm::all_reduce, py::arg("t"), py::arg("op") = "sum")
      .def("all_reduce_here", &PyRcclComm::all_reduce_here, py::arg("t"), py::arg("op") = "sum")
      .def("broadcast", &PyRcclComm::broadcast)
      .def("gather", &PyRcclComm::gather)
      .def("reduce_scatter", &PyRcclComm::reduce_scatter, py::arg("send"), py::arg("recv"), py::arg("op") = "sum")
      .def("all_gather", &PyRcclComm::all_gather)
      .def("send", &PyRcclComm::send)
      .def("recv", &PyRcclComm::recv)
      .def("wait", &PyRcclComm::wait)
      .def("synchronize", &PyRcclComm::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &PyRcclComm::async_error)
      .def("abort", &PyRcclComm::abort)
      .def("stream_ptr", &PyRcclComm::stream_ptr)
      .def_property_readonly("rank", &PyRcclComm::rank)
      .def_property_readonly("world", &PyRcclComm::world);
}
