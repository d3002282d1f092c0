// torch.library registration of the apneauq HIP kernels (namespace torch.ops.apneauq).
// Compiled as plain host C++; every kernel lives in a .hip translation unit built for gfx950.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime_api.h>

#include <vector>

namespace apneauq {
hipError_t launch_fused_forward(const void* x, const uint8_t* blob, long long blob_stride, float* out, int n_win,
                                int n_pass, int n_member, unsigned window_offset, unsigned pass_offset,
                                unsigned long long seed, int dropout, int out_logits, const unsigned* thr,
                                const float* dscale, int grid, hipStream_t stream);
int fused_blob_bytes();
int fused_lds_bytes();
void fused_layout(int* woffs, int* eoffs, int* dense_off);
hipError_t launch_uq_reduce(const float* probs, int t_count, int n, float* out, hipStream_t stream);
hipError_t launch_bootstrap(const float* metrics, const int* y, const int* idx, unsigned seed, int n, int n_boot,
                            double* out, hipStream_t stream);
hipError_t launch_adam(float* p, const float* g, float* m, float* v, long long n, float b1, float b2, float alpha,
                       float eps, float gscale, hipStream_t stream);
}  // namespace apneauq

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

at::Tensor fused_forward(const at::Tensor& x, const at::Tensor& blob, int64_t n_pass, int64_t window_offset,
                         int64_t pass_offset, int64_t seed, bool dropout, bool out_logits, at::IntArrayRef thr,
                         at::ArrayRef<double> dscale, int64_t grid) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda(), "fused_forward: tensors must be on the GPU");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "fused_forward: x must be contiguous bf16");
  TORCH_CHECK(x.dim() == 3 && x.size(1) == 60 && x.size(2) == 4, "fused_forward: x must be (N, 60, 4), got ",
              x.sizes());
  TORCH_CHECK(blob.scalar_type() == at::kByte && blob.dim() == 2 && blob.is_contiguous(),
              "fused_forward: blob must be contiguous uint8 (members, bytes)");
  TORCH_CHECK(blob.size(1) == apneauq::fused_blob_bytes(), "fused_forward: blob has ", blob.size(1),
              " bytes per member, kernel expects ", apneauq::fused_blob_bytes());
  TORCH_CHECK(thr.size() == 6 && dscale.size() == 6, "fused_forward: need 6 dropout thresholds/scales");
  TORCH_CHECK(n_pass >= 1, "fused_forward: n_pass >= 1");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(blob.data_ptr()) % 16 == 0,
              "fused_forward: 16-B alignment required");
  const int64_t n_win = x.size(0), n_member = blob.size(0);
  TORCH_CHECK(n_pass * n_win < (int64_t(1) << 31), "fused_forward: too many samples for one launch");
  const at::DeviceGuard guard(x.device());
  auto out = at::empty({n_member, n_pass, n_win}, x.options().dtype(at::kFloat));
  if (n_win == 0) return out;
  unsigned t[6];
  float d[6];
  for (int i = 0; i < 6; ++i) {
    t[i] = static_cast<unsigned>(thr[i]);
    d[i] = static_cast<float>(dscale[i]);
  }
  check(apneauq::launch_fused_forward(x.data_ptr(), blob.data_ptr<uint8_t>(),
                                      blob.stride(0), out.data_ptr<float>(), (int)n_win, (int)n_pass, (int)n_member,
                                      (unsigned)window_offset, (unsigned)pass_offset, (unsigned long long)seed,
                                      dropout ? 1 : 0, out_logits ? 1 : 0, t, d, (int)grid, cur_stream()),
        "fused_forward");
  return out;
}

at::Tensor uq_reduce(const at::Tensor& probs) {
  TORCH_CHECK(probs.is_cuda() && probs.scalar_type() == at::kFloat && probs.dim() == 2,
              "uq_reduce: probs must be a (T, N) float32 GPU tensor");
  auto p = probs.contiguous();
  const at::DeviceGuard guard(p.device());
  auto out = at::empty({7, p.size(1)}, p.options());
  check(apneauq::launch_uq_reduce(p.data_ptr<float>(), (int)p.size(0), (int)p.size(1), out.data_ptr<float>(),
                                  cur_stream()),
        "uq_reduce");
  return out;
}

at::Tensor bootstrap(const at::Tensor& metrics, const at::Tensor& y, const c10::optional<at::Tensor>& idx,
                     int64_t seed, int64_t n_boot) {
  TORCH_CHECK(metrics.is_cuda() && metrics.scalar_type() == at::kFloat && metrics.dim() == 2 && metrics.size(0) == 7,
              "bootstrap: metrics must be the (7, N) output of uq_reduce");
  const int64_t n = metrics.size(1);
  auto m = metrics.contiguous();
  auto yy = y.to(at::kInt).contiguous();
  TORCH_CHECK(yy.is_cuda() && yy.numel() == n, "bootstrap: y must be (N,) on the GPU");
  const int* ip = nullptr;
  at::Tensor ii;
  if (idx.has_value()) {
    ii = idx->to(at::kInt).contiguous();
    TORCH_CHECK(ii.is_cuda() && ii.dim() == 2 && ii.size(0) == n_boot && ii.size(1) == n,
                "bootstrap: idx must be (B, N) on the GPU");
    ip = ii.data_ptr<int>();
  }
  const at::DeviceGuard guard(m.device());
  auto out = at::empty({n_boot, 6}, m.options().dtype(at::kDouble));
  check(apneauq::launch_bootstrap(m.data_ptr<float>(), yy.data_ptr<int>(), ip, (unsigned)seed, (int)n, (int)n_boot,
                                  out.data_ptr<double>(), cur_stream()),
        "bootstrap");
  return out;
}

void adam_step(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v, double b1, double b2, double alpha,
               double eps, double gscale) {
  TORCH_CHECK(p.is_cuda() && g.is_cuda() && m.is_cuda() && v.is_cuda(), "adam_step: GPU tensors required");
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&p, &g, &m, &v})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == p.numel() &&
                    reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "adam_step: contiguous, 16-B aligned fp32 tensors of equal size required");
  const at::DeviceGuard guard(p.device());
  check(apneauq::launch_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                             p.numel(), (float)b1, (float)b2, (float)alpha, (float)eps, (float)gscale, cur_stream()),
        "adam_step");
}

std::vector<int64_t> fused_layout() {
  int w[6], e[6], d;
  apneauq::fused_layout(w, e, &d);
  std::vector<int64_t> v;
  for (int i = 0; i < 6; ++i) v.push_back(w[i]);
  for (int i = 0; i < 6; ++i) v.push_back(e[i]);
  v.push_back(d);
  v.push_back(apneauq::fused_blob_bytes());
  v.push_back(apneauq::fused_lds_bytes());
  return v;
}

}  // namespace

TORCH_LIBRARY(apneauq, m) {
  m.def("fused_forward(Tensor x, Tensor blob, int n_pass, int window_offset, int pass_offset, int seed, "
        "bool dropout, bool out_logits, int[] thr, float[] dscale, int grid) -> Tensor");
  m.def("uq_reduce(Tensor probs) -> Tensor");
  m.def("bootstrap(Tensor metrics, Tensor y, Tensor? idx, int seed, int n_boot) -> Tensor");
  m.def("fused_layout() -> int[]", &fused_layout);
  m.def("adam_step(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, float b1, float b2, float alpha, float eps, "
        "float gscale) -> ()");
}

TORCH_LIBRARY_IMPL(apneauq, CUDA, m) {
  m.impl("fused_forward", &fused_forward);
  m.impl("uq_reduce", &uq_reduce);
  m.impl("bootstrap", &bootstrap);
  m.impl("adam_step", &adam_step);
}
