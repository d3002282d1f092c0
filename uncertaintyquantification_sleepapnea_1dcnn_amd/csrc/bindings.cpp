// torch.library registration of the apneauq HIP kernels (namespace torch.ops.apneauq).
// Compiled as plain host C++; every kernel lives in a .hip translation unit built for gfx950.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime_api.h>

#include <cstring>
#include <vector>

namespace apneauq {
hipError_t launch_fused_forward(const void* x, const uint8_t* blob, long long blob_stride, float* out, int n_win,
                                int n_pass, int n_member, unsigned window_offset, unsigned pass_offset,
                                unsigned long long seed, int dropout, int out_logits, const unsigned* thr,
                                const float* dscale, int grid, hipStream_t stream);
int fused_blob_bytes();
int fused_lds_bytes();
hipError_t launch_fused_tiled(int net, const void* x, const uint8_t* blob, long long blob_stride, float* out,
                              int n_win, int n_pass, int n_member, unsigned window_offset, unsigned pass_offset,
                              unsigned long long seed, int dropout, int out_logits, const unsigned* thr,
                              hipStream_t stream);
int fused_pooled_lds_bytes();
void fused_layout(int* woffs, int* eoffs, int* dense_off);
hipError_t launch_fused_tiled_x3(int net, const float* x, const uint8_t* blob, long long blob_stride, float* out,
                                 int n_win, int n_pass, int n_member, unsigned window_offset, unsigned pass_offset,
                                 unsigned long long seed, int dropout, int out_logits, const unsigned* thr,
                                 hipStream_t stream);
void fused_layout_x3(int* woffs, int* eoffs, int* dense_off, int* bytes, int* lds);
hipError_t launch_uq_reduce(const float* probs, int t_count, int n, float* out, hipStream_t stream);
hipError_t launch_bootstrap(const float* metrics, const int* y, const int* idx, unsigned seed, int n, int n_boot,
                            double* out, hipStream_t stream);
hipError_t launch_bootstrap_partial(const float* metrics, const int* y, const int* idx, unsigned seed, int n, int lo,
                                    int n_loc, int n_boot, double* out, hipStream_t stream);
int zero_max_buffers();
hipError_t launch_zero(int nb, void* const* ptrs, const long long* words, hipStream_t stream);
int adam_max_sets();
hipError_t launch_adam_multi(int ns, float* const* p, const float* const* g, float* const* m, float* const* v,
                             const int* const* step, long long n, float b1, float b2, float alpha, float eps,
                             hipStream_t stream);
hipError_t launch_adam(float* p, const float* g, float* m, float* v, long long n, float b1, float b2, float alpha,
                       float eps, float gscale, const int* step_dev, hipStream_t stream);
hipError_t train_bump_counters(int* c, int n, hipStream_t st);
hipError_t train_stream_keys(unsigned* keys, const int* c, int n, unsigned long long seed, unsigned pass_base,
                             hipStream_t st);
hipError_t launch_generic_conv(const void* x, const void* wfrag, const float* epi, void* y, int n, int L, int cin,
                               int cout, int cout_pad, int ksize, int pool, int dropout, unsigned thr, int layer,
                               int n_win, unsigned pass_offset, unsigned window_offset, unsigned long long seed,
                               hipStream_t stream, int mode, int in_rs, int in_off, float* stats, long long x_rows,
                               int det_slots);
hipError_t launch_gt_bn_finalize(const float* st, int nslots, int C, float inv_count, const float* gamma,
                                 const float* beta, float eps, float momentum, float* mmean, float* mvar, int update,
                                 float* bn, hipStream_t stream);
hipError_t launch_gt_apply(const void* z, const float* bn, void* out, int n, int L, int C, int pool, int out_rs,
                           int out_off, int dropout, unsigned thr, float inv_keep, unsigned skey,
                           unsigned window_offset, hipStream_t stream, const unsigned* skey_dev, int f32);
hipError_t launch_gt_bwd(int dz_mode, const void* z, const float* bn, const void* dh, const float* dlog,
                         const float* w, float invL, int n, int L, int C, int pool, int dropout, unsigned thr,
                         float inv_keep, unsigned skey, unsigned window_offset, float* bst, const float* coef,
                         const float* gamma, void* dz, int dz_rs, int dz_off, float* gbias, hipStream_t stream,
                         const unsigned* skey_dev, int det_slots, int f32);
hipError_t launch_gt_bwd_finalize(const float* bst, int nslots, int C, float inv_count, float* coef, float* ggamma,
                                  float* gbeta, const float* dbs, int bslots, int BC, float* gbias,
                                  hipStream_t stream);
hipError_t launch_metrics_update(const float* p, const float* y, long long n, const float* thr, int n_thr,
                                 unsigned long long* counts, hipStream_t stream);
hipError_t launch_generic_head(const void* y, const float* w, float b, int n, int L, int C, int out_logits, float* out,
                               hipStream_t stream);
hipError_t launch_gt_wgrad(const void* x, long long x_rows, const void* dz, long long R, int cin, int cout, int k,
                           float* gw, hipStream_t st, float* part, long long part_floats);
hipError_t launch_gt_head(const void* h, const float* w, const float* b, const float* y, float* prob, float* dlog,
                          float* loss, float* gw, float* gb, int n, int L, int C, float inv_gb, hipStream_t st,
                          float* part, long long part_floats, int f32);
hipError_t launch_gf32_conv(const float* x, const float* w, const float* bias, float* y, float* stats, int n, int L,
                            int cin, int cout, int ksize, int mode, int in_rs, int in_off, int flip, int det_slots,
                            hipStream_t st);
hipError_t launch_gf32_wgrad(const float* x, const float* dz, long long R, int cin, int cout, int k, float* gw,
                             float* part, long long part_floats, hipStream_t st);
int gt_pack_max_blocks();
int gx3_max_blocks();
hipError_t launch_gx3_pack(int nb, const float* const* w, void* const* fwd, void* const* dgr, float* const* wsc,
                           const int* k, const int* cin, const int* cout, float* wpart, hipStream_t st);
hipError_t launch_gx3_amax(const float* x, long long n, unsigned* out, hipStream_t st);
hipError_t launch_gx3_conv(const float* x, long long x_rows, const void* wfrag, const float* wsc, const float* bias,
                           float* y, float* stats, unsigned* amax_out, int n, int L, int cin, int cout, int ksize,
                           int mode, int in_rs, int in_off, int det_slots, hipStream_t st);
hipError_t launch_gx3_wgrad(const float* x, const float* dz, const unsigned* amax_x, const unsigned* amax_dz,
                            long long R, int cin, int cout, int k, float* gw, float* part, long long part_floats,
                            hipStream_t st);
long long train_wgrad_part_floats(int B);
int train_det_floats(int B);
hipError_t launch_gt_pack(int nb, const float* const* w, void* const* fwd, void* const* dgr, const int* k,
                          const int* cin, const int* cout, hipStream_t st, int nz, void* const* zp,
                          const long long* zw);
int gt_pack_max_zero();
int train_tail_max();
hipError_t launch_train_tail(int* counters, int ncounters, int members, const float* const* logits,
                             float* const* probs, int n, hipStream_t stream);
hipError_t launch_train_inputs(int members, const float* const* x, void* const* xd, const float* const* y,
                               float* const* yd, int n, int L, int C, int SR, hipStream_t stream);
namespace train {
struct Layer {
  const void* wf; const void* wd; const float* bias; const float* gamma; const float* beta;
  float* mmean; float* mvar; float* gw; float* gb; float* ggamma; float* gbeta;
  void* R; void* dY; void* dZ; double* st; double* bst; unsigned thr; float dsc;
};
struct Args {
  Layer L[6];
  const void* x; const float* y; const float* dense_w; const float* dense_b; float* g_dense_w; float* g_dense_b;
  float* logits; float* dlogit; float* loss_sum;
  int B; int n_win; int groups; unsigned pass_base; unsigned window_offset; unsigned long long seed; int dropout;
  float inv_count; float inv_batch; float eps; float momentum; const unsigned* pass_dev; int st_groups; float* wpart; float* det; int shared0; float* tab; float* hpart;
  int bwd_self;
};
}  // namespace train
int train_args_size();
hipError_t launch_standardize(const double* x, double* out, long long n_win, int L, int C, double eps, hipStream_t stream);
hipError_t launch_knn(const double* X, int n, int D, long long* out, int k, hipStream_t stream);
int knn_lds_bytes(int D, int K);
int train_layer_size();
hipError_t train_launch_fwd(const train::Args& A, int l, hipStream_t st);
hipError_t train_launch_head(const train::Args& A, int backward, hipStream_t st, bool with_tab);
hipError_t train_launch_dgrad(const train::Args& A, int l, hipStream_t st, bool fused);
hipError_t train_launch_wgrad(const train::Args& A, int l, hipStream_t st, bool fused);
hipError_t train_launch_finalize(const train::Args& A, int update_moving, int grads, hipStream_t st, bool fused);
hipError_t train_launch_tab(const apneauq::train::Args& A, int mode, int l, hipStream_t st);
hipError_t train_launch_mb(const train::Args& A0, const train::Args* Am, int M, int op, int layer, int flag,
                           hipStream_t st);
}  // namespace apneauq

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

// net -1: fused_forward.hip (the reference no-pool CNN); 0 / 1: fused_tiled.hip (MaxPool1D(2) after
// blocks 1-5 / the (30, 1) single-channel window).  Same parameter blob.
at::Tensor fused_forward_impl(const at::Tensor& x, const at::Tensor& blob, int64_t n_pass, int64_t window_offset,
                              int64_t pass_offset, int64_t seed, bool dropout, bool out_logits, at::IntArrayRef thr,
                              at::ArrayRef<double> dscale, int64_t grid, int net) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda(), "fused_forward: tensors must be on the GPU");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "fused_forward: x must be contiguous bf16");
  const int64_t want_l = net == 1 ? 30 : 60, want_c = net == 1 ? 1 : 4;
  TORCH_CHECK(x.dim() == 3 && x.size(1) == want_l && x.size(2) == want_c, "fused_forward: x must be (N, ", want_l,
              ", ", want_c, "), got ", x.sizes());
  TORCH_CHECK(blob.scalar_type() == at::kByte && blob.dim() == 2 && blob.is_contiguous(),
              "fused_forward: blob must be contiguous uint8 (members, bytes)");
  TORCH_CHECK(blob.size(1) == apneauq::fused_blob_bytes(), "fused_forward: blob has ", blob.size(1),
              " bytes per member, kernel expects ", apneauq::fused_blob_bytes());
  TORCH_CHECK(thr.size() == 6 && dscale.size() == 6, "fused_forward: need 6 dropout thresholds/scales");
  TORCH_CHECK(n_pass >= 1, "fused_forward: n_pass >= 1");
  // x: 16-B vector loads except for the single-channel net (element loads into its im2col rows)
  TORCH_CHECK((net == 1 || reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0) &&
                  reinterpret_cast<uintptr_t>(blob.data_ptr()) % 16 == 0,
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
  if (net >= 0)
    check(apneauq::launch_fused_tiled(net, x.data_ptr(), blob.data_ptr<uint8_t>(), blob.stride(0),
                                      out.data_ptr<float>(), (int)n_win, (int)n_pass, (int)n_member,
                                      (unsigned)window_offset, (unsigned)pass_offset, (unsigned long long)seed,
                                      dropout ? 1 : 0, out_logits ? 1 : 0, t, cur_stream()),
          "fused_tiled_forward");
  else
    check(apneauq::launch_fused_forward(x.data_ptr(), blob.data_ptr<uint8_t>(), blob.stride(0), out.data_ptr<float>(),
                                        (int)n_win, (int)n_pass, (int)n_member, (unsigned)window_offset,
                                        (unsigned)pass_offset, (unsigned long long)seed, dropout ? 1 : 0,
                                        out_logits ? 1 : 0, t, d, (int)grid, cur_stream()),
          "fused_forward");
  return out;
}

at::Tensor fused_forward(const at::Tensor& x, const at::Tensor& blob, int64_t n_pass, int64_t window_offset,
                         int64_t pass_offset, int64_t seed, bool dropout, bool out_logits, at::IntArrayRef thr,
                         at::ArrayRef<double> dscale, int64_t grid) {
  return fused_forward_impl(x, blob, n_pass, window_offset, pass_offset, seed, dropout, out_logits, thr, dscale, grid,
                            -1);
}

at::Tensor fused_pooled_forward(const at::Tensor& x, const at::Tensor& blob, int64_t n_pass, int64_t window_offset,
                                int64_t pass_offset, int64_t seed, bool dropout, bool out_logits, at::IntArrayRef thr,
                                at::ArrayRef<double> dscale) {
  return fused_forward_impl(x, blob, n_pass, window_offset, pass_offset, seed, dropout, out_logits, thr, dscale, 0, 0);
}

at::Tensor fused_single_forward(const at::Tensor& x, const at::Tensor& blob, int64_t n_pass, int64_t window_offset,
                                int64_t pass_offset, int64_t seed, bool dropout, bool out_logits, at::IntArrayRef thr,
                                at::ArrayRef<double> dscale) {
  return fused_forward_impl(x, blob, n_pass, window_offset, pass_offset, seed, dropout, out_logits, thr, dscale, 0, 1);
}

// fp32-faithful fused inference of the pooled (net 0) / single-channel 30 s (net 1) CNN
// (csrc/fused_tiled_x3.hip): fp32 x, fp16x3 blob (ops/fused.py:pack_blob_x3)
at::Tensor fused_tiled_x3_forward(const at::Tensor& x, const at::Tensor& blob, int64_t net, int64_t n_pass,
                                  int64_t window_offset, int64_t pass_offset, int64_t seed, bool dropout,
                                  bool out_logits, at::IntArrayRef thr) {
  TORCH_CHECK(net == 0 || net == 1, "fused_tiled_x3: net 0 (pooled) or 1 (single-channel)");
  TORCH_CHECK(x.is_cuda() && blob.is_cuda(), "fused_tiled_x3: tensors must be on the GPU");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous(), "fused_tiled_x3: x must be contiguous fp32");
  const int64_t want_l = net == 1 ? 30 : 60, want_c = net == 1 ? 1 : 4;
  TORCH_CHECK(x.dim() == 3 && x.size(1) == want_l && x.size(2) == want_c, "fused_tiled_x3: x must be (N, ", want_l,
              ", ", want_c, "), got ", x.sizes());
  int w[6], e[6], d, nbytes, lds;
  apneauq::fused_layout_x3(w, e, &d, &nbytes, &lds);
  TORCH_CHECK(blob.scalar_type() == at::kByte && blob.dim() == 2 && blob.is_contiguous() && blob.size(1) == nbytes,
              "fused_tiled_x3: blob must be contiguous uint8 (members, ", nbytes, ")");
  TORCH_CHECK(thr.size() == 6, "fused_tiled_x3: need 6 dropout thresholds");
  TORCH_CHECK(n_pass >= 1, "fused_tiled_x3: n_pass >= 1");
  // x: 16-B row loads except for the single-channel net (element loads into its im2col rows)
  TORCH_CHECK((net == 1 || reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0) &&
                  reinterpret_cast<uintptr_t>(blob.data_ptr()) % 16 == 0,
              "fused_tiled_x3: 16-B alignment required");
  const int64_t n_win = x.size(0), n_member = blob.size(0);
  TORCH_CHECK(n_pass * n_win < (int64_t(1) << 31), "fused_tiled_x3: too many samples for one launch");
  const at::DeviceGuard guard(x.device());
  auto out = at::empty({n_member, n_pass, n_win}, x.options());
  if (n_win == 0) return out;
  unsigned t[6];
  for (int i = 0; i < 6; ++i) t[i] = static_cast<unsigned>(thr[i]);
  check(apneauq::launch_fused_tiled_x3((int)net, x.data_ptr<float>(), blob.data_ptr<uint8_t>(), blob.stride(0),
                                       out.data_ptr<float>(), (int)n_win, (int)n_pass, (int)n_member,
                                       (unsigned)window_offset, (unsigned)pass_offset, (unsigned long long)seed,
                                       dropout ? 1 : 0, out_logits ? 1 : 0, t, cur_stream()),
        "fused_tiled_x3");
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

// Sharded bootstrap: raw (B, 8) sums over the draws landing in this rank's windows
// [lo, lo + n_loc) of n_global; summed over ranks by the caller, then turned into the 6 means.
at::Tensor bootstrap_partial(const at::Tensor& metrics, const at::Tensor& y, const c10::optional<at::Tensor>& idx,
                             int64_t seed, int64_t n_boot, int64_t n_global, int64_t lo) {
  TORCH_CHECK(metrics.is_cuda() && metrics.scalar_type() == at::kFloat && metrics.dim() == 2 && metrics.size(0) == 7,
              "bootstrap_partial: metrics must be the (7, n_loc) output of uq_reduce");
  const int64_t n_loc = metrics.size(1);
  TORCH_CHECK(lo >= 0 && lo + n_loc <= n_global && n_global < (int64_t(1) << 31), "bootstrap_partial: bad shard");
  auto m = metrics.contiguous();
  auto yy = y.to(at::kInt).contiguous();
  TORCH_CHECK(yy.is_cuda() && yy.numel() == n_loc, "bootstrap_partial: y must be (n_loc,) on the GPU");
  const int* ip = nullptr;
  at::Tensor ii;
  if (idx.has_value()) {
    ii = idx->to(at::kInt).contiguous();
    TORCH_CHECK(ii.is_cuda() && ii.dim() == 2 && ii.size(0) == n_boot && ii.size(1) == n_global,
                "bootstrap_partial: idx must be (B, n_global) on the GPU");
    ip = ii.data_ptr<int>();
  }
  const at::DeviceGuard guard(m.device());
  auto out = at::empty({n_boot, 8}, m.options().dtype(at::kDouble));
  check(apneauq::launch_bootstrap_partial(m.data_ptr<float>(), yy.data_ptr<int>(), ip, (unsigned)seed, (int)n_global,
                                          (int)lo, (int)n_loc, (int)n_boot, out.data_ptr<double>(), cur_stream()),
        "bootstrap_partial");
  return out;
}

void adam_step(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v, double b1, double b2, double alpha,
               double eps, double gscale, const c10::optional<at::Tensor>& counters) {
  TORCH_CHECK(p.is_cuda() && g.is_cuda() && m.is_cuda() && v.is_cuda(), "adam_step: GPU tensors required");
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&p, &g, &m, &v})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == p.numel() &&
                    reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "adam_step: contiguous, 16-B aligned fp32 tensors of equal size required");
  const at::DeviceGuard guard(p.device());
  const int* step_dev = nullptr;
  if (counters.has_value()) {  // [pass offset, iterations]: alpha = lr, corrected on the device
    TORCH_CHECK(counters->is_cuda() && counters->scalar_type() == at::kInt && counters->numel() >= 2,
                "adam_step: counters must be an int32 GPU tensor [pass, iterations]");
    step_dev = counters->data_ptr<int>() + 1;
  }
  check(apneauq::launch_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                             p.numel(), (float)b1, (float)b2, (float)alpha, (float)eps, (float)gscale, step_dev,
                             cur_stream()),
        "adam_step");
}

// Adam over M members' flat buffers in one launch (same size and hyper-parameters; per-member device
// iteration counters [pass, iterations] as in adam_step).
void adam_step_multi(at::TensorList p, at::TensorList g, at::TensorList m, at::TensorList v, double b1, double b2,
                     double alpha, double eps, at::TensorList counters) {
  const int ns = (int)p.size();
  TORCH_CHECK(ns >= 1 && ns <= apneauq::adam_max_sets() && (int)g.size() == ns && (int)m.size() == ns &&
                  (int)v.size() == ns && (int)counters.size() == ns,
              "adam_step_multi: 1..", apneauq::adam_max_sets(), " equally long lists");
  std::vector<float*> pp(ns), mm(ns), vv(ns);
  std::vector<const float*> gg(ns);
  std::vector<const int*> st(ns);
  const int64_t n = p[0].numel();
  for (int i = 0; i < ns; ++i) {
    for (const at::Tensor* t : {&p[i], &g[i], &m[i], &v[i]})
      TORCH_CHECK(t->is_cuda() && t->device() == p[0].device() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                      t->numel() == n && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                  "adam_step_multi: contiguous, 16-B aligned fp32 GPU tensors of equal size on one device required");
    TORCH_CHECK(counters[i].is_cuda() && counters[i].scalar_type() == at::kInt && counters[i].numel() >= 2,
                "adam_step_multi: counters must be int32 GPU tensors [pass, iterations]");
    pp[i] = p[i].data_ptr<float>();
    gg[i] = g[i].data_ptr<float>();
    mm[i] = m[i].data_ptr<float>();
    vv[i] = v[i].data_ptr<float>();
    st[i] = counters[i].data_ptr<int>() + 1;
  }
  const at::DeviceGuard guard(p[0].device());
  check(apneauq::launch_adam_multi(ns, pp.data(), gg.data(), mm.data(), vv.data(), st.data(), n, (float)b1, (float)b2,
                                   (float)alpha, (float)eps, cur_stream()),
        "adam_step_multi");
}

// Zero several GPU buffers (4-byte multiples) in one launch.
void zero_buffers(at::TensorList ts) {
  const int nb = (int)ts.size();
  TORCH_CHECK(nb >= 1 && nb <= apneauq::zero_max_buffers(), "zero_buffers: 1..", apneauq::zero_max_buffers(), " tensors");
  std::vector<void*> p(nb);
  std::vector<long long> w(nb);
  for (int i = 0; i < nb; ++i) {
    TORCH_CHECK(ts[i].is_cuda() && ts[i].is_contiguous() && ts[i].device() == ts[0].device() &&
                    (ts[i].numel() * ts[i].element_size()) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(ts[i].data_ptr()) % 4 == 0,
                "zero_buffers: contiguous GPU tensors of whole 4-byte words on one device required");
    p[i] = ts[i].data_ptr();
    w[i] = (long long)(ts[i].numel() * ts[i].element_size() / 4);
  }
  const at::DeviceGuard guard(ts[0].device());
  check(apneauq::launch_zero(nb, p.data(), w.data(), cur_stream()), "zero_buffers");
}

void bump_counters(at::Tensor& counters) {
  TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == at::kInt && counters.numel() <= 64,
              "bump_counters: int32 GPU tensor of <= 64 counters");
  const at::DeviceGuard guard(counters.device());
  check(apneauq::train_bump_counters(counters.data_ptr<int>(), (int)counters.numel(), cur_stream()), "bump_counters");
}

void stream_keys(at::Tensor& keys, const at::Tensor& counters, int64_t seed, int64_t pass_base) {
  TORCH_CHECK(keys.is_cuda() && keys.scalar_type() == at::kInt && keys.is_contiguous() && keys.numel() <= 64,
              "stream_keys: contiguous int32 GPU tensor of <= 64 keys");
  TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == at::kInt && counters.numel() >= 1 &&
                  counters.device() == keys.device(), "stream_keys: int32 GPU counters on the keys' device");
  const at::DeviceGuard guard(keys.device());
  check(apneauq::train_stream_keys(reinterpret_cast<unsigned*>(keys.data_ptr<int>()), counters.data_ptr<int>(),
                                   (int)keys.numel(), static_cast<unsigned long long>(seed),
                                   static_cast<unsigned>(pass_base), cur_stream()),
        "stream_keys");
}

// ctx: int64 CPU tensor of device pointers / scalars built once per workspace (ops/train_ops.py)
constexpr int kCtxLayer = 18, kCtxLen = 6 * kCtxLayer + 27;

float bits_to_float(int64_t v) {
  uint32_t u = static_cast<uint32_t>(v);
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

apneauq::train::Args args_from_ctx(const at::Tensor& ctx, int64_t pass_base) {
  TORCH_CHECK(apneauq::train_args_size() == (int)sizeof(apneauq::train::Args) &&
                  apneauq::train_layer_size() == (int)sizeof(apneauq::train::Layer),
              "train Args ABI mismatch between bindings and kernels");
  TORCH_CHECK(ctx.device().is_cpu() && ctx.scalar_type() == at::kLong && ctx.numel() == kCtxLen,
              "train ctx must be an int64 CPU tensor of length ", kCtxLen);
  const int64_t* c = ctx.data_ptr<int64_t>();
  apneauq::train::Args A;
  for (int l = 0; l < 6; ++l) {
    const int64_t* q = c + l * kCtxLayer;
    auto& L = A.L[l];
    L.wf = reinterpret_cast<const void*>(q[0]);
    L.wd = reinterpret_cast<const void*>(q[1]);
    L.bias = reinterpret_cast<const float*>(q[2]);
    L.gamma = reinterpret_cast<const float*>(q[3]);
    L.beta = reinterpret_cast<const float*>(q[4]);
    L.mmean = reinterpret_cast<float*>(q[5]);
    L.mvar = reinterpret_cast<float*>(q[6]);
    L.gw = reinterpret_cast<float*>(q[7]);
    L.gb = reinterpret_cast<float*>(q[8]);
    L.ggamma = reinterpret_cast<float*>(q[9]);
    L.gbeta = reinterpret_cast<float*>(q[10]);
    L.R = reinterpret_cast<void*>(q[11]);
    L.dY = reinterpret_cast<void*>(q[12]);
    L.st = reinterpret_cast<double*>(q[13]);
    L.bst = reinterpret_cast<double*>(q[14]);
    L.thr = static_cast<unsigned>(q[15]);
    L.dsc = bits_to_float(q[16]);
    L.dZ = reinterpret_cast<void*>(q[17]);
  }
  const int64_t* g = c + 6 * kCtxLayer;
  A.x = reinterpret_cast<const void*>(g[0]);
  A.y = reinterpret_cast<const float*>(g[1]);
  A.dense_w = reinterpret_cast<const float*>(g[2]);
  A.dense_b = reinterpret_cast<const float*>(g[3]);
  A.g_dense_w = reinterpret_cast<float*>(g[4]);
  A.g_dense_b = reinterpret_cast<float*>(g[5]);
  A.logits = reinterpret_cast<float*>(g[6]);
  A.dlogit = reinterpret_cast<float*>(g[7]);
  A.loss_sum = reinterpret_cast<float*>(g[8]);
  A.B = static_cast<int>(g[9]);
  A.n_win = static_cast<int>(g[10]);
  A.groups = static_cast<int>(g[11]);
  A.pass_base = static_cast<unsigned>(pass_base >= 0 ? pass_base : g[12]);
  A.window_offset = static_cast<unsigned>(g[13]);
  A.seed = static_cast<unsigned long long>(g[14]);
  A.dropout = static_cast<int>(g[15]);
  A.inv_count = bits_to_float(g[16]);
  A.inv_batch = bits_to_float(g[17]);
  A.eps = bits_to_float(g[18]);
  A.momentum = bits_to_float(g[19]);
  A.pass_dev = reinterpret_cast<const unsigned*>(g[20]);
  A.st_groups = static_cast<int>(g[21]);
  A.shared0 = static_cast<int>(g[22]);
  A.wpart = reinterpret_cast<float*>(g[23]);
  A.det = reinterpret_cast<float*>(g[24]);
  A.tab = reinterpret_cast<float*>(g[25]);
  A.hpart = reinterpret_cast<float*>(g[26]);
  A.bwd_self = 0;
  TORCH_CHECK(A.hpart == nullptr || A.det == nullptr, "train ctx: head slots are for the atomic mode");
  TORCH_CHECK(A.tab == nullptr || (A.det == nullptr && A.groups == 1 && A.wpart != nullptr),
              "train ctx: the parameter table needs one stats group, no deterministic partials and wgrad partials "
              "(wgrad_reduce writes its backward rows)");
  TORCH_CHECK(A.st_groups >= A.groups, "train ctx: moment buffers hold fewer groups than requested");
  return A;
}

// op: 0 fwd(layer; flag=1: the pass-shared block 1 of batch-BN MC Dropout, over the n_win windows)
//     | 1 head(flag bit 0 = backward, bit 1 = + the table's forward rows, replacing op 5) | 2 dgrad(layer) | 3 wgrad(layer) | 4 finalize(layer=update_moving, flag=grads)
//     (2 / 3: flag bit 0 = Args::bwd_self, the backward BN rows from the slots instead of the table; bit 1 =
//     the fused single-device step: wgrad launches no reduce, dgrad<l> reduces wgrad<l+1>'s partials, and
//     finalize (flag bit 1, bit 0 = grads) those of wgrad<1> / wgrad<0>)
//     | 5 parameter table (flag 0: forward rows of every block, 1: backward rows of block ``layer``)
void train_call(const at::Tensor& ctx, int64_t op, int64_t layer, int64_t flag, int64_t pass_base, int64_t device) {
  const at::DeviceGuard guard(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device)));
  auto A = args_from_ctx(ctx, pass_base);
  TORCH_CHECK(A.B > 0 && A.n_win > 0 && A.groups > 0, "train_call: bad sizes");
  hipStream_t s = cur_stream();
  switch (op) {
    case 0:
      TORCH_CHECK(layer >= 0 && layer < 6);
      if (flag == 1) {
        TORCH_CHECK(layer == 0 && A.shared0, "train fwd: flag 1 = shared block 1 (layer 0, shared0 ctx)");
        A.B = A.n_win;  // one copy per window; stats group 0 (the buffers keep the ctx's group stride)
      }
      check(apneauq::train_launch_fwd(A, (int)layer, s), "train fwd");
      break;
    case 1: check(apneauq::train_launch_head(A, (int)(flag & 1), s, (flag & 2) != 0), "train head"); break;
    case 2:
      TORCH_CHECK(layer >= 1 && layer < 6);
      A.bwd_self = (int)(flag & 1);
      check(apneauq::train_launch_dgrad(A, (int)layer, s, (flag & 2) != 0), "train dgrad");
      break;
    case 3:
      TORCH_CHECK(layer >= 0 && layer < 6);
      A.bwd_self = (int)(flag & 1);
      check(apneauq::train_launch_wgrad(A, (int)layer, s, (flag & 2) != 0), "train wgrad");
      break;
    case 4: check(apneauq::train_launch_finalize(A, (int)layer, (int)(flag & 1), s, (flag & 2) != 0), "train finalize"); break;
    case 5: check(apneauq::train_launch_tab(A, (int)flag, (int)layer, s), "train param table"); break;
    default: TORCH_CHECK(false, "train_call: unknown op ", op);
  }
}

// Member-batched training (train_conv.hip train_launch_mb): the Args of M members' contexts in one device
// array, validated to share every size / mode the launch geometry depends on.
at::Tensor train_args_dev(const std::vector<at::Tensor>& ctxs, int64_t device) {
  const int64_t M = (int64_t)ctxs.size();
  TORCH_CHECK(M >= 1 && M <= 65535, "train_args_dev: 1..65535 member contexts");
  std::vector<apneauq::train::Args> v;
  v.reserve(M);
  for (const auto& c : ctxs) v.push_back(args_from_ctx(c, -1));
  const auto& a = v[0];
  for (const auto& x : v) {
    TORCH_CHECK(x.B == a.B && x.n_win == a.n_win && x.groups == 1 && x.st_groups == a.st_groups && (x.det == nullptr) == (a.det == nullptr) &&
                    !x.shared0 && (x.tab == nullptr) == (a.tab == nullptr) && x.wpart != nullptr &&
                    (x.hpart == nullptr) == (a.hpart == nullptr) && x.pass_dev != nullptr,
                "train_args_dev: member contexts must share batch size, stats groups and modes (atomic or "
                "deterministic, device counters, wgrad partials)");
  }
  auto cpu = at::empty({M * (int64_t)sizeof(apneauq::train::Args)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(cpu.data_ptr(), v.data(), M * sizeof(apneauq::train::Args));
  return cpu.to(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device)));
}

void train_call_mb(const at::Tensor& args_dev, const at::Tensor& ctx0, int64_t M, int64_t op, int64_t layer, int64_t flag) {
  TORCH_CHECK(args_dev.is_cuda() && args_dev.scalar_type() == at::kByte && args_dev.is_contiguous() &&
                  args_dev.numel() == M * (int64_t)sizeof(apneauq::train::Args),
              "train_call_mb: args_dev must hold M device Args (train_args_dev)");
  const auto A0 = args_from_ctx(ctx0, -1);
  TORCH_CHECK(op >= 0 && op <= 5, "train_call_mb: unknown op ", op);
  TORCH_CHECK((op != 0 || (layer >= 0 && layer < 6)) && (op != 2 || (layer >= 1 && layer < 6)) &&
                  (op != 3 || (layer >= 0 && layer < 6)),
              "train_call_mb: bad layer");
  const at::DeviceGuard guard(args_dev.device());
  check(apneauq::train_launch_mb(A0, reinterpret_cast<const apneauq::train::Args*>(args_dev.data_ptr()), (int)M,
                                 (int)op, (int)layer, (int)flag, cur_stream()),
        "train_call_mb");
}

int64_t train_wgrad_part_size(int64_t B) { return apneauq::train_wgrad_part_floats((int)B); }
int64_t train_det_size(int64_t B) { return apneauq::train_det_floats((int)B); }


// Generic-spec conv block (csrc/generic_conv.hip): x (N, L, Cin) bf16 -> (N, L or L/2, Cout) bf16.
at::Tensor generic_conv(const at::Tensor& x, const at::Tensor& wfrag, const at::Tensor& epi, int64_t cout,
                        int64_t ksize, bool pool, bool dropout, int64_t thr, int64_t layer, int64_t n_win,
                        int64_t pass_offset, int64_t window_offset, int64_t seed) {
  TORCH_CHECK(x.is_cuda() && wfrag.is_cuda() && epi.is_cuda(), "generic_conv: tensors must be on the GPU");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 3, "generic_conv: x must be contiguous bf16 (N, L, C)");
  TORCH_CHECK(wfrag.scalar_type() == at::kBFloat16 && wfrag.is_contiguous() && wfrag.dim() == 4 && wfrag.size(2) == 64 &&
              wfrag.size(3) == 8, "generic_conv: wfrag must be (nstep, Cout_pad/16, 64, 8) bf16");
  const int64_t n = x.size(0), L = x.size(1), cin = x.size(2), cout_pad = wfrag.size(1) * 16;
  TORCH_CHECK(wfrag.size(0) == (ksize * cin + 31) / 32, "generic_conv: wfrag k-steps do not match k*Cin");
  TORCH_CHECK(cout > 0 && cout % 4 == 0 && cout <= cout_pad && cout_pad - cout < 16, "generic_conv: Cout must be a multiple of 4");
  TORCH_CHECK(cout_pad <= 1024 && L < (1 << 22), "generic_conv: dropout hash needs C <= 1024, L < 2^22");
  TORCH_CHECK(epi.scalar_type() == at::kFloat && epi.is_contiguous() && epi.numel() == 8 * cout_pad, "generic_conv: epi must be (8, Cout_pad) fp32");
  TORCH_CHECK(ksize % 2 == 1, "generic_conv: odd kernel sizes only ('same' padding)");
  TORCH_CHECK(n_win >= 1 && n % n_win == 0, "generic_conv: N must be n_pass * n_win");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "generic_conv: 16-B alignment required");
  TORCH_CHECK(n * L < (int64_t(1) << 31), "generic_conv: too many rows");
  const at::DeviceGuard guard(x.device());
  const int64_t lout = pool ? L / 2 : L;
  auto y = at::empty({n, lout, cout}, x.options());
  check(apneauq::launch_generic_conv(x.data_ptr(), wfrag.data_ptr(), epi.data_ptr<float>(), y.data_ptr(), (int)n, (int)L,
                                     (int)cin, (int)cout, (int)cout_pad, (int)ksize, pool ? 1 : 0, dropout ? 1 : 0,
                                     (unsigned)thr, (int)layer, (int)n_win, (unsigned)pass_offset, (unsigned)window_offset,
                                     (unsigned long long)seed, cur_stream(), 0, (int)L, 0, nullptr, n * L, 0),
        "generic_conv");
  return y;
}

// ---- generic-spec training (csrc/generic_train.hip); every buffer is preallocated by ops/generic_train.py ----
// activation buffers of the generic training path: bf16, or fp32 (precision="fp32"); one launch's
// activation tensors must share the dtype (need_same)
inline void need_rows(const at::Tensor& t, int64_t rows, int64_t c, const char* what) {
  TORCH_CHECK(t.is_cuda() && (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat) && t.is_contiguous(), what,
              ": bf16 or fp32 contiguous GPU tensor required");
  TORCH_CHECK(t.numel() >= rows * c, what, ": buffer too small (", t.numel(), " < ", rows * c, ")");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, what, ": 16-B alignment required");
}
inline void need_f32(const at::Tensor& t, int64_t n, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() >= n, what,
              ": fp32 contiguous GPU tensor of >= ", n, " elements required");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, what, ": 16-B alignment required");
}
constexpr int64_t kGtSlots = 16;
inline void need_same(const at::Tensor& a, const at::Tensor& b, const char* what) {
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), what, ": activation buffers must share one dtype");
}

// mode 1: y = relu(conv(x) + bias) (N, L, Cout) + BN moment slots; mode 2: y = conv(x) (dgrad).
// x row (n, t) lives at n * in_rs + in_off + t (zero-padded layouts); the conv reads rows
// in_off - pad .. in_off + L - 1 + pad of each sample, all of which must exist.
void gt_conv(const at::Tensor& x, const at::Tensor& wfrag, const c10::optional<at::Tensor>& bias, at::Tensor& y,
             const c10::optional<at::Tensor>& stats, int64_t n, int64_t L, int64_t cin, int64_t cout, int64_t ksize,
             int64_t mode, int64_t in_rs, int64_t in_off, bool det) {
  TORCH_CHECK(mode == 1 || mode == 2, "gt_conv: mode must be 1 (train) or 2 (linear)");
  TORCH_CHECK(ksize % 2 == 1 && cout % 4 == 0 && cout <= 1024 && n >= 0 && L >= 1, "gt_conv: bad shape");
  TORCH_CHECK(wfrag.is_cuda() && wfrag.scalar_type() == at::kBFloat16 && wfrag.is_contiguous() && wfrag.dim() == 4 &&
              wfrag.size(0) == (ksize * cin + 31) / 32 && wfrag.size(2) == 64 && wfrag.size(3) == 8 &&
              wfrag.size(1) * 16 >= cout && wfrag.size(1) * 16 - cout < 16, "gt_conv: wfrag shape mismatch");
  const int64_t pad = (ksize - 1) / 2;
  TORCH_CHECK(in_rs >= L && in_off >= 0, "gt_conv: bad input row layout");
  if (n > 0) need_rows(x, (n - 1) * in_rs + in_off + L, cin, "gt_conv x");
  (void)pad;  // rows outside [0, L) of a sample are masked in the kernel, never read
  need_rows(y, n * L, cout, "gt_conv y");
  const float* bp = nullptr;
  float* sp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(bias.has_value() && stats.has_value(), "gt_conv: mode 1 needs bias and stats");
    need_f32(*bias, cout, "gt_conv bias");
    need_f32(*stats, kGtSlots * 2 * cout, "gt_conv stats");
    bp = bias->data_ptr<float>();
    sp = stats->data_ptr<float>();
  }
  // deterministic mode: one plain-store slot per (workgroup, wave row); the launcher checks the count
  const int det_slots = (mode == 1 && det) ? (int)(stats->numel() / (2 * cout)) : 0;
  TORCH_CHECK(n * L < (int64_t(1) << 31), "gt_conv: too many rows");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16, "gt_conv: bf16 (fp32: gf_conv)");
  const at::DeviceGuard guard(y.device());
  check(apneauq::launch_generic_conv(x.data_ptr(), wfrag.data_ptr(), bp, y.data_ptr(), (int)n, (int)L, (int)cin,
                                     (int)cout, (int)(wfrag.size(1) * 16), (int)ksize, 0, 0, 0u, 0, 1, 0u, 0u, 0ull,
                                     cur_stream(), (int)mode, (int)in_rs, (int)in_off, sp, x.numel() / cin, det_slots),
        "gt_conv");
}

void gt_bn_finalize(const at::Tensor& st, int64_t C, double inv_count, const at::Tensor& gamma, const at::Tensor& beta,
                    double eps, double momentum, at::Tensor& mmean, at::Tensor& mvar, bool update, at::Tensor& bn) {
  need_f32(st, kGtSlots * 2 * C, "gt_bn_finalize st");
  TORCH_CHECK(gamma.is_cuda() && gamma.numel() == C && beta.numel() == C && mmean.numel() == C && mvar.numel() == C,
              "gt_bn_finalize: per-channel tensors must have C elements");
  need_f32(bn, 4 * C, "gt_bn_finalize bn");
  const at::DeviceGuard guard(bn.device());
  // every slot of the table is summed (in a fixed order): kGtSlots atomic copies or the deterministic slots
  // (large tables in 64-slot ranges whose sums overwrite the ranges' first slots: st is consumed)
  check(apneauq::launch_gt_bn_finalize(st.data_ptr<float>(), (int)(st.numel() / (2 * C)), (int)C, (float)inv_count,
                                       gamma.data_ptr<float>(),
                                       beta.data_ptr<float>(), (float)eps, (float)momentum, mmean.data_ptr<float>(),
                                       mvar.data_ptr<float>(), update ? 1 : 0, bn.data_ptr<float>(), cur_stream()),
        "gt_bn_finalize");
}

// optional device-resident dropout stream key (int32, one element): graph-replayed steps
inline const unsigned* skey_dev_ptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "skey_dev: int32 GPU tensor");
  return reinterpret_cast<const unsigned*>(t->data_ptr<int>());
}

void gt_apply(const at::Tensor& z, const at::Tensor& bn, at::Tensor& out, int64_t n, int64_t L, int64_t C, bool pool,
              int64_t out_rs, int64_t out_off, bool dropout, int64_t thr, double inv_keep, int64_t skey,
              int64_t window_offset, const c10::optional<at::Tensor>& skey_dev) {
  TORCH_CHECK(C % 4 == 0 && C <= 1024 && L >= 1, "gt_apply: bad shape");
  const unsigned* kd = skey_dev_ptr(skey_dev);
  const int64_t lout = pool ? L / 2 : L;
  need_rows(z, n * L, C, "gt_apply z");
  need_f32(bn, 4 * C, "gt_apply bn");
  TORCH_CHECK(out_rs >= lout && out_off >= 0, "gt_apply: bad output row layout");
  if (n > 0) need_rows(out, (n - 1) * out_rs + out_off + lout, C, "gt_apply out");
  need_same(z, out, "gt_apply");
  const at::DeviceGuard guard(out.device());
  check(apneauq::launch_gt_apply(z.data_ptr(), bn.data_ptr<float>(), out.data_ptr(), (int)n, (int)L, (int)C, pool ? 1 : 0,
                                 (int)out_rs, (int)out_off, dropout ? 1 : 0, (unsigned)thr, (float)inv_keep,
                                 (unsigned)skey, (unsigned)window_offset, cur_stream(), kd, z.scalar_type() == at::kFloat),
        "gt_apply");
}

// dz_mode 0: BN-backward sums into bst; 1: dz (zero-padded rows) + bias gradient.  The upstream
// gradient is dh (N, L/2 or L, C) bf16, or (head mode, dh undefined) dlog[n] * w[c] * invL.
void gt_bwd(bool dz_mode, const at::Tensor& z, const at::Tensor& bn, const c10::optional<at::Tensor>& dh,
            const c10::optional<at::Tensor>& dlog, const c10::optional<at::Tensor>& w, double invL, int64_t n, int64_t L,
            int64_t C, bool pool, bool dropout, int64_t thr, double inv_keep, int64_t skey, int64_t window_offset,
            const c10::optional<at::Tensor>& bst, const c10::optional<at::Tensor>& coef,
            const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& dz, int64_t dz_rs, int64_t dz_off,
            const c10::optional<at::Tensor>& gbias, const c10::optional<at::Tensor>& skey_dev, bool det) {
  TORCH_CHECK(C % 4 == 0 && C <= 1024 && L >= 1, "gt_bwd: bad shape");
  const int64_t lout = pool ? L / 2 : L;
  need_rows(z, n * L, C, "gt_bwd z");
  need_f32(bn, 4 * C, "gt_bwd bn");
  const void* dhp = nullptr;
  const float *dlp = nullptr, *wp = nullptr;
  if (dh.has_value()) {
    need_rows(*dh, n * lout, C, "gt_bwd dh");
    need_same(z, *dh, "gt_bwd");
    dhp = dh->data_ptr();
  } else {
    TORCH_CHECK(dlog.has_value() && w.has_value(), "gt_bwd: need dh or (dlog, w)");
    need_f32(*dlog, n, "gt_bwd dlog");
    need_f32(*w, C, "gt_bwd w");
    dlp = dlog->data_ptr<float>();
    wp = w->data_ptr<float>();
  }
  float* bp = nullptr;
  const float *cp = nullptr, *gp = nullptr;
  void* dzp = nullptr;
  float* gbp = nullptr;
  if (!dz_mode) {
    TORCH_CHECK(bst.has_value(), "gt_bwd: stats mode needs bst");
    need_f32(*bst, kGtSlots * 2 * C, "gt_bwd bst");
    bp = bst->data_ptr<float>();
  } else {
    TORCH_CHECK(coef.has_value() && gamma.has_value() && dz.has_value() && gbias.has_value(), "gt_bwd: dz mode args");
    need_f32(*coef, 2 * C, "gt_bwd coef");
    TORCH_CHECK(gamma->is_cuda() && gamma->numel() == C, "gt_bwd gamma");
    TORCH_CHECK(dz_rs >= L && dz_off >= 0, "gt_bwd: bad dz row layout");
    if (n > 0) need_rows(*dz, (n - 1) * dz_rs + dz_off + L, C, "gt_bwd dz");
    need_same(z, *dz, "gt_bwd");
    need_f32(*gbias, kGtSlots * C, "gt_bwd gbias slots");
    cp = coef->data_ptr<float>();
    gp = gamma->data_ptr<float>();
    dzp = dz->data_ptr();
    gbp = gbias->data_ptr<float>();
  }
  // deterministic mode: workgroup b writes slot b (the grid is capped to the slot count)
  const int det_slots = !det ? 0 : (int)(dz_mode ? gbias->numel() / C : bst->numel() / (2 * C));
  const at::DeviceGuard guard(z.device());
  check(apneauq::launch_gt_bwd(dz_mode ? 1 : 0, z.data_ptr(), bn.data_ptr<float>(), dhp, dlp, wp, (float)invL, (int)n,
                               (int)L, (int)C, pool ? 1 : 0, dropout ? 1 : 0, (unsigned)thr, (float)inv_keep,
                               (unsigned)skey, (unsigned)window_offset, bp, cp, gp, dzp, (int)dz_rs, (int)dz_off, gbp,
                               cur_stream(), skey_dev_ptr(skey_dev), det_slots, z.scalar_type() == at::kFloat),
        "gt_bwd");
}

// BN-backward finalize of one block (C > 0; C == 0: none) plus, as extra workgroups of the same launch,
// the bias gradient gbias (BC) = column sums of a (slots, BC) table (the block above's, done by now).
void gt_bwd_finalize(const at::Tensor& bst, int64_t C, double inv_count, at::Tensor& coef, at::Tensor& ggamma,
                     at::Tensor& gbeta, const c10::optional<at::Tensor>& dbs, const c10::optional<at::Tensor>& gbias) {
  TORCH_CHECK(C >= 0, "gt_bwd_finalize: C >= 0");
  if (C > 0) {
    need_f32(bst, kGtSlots * 2 * C, "gt_bwd_finalize bst");
    need_f32(coef, 2 * C, "gt_bwd_finalize coef");
    TORCH_CHECK(ggamma.is_cuda() && ggamma.scalar_type() == at::kFloat && ggamma.numel() == C && gbeta.numel() == C,
                "gt_bwd_finalize: grads must have C elements");
  }
  TORCH_CHECK(dbs.has_value() == gbias.has_value(), "gt_bwd_finalize: dbs and gbias go together");
  int bslots = 0, BC = 0;
  float* gbp = nullptr;
  const float* dbp = nullptr;
  if (gbias.has_value()) {
    const at::Tensor& d = *dbs;
    const at::Tensor& gbt = *gbias;
    TORCH_CHECK(d.is_cuda() && d.scalar_type() == at::kFloat && d.is_contiguous() && d.dim() == 2,
                "gt_bwd_finalize: dbs must be a contiguous (slots, C) fp32 GPU tensor");
    TORCH_CHECK(gbt.is_cuda() && gbt.scalar_type() == at::kFloat && gbt.is_contiguous() && gbt.numel() == d.size(1),
                "gt_bwd_finalize: gbias must have dbs.size(1) fp32 elements");
    bslots = (int)d.size(0);
    BC = (int)d.size(1);
    dbp = d.data_ptr<float>();
    gbp = gbt.data_ptr<float>();
  }
  const at::DeviceGuard guard(C > 0 ? coef.device() : gbias->device());
  check(apneauq::launch_gt_bwd_finalize(C > 0 ? bst.data_ptr<float>() : nullptr, C > 0 ? (int)(bst.numel() / (2 * C)) : 0,
                                        (int)C, (float)inv_count, C > 0 ? coef.data_ptr<float>() : nullptr,
                                        C > 0 ? ggamma.data_ptr<float>() : nullptr,
                                        C > 0 ? gbeta.data_ptr<float>() : nullptr, dbp, bslots, BC, gbp, cur_stream()),
        "gt_bwd_finalize");
}

// Generic wgrad (csrc/generic_wgrad.hip): gw (k, cin, cout) fp32 += sum_R x[R + tap] dz[R]; gw pre-zeroed.
// part (deterministic mode): fp32 scratch for the per-row-group partials, summed in order into gw.
void gt_wgrad(const at::Tensor& x, const at::Tensor& dz, int64_t R, int64_t cin, int64_t cout, int64_t k, at::Tensor& gw,
              const c10::optional<at::Tensor>& part) {
  need_rows(x, R + k - 1, cin, "gt_wgrad x");
  need_rows(dz, R, cout, "gt_wgrad dz");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dz.scalar_type() == at::kBFloat16, "gt_wgrad: bf16 (fp32: gf_wgrad)");
  need_f32(gw, k * cin * cout, "gt_wgrad gw");
  TORCH_CHECK(k >= 1 && k <= 15 && cin >= 1 && cout >= 1, "gt_wgrad: 1 <= k <= 15");
  const at::DeviceGuard guard(x.device());
  float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    need_f32(*part, k * cin * cout, "gt_wgrad part");
    pp = part->data_ptr<float>();
  }
  check(apneauq::launch_gt_wgrad(x.data_ptr(), x.numel() / cin, dz.data_ptr(), R, (int)cin, (int)cout, (int)k,
                                 gw.data_ptr<float>(), cur_stream(), pp, pp ? part->numel() : 0),
        "gt_wgrad");
}

// Generic head (csrc/generic_wgrad.hip): GAP + Dense + BCE + dlogit + dense grads, n samples.
void gt_head(const at::Tensor& h, const at::Tensor& w, const at::Tensor& b, const at::Tensor& y, at::Tensor& prob,
             at::Tensor& dlog, at::Tensor& loss, at::Tensor& gw, at::Tensor& gb, int64_t n, int64_t L, int64_t C,
             double inv_gb, const c10::optional<at::Tensor>& part) {
  need_rows(h, n * L, C, "gt_head h");
  need_f32(w, C, "gt_head w");
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&b, &loss, &gb}) need_f32(*t, 1, "gt_head scalar");
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&y, &prob, &dlog}) need_f32(*t, n, "gt_head per-sample");
  need_f32(gw, C, "gt_head gw");
  TORCH_CHECK(C >= 1 && C <= 4096 && L >= 1, "gt_head: bad shape");
  float* pp = nullptr;  // deterministic mode: per-workgroup records, summed in order
  if (part.has_value() && part->defined()) {
    need_f32(*part, ((n + 3) / 4) * (C + 2), "gt_head part");
    pp = part->data_ptr<float>();
  }
  const at::DeviceGuard guard(h.device());
  check(apneauq::launch_gt_head(h.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr<float>(),
                                prob.data_ptr<float>(), dlog.data_ptr<float>(), loss.data_ptr<float>(),
                                gw.data_ptr<float>(), gb.data_ptr<float>(), (int)n, (int)L, (int)C, (float)inv_gb,
                                cur_stream(), pp, pp ? part->numel() : 0, h.scalar_type() == at::kFloat),
        "gt_head");
}

// fp32 conv (csrc/gf32_conv.hip): mode 1 y = relu(conv(x) + bias) + BN moment slots (det: one slot per
// (workgroup, wave row)); mode 2 y = conv(x) with the flipped kernel (flip, dgrad).  w is the Keras kernel
// (k, Cin_k, Cout_k) read in place: forward cin = Cin_k, cout = Cout_k; dgrad cin = Cout_k, cout = Cin_k.
void gf_conv(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, at::Tensor& y,
             const c10::optional<at::Tensor>& stats, int64_t n, int64_t L, int64_t cin, int64_t cout, int64_t ksize,
             int64_t mode, int64_t in_rs, int64_t in_off, bool det) {
  TORCH_CHECK(mode == 1 || mode == 2, "gf_conv: mode must be 1 (train) or 2 (dgrad)");
  TORCH_CHECK(ksize % 2 == 1 && ksize <= 15 && cout % 4 == 0 && cin >= 1 && n >= 0 && L >= 1, "gf_conv: bad shape");
  TORCH_CHECK(x.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat, "gf_conv: fp32 activations");
  need_f32(w, ksize * cin * cout, "gf_conv w");
  TORCH_CHECK(w.dim() == 3 && w.size(0) == ksize &&
                  (mode == 1 ? (w.size(1) == cin && w.size(2) == cout) : (w.size(1) == cout && w.size(2) == cin)),
              "gf_conv: kernel shape must be (k, cin, cout) forward / (k, cout, cin) dgrad");
  TORCH_CHECK(in_rs >= L && in_off >= 0, "gf_conv: bad input row layout");
  if (n > 0) need_rows(x, (n - 1) * in_rs + in_off + L, cin, "gf_conv x");
  need_rows(y, n * L, cout, "gf_conv y");
  TORCH_CHECK(n * L < (int64_t(1) << 31), "gf_conv: too many rows");
  const float* bp = nullptr;
  float* sp = nullptr;
  int det_slots = 0;
  if (mode == 1) {
    TORCH_CHECK(bias.has_value() && stats.has_value(), "gf_conv: mode 1 needs bias and stats");
    need_f32(*bias, cout, "gf_conv bias");
    need_f32(*stats, kGtSlots * 2 * cout, "gf_conv stats");
    bp = bias->data_ptr<float>();
    sp = stats->data_ptr<float>();
    if (det) det_slots = (int)(stats->numel() / (2 * cout));
  }
  const at::DeviceGuard guard(y.device());
  check(apneauq::launch_gf32_conv(x.data_ptr<float>(), w.data_ptr<float>(), bp, y.data_ptr<float>(), sp, (int)n, (int)L,
                                  (int)cin, (int)cout, (int)ksize, (int)mode, (int)in_rs, (int)in_off, mode == 2 ? 1 : 0,
                                  det_slots, cur_stream()),
        "gf_conv");
}

// fp32 wgrad (csrc/gf32_conv.hip): gw (k, cin, cout) = sum_R x[R + tap] dz[R], row-group partials in part
// summed in a fixed order (deterministic).
void gf_wgrad(const at::Tensor& x, const at::Tensor& dz, int64_t R, int64_t cin, int64_t cout, int64_t k, at::Tensor& gw,
              at::Tensor& part) {
  TORCH_CHECK(x.scalar_type() == at::kFloat && dz.scalar_type() == at::kFloat, "gf_wgrad: fp32 activations");
  need_rows(x, R + k - 1, cin, "gf_wgrad x");
  need_rows(dz, R, cout, "gf_wgrad dz");
  need_f32(gw, k * cin * cout, "gf_wgrad gw");
  need_f32(part, k * cin * cout, "gf_wgrad part");
  TORCH_CHECK(k >= 1 && k <= 15 && cin >= 1 && cout >= 1, "gf_wgrad: 1 <= k <= 15");
  const at::DeviceGuard guard(x.device());
  check(apneauq::launch_gf32_wgrad(x.data_ptr<float>(), dz.data_ptr<float>(), R, (int)cin, (int)cout, (int)k,
                                   gw.data_ptr<float>(), part.data_ptr<float>(), part.numel(), cur_stream()),
        "gf_wgrad");
}

// All blocks' forward (+ dgrad) MFMA fragments in one launch (csrc/generic_wgrad.hip pack_kernel), and
// optionally (zero) a list of accumulators cleared by the same launch.
void gt_pack_impl(at::TensorList w, at::TensorList fwd, at::TensorList dgr, at::IntArrayRef k, at::IntArrayRef cin,
                  at::IntArrayRef cout, at::TensorList zero) {
  const int64_t nb = (int64_t)w.size();
  TORCH_CHECK(nb >= 1 && nb <= apneauq::gt_pack_max_blocks() && (int64_t)fwd.size() == nb && (int64_t)dgr.size() == nb &&
                  (int64_t)k.size() == nb && (int64_t)cin.size() == nb && (int64_t)cout.size() == nb,
              "gt_pack: inconsistent block lists");
  std::vector<const float*> wp(nb);
  std::vector<void*> fp(nb), dp(nb);
  std::vector<int> kk(nb), ci(nb), co(nb);
  for (int64_t i = 0; i < nb; ++i) {
    kk[i] = (int)k[i];
    ci[i] = (int)cin[i];
    co[i] = (int)cout[i];
    TORCH_CHECK(w[i].is_cuda() && w[i].scalar_type() == at::kFloat && w[i].is_contiguous() &&
                    w[i].numel() == k[i] * cin[i] * cout[i],
                "gt_pack: w must be contiguous fp32 (k, cin, cout)");
    const int64_t nf = ((k[i] * cin[i] + 31) / 32) * 512 * ((cout[i] + 15) / 16);
    const int64_t nd = ((k[i] * cout[i] + 31) / 32) * 512 * ((cin[i] + 15) / 16);
    TORCH_CHECK(fwd[i].scalar_type() == at::kBFloat16 && fwd[i].is_contiguous() && fwd[i].numel() == nf,
                "gt_pack: forward fragment buffer has the wrong size");
    TORCH_CHECK(dgr[i].numel() == 0 || (dgr[i].scalar_type() == at::kBFloat16 && dgr[i].is_contiguous() &&
                                        dgr[i].numel() == nd),
                "gt_pack: dgrad fragment buffer has the wrong size");
    wp[i] = w[i].data_ptr<float>();
    fp[i] = fwd[i].data_ptr();
    dp[i] = dgr[i].numel() ? dgr[i].data_ptr() : nullptr;
  }
  const int nz = (int)zero.size();
  TORCH_CHECK(nz <= apneauq::gt_pack_max_zero(), "gt_pack_zero: at most ", apneauq::gt_pack_max_zero(), " buffers");
  std::vector<void*> zp(nz);
  std::vector<long long> zw(nz);
  for (int i = 0; i < nz; ++i) {
    TORCH_CHECK(zero[i].is_cuda() && zero[i].is_contiguous() && zero[i].device() == w[0].device() &&
                    (zero[i].numel() * zero[i].element_size()) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(zero[i].data_ptr()) % 4 == 0,
                "gt_pack_zero: contiguous GPU buffers of whole 4-byte words on the weights' device required");
    zp[i] = zero[i].data_ptr();
    zw[i] = (long long)(zero[i].numel() * zero[i].element_size() / 4);
  }
  const at::DeviceGuard guard(w[0].device());
  check(apneauq::launch_gt_pack((int)nb, wp.data(), fp.data(), dp.data(), kk.data(), ci.data(), co.data(), cur_stream(),
                                nz, zp.data(), zw.data()),
        "gt_pack");
}

void gt_pack(at::TensorList w, at::TensorList fwd, at::TensorList dgr, at::IntArrayRef k, at::IntArrayRef cin,
             at::IntArrayRef cout) {
  gt_pack_impl(w, fwd, dgr, k, cin, cout, {});
}

void gt_pack_zero(at::TensorList w, at::TensorList fwd, at::TensorList dgr, at::IntArrayRef k, at::IntArrayRef cin,
                  at::IntArrayRef cout, at::TensorList zero) {
  gt_pack_impl(w, fwd, dgr, k, cin, cout, zero);
}

// The training step's tail: bump the device counters, probs = sigmoid(logits[:n]) of every member.
void train_tail(at::Tensor& counters, at::TensorList logits, at::TensorList probs) {
  const int M = (int)logits.size();
  TORCH_CHECK(M >= 1 && M <= apneauq::train_tail_max() && (int)probs.size() == M, "train_tail: 1..",
              apneauq::train_tail_max(), " members, one probs buffer each");
  TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == at::kInt && counters.is_contiguous(),
              "train_tail: contiguous int32 GPU counters");
  const int64_t n = logits[0].numel();
  std::vector<const float*> lp(M);
  std::vector<float*> pp(M);
  for (int i = 0; i < M; ++i) {
    TORCH_CHECK(logits[i].is_cuda() && logits[i].scalar_type() == at::kFloat && logits[i].is_contiguous() &&
                    logits[i].numel() == n && probs[i].scalar_type() == at::kFloat && probs[i].is_contiguous() &&
                    probs[i].numel() == n && probs[i].device() == counters.device() &&
                    logits[i].device() == counters.device(),
                "train_tail: contiguous fp32 logits / probs of one length on the counters' device");
    lp[i] = logits[i].data_ptr<float>();
    pp[i] = probs[i].data_ptr<float>();
  }
  const at::DeviceGuard guard(counters.device());
  check(apneauq::launch_train_tail(counters.data_ptr<int>(), (int)counters.numel(), M, lp.data(), pp.data(), (int)n,
                                   cur_stream()),
        "train_tail");
}

// The step's inputs of every member in one launch: x (n, L, C) fp32 into the padded-row bf16 buffer
// (rows of SR, the first n * SR * C elements of xd), y (n) fp32 into yd.
void train_inputs(at::TensorList x, at::TensorList y, at::TensorList xd, at::TensorList yd, int64_t sr) {
  const int M = (int)x.size();
  TORCH_CHECK(M >= 1 && M <= apneauq::train_tail_max() && (int)y.size() == M && (int)xd.size() == M &&
                  (int)yd.size() == M,
              "train_inputs: 1..", apneauq::train_tail_max(), " members with x, y, xd, yd each");
  const int64_t n = x[0].size(0), L = x[0].size(1), C = x[0].size(2);
  std::vector<const float*> xp(M), yp(M);
  std::vector<void*> xdp(M);
  std::vector<float*> ydp(M);
  for (int i = 0; i < M; ++i) {
    TORCH_CHECK(x[i].is_cuda() && x[i].scalar_type() == at::kFloat && x[i].is_contiguous() && x[i].dim() == 3 &&
                    x[i].size(0) == n && x[i].size(1) == L && x[i].size(2) == C,
                "train_inputs: contiguous fp32 (n, L, C) inputs of one shape");
    TORCH_CHECK(y[i].is_cuda() && y[i].scalar_type() == at::kFloat && y[i].is_contiguous() && y[i].numel() == n,
                "train_inputs: contiguous fp32 labels (n)");
    TORCH_CHECK(xd[i].scalar_type() == at::kBFloat16 && xd[i].is_contiguous() && xd[i].numel() >= n * sr * C &&
                    yd[i].scalar_type() == at::kFloat && yd[i].is_contiguous() && yd[i].numel() >= n,
                "train_inputs: destination buffers too small");
    TORCH_CHECK(x[i].device() == xd[i].device() && y[i].device() == xd[i].device() && yd[i].device() == xd[i].device(),
                "train_inputs: one device per member");
    xp[i] = x[i].data_ptr<float>();
    yp[i] = y[i].data_ptr<float>();
    xdp[i] = xd[i].data_ptr();
    ydp[i] = yd[i].data_ptr<float>();
  }
  const at::DeviceGuard guard(xd[0].device());
  check(apneauq::launch_train_inputs(M, xp.data(), xdp.data(), yp.data(), ydp.data(), (int)n, (int)L, (int)C, (int)sr,
                                     cur_stream()),
        "train_inputs");
}

// ---- fp32-faithful (fp16x3) generic conv kernels (csrc/gx3_conv.hip): the precision="fp32" path ----
// packed hi/lo fragments of nb blocks' kernels (forward; + dgrad where dgr[i] is non-empty), per-tensor
// scales wsc[i] (one fp32 each), wpart: >= 16 nb floats of scratch
void gx3_pack(at::TensorList w, at::TensorList fwd, at::TensorList dgr, at::TensorList wsc, at::IntArrayRef k,
              at::IntArrayRef cin, at::IntArrayRef cout, at::Tensor& wpart) {
  const int64_t nb = (int64_t)w.size();
  TORCH_CHECK(nb >= 1 && nb <= apneauq::gx3_max_blocks() && (int64_t)fwd.size() == nb && (int64_t)dgr.size() == nb &&
                  (int64_t)wsc.size() == nb && (int64_t)k.size() == nb && (int64_t)cin.size() == nb &&
                  (int64_t)cout.size() == nb,
              "gx3_pack: inconsistent block lists");
  need_f32(wpart, 16 * nb, "gx3_pack wpart");
  std::vector<const float*> wp(nb);
  std::vector<void*> fp(nb), dp(nb);
  std::vector<float*> sp(nb);
  std::vector<int> kk(nb), ci(nb), co(nb);
  for (int64_t i = 0; i < nb; ++i) {
    kk[i] = (int)k[i];
    ci[i] = (int)cin[i];
    co[i] = (int)cout[i];
    TORCH_CHECK(k[i] >= 1 && cin[i] >= 1 && cout[i] % 4 == 0, "gx3_pack: cout must be a multiple of 4");
    TORCH_CHECK(w[i].is_cuda() && w[i].scalar_type() == at::kFloat && w[i].is_contiguous() &&
                    w[i].numel() == k[i] * cin[i] * cout[i] && reinterpret_cast<uintptr_t>(w[i].data_ptr()) % 16 == 0,
                "gx3_pack: w must be contiguous, 16-B aligned fp32 (k, cin, cout)");
    const int64_t nf = 2 * ((k[i] * cin[i] + 31) / 32) * 512 * ((cout[i] + 15) / 16);
    const int64_t nd = 2 * ((k[i] * cout[i] + 31) / 32) * 512 * ((cin[i] + 15) / 16);
    TORCH_CHECK(fwd[i].scalar_type() == at::kHalf && fwd[i].is_contiguous() && fwd[i].numel() == nf,
                "gx3_pack: forward fragment buffer must be fp16 of the packed size");
    TORCH_CHECK(dgr[i].numel() == 0 || (dgr[i].scalar_type() == at::kHalf && dgr[i].is_contiguous() && dgr[i].numel() == nd),
                "gx3_pack: dgrad fragment buffer must be fp16 of the packed size");
    need_f32(wsc[i], 1, "gx3_pack wsc");
    wp[i] = w[i].data_ptr<float>();
    fp[i] = fwd[i].data_ptr();
    dp[i] = dgr[i].numel() ? dgr[i].data_ptr() : nullptr;
    sp[i] = const_cast<float*>(wsc[i].data_ptr<float>());
  }
  const at::DeviceGuard guard(w[0].device());
  check(apneauq::launch_gx3_pack((int)nb, wp.data(), fp.data(), dp.data(), sp.data(), kk.data(), ci.data(), co.data(),
                                 wpart.data_ptr<float>(), cur_stream()),
        "gx3_pack");
}

// amax (int32, >= 1): atomicMax of max |x| (fp32 bits) over x's first n elements
void gx3_amax(const at::Tensor& x, int64_t n, at::Tensor& amax) {
  need_f32(x, n, "gx3_amax x");
  TORCH_CHECK(amax.is_cuda() && amax.scalar_type() == at::kInt && amax.numel() >= 1, "gx3_amax: amax must be int32");
  const at::DeviceGuard guard(x.device());
  check(apneauq::launch_gx3_amax(x.data_ptr<float>(), n, reinterpret_cast<unsigned*>(amax.data_ptr<int32_t>()),
                                 cur_stream()),
        "gx3_amax");
}

// mode 1: y = relu(conv(x) + bias) + BN moment slots (det: one per (workgroup, wave row)); mode 2:
// y = conv(x) with the flipped packed kernel (dgrad; cin = the forward Cout).  wfrag: gx3_pack output of
// that orientation, wsc its scale.  The input's row layout must keep >= pad zero rows around every
// sample's data (in_off >= pad, in_rs - L >= pad): taps never reach a neighbour's rows.
// amax (int32, nullable): atomicMax of the input's max |x| (the tensor maximum, for gx3_wgrad).
void gx3_conv(const at::Tensor& x, const at::Tensor& wfrag, const at::Tensor& wsc, const c10::optional<at::Tensor>& bias,
              at::Tensor& y, const c10::optional<at::Tensor>& stats, const c10::optional<at::Tensor>& amax, int64_t n,
              int64_t L, int64_t cin, int64_t cout, int64_t ksize, int64_t mode, int64_t in_rs, int64_t in_off, bool det) {
  TORCH_CHECK(mode == 1 || mode == 2, "gx3_conv: mode must be 1 (train) or 2 (dgrad)");
  TORCH_CHECK(ksize % 2 == 1 && cout % 4 == 0 && cin >= 1 && n >= 0 && L >= 1, "gx3_conv: bad shape");
  const int64_t pad = (ksize - 1) / 2;
  TORCH_CHECK(in_off >= pad && in_rs - L >= pad, "gx3_conv: input rows need >= pad zero rows around each sample");
  TORCH_CHECK(x.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat, "gx3_conv: fp32 activations");
  need_rows(x, n > 0 ? (n - 1) * in_rs + in_off + L + pad : 0, cin, "gx3_conv x");
  need_rows(y, n * L, cout, "gx3_conv y");
  TORCH_CHECK(wfrag.is_cuda() && wfrag.scalar_type() == at::kHalf && wfrag.is_contiguous() &&
                  wfrag.numel() == 2 * ((ksize * cin + 31) / 32) * 512 * ((cout + 15) / 16),
              "gx3_conv: wfrag must be the fp16 hi/lo fragments of this orientation");
  need_f32(wsc, 1, "gx3_conv wsc");
  TORCH_CHECK(n * L < (int64_t(1) << 31), "gx3_conv: too many rows");
  const float* bp = nullptr;
  float* sp = nullptr;
  int det_slots = 0;
  if (mode == 1) {
    TORCH_CHECK(bias.has_value() && stats.has_value(), "gx3_conv: mode 1 needs bias and stats");
    need_f32(*bias, cout, "gx3_conv bias");
    need_f32(*stats, kGtSlots * 2 * cout, "gx3_conv stats");
    bp = bias->data_ptr<float>();
    sp = stats->data_ptr<float>();
    if (det) det_slots = (int)(stats->numel() / (2 * cout));
  }
  unsigned* ap = nullptr;
  if (amax.has_value()) {
    TORCH_CHECK(amax->is_cuda() && amax->scalar_type() == at::kInt && amax->numel() >= 1, "gx3_conv: amax must be int32");
    ap = reinterpret_cast<unsigned*>(amax->data_ptr<int32_t>());
  }
  const at::DeviceGuard guard(y.device());
  check(apneauq::launch_gx3_conv(x.data_ptr<float>(), x.numel() / cin, wfrag.data_ptr(), wsc.data_ptr<float>(), bp,
                                 y.data_ptr<float>(), sp, ap, (int)n, (int)L, (int)cin, (int)cout, (int)ksize, (int)mode,
                                 (int)in_rs, (int)in_off, det_slots, cur_stream()),
        "gx3_conv");
}

// gw (k, cin, cout) = sum_R x[R + tap] dz[R] on the fp16x3 MFMA, the operands prescaled by their tensor
// maxima amax_x / amax_dz (int32 fp32 bits, >= the true maxima); row-group partials in part summed in a
// fixed order (deterministic)
void gx3_wgrad(const at::Tensor& x, const at::Tensor& dz, const at::Tensor& amax_x, const at::Tensor& amax_dz, int64_t R,
               int64_t cin, int64_t cout, int64_t k, at::Tensor& gw, at::Tensor& part) {
  TORCH_CHECK(x.scalar_type() == at::kFloat && dz.scalar_type() == at::kFloat, "gx3_wgrad: fp32 activations");
  TORCH_CHECK(k >= 1 && k <= 15 && cin >= 1 && cout % 4 == 0, "gx3_wgrad: 1 <= k <= 15, cout % 4 == 0");
  need_rows(x, R + k - 1, cin, "gx3_wgrad x");
  need_rows(dz, R, cout, "gx3_wgrad dz");
  need_f32(gw, k * cin * cout, "gx3_wgrad gw");
  need_f32(part, k * cin * cout, "gx3_wgrad part");
  TORCH_CHECK(amax_x.is_cuda() && amax_x.scalar_type() == at::kInt && amax_dz.is_cuda() && amax_dz.scalar_type() == at::kInt,
              "gx3_wgrad: amax must be int32");
  const at::DeviceGuard guard(x.device());
  check(apneauq::launch_gx3_wgrad(x.data_ptr<float>(), dz.data_ptr<float>(),
                                  reinterpret_cast<const unsigned*>(amax_x.data_ptr<int32_t>()),
                                  reinterpret_cast<const unsigned*>(amax_dz.data_ptr<int32_t>()), R, (int)cin, (int)cout,
                                  (int)k, gw.data_ptr<float>(), part.data_ptr<float>(), part.numel(), cur_stream()),
        "gx3_wgrad");
}

at::Tensor generic_head(const at::Tensor& y, const at::Tensor& w, double b, bool out_logits) {
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.dim() == 3, "generic_head: y must be (N, L, C) bf16");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == y.size(2), "generic_head: w must be (C,) fp32");
  const at::DeviceGuard guard(y.device());
  auto out = at::empty({y.size(0)}, y.options().dtype(at::kFloat));
  check(apneauq::launch_generic_head(y.data_ptr(), w.data_ptr<float>(), (float)b, (int)y.size(0), (int)y.size(1), (int)y.size(2),
                                     out_logits ? 1 : 0, out.data_ptr<float>(), cur_stream()),
        "generic_head");
  return out;
}

// K10 (csrc/metrics.hip): counts (int64, 1 + 2 (n_thr + 1)) += accuracy / AUC-bucket counts of a batch.
void metrics_update(const at::Tensor& p, const at::Tensor& y, const at::Tensor& thr, at::Tensor& counts) {
  TORCH_CHECK(p.is_cuda() && y.is_cuda() && thr.is_cuda() && counts.is_cuda(), "metrics_update: GPU tensors required");
  TORCH_CHECK(p.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat && thr.scalar_type() == at::kFloat &&
              p.is_contiguous() && y.is_contiguous() && thr.is_contiguous() && p.numel() == y.numel(),
              "metrics_update: contiguous fp32 p, y of equal size and fp32 thresholds required");
  TORCH_CHECK(thr.numel() >= 1 && thr.numel() <= 1024, "metrics_update: 1..1024 thresholds");
  TORCH_CHECK(counts.scalar_type() == at::kLong && counts.is_contiguous() && counts.numel() == 1 + 2 * (thr.numel() + 1),
              "metrics_update: counts must be int64 (1 + 2 (n_thr + 1))");
  const at::DeviceGuard guard(p.device());
  check(apneauq::launch_metrics_update(p.data_ptr<float>(), y.data_ptr<float>(), p.numel(), thr.data_ptr<float>(),
                                       (int)thr.numel(), reinterpret_cast<unsigned long long*>(counts.data_ptr<int64_t>()),
                                       cur_stream()),
        "metrics_update");
}

// K14 (csrc/prep.hip): per-window z-score of an (N, L, C) float64 tensor; exact fp64 k-NN of SMOTE
at::Tensor prep_standardize(const at::Tensor& x, double eps) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kDouble && x.dim() == 3, "prep_standardize: (N, L, C) float64 GPU tensor");
  auto xc = x.contiguous();
  TORCH_CHECK(xc.size(1) * xc.size(2) * 8 <= 64 * 1024 && xc.size(2) <= 256, "prep_standardize: window too large");
  const at::DeviceGuard guard(xc.device());
  auto out = at::empty_like(xc);
  check(apneauq::launch_standardize(xc.data_ptr<double>(), out.data_ptr<double>(), xc.size(0), (int)xc.size(1),
                                    (int)xc.size(2), eps, cur_stream()),
        "prep_standardize");
  return out;
}

at::Tensor prep_knn(const at::Tensor& X, int64_t k) {
  TORCH_CHECK(X.is_cuda() && X.scalar_type() == at::kDouble && X.dim() == 2, "prep_knn: (n, D) float64 GPU tensor");
  TORCH_CHECK(k >= 1 && k <= 16, "prep_knn: 1 <= k <= 16");
  TORCH_CHECK(X.size(0) < (int64_t(1) << 31), "prep_knn: too many rows");
  auto xc = X.contiguous();
  TORCH_CHECK(apneauq::knn_lds_bytes((int)xc.size(1), k <= 8 ? 8 : 16) <= 160 * 1024, "prep_knn: rows too wide for LDS");
  const at::DeviceGuard guard(xc.device());
  auto out = at::empty({xc.size(0), k}, xc.options().dtype(at::kLong));
  check(apneauq::launch_knn(xc.data_ptr<double>(), (int)xc.size(0), (int)xc.size(1),
                            reinterpret_cast<long long*>(out.data_ptr<int64_t>()), (int)k, cur_stream()),
        "prep_knn");
  return out;
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
  v.push_back(apneauq::fused_pooled_lds_bytes());
  return v;
}

// [woff x6, eoff x6, dense, bytes, lds(pooled), lds(single)] of the fp16x3 blob / kernel
std::vector<int64_t> fused_layout_x3() {
  int w[6], e[6], d, nbytes, lds[2];
  apneauq::fused_layout_x3(w, e, &d, &nbytes, lds);
  std::vector<int64_t> v(w, w + 6);
  v.insert(v.end(), e, e + 6);
  v.push_back(d);
  v.push_back(nbytes);
  v.push_back(lds[0]);
  v.push_back(lds[1]);
  return v;
}

}  // namespace

TORCH_LIBRARY(apneauq, m) {
  m.def("fused_forward(Tensor x, Tensor blob, int n_pass, int window_offset, int pass_offset, int seed, "
        "bool dropout, bool out_logits, int[] thr, float[] dscale, int grid) -> Tensor");
  m.def("fused_pooled_forward(Tensor x, Tensor blob, int n_pass, int window_offset, int pass_offset, int seed, "
        "bool dropout, bool out_logits, int[] thr, float[] dscale) -> Tensor");
  m.def("fused_single_forward(Tensor x, Tensor blob, int n_pass, int window_offset, int pass_offset, int seed, "
        "bool dropout, bool out_logits, int[] thr, float[] dscale) -> Tensor");
  m.def("uq_reduce(Tensor probs) -> Tensor");
  m.def("bootstrap(Tensor metrics, Tensor y, Tensor? idx, int seed, int n_boot) -> Tensor");
  m.def("bootstrap_partial(Tensor metrics, Tensor y, Tensor? idx, int seed, int n_boot, int n_global, int lo) -> Tensor");
  m.def("fused_layout() -> int[]", &fused_layout);
  m.def("fused_layout_x3() -> int[]", &fused_layout_x3);
  m.def("fused_tiled_x3_forward(Tensor x, Tensor blob, int net, int n_pass, int window_offset, int pass_offset, "
        "int seed, bool dropout, bool out_logits, int[] thr) -> Tensor");
  m.def("train_call(Tensor ctx, int op, int layer, int flag, int pass_base, int device) -> ()", &train_call);
  m.def("train_args_dev(Tensor[] ctxs, int device) -> Tensor", &train_args_dev);
  m.def("train_call_mb(Tensor args_dev, Tensor ctx0, int M, int op, int layer, int flag) -> ()", &train_call_mb);
  m.def("train_wgrad_part_size(int B) -> int", &train_wgrad_part_size);
  m.def("train_det_size(int B) -> int", &train_det_size);
  m.def("prep_standardize(Tensor x, float eps) -> Tensor");
  m.def("prep_knn(Tensor X, int k) -> Tensor");
  m.def("adam_step(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, float b1, float b2, float alpha, float eps, "
        "float gscale, Tensor? counters=None) -> ()");
  m.def("adam_step_multi(Tensor(a!)[] p, Tensor[] g, Tensor(b!)[] m, Tensor(c!)[] v, float b1, float b2, float alpha, "
        "float eps, Tensor[] counters) -> ()");
  m.def("bump_counters(Tensor(a!) counters) -> ()");
  m.def("stream_keys(Tensor(a!) keys, Tensor counters, int seed, int pass_base) -> ()");
  m.def("zero_buffers(Tensor(a!)[] ts) -> ()");
  m.def("generic_conv(Tensor x, Tensor wfrag, Tensor epi, int cout, int ksize, bool pool, bool dropout, int thr, "
        "int layer, int n_win, int pass_offset, int window_offset, int seed) -> Tensor");
  m.def("generic_head(Tensor y, Tensor w, float b, bool logits) -> Tensor");
  m.def("metrics_update(Tensor p, Tensor y, Tensor thr, Tensor(a!) counts) -> ()");
  m.def("gt_conv(Tensor x, Tensor wfrag, Tensor? bias, Tensor(a!) y, Tensor(b!)? stats, int n, int L, int cin, "
        "int cout, int ksize, int mode, int in_rs, int in_off, bool det=False) -> ()");
  m.def("gt_bn_finalize(Tensor st, int C, float inv_count, Tensor gamma, Tensor beta, float eps, float momentum, "
        "Tensor(a!) mmean, Tensor(b!) mvar, bool update, Tensor(c!) bn) -> ()");
  m.def("gt_apply(Tensor z, Tensor bn, Tensor(a!) out, int n, int L, int C, bool pool, int out_rs, int out_off, "
        "bool dropout, int thr, float inv_keep, int skey, int window_offset, Tensor? skey_dev=None) -> ()");
  m.def("gt_bwd(bool dz_mode, Tensor z, Tensor bn, Tensor? dh, Tensor? dlog, Tensor? w, float invL, int n, int L, "
        "int C, bool pool, bool dropout, int thr, float inv_keep, int skey, int window_offset, Tensor(a!)? bst, "
        "Tensor? coef, Tensor? gamma, Tensor(b!)? dz, int dz_rs, int dz_off, Tensor(c!)? gbias, Tensor? skey_dev=None, "
        "bool det=False) -> ()");
  m.def("gt_bwd_finalize(Tensor bst, int C, float inv_count, Tensor(a!) coef, Tensor(b!) ggamma, Tensor(c!) gbeta, Tensor? dbs=None, Tensor(d!)? gbias=None) -> ()");
  m.def("gt_wgrad(Tensor x, Tensor dz, int R, int cin, int cout, int k, Tensor(a!) gw, Tensor(b!)? part=None) -> ()");
  m.def("gt_head(Tensor h, Tensor w, Tensor b, Tensor y, Tensor(a!) prob, Tensor(b!) dlog, Tensor(c!) loss, "
        "Tensor(d!) gw, Tensor(e!) gb, int n, int L, int C, float inv_gb, Tensor(f!)? part=None) -> ()");
  m.def("gt_pack(Tensor[] w, Tensor(a!)[] fwd, Tensor(b!)[] dgr, int[] k, int[] cin, int[] cout) -> ()");
  m.def("gt_pack_zero(Tensor[] w, Tensor(a!)[] fwd, Tensor(b!)[] dgr, int[] k, int[] cin, int[] cout, "
        "Tensor(c!)[] zero) -> ()");
  m.def("train_tail(Tensor(a!) counters, Tensor[] logits, Tensor(b!)[] probs) -> ()");
  m.def("train_inputs(Tensor[] x, Tensor[] y, Tensor(a!)[] xd, Tensor(b!)[] yd, int sr) -> ()");
  m.def("gf_conv(Tensor x, Tensor w, Tensor? bias, Tensor(a!) y, Tensor(b!)? stats, int n, int L, int cin, int cout, "
        "int ksize, int mode, int in_rs, int in_off, bool det=False) -> ()");
  m.def("gf_wgrad(Tensor x, Tensor dz, int R, int cin, int cout, int k, Tensor(a!) gw, Tensor(b!) part) -> ()");
  m.def("gx3_pack(Tensor[] w, Tensor(a!)[] fwd, Tensor(b!)[] dgr, Tensor(c!)[] wsc, int[] k, int[] cin, int[] cout, "
        "Tensor(d!) wpart) -> ()");
  m.def("gx3_amax(Tensor x, int n, Tensor(a!) amax) -> ()");
  m.def("gx3_conv(Tensor x, Tensor wfrag, Tensor wsc, Tensor? bias, Tensor(a!) y, Tensor(b!)? stats, Tensor(c!)? amax, "
        "int n, int L, int cin, int cout, int ksize, int mode, int in_rs, int in_off, bool det=False) -> ()");
  m.def("gx3_wgrad(Tensor x, Tensor dz, Tensor amax_x, Tensor amax_dz, int R, int cin, int cout, int k, Tensor(a!) gw, "
        "Tensor(b!) part) -> ()");
}

TORCH_LIBRARY_IMPL(apneauq, CUDA, m) {
  m.impl("fused_forward", &fused_forward);
  m.impl("fused_pooled_forward", &fused_pooled_forward);
  m.impl("fused_single_forward", &fused_single_forward);
  m.impl("fused_tiled_x3_forward", &fused_tiled_x3_forward);
  m.impl("uq_reduce", &uq_reduce);
  m.impl("bootstrap", &bootstrap);
  m.impl("bootstrap_partial", &bootstrap_partial);
  m.impl("adam_step", &adam_step);
  m.impl("adam_step_multi", &adam_step_multi);
  m.impl("bump_counters", &bump_counters);
  m.impl("stream_keys", &stream_keys);
  m.impl("zero_buffers", &zero_buffers);
  m.impl("generic_conv", &generic_conv);
  m.impl("generic_head", &generic_head);
  m.impl("metrics_update", &metrics_update);
  m.impl("gt_conv", &gt_conv);
  m.impl("gt_bn_finalize", &gt_bn_finalize);
  m.impl("gt_apply", &gt_apply);
  m.impl("gt_bwd", &gt_bwd);
  m.impl("gt_bwd_finalize", &gt_bwd_finalize);
  m.impl("gt_wgrad", &gt_wgrad);
  m.impl("gt_head", &gt_head);
  m.impl("gt_pack", &gt_pack);
  m.impl("gt_pack_zero", &gt_pack_zero);
  m.impl("train_tail", &train_tail);
  m.impl("train_inputs", &train_inputs);
  m.impl("gf_conv", &gf_conv);
  m.impl("gf_wgrad", &gf_wgrad);
  m.impl("gx3_pack", &gx3_pack);
  m.impl("gx3_amax", &gx3_amax);
  m.impl("gx3_conv", &gx3_conv);
  m.impl("gx3_wgrad", &gx3_wgrad);
  m.impl("prep_standardize", &prep_standardize);
  m.impl("prep_knn", &prep_knn);
}
