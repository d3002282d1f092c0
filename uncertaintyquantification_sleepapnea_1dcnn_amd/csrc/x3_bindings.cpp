// torch.library registration of the fp32-faithful (fp16x3) layer-wise inference kernels
// (x3_layers.hip): torch.ops.apneauq.x3_*.  Host C++; shapes are checked here against what the
// kernels and their grids assume before anything is launched.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime_api.h>

#include "x3_args.h"

namespace apneauq {
int x3_lds_bytes(int layer);
int x3_tile_samples(int layer);
int x3_wg_per_cu(int layer);
hipError_t x3_launch_layer(int layer, const x3::LayerArgs& A, int grid, hipStream_t stream);
hipError_t x3_launch_l1(const x3::L1Args& A, hipStream_t stream);
hipError_t x3_launch_aff(const x3::AffArgs& A, hipStream_t stream);
hipError_t x3_launch_head(const x3::HeadArgs& A, hipStream_t stream);
}  // namespace apneauq

namespace {

constexpr int kCh[7] = {4, 128, 192, 224, 96, 256, 96};
constexpr int kKs[6] = {7, 5, 3, 7, 9, 9};

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
inline void check(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e)); }

inline void need(const at::Tensor& t, at::ScalarType dt, int64_t min_numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous(), what, ": contiguous GPU tensor of dtype ", dt,
              " required");
  TORCH_CHECK(t.numel() >= min_numel, what, ": ", t.numel(), " elements, need >= ", min_numel);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, what, ": 16-B alignment required");
}

int num_cus(const at::Tensor& t) {
  int n = 0;
  check(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, t.device().index()), "hipDeviceGetAttribute");
  return n > 0 ? n : 256;
}

// Block l (1..5, 0-based) of the reference architecture for samples = groups x n_win.
void x3_layer(int64_t layer, const at::Tensor& in, at::Tensor& out, const at::Tensor& wfrag, int64_t w_gstride,
              const at::Tensor& bias, const at::Tensor& wscale, int64_t p_gstride, const at::Tensor& aff_in,
              int64_t aff_gstride, const c10::optional<at::Tensor>& stats, int64_t n_win, int64_t groups,
              bool in_shared, int64_t thr_in, int64_t thr_out, int64_t seed, int64_t pass_base,
              int64_t window_offset, int64_t grid, const c10::optional<at::Tensor>& smax_in,
              const c10::optional<at::Tensor>& amax_in, const c10::optional<at::Tensor>& smax_out,
              const c10::optional<at::Tensor>& gscale_in, bool sign_in, bool sign_out) {
  TORCH_CHECK(layer >= 1 && layer <= 5, "x3_layer: layer must be 1..5 (block 2..6)");
  TORCH_CHECK(n_win >= 1 && groups >= 1, "x3_layer: empty launch");
  const int cin = kCh[layer], cout = kCh[layer + 1], ks = kKs[layer];
  const int64_t samples = n_win * groups, samples_in = in_shared ? n_win : samples;
  const int ts = apneauq::x3_tile_samples((int)layer);
  const int64_t tpg = (n_win + ts - 1) / ts;
  TORCH_CHECK(tpg * groups < (int64_t(1) << 31), "x3_layer: too many tiles");
  const int64_t wgroups = w_gstride ? groups : 1, pgroups = p_gstride ? groups : 1;
  need(in, at::kFloat, samples_in * 60 * cin, "x3_layer: in");
  need(out, at::kFloat, layer == 5 ? samples * 2 * cout : samples * 60 * cout, "x3_layer: out");
  const int64_t frag = (int64_t)(cin / 32) * ks * (cout / 16) * 128;  // 16-B fragments per weight group
  TORCH_CHECK(w_gstride == 0 || w_gstride == frag, "x3_layer: w_gstride must be 0 or ", frag);
  need(wfrag, at::kHalf, wgroups * frag * 8, "x3_layer: wfrag");
  TORCH_CHECK(p_gstride == 0 || p_gstride == cout, "x3_layer: p_gstride must be 0 or ", cout);
  need(bias, at::kFloat, pgroups * cout, "x3_layer: bias");
  need(wscale, at::kFloat, pgroups, "x3_layer: wscale");
  TORCH_CHECK(aff_gstride == 0 || aff_gstride == 2 * cin, "x3_layer: aff_gstride must be 0 or ", 2 * cin);
  need(aff_in, at::kFloat, (aff_gstride ? groups : 1) * 2 * cin, "x3_layer: aff_in");
  double* st = nullptr;
  if (stats.has_value()) {
    need(*stats, at::kDouble, groups * apneauq::x3::kStatSlots * 2 * cout, "x3_layer: stats");
    st = stats->data_ptr<double>();
  }
  TORCH_CHECK(thr_in >= 0 && thr_in <= 65536 && thr_out >= 0 && thr_out <= 65536, "x3_layer: thresholds");
  // range-safe split: per-sample maxima of the input (indexed like its rows) + the affine's channel maxima
  const bool pre = smax_in.has_value() && smax_in->defined();
  TORCH_CHECK(pre == (amax_in.has_value() && amax_in->defined()), "x3_layer: smax_in and amax_in go together");
  if (pre) {
    need(*smax_in, at::kInt, samples_in, "x3_layer: smax_in");
    need(*amax_in, at::kFloat, (aff_gstride ? groups : 1) * 2, "x3_layer: amax_in");
  }
  // or: a per-group prescale folded into aff_in (batch moments; x3_aff gscale)
  const bool gpre = gscale_in.has_value() && gscale_in->defined();
  TORCH_CHECK(!(pre && gpre), "x3_layer: per-sample and per-group prescale are exclusive");
  if (gpre) need(*gscale_in, at::kFloat, aff_gstride ? groups : 1, "x3_layer: gscale_in");
  unsigned* smo = nullptr;
  if (smax_out.has_value() && smax_out->defined()) {
    TORCH_CHECK(layer < 5, "x3_layer: block 6 feeds the fp32 head (no smax_out)");
    need(*smax_out, at::kInt, samples, "x3_layer: smax_out");
    smo = reinterpret_cast<unsigned*>(smax_out->data_ptr<int>());
  }
  const at::DeviceGuard guard(in.device());
  apneauq::x3::LayerArgs A;
  A.in = in.data_ptr<float>();
  A.out = out.data_ptr<float>();
  A.wfrag = wfrag.data_ptr();
  A.w_gstride = w_gstride;
  A.bias = bias.data_ptr<float>();
  A.wscale = wscale.data_ptr<float>();
  A.p_gstride = (int)p_gstride;
  A.aff_in = aff_in.data_ptr<float>();
  A.aff_gstride = (int)aff_gstride;
  A.stats = st;
  A.smax_in = pre ? reinterpret_cast<const unsigned*>(smax_in->data_ptr<int>()) : nullptr;
  A.amax_in = pre ? amax_in->data_ptr<float>() : nullptr;
  A.smax_out = smo;
  A.gscale_in = gpre ? gscale_in->data_ptr<float>() : nullptr;
  A.n_win = (int)n_win;
  A.groups = (int)groups;
  A.tiles_per_group = (int)tpg;
  A.total_tiles = (int)(tpg * groups);
  A.in_shared = in_shared ? 1 : 0;
  TORCH_CHECK(!(sign_in && in_shared), "x3_layer: the shared block-1 output carries no masks");
  TORCH_CHECK(!(sign_out && layer == 5), "x3_layer: block 6 reduces its masked output in place");
  A.sign_in = sign_in ? 1 : 0;
  A.sign_out = sign_out ? 1 : 0;
  A.thr_in = (unsigned)thr_in;
  A.thr_out = (unsigned)thr_out;
  A.layer = (int)layer;
  A.pass_base = (unsigned)pass_base;
  A.window_offset = (unsigned)window_offset;
  A.seed = (unsigned long long)seed;
  int g = grid > 0 ? (int)grid : num_cus(in) * apneauq::x3_wg_per_cu((int)layer);
  if (g > A.total_tiles) g = A.total_tiles;
  check(apneauq::x3_launch_layer((int)layer, A, g, cur_stream()), "x3_layer");
}

void x3_l1(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, at::Tensor& out,
           const c10::optional<at::Tensor>& stats, int64_t n_win, int64_t groups, const c10::optional<at::Tensor>& smax) {
  TORCH_CHECK(n_win >= 1 && groups >= 1, "x3_l1: empty launch");
  need(x, at::kFloat, n_win * 60 * 4, "x3_l1: x");
  need(w, at::kFloat, groups * 7 * 4 * 128, "x3_l1: w");
  need(b, at::kFloat, groups * 128, "x3_l1: b");
  need(out, at::kFloat, groups * n_win * 60 * 128, "x3_l1: out");
  double* st = nullptr;
  if (stats.has_value()) {
    need(*stats, at::kDouble, groups * apneauq::x3::kStatSlots * 2 * 128, "x3_l1: stats");
    st = stats->data_ptr<double>();
  }
  unsigned* smp = nullptr;
  if (smax.has_value() && smax->defined()) {
    need(*smax, at::kInt, groups * n_win, "x3_l1: smax");
    smp = reinterpret_cast<unsigned*>(smax->data_ptr<int>());
  }
  const int64_t bpg = (n_win + apneauq::x3::kL1Win - 1) / apneauq::x3::kL1Win;
  TORCH_CHECK(bpg * groups < (int64_t(1) << 31), "x3_l1: too many blocks");
  const at::DeviceGuard guard(x.device());
  apneauq::x3::L1Args A{x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(), out.data_ptr<float>(), st, smp,
                        (int)n_win, (int)groups, (int)bpg};
  check(apneauq::x3_launch_l1(A, cur_stream()), "x3_l1");
}

void x3_aff(const c10::optional<at::Tensor>& stats, const at::Tensor& gamma, const at::Tensor& beta, at::Tensor& mmean,
            at::Tensor& mvar, at::Tensor& aff, int64_t C, int64_t groups, int64_t p_gstride, bool update,
            int64_t repeat, double inv_count, double eps, double momentum, double dsc,
            const c10::optional<at::Tensor>& amax, const c10::optional<at::Tensor>& gscale, bool running) {
  TORCH_CHECK(C >= 1 && C <= 4096 && groups >= 1, "x3_aff: bad sizes");
  TORCH_CHECK(!(running && update), "x3_aff: running affine and the moving update are exclusive");
  TORCH_CHECK(p_gstride == 0 || p_gstride == C, "x3_aff: p_gstride must be 0 or C");
  const int64_t pg = p_gstride ? groups : 1;
  need(gamma, at::kFloat, pg * C, "x3_aff: gamma");
  need(beta, at::kFloat, pg * C, "x3_aff: beta");
  need(mmean, at::kFloat, pg * C, "x3_aff: moving_mean");
  need(mvar, at::kFloat, pg * C, "x3_aff: moving_variance");
  need(aff, at::kFloat, groups * 2 * C, "x3_aff: aff");
  const double* st = nullptr;
  if (stats.has_value()) {
    need(*stats, at::kDouble, groups * apneauq::x3::kStatSlots * 2 * C, "x3_aff: stats");
    st = stats->data_ptr<double>();
  }
  TORCH_CHECK(!update || st != nullptr, "x3_aff: the moving update needs batch moments");
  float* amp = nullptr;
  if (amax.has_value() && amax->defined()) {
    need(*amax, at::kFloat, groups * 2, "x3_aff: amax");
    amp = amax->data_ptr<float>();
  }
  float* gsp = nullptr;
  if (gscale.has_value() && gscale->defined()) {
    TORCH_CHECK(st != nullptr && amp == nullptr, "x3_aff: gscale needs batch moments and excludes amax");
    need(*gscale, at::kFloat, groups, "x3_aff: gscale");
    gsp = gscale->data_ptr<float>();
  }
  const at::DeviceGuard guard(gamma.device());
  apneauq::x3::AffArgs A{st, gamma.data_ptr<float>(), beta.data_ptr<float>(), mmean.data_ptr<float>(),
                         mvar.data_ptr<float>(), aff.data_ptr<float>(), amp, gsp, (int)C, (int)groups, (int)p_gstride,
                         update ? 1 : 0, (int)repeat, inv_count, (float)eps, (float)momentum, (float)dsc,
                         running ? 1 : 0};
  check(apneauq::x3_launch_aff(A, cur_stream()), "x3_aff");
}

void x3_head(const at::Tensor& sums, const at::Tensor& aff, int64_t aff_gstride, const at::Tensor& dw,
             const at::Tensor& db, int64_t p_gstride, at::Tensor& out, int64_t n_win, int64_t groups, bool logits) {
  const int C = kCh[6];
  const int64_t samples = n_win * groups;
  TORCH_CHECK(samples >= 1 && samples < (int64_t(1) << 31), "x3_head: bad sample count");
  TORCH_CHECK(aff_gstride == 0 || aff_gstride == 2 * C, "x3_head: aff_gstride");
  TORCH_CHECK(p_gstride == 0 || p_gstride == C, "x3_head: p_gstride");
  need(sums, at::kFloat, samples * 2 * C, "x3_head: sums");
  need(aff, at::kFloat, (aff_gstride ? groups : 1) * 2 * C, "x3_head: aff");
  need(dw, at::kFloat, (p_gstride ? groups : 1) * C, "x3_head: dense w");
  need(db, at::kFloat, p_gstride ? groups : 1, "x3_head: dense b");
  need(out, at::kFloat, samples, "x3_head: out");
  const at::DeviceGuard guard(sums.device());
  apneauq::x3::HeadArgs A{sums.data_ptr<float>(), aff.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(),
                          out.data_ptr<float>(), C, (int)n_win, (int)samples, (int)aff_gstride, (int)p_gstride,
                          logits ? 1 : 0};
  check(apneauq::x3_launch_head(A, cur_stream()), "x3_head");
}

int64_t x3_lds(int64_t layer) { return apneauq::x3_lds_bytes((int)layer); }

}  // namespace

TORCH_LIBRARY_FRAGMENT(apneauq, m) {
  m.def("x3_layer(int layer, Tensor input, Tensor(a!) out, Tensor wfrag, int w_gstride, Tensor bias, Tensor wscale, "
        "int p_gstride, Tensor aff_in, int aff_gstride, Tensor(b!)? stats, int n_win, int groups, bool in_shared, "
        "int thr_in, int thr_out, int seed, int pass_base, int window_offset, int grid, Tensor? smax_in=None, "
        "Tensor? amax_in=None, Tensor(c!)? smax_out=None, Tensor? gscale_in=None, bool sign_in=False, bool sign_out=False) -> ()");
  m.def("x3_l1(Tensor x, Tensor w, Tensor b, Tensor(a!) out, Tensor(b!)? stats, int n_win, int groups, "
        "Tensor(c!)? smax=None) -> ()");
  m.def("x3_aff(Tensor? stats, Tensor gamma, Tensor beta, Tensor(a!) mmean, Tensor(b!) mvar, Tensor(c!) aff, int C, "
        "int groups, int p_gstride, bool update, int repeat, float inv_count, float eps, float momentum, float dsc, "
        "Tensor(d!)? amax=None, Tensor(e!)? gscale=None, bool running=False) -> ()");
  m.def("x3_head(Tensor sums, Tensor aff, int aff_gstride, Tensor dw, Tensor db, int p_gstride, Tensor(a!) out, "
        "int n_win, int groups, bool logits) -> ()");
  m.def("x3_lds(int layer) -> int", &x3_lds);
}

TORCH_LIBRARY_IMPL(apneauq, CUDA, m) {
  m.impl("x3_layer", &x3_layer);
  m.impl("x3_l1", &x3_l1);
  m.impl("x3_head", &x3_head);
  m.impl("x3_aff", &x3_aff);
}
