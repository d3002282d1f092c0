// On-device uncertainty metrics and bootstrap confidence intervals (gfx950).
//
// uq_reduce  replaces the NumPy/SciPy per-window math of uq_techniques.py:62-91 (mean, ddof=0
//            variance, H(E[p]) and E[H(p)] in nats with the SciPy clip to [1e-10, 1-1e-10],
//            MI = max(H - E[H], 0)) plus the per-window CSV columns of
//            analyze_mcd_patient_level.py:107-117 (entropy in BITS with log2(p + 1e-9), label p>0.5).
//            One thread per window, one pass over the T (or M) samples, fp32 like the reference.
// bootstrap  replaces uq_techniques.py:137-157, which re-runs the whole metric computation for
//            each of B resamples.  The per-window metrics do not change under resampling, so every
//            replicate is a gather + masked mean; one workgroup per replicate, fp64 accumulation.
#include "common.h"

namespace apneauq {

// metric rows written by uq_reduce (out[k * n + i])
enum UqRow { kMean = 0, kVar, kEntNats, kExpEnt, kMI, kEntBits, kLabel, kUqRows };

__device__ __forceinline__ float bin_entropy_nats(float p) {
  // scipy.stats.entropy([1-p, p]) after np.clip(., 1e-10, 1-1e-10) in float32 (the upper bound
  // rounds to 1.0f), including SciPy's renormalisation by the sum.
  float q = 1.0f - p;
  p = fminf(fmaxf(p, 1e-10f), 1.0f);
  q = fminf(fmaxf(q, 1e-10f), 1.0f);
  const float s = p + q;
  p = p / s;
  q = q / s;
  return -(p * __logf(p) + q * __logf(q));
}

__global__ __launch_bounds__(256) void uq_reduce_kernel(const float* __restrict__ probs, int t_count, int n,
                                                         float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f, eh = 0.f;
  for (int t = 0; t < t_count; ++t) {
    const float p = probs[(long long)t * n + i];
    s += p;
    eh += bin_entropy_nats(p);
  }
  const float mean = s / (float)t_count;
  float v = 0.f;
  for (int t = 0; t < t_count; ++t) {
    const float d = probs[(long long)t * n + i] - mean;
    v += d * d;
  }
  const float var = v / (float)t_count;
  const float h = bin_entropy_nats(mean);
  const float e = eh / (float)t_count;
  const float bits = -(mean * log2f(mean + 1e-9f) + (1.0f - mean) * log2f(1.0f - mean + 1e-9f));
  out[kMean * (long long)n + i] = mean;
  out[kVar * (long long)n + i] = var;
  out[kEntNats * (long long)n + i] = h;
  out[kExpEnt * (long long)n + i] = e;
  out[kMI * (long long)n + i] = fmaxf(h - e, 0.f);
  out[kEntBits * (long long)n + i] = bits;
  out[kLabel * (long long)n + i] = mean > 0.5f ? 1.f : 0.f;
}

// Bootstrap: replicate b draws n indices (host-supplied parity indices, or device counter hash).
// Output per replicate: overall_mean_variance, mean_variance_class_0, mean_variance_class_1,
// mean_total_pred_entropy, mean_expected_aleatoric_entropy, mean_mutual_info.
constexpr int kBootThreads = 512;

// PARTIAL (sharded windows): this rank holds the metrics of global windows [lo, lo + n_loc);
// every draw is enumerated, only those landing in the shard are summed, and the 8 raw sums per
// replicate go out for an all-reduce (ops/uq.py bootstrap_partial) instead of the 6 means.  What the
// sharding divides is the window data (metric rows, memory, the per-window metric pass); the B x n draw
// enumeration (index reads or hashes, ~1 integer op per draw) is replicated on every rank.
template <bool PARTIAL>
__global__ __launch_bounds__(kBootThreads) void bootstrap_kernel(const float* __restrict__ metrics, const int* __restrict__ y,
                                                                 const int* __restrict__ idx, unsigned seed, int n,
                                                                 int lo, int n_loc, double* __restrict__ out) {
  const int b = blockIdx.x;
  APNEAUQ_DASSERT(blockDim.x == kBootThreads && n > 0);
  const int ld = PARTIAL ? n_loc : n;  // leading dimension of the metric rows
  const float* var = metrics + kVar * (long long)ld;
  const float* ent = metrics + kEntNats * (long long)ld;
  const float* eent = metrics + kExpEnt * (long long)ld;
  const float* mi = metrics + kMI * (long long)ld;
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};  // sum var, sum var|0, cnt0, sum var|1, cnt1, sum H, sum EH  (+MI below)
  double smi = 0.0;
  const unsigned bkey = mix32(seed ^ mix32((unsigned)b * 0x9E3779B9u + 0x7F4A7C15u));
  for (int j = threadIdx.x; j < n; j += kBootThreads) {
    int k;
    if (idx) {
      k = idx[(long long)b * n + j];
    } else {
      const unsigned hsh = mix32(bkey ^ mix32((unsigned)j));
      k = (int)(((unsigned long long)hsh * (unsigned long long)n) >> 32);
    }
    if constexpr (PARTIAL) {
      k -= lo;
      if (k < 0 || k >= n_loc) continue;
    }
    const float v = var[k];
    const int yy = y[k];
    acc[0] += v;
    if (yy == 0) { acc[1] += v; acc[2] += 1.0; }
    if (yy == 1) { acc[3] += v; acc[4] += 1.0; }
    acc[5] += ent[k];
    acc[6] += eent[k];
    smi += mi[k];
  }
  __shared__ double red[8][kBootThreads / kWave];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double vals[8] = {acc[0], acc[1], acc[2], acc[3], acc[4], acc[5], acc[6], smi};
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    double x = vals[q];
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, kWave);
    if (lane == 0) red[q][wave] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[8];
    for (int q = 0; q < 8; ++q) {
      t[q] = 0.0;
      for (int w = 0; w < kBootThreads / kWave; ++w) t[q] += red[q][w];
    }
    if constexpr (PARTIAL) {
      for (int q = 0; q < 8; ++q) out[b * 8 + q] = t[q];
      return;
    }
    out[b * 6 + 0] = t[0] / n;
    out[b * 6 + 1] = t[2] > 0 ? t[1] / t[2] : 0.0;
    out[b * 6 + 2] = t[4] > 0 ? t[3] / t[4] : 0.0;
    out[b * 6 + 3] = t[5] / n;
    out[b * 6 + 4] = t[6] / n;
    out[b * 6 + 5] = t[7] / n;
  }
}

hipError_t launch_uq_reduce(const float* probs, int t_count, int n, float* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(uq_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, probs, t_count, n, out);
  return hipGetLastError();
}

hipError_t launch_bootstrap(const float* metrics, const int* y, const int* idx, unsigned seed, int n, int n_boot,
                            double* out, hipStream_t stream) {
  if (n_boot <= 0) return hipSuccess;
  hipLaunchKernelGGL(bootstrap_kernel<false>, dim3(n_boot), dim3(kBootThreads), 0, stream, metrics, y, idx, seed, n, 0, n,
                     out);
  return hipGetLastError();
}

hipError_t launch_bootstrap_partial(const float* metrics, const int* y, const int* idx, unsigned seed, int n, int lo,
                                    int n_loc, int n_boot, double* out, hipStream_t stream) {
  if (n_boot <= 0) return hipSuccess;
  hipLaunchKernelGGL(bootstrap_kernel<true>, dim3(n_boot), dim3(kBootThreads), 0, stream, metrics, y, idx, seed, n, lo,
                     n_loc, out);
  return hipGetLastError();
}

}  // namespace apneauq
