// K10: streaming training / evaluation metrics on the device (gfx950 / MI355X).
//
// Keras compiles the model with metrics ['accuracy', AUC(name='auc')] (cnn_baseline_train.py:100-102):
// binary accuracy at 0.5 and the 200-threshold ROC AUC, both accumulated over the epoch.  One
// launch per batch adds the batch into device-resident int64 counters -- no host synchronisation
// inside the epoch; the host reads the counters once at epoch end (training/metrics.py).
//
//   counts[0]                 #(pred > 0.5) == (y > 0.5)
//   counts[1 .. nb]           positives per bucket, bucket = #thresholds strictly below pred
//   counts[1 + nb .. 2 nb]    negatives per bucket                      (nb = n_thr + 1)
//
// The bucket is a lower_bound over the fp32 threshold table staged in LDS, so it equals
// torch.bucketize(p, thr) bit for bit; per-block LDS histograms are flushed with one 64-bit
// atomic per non-empty bin.
#include "common.h"

namespace apneauq {
namespace metrics {

constexpr int kMaxThr = 1024;

__global__ __launch_bounds__(256) void update_kernel(const float* p, const float* y, long long n, const float* thr,
                                                     int n_thr, unsigned long long* counts) {
  __shared__ float t[kMaxThr];
  __shared__ unsigned int hist[2 * (kMaxThr + 1)];
  __shared__ unsigned int correct;
  const int nb = n_thr + 1;
  for (int i = threadIdx.x; i < n_thr; i += 256) t[i] = thr[i];
  for (int i = threadIdx.x; i < 2 * nb; i += 256) hist[i] = 0u;
  if (threadIdx.x == 0) correct = 0u;
  __syncthreads();
  unsigned int mine = 0u;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float pi = p[i];
    const bool pos = y[i] > 0.5f;
    mine += ((pi > 0.5f) == pos) ? 1u : 0u;
    int lo = 0, hi = n_thr;  // first index with t[idx] >= pi
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (t[mid] < pi)
        lo = mid + 1;
      else
        hi = mid;
    }
    atomicAdd(&hist[(pos ? 0 : nb) + lo], 1u);
  }
  mine = (unsigned int)wave_sum((float)mine);  // <= 64 * per-thread count: exact in fp32 below 2^24
  if ((threadIdx.x & 63) == 0) atomicAdd(&correct, mine);
  __syncthreads();
  if (threadIdx.x == 0 && correct) atomicAdd(counts, (unsigned long long)correct);
  for (int i = threadIdx.x; i < 2 * nb; i += 256)
    if (hist[i]) atomicAdd(counts + 1 + i, (unsigned long long)hist[i]);
}

}  // namespace metrics

hipError_t launch_metrics_update(const float* p, const float* y, long long n, const float* thr, int n_thr,
                                 unsigned long long* counts, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  long long g = (n + 255) / 256;
  if (g > 512) g = 512;
  hipLaunchKernelGGL(metrics::update_kernel, dim3((unsigned)g), dim3(256), 0, stream, p, y, n, thr, n_thr, counts);
  return hipGetLastError();
}

}  // namespace apneauq
