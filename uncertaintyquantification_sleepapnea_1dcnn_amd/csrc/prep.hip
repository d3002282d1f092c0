// K14: data-preparation kernels on gfx950 (MI355X) -- per-window standardisation and the exact
// k-nearest-neighbour search of SMOTE.
//
// Replaces the host NumPy / scikit-learn work of prepare_numpy_datasets.py:
//   * standardize_data (prepare_numpy_datasets.py:83-95): per window, per channel z-score over the
//     time axis, ddof 0, (x - mean) / (std + 1e-8), float64 like the reference;
//   * SMOTE's NearestNeighbors(k+1).kneighbors(X_class) (imblearn, prepare_numpy_datasets.py:185-187):
//     brute force over the minority class, self excluded, ties broken by index.
//
// Both are fp64 end to end: a resampled training set must not depend on whether the k-NN ran on the
// host or here, so distances are the exact sum of squared differences in a fixed feature order (no
// ||a||^2 + ||b||^2 - 2ab cancellation) and the neighbour order is (distance, index) lexicographic.
#include "common.h"

namespace apneauq {
namespace prep {

// ---- standardisation: one thread per (window, channel); the window's L x C block is staged through
// LDS by the workgroup with coalesced loads, so the strided per-channel sweeps hit LDS, not L2.
constexpr int kStdThreads = 256;

__global__ __launch_bounds__(kStdThreads) void standardize_kernel(const double* __restrict__ x, double* __restrict__ out,
                                                                  long long n_win, int L, int C, int wpb, double eps) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  double* s = reinterpret_cast<double*>(smem_raw);
  const long long w0 = (long long)blockIdx.x * wpb;
  const int nw = (int)min((long long)wpb, n_win - w0);
  const int elems = nw * L * C;
  const double* src = x + w0 * L * C;
  for (int i = threadIdx.x; i < elems; i += kStdThreads) s[i] = src[i];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < nw * C) {
    const int w = t / C, c = t - w * C;
    const double* p = s + w * L * C + c;
    double m = 0.0;
    for (int i = 0; i < L; ++i) m += p[i * C];
    m /= (double)L;
    double v = 0.0;
    for (int i = 0; i < L; ++i) {
      const double d = p[i * C] - m;
      v += d * d;
    }
    const double inv = 1.0 / (sqrt(v / (double)L) + eps);
    double* q = s + w * L * C + c;
    for (int i = 0; i < L; ++i) q[i * C] = (p[i * C] - m) * inv;
  }
  __syncthreads();
  double* dst = out + w0 * L * C;
  for (int i = threadIdx.x; i < elems; i += kStdThreads) dst[i] = s[i];
}

// ---- exact k-NN.  A workgroup owns kQ query rows (LDS) and streams the candidate rows through LDS in
// tiles of kCT rows; thread (q, sub) scans candidates sub, sub + kSub, ... of every tile for query q and
// keeps its own sorted top-K in registers; the kSub partial lists of a query are merged at the end.
constexpr int kQ = 32, kSub = 8, kCT = 32, kMaxK = 16, kKnnThreads = kQ * kSub;
static_assert(kKnnThreads == 256, "one wave per 8 queries");

template <int K>
__device__ __forceinline__ void topk_insert(double (&bd)[K], int (&bi)[K], double d, int j) {
  // (d, j) < (bd[K-1], bi[K-1]) lexicographically -> insert, keeping (distance, index) order
  if (d > bd[K - 1] || (d == bd[K - 1] && j > bi[K - 1])) return;
#pragma unroll
  for (int i = K - 1; i > 0; --i) {
    const bool shift = d < bd[i - 1] || (d == bd[i - 1] && j < bi[i - 1]);
    // slot i takes slot i-1 when the new pair sorts before it, else the new pair if it sorts before slot i
    const bool here = !shift && (d < bd[i] || (d == bd[i] && j < bi[i]));
    const double nd = shift ? bd[i - 1] : (here ? d : bd[i]);
    const int ni = shift ? bi[i - 1] : (here ? j : bi[i]);
    bd[i] = nd;
    bi[i] = ni;
  }
  if (d < bd[0] || (d == bd[0] && j < bi[0])) {
    bd[0] = d;
    bi[0] = j;
  }
}

template <int K>
__global__ __launch_bounds__(kKnnThreads) void knn_kernel(const double* __restrict__ X, int n, int D,
                                                          long long* __restrict__ out, int k) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  double* qs = reinterpret_cast<double*>(smem_raw);  // [kQ][D]
  double* cs = qs + kQ * D;                          // [kCT][D]
  const int q0 = blockIdx.x * kQ;
  const int nq = min(kQ, n - q0);
  for (int i = threadIdx.x; i < nq * D; i += kKnnThreads) qs[i] = X[(long long)q0 * D + i];
  const int q = threadIdx.x / kSub, sub = threadIdx.x % kSub;
  double bd[K];
  int bi[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    bd[i] = __builtin_huge_val();
    bi[i] = 0x7FFFFFFF;
  }
  for (int c0 = 0; c0 < n; c0 += kCT) {
    const int nc = min(kCT, n - c0);
    __syncthreads();  // previous tile fully read (and, first time round, the queries staged)
    for (int i = threadIdx.x; i < nc * D; i += kKnnThreads) cs[i] = X[(long long)c0 * D + i];
    __syncthreads();
    if (q < nq) {
      const double* qr = qs + q * D;
      for (int cc = sub; cc < nc; cc += kSub) {
        const int j = c0 + cc;
        if (j == q0 + q) continue;  // the query itself is not its own neighbour
        const double* cr = cs + cc * D;
        double d = 0.0;
        for (int f = 0; f < D; ++f) {
          const double t = qr[f] - cr[f];
          d = __builtin_fma(t, t, d);
        }
        topk_insert<K>(bd, bi, d, j);
      }
    }
  }
  __syncthreads();
  // merge the kSub partial lists of each query through LDS (reuses the query tile)
  double* md = qs;                                        // [kQ][kSub][K]
  int* mi = reinterpret_cast<int*>(qs + kQ * kSub * K);   // [kQ][kSub][K]
#pragma unroll
  for (int i = 0; i < K; ++i) {
    md[(q * kSub + sub) * K + i] = bd[i];
    mi[(q * kSub + sub) * K + i] = bi[i];
  }
  __syncthreads();
  if (sub == 0 && q < nq) {
    int pos[kSub];
#pragma unroll
    for (int s = 0; s < kSub; ++s) pos[s] = 0;
    for (int r = 0; r < k; ++r) {
      int best = 0;
      double bdv = __builtin_huge_val();
      int biv = 0x7FFFFFFF;
#pragma unroll
      for (int s = 0; s < kSub; ++s) {
        const double d = pos[s] < K ? md[(q * kSub + s) * K + pos[s]] : __builtin_huge_val();
        const int j = pos[s] < K ? mi[(q * kSub + s) * K + pos[s]] : 0x7FFFFFFF;
        if (d < bdv || (d == bdv && j < biv)) {
          bdv = d;
          biv = j;
          best = s;
        }
      }
      pos[best] += 1;
      out[(long long)(q0 + q) * k + r] = biv == 0x7FFFFFFF ? -1 : biv;
    }
  }
}

}  // namespace prep

hipError_t launch_standardize(const double* x, double* out, long long n_win, int L, int C, double eps,
                              hipStream_t stream) {
  if (n_win == 0) return hipSuccess;
  const int per = L * C * 8;
  int wpb = prep::kStdThreads / C;  // one thread per (window, channel)
  while (wpb > 1 && wpb * per > 64 * 1024) --wpb;
  if (wpb * C > prep::kStdThreads || wpb * per > 64 * 1024) return hipErrorInvalidValue;
  const long long grid = (n_win + wpb - 1) / wpb;
  hipLaunchKernelGGL(prep::standardize_kernel, dim3((unsigned)grid), dim3(prep::kStdThreads), wpb * per, stream, x, out,
                     n_win, L, C, wpb, eps);
  return hipGetLastError();
}

int knn_lds_bytes(int D, int K) {
  const int tiles = (prep::kQ + prep::kCT) * D * 8;
  const int merge = prep::kQ * prep::kSub * K * (8 + 4);
  return tiles > merge ? tiles : merge;
}

hipError_t launch_knn(const double* X, int n, int D, long long* out, int k, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (k < 1 || k > prep::kMaxK) return hipErrorInvalidValue;
  const int K = k <= 8 ? 8 : 16;
  const int lds = knn_lds_bytes(D, K);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int grid = (n + prep::kQ - 1) / prep::kQ;
  if (K == 8)
    hipLaunchKernelGGL(prep::knn_kernel<8>, dim3(grid), dim3(prep::kKnnThreads), lds, stream, X, n, D, out, k);
  else
    hipLaunchKernelGGL(prep::knn_kernel<16>, dim3(grid), dim3(prep::kKnnThreads), lds, stream, X, n, D, out, k);
  return hipGetLastError();
}

}  // namespace apneauq
