// Multi-tensor Adam over the model's single flat fp32 parameter buffer (gfx950).
//
// Keras 2.12 Adam (the optimizer of cnn_baseline_train.py:100, lr 1e-3):
//   m += (g - m) * (1 - b1);  v += (g^2 - v) * (1 - b2)
//   p -= alpha * m / (sqrt(v) + eps),   alpha = lr * sqrt(1 - b2^t) / (1 - b1^t),  eps = 1e-7
// One launch updates all 26 trainable tensors (851,457 values): 16-B vector loads/stores, grid
// sized to the chip and grid-strided.  Optionally averages a data-parallel gradient (scale).  With
// step_dev the bias correction is computed on the device from the iteration counter, so a captured
// HIP graph of the training step replays correctly (ops/train_ops.py:GraphedTrainStep).
#include "common.h"

namespace apneauq {

__device__ __forceinline__ void adam_body(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                          float* __restrict__ v, long long n, float b1, float b2, float alpha,
                                          float eps, float gscale, const int* __restrict__ step_dev) {
  if (step_dev != nullptr) {  // HIP-graph replays: alpha_t from the device iteration counter (alpha = lr)
    const float t = (float)(*step_dev + 1);
    alpha = alpha * sqrtf(1.f - powf(b2, t)) / (1.f - powf(b1, t));
  }
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float c1 = 1.f - b1, c2 = 1.f - b2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i] * gscale;
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mm[k] += (gg[k] - mm[k]) * c1;
      vv[k] += (gg[k] * gg[k] - vv[k]) * c2;
      pp[k] -= alpha * mm[k] / (sqrtf(vv[k]) + eps);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  // scalar tail
  const long long t = (n4 << 2) + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t < n && t < (n4 << 2) + 4) {
    const float gg = g[t] * gscale;
    float mm = m[t] + (gg - m[t]) * c1;
    float vv = v[t] + (gg * gg - v[t]) * c2;
    p[t] -= alpha * mm / (sqrtf(vv) + eps);
    m[t] = mm;
    v[t] = vv;
  }
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, long long n,
                                                    float b1, float b2, float alpha, float eps, float gscale,
                                                    const int* __restrict__ step_dev) {
  adam_body(p, g, m, v, n, b1, b2, alpha, eps, gscale, step_dev);
}

// Member-batched Adam (ensemble members of one architecture sharing the hyper-parameters): set
// blockIdx.y = one member's (params, grads, moments, device iteration counter), one launch for all.
constexpr int kAdamMaxSets = 16;
struct AdamSets {
  float* p[kAdamMaxSets];
  const float* g[kAdamMaxSets];
  float* m[kAdamMaxSets];
  float* v[kAdamMaxSets];
  const int* step[kAdamMaxSets];
};

__global__ __launch_bounds__(256) void adam_multi_kernel(AdamSets S, long long n, float b1, float b2, float alpha,
                                                          float eps) {
  const int i = blockIdx.y;
  adam_body(S.p[i], S.g[i], S.m[i], S.v[i], n, b1, b2, alpha, eps, 1.f, S.step[i]);
}

int adam_max_sets() { return kAdamMaxSets; }

hipError_t launch_adam_multi(int ns, float* const* p, const float* const* g, float* const* m, float* const* v,
                             const int* const* step, long long n, float b1, float b2, float alpha, float eps,
                             hipStream_t stream) {
  if (ns < 1 || ns > kAdamMaxSets) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  AdamSets S = {};
  for (int i = 0; i < ns; ++i) {
    S.p[i] = p[i];
    S.g[i] = g[i];
    S.m[i] = m[i];
    S.v[i] = v[i];
    S.step[i] = step[i];
  }
  long long blocks = ((n >> 2) + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks, (unsigned)ns), dim3(256), 0, stream, S, n, b1, b2, alpha,
                     eps);
  return hipGetLastError();
}

hipError_t launch_adam(float* p, const float* g, float* m, float* v, long long n, float b1, float b2, float alpha,
                       float eps, float gscale, const int* step_dev, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  long long blocks = ((n >> 2) + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p, g, m, v, n, b1, b2, alpha, eps, gscale,
                     step_dev);
  return hipGetLastError();
}

// Zero up to kZeroMax buffers in ONE launch (the training step clears its moment / gradient / loss
// accumulators: four fill kernels, ~5 us per graph node each, became one).  Buffer y = blockIdx.y;
// sizes in 4-byte words, 16-B stores where the buffer allows.
constexpr int kZeroMax = 64;  // 8 ensemble members x 5 accumulators in one member-batched step
struct ZeroArgs {
  uint32_t* p[kZeroMax];
  long long words[kZeroMax];
};

__global__ __launch_bounds__(256) void zero_kernel(ZeroArgs Z) {
  uint32_t* p = Z.p[blockIdx.y];
  const long long n = Z.words[blockIdx.y];
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const bool vec = (reinterpret_cast<uintptr_t>(p) & 15) == 0;  // block-uniform
  const long long n4 = vec ? n >> 2 : 0;
  for (long long i = t0; i < n4; i += stride) reinterpret_cast<uint4*>(p)[i] = uint4{0u, 0u, 0u, 0u};
  for (long long i = (n4 << 2) + t0; i < n; i += stride) p[i] = 0u;
}

int zero_max_buffers() { return kZeroMax; }

// Training-step tail (the graph's last node): bump every member's device counters [dropout step, Adam
// iterations] and write probs = sigmoid(logits) of up to kTailMax members -- what a bump launch plus one
// torch sigmoid per member did.
constexpr int kTailMax = 32;
struct TailArgs {
  const float* logits[kTailMax];
  float* probs[kTailMax];
  int* counters;
  int ncounters, n;
};

__global__ __launch_bounds__(256) void train_tail_kernel(TailArgs T) {
  const int m = blockIdx.y;
  if (m == 0 && blockIdx.x == 0)
    for (int i = threadIdx.x; i < T.ncounters; i += blockDim.x) T.counters[i] += 1;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < T.n; i += gridDim.x * blockDim.x)
    T.probs[m][i] = 1.0f / (1.0f + __expf(-T.logits[m][i]));
}

int train_tail_max() { return kTailMax; }

hipError_t launch_train_tail(int* counters, int ncounters, int members, const float* const* logits,
                             float* const* probs, int n, hipStream_t stream) {
  if (members < 1 || members > kTailMax || n < 0) return hipErrorInvalidValue;
  TailArgs T = {};
  for (int i = 0; i < members; ++i) {
    T.logits[i] = logits[i];
    T.probs[i] = probs[i];
  }
  T.counters = counters;
  T.ncounters = ncounters;
  T.n = n;
  int gx = (n + 255) / 256;
  gx = gx < 1 ? 1 : (gx > 64 ? 64 : gx);
  hipLaunchKernelGGL(train_tail_kernel, dim3(gx, members), dim3(256), 0, stream, T);
  return hipGetLastError();
}

// The step's inputs for up to kTailMax members in one launch: x (n, L, C) fp32 -> the workspace's
// padded-row bf16 layout (row stride SR*C per sample), y (n) fp32 -> the label buffer.
struct InputArgs {
  const float* x[kTailMax];
  __bf16* xd[kTailMax];
  const float* y[kTailMax];
  float* yd[kTailMax];
  int n, L, C, SR;
};

__global__ __launch_bounds__(256) void train_inputs_kernel(InputArgs A) {
  const int m = blockIdx.y;
  const long long nx = (long long)A.n * A.L * A.C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nx + A.n; i += stride) {
    if (i < nx) {
      const long long b = i / ((long long)A.L * A.C), r = i - b * A.L * A.C;
      A.xd[m][b * A.SR * A.C + r] = (__bf16)A.x[m][i];
    } else {
      A.yd[m][i - nx] = A.y[m][i - nx];
    }
  }
}

hipError_t launch_train_inputs(int members, const float* const* x, void* const* xd, const float* const* y,
                               float* const* yd, int n, int L, int C, int SR, hipStream_t stream) {
  if (members < 1 || members > kTailMax || n < 0 || SR < L) return hipErrorInvalidValue;
  InputArgs A = {};
  for (int i = 0; i < members; ++i) {
    A.x[i] = x[i];
    A.xd[i] = reinterpret_cast<__bf16*>(xd[i]);
    A.y[i] = y[i];
    A.yd[i] = yd[i];
  }
  A.n = n;
  A.L = L;
  A.C = C;
  A.SR = SR;
  long long gx = ((long long)n * L * C + n + 255) / 256;
  gx = gx < 1 ? 1 : (gx > 512 ? 512 : gx);
  hipLaunchKernelGGL(train_inputs_kernel, dim3((unsigned)gx, members), dim3(256), 0, stream, A);
  return hipGetLastError();
}

hipError_t launch_zero(int nb, void* const* ptrs, const long long* words, hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  if (nb > kZeroMax) return hipErrorInvalidValue;
  ZeroArgs Z = {};
  long long mx = 0;
  for (int i = 0; i < nb; ++i) {
    Z.p[i] = reinterpret_cast<uint32_t*>(ptrs[i]);
    Z.words[i] = words[i];
    mx = words[i] > mx ? words[i] : mx;
  }
  long long blocks = ((mx >> 2) + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 512 ? 512 : blocks);
  hipLaunchKernelGGL(zero_kernel, dim3((unsigned)blocks, (unsigned)nb), dim3(256), 0, stream, Z);
  return hipGetLastError();
}

}  // namespace apneauq
