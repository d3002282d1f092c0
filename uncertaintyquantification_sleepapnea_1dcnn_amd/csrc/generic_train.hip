// Layer-wise HIP training kernels for ANY ModelSpec (gfx950 / MI355X): the opt-in MaxPool1D blocks,
// other window shapes (the "30 s single-channel" ModelSpec(30, 1)), other filter / kernel sizes.
// Reference semantics: one Keras train_on_batch of the SURVEY §2.2 stack (cnn_baseline_train.py:55-102):
//   z = relu(conv(h) + b);  y = BN_batch(z);  [y = MaxPool1D(2)(y)];  h' = Dropout(y)
// The reference architecture has its own persistent, LDS-resident kernels (train_conv.hip); this
// path is built from the generic implicit-GEMM MFMA conv (generic_conv.hip, modes kTrain / kLinear)
// plus the memory-bound pieces below, each one pass over bf16 activations:
//
//   bn_finalize   moment slots -> (scale, shift, mean, rstd) + Keras moving-average update
//   apply         BN affine + 2:1 max pool + counter-based dropout -> next layer's input, written in
//                 the consumer's zero-padded row layout (so wgrad is a plain strided GEMM)
//   bwd_stats     upstream grad routed back through dropout (same keys) and the pool (argmax
//                 recomputed from z) -> per-channel sum(dy), sum(dy * xhat)
//   bwd_finalize  -> dgamma, dbeta and the two BN-backward coefficients
//   bwd_dz        dz = relu'(z) * gamma * rstd * (dy - E[dy] - xhat E[dy xhat]) written zero-padded,
//                 bias gradient as a fused column sum (kSlots interleaved copies: one
//                 same-address atomic per block and channel serialised at L2 cost 5x the kernel)
//
// Channel-group mapping of the elementwise kernels: a thread owns 4 consecutive channels of one
// row (8-byte bf16x4 accesses), G = C/4 <= 256 groups across the block, 256 / G rows per sweep.
#include "common.h"

namespace apneauq {
namespace gtrain {

constexpr int kSlots = 16;  // == generic::kStatSlots

// Ordered sums of the two C-wide rows of every slot of an (nslots, 2, C) table, 16 channels x 16 slot
// lanes per 256-thread block: lane j adds slots j, j + 16, ... in order (fp64), then the block's first
// 16 threads add the 16 lane sums in order.  The association depends on nslots only, so the result is
// bitwise reproducible for a fixed slot layout: atomic mode (kSlots interleaved copies, each itself an
// atomic sum) and deterministic mode (one slot per producing workgroup, written with plain stores).
__device__ __forceinline__ bool slot_pair_sums(const float* st, int nslots, int C, double (&red)[2][256], double& s1,
                                               double& s2, int& c) {
  const int chl = threadIdx.x & 15, lane = threadIdx.x >> 4;
  c = blockIdx.x * 16 + chl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    for (int s = lane; s < nslots; s += 16) {
      a += (double)st[(long long)s * 2 * C + c];
      b += (double)st[(long long)s * 2 * C + C + c];
    }
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  s1 = 0.0;
  s2 = 0.0;
  if (threadIdx.x >= 16 || c >= C) return false;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    s1 += red[0][j * 16 + chl];
    s2 += red[1][j * 16 + chl];
  }
  return true;
}

// Large slot tables (deterministic mode: one slot per producing workgroup, ~15 k for a 16384-window
// batch-statistics MC-Dropout pass) are summed in two launches: slot_partial_kernel adds every range of
// kRange consecutive slots (fixed order, fp64) and parks the two sums in the range's first two slots
// (their fp32 words hold the fp64 bits: the raw table is dead after the finalize), then the finalize
// adds the ranges in order.  One 16-channel block per C / 16 with a serial pass over 15 k slots took
// ~130 us per call.  The packed sums take four words per channel = two slots, so no range may hold a
// single slot: a one-slot tail joins the range before it (the last range runs to nslots; see
// partial_ranges).
constexpr int kRange = 64;

__host__ __device__ inline int partial_ranges(int nslots) {
  const int r = (nslots + kRange - 1) / kRange;
  return (nslots % kRange == 1 && r > 1) ? r - 1 : r;
}

__global__ __launch_bounds__(256) void slot_partial_kernel(float* st, int nslots, int C) {
  __shared__ double red[2][256];
  const int chl = threadIdx.x & 15, lane = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + chl;
  const int s0 = blockIdx.y * kRange, s1e = blockIdx.y + 1 == gridDim.y ? nslots : s0 + kRange;
  APNEAUQ_DASSERT(s1e - s0 >= 2 && s1e <= nslots);
  double a = 0.0, b = 0.0;
  if (c < C) {
    for (int s = s0 + lane; s < s1e; s += 16) {
      a += (double)st[(long long)s * 2 * C + c];
      b += (double)st[(long long)s * 2 * C + C + c];
    }
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();  // every read of this range is done before the range's first slots are overwritten
  if (threadIdx.x >= 16 || c >= C) return;
  double t1 = 0.0, t2 = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    t1 += red[0][j * 16 + chl];
    t2 += red[1][j * 16 + chl];
  }
  unsigned* w = reinterpret_cast<unsigned*>(st) + (long long)s0 * 2 * C;
  const unsigned long long b1 = __double_as_longlong(t1), b2 = __double_as_longlong(t2);
  w[c] = (unsigned)b1;
  w[C + c] = (unsigned)(b1 >> 32);
  w[2 * C + c] = (unsigned)b2;
  w[3 * C + c] = (unsigned)(b2 >> 32);
}

__device__ __forceinline__ double packed_sum(const float* st, int C, int range, int word) {
  const unsigned* w = reinterpret_cast<const unsigned*>(st) + (long long)range * kRange * 2 * C;
  return __longlong_as_double((long long)(((unsigned long long)w[word + C] << 32) | w[word]));
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* st, int nslots, int C, float inv_count,
                                                          const float* gamma, const float* beta, float eps,
                                                          float momentum, float* mmean, float* mvar, int update,
                                                          float* bn, int packed) {
  __shared__ double red[2][256];
  double s1, s2;
  int c;
  if (packed) {  // nslots = ranges of slot_partial_kernel: their fp64 sums, added in range order
    const int chl = threadIdx.x & 15, lane = threadIdx.x >> 4;
    c = blockIdx.x * 16 + chl;
    double a = 0.0, b = 0.0;
    if (c < C) {
      for (int r = lane; r < nslots; r += 16) {
        a += packed_sum(st, C, r, c);
        b += packed_sum(st, C, r, 2 * C + c);
      }
    }
    red[0][threadIdx.x] = a;
    red[1][threadIdx.x] = b;
    __syncthreads();
    if (threadIdx.x >= 16 || c >= C) return;
    s1 = s2 = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      s1 += red[0][j * 16 + chl];
      s2 += red[1][j * 16 + chl];
    }
  } else if (!slot_pair_sums(st, nslots, C, red, s1, s2, c)) {
    return;
  }
  const double meand = s1 * inv_count;
  const float mean = (float)meand;
  const float var = (float)fmax(s2 * inv_count - meand * meand, 0.0);
  const float rstd = rsqrtf(var + eps);
  const float scale = gamma[c] * rstd;
  bn[c] = scale;
  bn[C + c] = beta[c] - mean * scale;
  bn[2 * C + c] = mean;
  bn[3 * C + c] = rstd;
  if (update) {
    mmean[c] = mmean[c] * momentum + mean * (1.f - momentum);
    mvar[c] = mvar[c] * momentum + var * (1.f - momentum);
  }
}

// Activation storage: bf16 (the bf16 training path) or fp32 (precision="fp32", csrc/gf32_conv.hip);
// the kernels below are templated on it (4 consecutive channels per thread either way).
__device__ __forceinline__ f32x4 load4(const __bf16* p) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
__device__ __forceinline__ f32x4 load4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void store4(__bf16* p, const f32x4& v) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}
__device__ __forceinline__ void store4(float* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }

template <typename T>
struct ApplyArgs {
  const T* z;       // (N, L, C) pre-BN activations
  const float* bn;  // (4, C): scale, shift, mean, rstd
  T* out;           // row (n, t) at n * out_rs + out_off + t
  int n, L, C, pool, lout, out_rs, out_off, dropout;
  unsigned thr;
  float inv_keep;
  unsigned skey;  // stream_key(seed, layer, pass)
  unsigned window_offset;
  const unsigned* skey_dev;  // optional: the key read from device memory (HIP-graph replays)
};

template <typename T>
__global__ __launch_bounds__(256) void apply_kernel(ApplyArgs<T> A) {
  if (A.skey_dev != nullptr) A.skey = *A.skey_dev;
  const int G = A.C >> 2;
  const long long total = (long long)A.n * A.lout * G;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % G) * 4;
    const long long row = i / G;
    const int ns = (int)(row / A.lout), to = (int)(row - (long long)ns * A.lout);
    const int t0 = A.pool ? 2 * to : to;
    const T* zr = A.z + ((long long)ns * A.L + t0) * A.C + c;
    const f32x4 sc = *reinterpret_cast<const f32x4*>(A.bn + c);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(A.bn + A.C + c);
    f32x4 y = load4(zr);
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = __builtin_fmaf(y[j], sc[j], sh[j]);
    if (A.pool) {
      const f32x4 y1 = load4(zr + A.C);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = fmaxf(y[j], __builtin_fmaf(y1[j], sc[j], sh[j]));
    }
    if (A.dropout) {
      const unsigned key = sample_key(A.skey, A.window_offset + (unsigned)ns);
      const unsigned b01 = dropout_bits2(key, (unsigned)to, (unsigned)c);
      const unsigned b23 = dropout_bits2(key, (unsigned)to, (unsigned)c + 2);
      y[0] = (b01 & 0xFFFFu) >= A.thr ? y[0] * A.inv_keep : 0.f;
      y[1] = (b01 >> 16) >= A.thr ? y[1] * A.inv_keep : 0.f;
      y[2] = (b23 & 0xFFFFu) >= A.thr ? y[2] * A.inv_keep : 0.f;
      y[3] = (b23 >> 16) >= A.thr ? y[3] * A.inv_keep : 0.f;
    }
    store4(A.out + ((long long)ns * A.out_rs + A.out_off + to) * A.C + c, y);
  }
}

template <typename T>
struct BwdArgs {
  const T* z;          // (N, L, C)
  const float* bn;     // (4, C)
  const T* dh;         // (N, lout, C) upstream gradient, or nullptr in head mode
  const float* dlog;   // head mode: dh[n, t, c] = dlog[n] * w[c] * invL
  const float* w;
  float invL;
  int n, L, C, pool, lout, dropout;
  unsigned thr;
  float inv_keep;
  unsigned skey, window_offset;
  const unsigned* skey_dev;  // optional: the key read from device memory (HIP-graph replays)
  float* bst;          // bwd_stats: (kSlots, 2, C) sums of dy, dy * xhat
  const float* coef;   // bwd_dz: (2, C) E[dy], E[dy xhat]
  const float* gamma;
  T* dz;               // bwd_dz: row (n, t) at n * dz_rs + dz_off + t
  int dz_rs, dz_off;
  float* gbias;        // bwd_dz: bias-gradient slots (kSlots, C), summed by the host
  int det;             // deterministic mode: block b writes slot b with plain stores (grid <= slots)
};

// Gradient w.r.t. the BN output y at pre-pool row (ns, t), channels c .. c+3.
template <typename T>
__device__ __forceinline__ f32x4 upstream_dy(const BwdArgs<T>& A, int ns, int t, int c, const f32x4& sc,
                                             const f32x4& sh) {
  f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
  const int to = A.pool ? (t >> 1) : t;
  if (to >= A.lout) return g;  // odd L with pool: the last step is dropped by the valid pool
  if (A.dh != nullptr) {
    g = load4(A.dh + ((long long)ns * A.lout + to) * A.C + c);
  } else {
    const float d = A.dlog[ns] * A.invL;
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = d * A.w[c + j];
  }
  if (A.dropout) {
    const unsigned key = sample_key(A.skey, A.window_offset + (unsigned)ns);
    const unsigned b01 = dropout_bits2(key, (unsigned)to, (unsigned)c);
    const unsigned b23 = dropout_bits2(key, (unsigned)to, (unsigned)c + 2);
    g[0] = (b01 & 0xFFFFu) >= A.thr ? g[0] * A.inv_keep : 0.f;
    g[1] = (b01 >> 16) >= A.thr ? g[1] * A.inv_keep : 0.f;
    g[2] = (b23 & 0xFFFFu) >= A.thr ? g[2] * A.inv_keep : 0.f;
    g[3] = (b23 >> 16) >= A.thr ? g[3] * A.inv_keep : 0.f;
  }
  if (A.pool) {  // max-pool backward: the gradient goes to the (first) maximum of the pair
    const T* zr = A.z + (long long)ns * A.L * A.C + c;
    const f32x4 za = load4(zr + (long long)t * A.C), zb = load4(zr + (long long)(t ^ 1) * A.C);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float ya = __builtin_fmaf(za[j], sc[j], sh[j]), yb = __builtin_fmaf(zb[j], sc[j], sh[j]);
      const bool win = (t & 1) == 0 ? ya >= yb : ya > yb;
      g[j] = win ? g[j] : 0.f;
    }
  }
  return g;
}

// Block reduction of 8 per-thread partial sums per channel group; returns in threads tid < G.
__device__ __forceinline__ void block_reduce8(float* lds, float (&v)[8], int G, int rpb) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) lds[j * 256 + tid] = v[j];
  __syncthreads();
  if (tid < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
      for (int r = 1; r < rpb; ++r) s += lds[j * 256 + r * G + tid];
      v[j] += s;
    }
  }
}

template <bool DZ, typename T>
__global__ __launch_bounds__(256) void bwd_kernel(BwdArgs<T> A) {
  __shared__ float lds[8 * 256];
  if (A.skey_dev != nullptr) A.skey = *A.skey_dev;
  const int G = A.C >> 2;
  const int rpb = 256 / G;
  const int cg = threadIdx.x % G, rl = threadIdx.x / G;
  const int c = cg * 4;
  const bool active = rl < rpb;
  const long long rows = (long long)A.n * A.L;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    const f32x4 sc = *reinterpret_cast<const f32x4*>(A.bn + c);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(A.bn + A.C + c);
    const f32x4 mu = *reinterpret_cast<const f32x4*>(A.bn + 2 * A.C + c);
    const f32x4 rs = *reinterpret_cast<const f32x4*>(A.bn + 3 * A.C + c);
    f32x4 k0 = f32x4{0.f, 0.f, 0.f, 0.f}, k1 = k0, gr = k0;
    if constexpr (DZ) {
      k0 = *reinterpret_cast<const f32x4*>(A.coef + c);
      k1 = *reinterpret_cast<const f32x4*>(A.coef + A.C + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) gr[j] = A.gamma[c + j] * rs[j];
    }
    for (long long row = (long long)blockIdx.x * rpb + rl; row < rows; row += (long long)gridDim.x * rpb) {
      const int ns = (int)(row / A.L), t = (int)(row - (long long)ns * A.L);
      const f32x4 dy = upstream_dy(A, ns, t, c, sc, sh);
      const f32x4 z = load4(A.z + row * A.C + c);
      if constexpr (!DZ) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j] += dy[j];
          acc[4 + j] += dy[j] * (z[j] - mu[j]) * rs[j];
        }
      } else {
        f32x4 d;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = (z[j] - mu[j]) * rs[j];
          d[j] = z[j] > 0.f ? gr[j] * (dy[j] - k0[j] - xh * k1[j]) : 0.f;
          acc[j] += d[j];
        }
        store4(A.dz + ((long long)ns * A.dz_rs + A.dz_off + t) * A.C + c, d);
      }
    }
  }
  block_reduce8(lds, acc, G, rpb);
  if (threadIdx.x < G) {
    const int slot = A.det ? blockIdx.x : blockIdx.x % kSlots;
    if constexpr (!DZ) {
      float* st = A.bst + (long long)slot * 2 * A.C;
      if (A.det) {
        *reinterpret_cast<f32x4*>(st + c) = f32x4{acc[0], acc[1], acc[2], acc[3]};
        *reinterpret_cast<f32x4*>(st + A.C + c) = f32x4{acc[4], acc[5], acc[6], acc[7]};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          atomicAdd(st + c + j, acc[j]);
          atomicAdd(st + A.C + c + j, acc[4 + j]);
        }
      }
    } else {
      float* gb = A.gbias + (long long)slot * A.C + c;
      if (A.det) {
        *reinterpret_cast<f32x4*>(gb) = f32x4{acc[0], acc[1], acc[2], acc[3]};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(gb + j, acc[j]);
      }
    }
  }
}

// Blocks [0, ceil(C / 16)) finalize the BN backward of one block; blocks after that (side job, no
// node of its own) add the bias-gradient slot table (bslots, BC) of the block above it in fixed order:
// lane j sums slots j, j + 16, ... (fp64), then the 16 lane sums in order -> reproducible.
__global__ __launch_bounds__(256) void bwd_finalize_kernel(const float* bst, int nslots, int C, float inv_count,
                                                           float* coef, float* ggamma, float* gbeta, const float* dbs,
                                                           int bslots, int BC, float* gbias) {
  __shared__ double red[2][256];
  const int nfin = (C + 15) / 16;
  if ((int)blockIdx.x >= nfin) {
    const int chl = threadIdx.x & 15, lane = threadIdx.x >> 4;
    const int c = ((int)blockIdx.x - nfin) * 16 + chl;
    double a = 0.0;
    if (c < BC)
      for (int s = lane; s < bslots; s += 16) a += (double)dbs[(long long)s * BC + c];
    red[0][threadIdx.x] = a;
    __syncthreads();
    if (threadIdx.x >= 16 || c >= BC) return;
    double t = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[0][j * 16 + chl];
    gbias[c] = (float)t;
    return;
  }
  double s1, s2;
  int c;
  if (!slot_pair_sums(bst, nslots, C, red, s1, s2, c)) return;
  gbeta[c] = (float)s1;
  ggamma[c] = (float)s2;
  coef[c] = (float)(s1 * inv_count);
  coef[C + c] = (float)(s2 * inv_count);
}

inline int elem_grid(long long items, int per_block) {
  long long g = (items + per_block - 1) / per_block;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace gtrain

hipError_t launch_gt_bn_finalize(const float* st, int nslots, int C, float inv_count, const float* gamma,
                                 const float* beta, float eps, float momentum, float* mmean, float* mvar, int update,
                                 float* bn, hipStream_t stream) {
  if (nslots >= 4 * gtrain::kRange) {
    const int ranges = gtrain::partial_ranges(nslots);
    hipLaunchKernelGGL(gtrain::slot_partial_kernel, dim3((C + 15) / 16, ranges), dim3(256), 0, stream,
                       const_cast<float*>(st), nslots, C);
    hipLaunchKernelGGL(gtrain::bn_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, stream, st, ranges, C, inv_count,
                       gamma, beta, eps, momentum, mmean, mvar, update, bn, 1);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(gtrain::bn_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, stream, st, nslots, C, inv_count,
                     gamma, beta, eps, momentum, mmean, mvar, update, bn, 0);
  return hipGetLastError();
}

template <typename T>
static hipError_t gt_apply_t(const void* z, const float* bn, void* out, int n, int L, int C, int pool, int out_rs,
                             int out_off, int dropout, unsigned thr, float inv_keep, unsigned skey,
                             unsigned window_offset, hipStream_t stream, const unsigned* skey_dev) {
  gtrain::ApplyArgs<T> A;
  A.skey_dev = skey_dev;
  A.z = reinterpret_cast<const T*>(z);
  A.bn = bn;
  A.out = reinterpret_cast<T*>(out);
  A.n = n;
  A.L = L;
  A.C = C;
  A.pool = pool;
  A.lout = pool ? L / 2 : L;
  A.out_rs = out_rs;
  A.out_off = out_off;
  A.dropout = dropout;
  A.thr = thr;
  A.inv_keep = inv_keep;
  A.skey = skey;
  A.window_offset = window_offset;
  const long long items = (long long)n * A.lout * (C / 4);
  if (items == 0) return hipSuccess;
  hipLaunchKernelGGL(gtrain::apply_kernel<T>, dim3(gtrain::elem_grid(items, 256)), dim3(256), 0, stream, A);
  return hipGetLastError();
}

hipError_t launch_gt_apply(const void* z, const float* bn, void* out, int n, int L, int C, int pool, int out_rs,
                           int out_off, int dropout, unsigned thr, float inv_keep, unsigned skey,
                           unsigned window_offset, hipStream_t stream, const unsigned* skey_dev, int f32) {
  return f32 ? gt_apply_t<float>(z, bn, out, n, L, C, pool, out_rs, out_off, dropout, thr, inv_keep, skey,
                                 window_offset, stream, skey_dev)
             : gt_apply_t<__bf16>(z, bn, out, n, L, C, pool, out_rs, out_off, dropout, thr, inv_keep, skey,
                                  window_offset, stream, skey_dev);
}

template <typename T>
static hipError_t gt_bwd_t(int dz_mode, const void* z, const float* bn, const void* dh, const float* dlog,
                           const float* w, float invL, int n, int L, int C, int pool, int dropout, unsigned thr,
                           float inv_keep, unsigned skey, unsigned window_offset, float* bst, const float* coef,
                           const float* gamma, void* dz, int dz_rs, int dz_off, float* gbias, hipStream_t stream,
                           const unsigned* skey_dev, int det_slots) {
  gtrain::BwdArgs<T> A;
  A.skey_dev = skey_dev;
  A.z = reinterpret_cast<const T*>(z);
  A.bn = bn;
  A.dh = reinterpret_cast<const T*>(dh);
  A.dlog = dlog;
  A.w = w;
  A.invL = invL;
  A.n = n;
  A.L = L;
  A.C = C;
  A.pool = pool;
  A.lout = pool ? L / 2 : L;
  A.dropout = dropout;
  A.thr = thr;
  A.inv_keep = inv_keep;
  A.skey = skey;
  A.window_offset = window_offset;
  A.bst = bst;
  A.coef = coef;
  A.gamma = gamma;
  A.dz = reinterpret_cast<T*>(dz);
  A.dz_rs = dz_rs;
  A.dz_off = dz_off;
  A.gbias = gbias;
  A.det = det_slots > 0;
  const int rpb = 256 / (C / 4);
  const long long rows = (long long)n * L;
  if (rows == 0) return hipSuccess;
  int g = gtrain::elem_grid(rows, rpb * 4);  // ~4 rows per thread
  if (A.det && g > det_slots) g = det_slots;  // one slot per block (grid-stride rows)
  const dim3 grid(g);
  if (dz_mode)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gtrain::bwd_kernel<true, T>), grid, dim3(256), 0, stream, A);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gtrain::bwd_kernel<false, T>), grid, dim3(256), 0, stream, A);
  return hipGetLastError();
}

hipError_t launch_gt_bwd(int dz_mode, const void* z, const float* bn, const void* dh, const float* dlog,
                         const float* w, float invL, int n, int L, int C, int pool, int dropout, unsigned thr,
                         float inv_keep, unsigned skey, unsigned window_offset, float* bst, const float* coef,
                         const float* gamma, void* dz, int dz_rs, int dz_off, float* gbias, hipStream_t stream,
                         const unsigned* skey_dev, int det_slots, int f32) {
  return f32 ? gt_bwd_t<float>(dz_mode, z, bn, dh, dlog, w, invL, n, L, C, pool, dropout, thr, inv_keep, skey,
                               window_offset, bst, coef, gamma, dz, dz_rs, dz_off, gbias, stream, skey_dev, det_slots)
             : gt_bwd_t<__bf16>(dz_mode, z, bn, dh, dlog, w, invL, n, L, C, pool, dropout, thr, inv_keep, skey,
                                window_offset, bst, coef, gamma, dz, dz_rs, dz_off, gbias, stream, skey_dev, det_slots);
}

hipError_t launch_gt_bwd_finalize(const float* bst, int nslots, int C, float inv_count, float* coef, float* ggamma,
                                  float* gbeta, const float* dbs, int bslots, int BC, float* gbias,
                                  hipStream_t stream) {
  if (gbias == nullptr) BC = 0;
  const int blocks = (C + 15) / 16 + (BC + 15) / 16;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(gtrain::bwd_finalize_kernel, dim3(blocks), dim3(256), 0, stream, bst, nslots, C, inv_count, coef,
                     ggamma, gbeta, dbs, bslots, BC, gbias);
  return hipGetLastError();
}

}  // namespace apneauq
