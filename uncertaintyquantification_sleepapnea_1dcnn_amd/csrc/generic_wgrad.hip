// Generic-spec training kernels that replace library GEMMs and torch ops on the generic hot path
// (gfx950 / MI355X): any ModelSpec -- pooled blocks, the "30 s single-channel" ModelSpec(30, 1), other
// filter / kernel sizes -- trains on the layer-wise kernels of generic_train.hip plus these:
//
//   wgrad_kernel  dW[tap][ci][co] = sum_R Xpad[R + tap][ci] * dZpad[R][co]   (split-K over rows)
//                 on v_mfma_f32_16x16x32_bf16.  Both operands are row-major (rows x channels) bf16
//                 tiles staged in LDS and read with the transposing ds_read_b64_tr_b16 (K = rows);
//                 the row order inside a 32-row k-step makes every read conflict-free on strides
//                 that are odd multiples of 32 B (train_conv.hip tr_frag).  A workgroup owns one
//                 16-channel ci tile x 4*NCO co tiles and a contiguous range of 64-row chunks; every
//                 tap's fragment is re-read from the same staged rows (shifted by the tap).  Few
//                 input channels (Cin * k <= 32, the first block) use an im2col tile instead:
//                 kk = tap * Cin + ci as the M dimension.  fp32 results are atomically added.
//                 (Round 1 ran this as hipBLASLt strided-batched GEMMs.)
//   head_kernel   GAP + Dense(C -> 1) + BCE on logits + dlogit + dense gradients, one wave/sample
//                 (round 1: six torch ops).
//   pack_kernel   fp32 (k, Cin, Cout) kernels of every block -> forward and dgrad (flipped,
//                 transposed) MFMA A fragments, channels zero-padded to 16, in one launch
//                 (round 1: torch pad / flip / permute / cast per block and step).
//
// Reference: models/train_deep_ensemble_cnns.py:30-71 (the pooled variants), cnn_baseline_train.py:
// 100-102 (Adam, BCE) -- the Keras train step these kernels implement.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace apneauq {
namespace gwgrad {

typedef short v4i16 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kChunk = 64;  // rows staged per step (two 32-row k-steps)

__host__ __device__ constexpr int odd32(int bytes) { return ((bytes + 31) / 32) % 2 ? (bytes + 31) / 32 * 32 : (bytes + 31) / 32 * 32 + 32; }

// fragment of a 16x16x32 operand whose K index is the LDS row (32 rows from row_base), 16 columns
// from col0: k-slot order as train_conv.hip tr_frag (conflict-free on odd-32B strides)
__device__ __forceinline__ bf16x8 tr_frag(const char* lds, int rs, int row_base, int col0) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const char* a0 = lds + (row_base + 4 * h + q) * rs + (col0 + 4 * p) * 2;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(a0 + 16 * rs));
  bf16x8 r;
  const __bf16* pl = reinterpret_cast<const __bf16*>(&lo);
  const __bf16* ph = reinterpret_cast<const __bf16*>(&hi);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = pl[j];
    r[4 + j] = ph[j];
  }
  return r;
}

struct WgArgs {
  const __bf16* x;   // Xpad rows (x_rows, cin)
  const __bf16* dz;  // dZpad rows (R, cout)
  float* gw;         // (k, cin, cout) fp32, accumulated
  long long R;       // reduction rows (n * rs)
  long long x_rows;  // rows of the x buffer (>= R + k - 1)
  int cin, cout, k;
  int n_ci, n_co;    // ci tiles (16) / co blocks (4 * NCO tiles) of the grid
  int chunks_per_wg;
  float* part;       // deterministic mode: (row groups, k * cin * cout) partials, plain stores (nullptr: atomics)
};

// IM2COL: M = kk = tap * cin + ci < 32 (two 16-row A tiles), one "tap".
template <int NCO, int KMAX, bool IM2COL>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(WgArgs A) {
  constexpr int COB = 64 * NCO;                        // co per workgroup
  constexpr int XCOLS = IM2COL ? 32 : 16;              // staged A columns (ci, or kk)
  constexpr int DZRS = odd32(COB * 2);
  constexpr int XRS = odd32(XCOLS * 2);
  constexpr int XROWS = kChunk + (IM2COL ? 0 : KMAX - 1) + 16;  // + slack: the last tr read of a tap
  constexpr int NT = IM2COL ? 1 : KMAX;                // taps held in accumulators
  constexpr int NM = IM2COL ? 2 : 1;                   // A tiles per tap
  __shared__ __attribute__((aligned(16))) char dz_lds[kChunk * DZRS];
  __shared__ __attribute__((aligned(16))) char x_lds[XROWS * XRS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // XCD-aware block order: the n_ci blocks sharing a chunk range run on one XCD (shared dZ rows in L2)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = bid % 8;
  const int wg = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + bid / 8;
  const int ci_t = wg % A.n_ci;
  const int co_b = (wg / A.n_ci) % A.n_co;
  const int rg = wg / (A.n_ci * A.n_co);
  const int ci0 = ci_t * 16, co0 = co_b * COB;
  const int k = A.k;
  f32x4 acc[NT][NM][NCO];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mi = 0; mi < NM; ++mi)
#pragma unroll
      for (int c = 0; c < NCO; ++c) acc[t][mi][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const long long chunks = (A.R + kChunk - 1) / kChunk;
  const long long c_begin = (long long)rg * A.chunks_per_wg;
  const long long c_end = c_begin + A.chunks_per_wg < chunks ? c_begin + A.chunks_per_wg : chunks;
  // Software pipeline: chunk ch+1's rows are loaded into registers (DZI + XI 16-B pieces per
  // thread, IM2COL: 8 scalars) while chunk ch's MFMAs run; the staging otherwise paid one full
  // memory round trip per 64-row chunk with only ~600 MFMA cycles per wave to cover it.
  constexpr int DZI = kChunk * (COB / 8) / kThreads;      // 16-B dZ pieces per thread
  constexpr int XI = (XROWS * 2 + kThreads - 1) / kThreads;  // 16-B X pieces per thread (non-im2col)
  constexpr int XS = IM2COL ? kChunk * 32 / kThreads : 1;   // im2col scalars per thread
  static_assert(kChunk * (COB / 8) % kThreads == 0, "dZ staging must tile the workgroup");
  bf16x8 rdz[DZI];
  bf16x8 rx[XI];
  __bf16 rxs[XS];
  auto load = [&](long long r0) {
#pragma unroll
    for (int u = 0; u < DZI; ++u) {
      const int i = threadIdx.x + u * kThreads;
      const int r = i / (COB / 8), cw = i - r * (COB / 8);
      const int co = co0 + cw * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) rdz[u][j] = (__bf16)0.f;
      if (r0 + r < A.R) {
        const __bf16* src = A.dz + (r0 + r) * A.cout + co;
        if ((A.cout & 7) == 0 && co + 8 <= A.cout) {
          rdz[u] = *(const gbf16x8*)(src);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (co + j < A.cout) rdz[u][j] = src[j];
        }
      }
    }
    if constexpr (IM2COL) {
      // im2col: column kk = tap * cin + ci of row r is Xpad[r0 + r + tap][ci]
#pragma unroll
      for (int u = 0; u < XS; ++u) {
        const int i = threadIdx.x + u * kThreads;
        const int r = i >> 5, kk = i & 31;
        const int tap = kk / A.cin, ci = kk - tap * A.cin;
        rxs[u] = (__bf16)0.f;
        if (tap < k && r0 + r + tap < A.x_rows) rxs[u] = A.x[(r0 + r + tap) * A.cin + ci];
      }
    } else {
      // X rows [r0, r0 + 64 + k - 1) x channels [ci0, ci0 + 16)
      const int xr_n = kChunk + k - 1;
#pragma unroll
      for (int u = 0; u < XI; ++u) {
        const int i = threadIdx.x + u * kThreads;
        const int r = i >> 1, half = i & 1;
        const int ci = ci0 + half * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) rx[u][j] = (__bf16)0.f;
        if (i < XROWS * 2 && r < xr_n && r0 + r < A.x_rows) {
          const __bf16* src = A.x + (r0 + r) * A.cin + ci;
          if ((A.cin & 7) == 0 && ci + 8 <= A.cin) {
            rx[u] = *(const gbf16x8*)(src);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (ci + j < A.cin) rx[u][j] = src[j];
          }
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < DZI; ++u) {
      const int i = threadIdx.x + u * kThreads;
      const int r = i / (COB / 8), cw = i - r * (COB / 8);
      *reinterpret_cast<bf16x8*>(dz_lds + r * DZRS + cw * 16) = rdz[u];
    }
    if constexpr (IM2COL) {
#pragma unroll
      for (int u = 0; u < XS; ++u) {
        const int i = threadIdx.x + u * kThreads;
        *reinterpret_cast<__bf16*>(x_lds + (i >> 5) * XRS + (i & 31) * 2) = rxs[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < XI; ++u) {
        const int i = threadIdx.x + u * kThreads;
        if (i < XROWS * 2) *reinterpret_cast<bf16x8*>(x_lds + (i >> 1) * XRS + (i & 1) * 16) = rx[u];
      }
    }
  };
  if (c_begin < c_end) load(c_begin * kChunk);
  for (long long ch = c_begin; ch < c_end; ++ch) {
    __syncthreads();  // previous chunk's reads of the tiles are done
    store();
    __syncthreads();
    if (ch + 1 < c_end) load((ch + 1) * kChunk);  // in flight under this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < kChunk / 32; ++ks) {
      bf16x8 fb[NCO];
#pragma unroll
      for (int c = 0; c < NCO; ++c) fb[c] = tr_frag(dz_lds, DZRS, ks * 32, (wave * NCO + c) * 16);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (IM2COL || t < k) {  // uniform; t stays a compile-time index (acc in registers)
#pragma unroll
          for (int mi = 0; mi < NM; ++mi) {
            const bf16x8 fa = tr_frag(x_lds, XRS, ks * 32 + (IM2COL ? 0 : t), mi * 16);
#pragma unroll
            for (int c = 0; c < NCO; ++c) acc[t][mi][c] = mfma16(fa, fb[c], acc[t][mi][c]);
          }
        }
      }
    }
  }
  // D[m][n]: lane holds rows m = 4h + i (ci or kk), column n = lane & 15 (co)
  const int h = lane >> 4, nn = lane & 15;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (!IM2COL && t >= k) continue;
#pragma unroll
    for (int mi = 0; mi < NM; ++mi)
#pragma unroll
      for (int c = 0; c < NCO; ++c) {
        const int co = co0 + (wave * NCO + c) * 16 + nn;
        if (co >= A.cout) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mi * 16 + 4 * h + i;
          int tap, ci;
          if constexpr (IM2COL) {
            tap = m / A.cin;
            ci = m - tap * A.cin;
            if (tap >= k) continue;
          } else {
            tap = t;
            ci = ci0 + m;
            if (ci >= A.cin) continue;
          }
          const long long e = ((long long)tap * A.cin + ci) * A.cout + co;
          if (A.part != nullptr)
            A.part[(long long)rg * A.k * A.cin * A.cout + e] = acc[t][mi][c][i];
          else
            atomicAdd(A.gw + e, acc[t][mi][c][i]);
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
// head: GAP over time + Dense(C -> 1), BCE on logits, dlogit = (sigmoid - y) / global batch, dense
// gradients.  One wave per sample, lanes over channels; workgroup-level sums, then one atomic per
// channel / scalar per workgroup.
// ---------------------------------------------------------------------------------------------
template <typename T>
struct HeadArgs {
  const T* h;        // (n, L, C) bf16, or fp32 (precision="fp32")
  const float* w;    // (C)
  const float* b;    // (1)
  const float* y;    // (n)
  float* prob;       // (n)
  float* dlog;       // (n)
  float* loss;       // (1) summed BCE
  float* gw;         // (C)
  float* gb;         // (1)
  int n, L, C;
  float inv_gb;
  float* part;       // deterministic mode: per-workgroup records [loss, dense bias, dense weights (C)]
};

template <typename T>
__global__ __launch_bounds__(256) void head_kernel(HeadArgs<T> A) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];  // [4 waves][C] gap, then 2 sums
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s = blockIdx.x * 4 + wave;
  float* gap = hsm + wave * A.C;
  float part = 0.f;
  if (s < A.n) {
    const T* base = A.h + (long long)s * A.L * A.C;
    for (int c = lane; c < A.C; c += 64) {
      float acc = 0.f;
      for (int t = 0; t < A.L; ++t) acc += (float)base[(long long)t * A.C + c];
      const float g = acc / (float)A.L;
      gap[c] = g;
      part += g * A.w[c];
    }
  }
  const float z = wave_sum(part) + A.b[0];
  float dl = 0.f;
  if (s < A.n) {
    const float yv = A.y[s];
    const float p = 1.0f / (1.0f + __expf(-z));
    dl = (p - yv) * A.inv_gb;
    if (lane == 0) {
      A.prob[s] = p;
      A.dlog[s] = dl;
    }
  } else {
    for (int c = lane; c < A.C; c += 64) gap[c] = 0.f;
  }
  float* dls = hsm + 4 * A.C;
  float* wloss = dls + 4;
  if (lane == 0) {
    dls[wave] = dl;
    wloss[wave] = s < A.n ? fmaxf(z, 0.f) - z * A.y[s] + log1pf(__expf(-fabsf(z))) : 0.f;
  }
  __syncthreads();
  float* rec = A.part != nullptr ? A.part + (long long)blockIdx.x * (A.C + 2) : nullptr;
  for (int c = threadIdx.x; c < A.C; c += 256) {
    float g = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < 4; ++w2) g += dls[w2] * hsm[w2 * A.C + c];
    if (rec != nullptr)
      rec[2 + c] = g;
    else
      atomicAdd(A.gw + c, g);
  }
  if (threadIdx.x == 0) {
    const float lsum = (wloss[0] + wloss[1]) + (wloss[2] + wloss[3]);
    const float bsum = (dls[0] + dls[1]) + (dls[2] + dls[3]);
    if (rec != nullptr) {
      rec[0] = lsum;
      rec[1] = bsum;
    } else {
      atomicAdd(A.loss, lsum);
      atomicAdd(A.gb, bsum);
    }
  }
}

// Deterministic mode: column sums of an (nrows, ncols) fp32 partial table in a fixed order, 16 columns x
// 16 row lanes per block (lane j adds rows j, j + 16, ... in fp64, then 16 lane sums in order), written
// to up to three consecutive column segments.
struct RedSeg {
  float* ptr;
  long long cols;
};
struct RedDst {
  RedSeg seg[3];
};

__global__ __launch_bounds__(256) void ordered_reduce_kernel(const float* __restrict__ part, int nrows, long long ncols,
                                                             RedDst d) {
  __shared__ double red[256];
  const int cl = threadIdx.x & 15, lane = threadIdx.x >> 4;
  const long long c = (long long)blockIdx.x * 16 + cl;
  double a = 0.0;
  if (c < ncols)
    for (int r = lane; r < nrows; r += 16) a += (double)part[(long long)r * ncols + c];
  red[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x >= 16 || c >= ncols) return;
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += red[j * 16 + cl];
  long long k = c;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (k < d.seg[q].cols) {
      d.seg[q].ptr[k] = (float)s;
      return;
    }
    k -= d.seg[q].cols;
  }
}

// ---------------------------------------------------------------------------------------------
// pack: per block, fp32 kernel (k, cin, cout) -> forward fragments (nstep, cout16/16, 64, 8) with
// kk = tap*cin + ci, co = 16 ct + (lane & 15), and dgrad fragments of W'[tap'][co][ci] =
// W[k-1-tap'][ci][co] (output channels ci padded to 16).  Zero outside the real ranges.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxBlocks = 48;  // 8 ensemble members x 6 blocks in one member-batched pack
struct PackBlock {
  const float* w;
  __bf16* fwd;
  __bf16* dgr;  // nullptr: no dgrad fragments (block 1)
  int k, cin, cout;
  long long nf, nd;  // elements of each fragment array
};
// + up to kMaxZero buffers zeroed by the rows of blocks past the packs (the training step's
// accumulators: the step's first two graph nodes, one launch)
constexpr int kMaxZero = 48;
struct PackArgs {
  PackBlock b[kMaxBlocks];
  uint32_t* zp[kMaxZero];
  long long zw[kMaxZero];  // 4-byte words
  int nblocks, nzero;
};

__global__ void pack_kernel(PackArgs P) {
  if ((int)blockIdx.y >= P.nblocks) {  // zero rows (block-uniform)
    uint32_t* p = P.zp[blockIdx.y - P.nblocks];
    const long long n = P.zw[blockIdx.y - P.nblocks];
    const long long stride = (long long)gridDim.x * blockDim.x, t0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const long long n4 = (reinterpret_cast<uintptr_t>(p) & 15) == 0 ? n >> 2 : 0;
    for (long long i = t0; i < n4; i += stride) reinterpret_cast<uint4*>(p)[i] = uint4{0u, 0u, 0u, 0u};
    for (long long i = (n4 << 2) + t0; i < n; i += stride) p[i] = 0u;
    return;
  }
  const PackBlock B = P.b[blockIdx.y];
  const long long tot = B.nf + (B.dgr ? B.nd : 0);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const bool is_f = e < B.nf;
    const long long i = is_f ? e : e - B.nf;
    const int ci_ = is_f ? B.cin : B.cout;   // GEMM K channels
    const int co_ = is_f ? B.cout : B.cin;   // GEMM M channels (padded to 16)
    const int j = (int)(i & 7), lane = (int)((i >> 3) & 63);
    const long long fr = i >> 9;
    const int nct = (co_ + 15) / 16;
    const int ct = (int)(fr % nct), s = (int)(fr / nct);
    const int co = 16 * ct + (lane & 15);
    const int kk = 32 * s + 8 * (lane >> 4) + j;
    float v = 0.f;
    if (kk < ci_ * B.k && co < co_) {
      const int tap = kk / ci_, ci = kk - tap * ci_;
      v = is_f ? B.w[((long long)tap * B.cin + ci) * B.cout + co]
               : B.w[((long long)(B.k - 1 - tap) * B.cin + co) * B.cout + ci];
    }
    (is_f ? B.fwd : B.dgr)[i] = (__bf16)v;
  }
}

}  // namespace gwgrad

// ------------------------------------------------------------------------------------------- host
template <int NCO, int KMAX, bool IM2COL>
static void wg_go(const gwgrad::WgArgs& A, int grid, hipStream_t st) {
  hipLaunchKernelGGL((gwgrad::wgrad_kernel<NCO, KMAX, IM2COL>), dim3(grid), dim3(gwgrad::kThreads), 0, st, A);
}

template <int NCO>
static hipError_t wg_dispatch(const gwgrad::WgArgs& A, int grid, bool im2col, hipStream_t st) {
  if (im2col) {
    wg_go<NCO, 1, true>(A, grid, st);
  } else if (A.k <= 3) {
    wg_go<NCO, 3, false>(A, grid, st);
  } else if (A.k <= 5) {
    wg_go<NCO, 5, false>(A, grid, st);
  } else if (A.k <= 9) {
    wg_go<NCO, 9, false>(A, grid, st);
  } else if (A.k <= 15) {
    wg_go<NCO, 15, false>(A, grid, st);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// gw must be zeroed by the caller (the step zeroes the whole flat gradient).
hipError_t ordered_reduce(const float* part, int nrows, long long ncols, gwgrad::RedDst d, hipStream_t st) {
  hipLaunchKernelGGL(gwgrad::ordered_reduce_kernel, dim3((unsigned)((ncols + 15) / 16)), dim3(256), 0, st, part, nrows,
                     ncols, d);
  return hipGetLastError();
}

// out[c] = sum over the nrows rows of part[r][c], in the fixed order of ordered_reduce_kernel
hipError_t launch_ordered_sum(const float* part, int nrows, long long ncols, float* out, hipStream_t st) {
  gwgrad::RedDst d = {};
  d.seg[0] = {out, ncols};
  return ordered_reduce(part, nrows, ncols, d, st);
}

// part (deterministic mode, nullable): room for part_floats partials; the row groups are capped so that
// each writes its own (k, cin, cout) slice, then an ordered reduce writes gw.
hipError_t launch_gt_wgrad(const void* x, long long x_rows, const void* dz, long long R, int cin, int cout, int k,
                           float* gw, hipStream_t st, float* part, long long part_floats) {
  if (R <= 0) return hipSuccess;
  if (k < 1 || k > 15 || cin < 1 || cout < 1) return hipErrorInvalidValue;
  if (x_rows < R + k - 1) return hipErrorInvalidValue;  // every tap's rows must exist
  gwgrad::WgArgs A;
  A.x = reinterpret_cast<const __bf16*>(x);
  A.dz = reinterpret_cast<const __bf16*>(dz);
  A.gw = gw;
  A.R = R;
  A.x_rows = x_rows;
  A.cin = cin;
  A.cout = cout;
  A.k = k;
  A.part = part;
  const bool im2col = cin * k <= 32;
  // co tiles per wave: the fewest padded tile slots (4 waves x NCO per block), then the largest NCO; the
  // accumulators (k x NCO tiles) are capped so a workgroup keeps >= 2 waves per SIMD
  const int co_tiles = (cout + 15) / 16;
  const int nmax = k <= 5 ? 4 : k <= 9 ? 3 : 2;
  int nco = 1;
  for (int c = 2; c <= nmax; ++c) {
    const int slots_c = (co_tiles + 4 * c - 1) / (4 * c) * 4 * c, slots_b = (co_tiles + 4 * nco - 1) / (4 * nco) * 4 * nco;
    if (slots_c <= slots_b) nco = c;
  }
  A.n_ci = im2col ? 1 : (cin + 15) / 16;
  A.n_co = (co_tiles + 4 * nco - 1) / (4 * nco);
  const long long chunks = (R + gwgrad::kChunk - 1) / gwgrad::kChunk;
  // ~2048 workgroups (8 per CU over the 256 CUs), but at least minc chunks each: every workgroup ends
  // with k * 16 * 64 * NCO fp32 atomics, and the chip adds ~1.3 TB/s of atomic bytes, so at 4 chunks
  // per workgroup the k = 9 blocks of ModelSpec(30, 1) spent ~100 us of a ~106 us wgrad on them.
  const long long minc = k <= 3 ? 4 : 2 * k;
  const long long blocks = (long long)A.n_ci * A.n_co;
  long long rg = 2048 / blocks;
  if (rg < 1) rg = 1;
  if (rg > (chunks + minc - 1) / minc) rg = (chunks + minc - 1) / minc;
  const long long wfl = (long long)k * cin * cout;
  if (part != nullptr && rg > part_floats / wfl) rg = part_floats / wfl;  // one partial slice per row group
  if (rg < 1) rg = 1;
  A.chunks_per_wg = (int)((chunks + rg - 1) / rg);
  rg = (chunks + A.chunks_per_wg - 1) / A.chunks_per_wg;
  const long long grid = blocks * rg;
  if (grid > 0x7FFFFFFF) return hipErrorInvalidValue;
  if (part != nullptr && rg * wfl > part_floats) return hipErrorInvalidValue;
  hipError_t e;
  switch (nco) {
    case 1: e = wg_dispatch<1>(A, (int)grid, im2col, st); break;
    case 2: e = wg_dispatch<2>(A, (int)grid, im2col, st); break;
    case 3: e = wg_dispatch<3>(A, (int)grid, im2col, st); break;
    default: e = wg_dispatch<4>(A, (int)grid, im2col, st); break;
  }
  if (e != hipSuccess || part == nullptr) return e;
  gwgrad::RedDst d = {};
  d.seg[0] = {gw, wfl};
  return ordered_reduce(part, (int)rg, wfl, d, st);
}

// part (deterministic mode, nullable): ceil(n / 4) * (C + 2) floats of per-workgroup records.
hipError_t launch_gt_head(const void* h, const float* w, const float* b, const float* y, float* prob, float* dlog,
                          float* loss, float* gw, float* gb, int n, int L, int C, float inv_gb, hipStream_t st,
                          float* part, long long part_floats, int f32) {
  if (n <= 0) return hipSuccess;
  const int nblk = (n + 3) / 4;
  if (part != nullptr && (long long)nblk * (C + 2) > part_floats) return hipErrorInvalidValue;
  const size_t lds = (4 * (size_t)C + 8) * sizeof(float);
  if (f32) {
    gwgrad::HeadArgs<float> A{reinterpret_cast<const float*>(h), w, b, y, prob, dlog, loss, gw, gb, n, L, C, inv_gb, part};
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gwgrad::head_kernel<float>), dim3(nblk), dim3(256), lds, st, A);
  } else {
    gwgrad::HeadArgs<__bf16> A{reinterpret_cast<const __bf16*>(h), w, b, y, prob, dlog, loss, gw, gb, n, L, C, inv_gb,
                               part};
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gwgrad::head_kernel<__bf16>), dim3(nblk), dim3(256), lds, st, A);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || part == nullptr) return e;
  gwgrad::RedDst d = {};
  d.seg[0] = {loss, 1};
  d.seg[1] = {gb, 1};
  d.seg[2] = {gw, C};
  return ordered_reduce(part, nblk, C + 2, d, st);
}

int gt_pack_max_blocks() { return gwgrad::kMaxBlocks; }
int gt_pack_max_zero() { return gwgrad::kMaxZero; }

// blocks: nb descriptors (w, fwd, dgr-or-null, k, cin, cout); nz buffers (ptr, 4-byte words) zeroed in the
// same launch
hipError_t launch_gt_pack(int nb, const float* const* w, void* const* fwd, void* const* dgr, const int* k,
                          const int* cin, const int* cout, hipStream_t st, int nz, void* const* zp,
                          const long long* zw) {
  if (nb < 1 || nb > gwgrad::kMaxBlocks || nz < 0 || nz > gwgrad::kMaxZero) return hipErrorInvalidValue;
  gwgrad::PackArgs P;
  P.nblocks = nb;
  P.nzero = nz;
  for (int i = 0; i < nz; ++i) {
    P.zp[i] = reinterpret_cast<uint32_t*>(zp[i]);
    P.zw[i] = zw[i];
  }
  long long most = 0;
  for (int i = 0; i < nb; ++i) {
    auto& B = P.b[i];
    B.w = w[i];
    B.fwd = reinterpret_cast<__bf16*>(fwd[i]);
    B.dgr = reinterpret_cast<__bf16*>(dgr[i]);
    B.k = k[i];
    B.cin = cin[i];
    B.cout = cout[i];
    B.nf = (long long)((k[i] * cin[i] + 31) / 32) * 512 * ((cout[i] + 15) / 16);
    B.nd = (long long)((k[i] * cout[i] + 31) / 32) * 512 * ((cin[i] + 15) / 16);
    const long long t = B.nf + (B.dgr ? B.nd : 0);
    most = t > most ? t : most;
  }
  for (int i = 0; i < nz; ++i) most = std::max(most, zw[i] / 4);
  long long gx = (most + 255) / 256;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(gwgrad::pack_kernel, dim3((unsigned)gx, nb + nz), dim3(256), 0, st, P);
  return hipGetLastError();
}

}  // namespace apneauq
