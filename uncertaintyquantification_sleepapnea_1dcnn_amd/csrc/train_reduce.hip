// Reductions of the layer-wise training step (train_conv.hip): the wgrad partial sums, the
// deterministic-mode column sums and the BN finalize (moving averages, dgamma / dbeta) -- the
// gradient / BatchNorm bookkeeping of Keras model.fit (/root/reference/models/cnn_baseline_train.py:
// 100-102 compile with Adam + BCE, :210-217 fit; Keras BatchNormalization momentum 0.99, eps 1e-3).
#include "train_args.h"

namespace apneauq {
namespace train {

// The separate reduce launch (wgrad_reduce_cols, train_args.h) with its optional side job: the table's
// backward rows of the block the NEXT dgrad / wgrad read.
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ part, int rgs, int kcc, int cout,
                                                  float* __restrict__ gw, float* __restrict__ gb, int J,
                                                  const TabBwd& tb, int bx, int nbx, bool side_block) {
  __shared__ f32x4 red[256];
  if (side_block) {
    tab_bwd_rows(tb);
    return;
  }
  const RedJob jb = {part, gw, gb, rgs, kcc, cout, J, nbx};
  wgrad_reduce_cols(jb, bx, nbx, red);
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int rgs, int kcc, int cout,
                                                           float* __restrict__ gw, float* __restrict__ gb, int J,
                                                           TabBwd tb) {
  if (blockIdx.y == 1 && blockIdx.x != 0) return;
  wgrad_reduce_body(part, rgs, kcc, cout, gw, gb, J, tb, blockIdx.x, gridDim.x, blockIdx.y == 1);
}

// member-batched: the member's partial slots (written by its wgrad on its XCDs), gradients and table
// rows from its Args; with the table the last x-block of each member does the side job
__global__ __launch_bounds__(256) void wgrad_reduce_mb_kernel(const Args* __restrict__ Am, int l, int rgs, int kcc,
                                                              int cout, int J, int side) {
  const MbPos pos = mb_pos<true>();
  const Args& A = Am[pos.member];
  TabBwd tb = {};
  if (side) {
    tb.bst = A.L[l - 1].bst;
    tb.cc = C[l];
    tb.mdy = A.tab + ((l - 1) * kTabRows + kTabMdy) * 256;
    tb.mdyx = A.tab + ((l - 1) * kTabRows + kTabMdyx) * 256;
    tb.inv_count = A.inv_count;
  }
  const int nbx = gridDim.x - (side ? 1 : 0);
  wgrad_reduce_body(A.wpart, rgs, kcc, cout, A.L[l].gw, A.L[l].gb, J, tb, pos.bx, nbx, side && pos.bx == nbx);
}

// ------------------------------------------------------------------------------------------------
// BN finalize: moving averages (Keras momentum update on batch moments) and dgamma / dbeta.
// ------------------------------------------------------------------------------------------------
// Deterministic mode: column sums of an (n, w) row-major fp32 partial table in a fixed order (fp64
// accumulation), scattered to up to four destination segments (consecutive column ranges; fp64 or
// fp32 stores).  Two passes, both with a fixed association: pass 1 splits the rows into kDetSeg
// contiguous segments, each summed by 4 threads (row quarters, sequential) per column and combined
// as (q0 + q1) + (q2 + q3) into scratch[segment][column]; pass 2 adds the kDetSeg segment sums of a
// column in segment order.  (One thread per column over all rows -- the first version -- left the
// ~2-4 workgroups of a reduce latency-bound: the deterministic step took 1.8x / 2.2x the atomic one
// at batch 1024 / 8192.)

__device__ __forceinline__ void det_pass1(const float* __restrict__ part, int n, int w, double* __restrict__ scr,
                                          int cb, int seg) {
  __shared__ double red[4][64];
  const int cl = threadIdx.x & 63, sub = threadIdx.x >> 6, c = cb * 64 + cl;
  const int r0 = (int)((long long)n * seg / kDetSeg), r1 = (int)((long long)n * (seg + 1) / kDetSeg);
  const int s0 = r0 + (r1 - r0) * sub / 4, s1 = r0 + (r1 - r0) * (sub + 1) / 4;
  double acc = 0.0;
  if (c < w) {
#pragma unroll 8
    for (int i = s0; i < s1; ++i) acc += (double)part[(long long)i * w + c];
  }
  red[sub][cl] = acc;
  __syncthreads();
  if (sub == 0 && c < w) scr[(long long)seg * w + c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

__device__ __forceinline__ void det_pass2(const double* __restrict__ scr, int w, const DetDst& d, int c) {
  double acc = 0.0;
#pragma unroll 8
  for (int sg = 0; sg < kDetSeg; ++sg) acc += scr[(long long)sg * w + c];
  int k = c;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (k < d.seg[q].cols) {
      if (d.seg[q].f64)
        reinterpret_cast<double*>(d.seg[q].ptr)[k] = acc;
      else
        reinterpret_cast<float*>(d.seg[q].ptr)[k] = (float)acc;
      return;
    }
    k -= d.seg[q].cols;
  }
}

// grid (ceil(w / 64), kDetSeg), 256 threads
__global__ __launch_bounds__(256) void det_pass1_kernel(const float* __restrict__ part, int n, int w,
                                                        double* __restrict__ scr) {
  det_pass1(part, n, w, scr, blockIdx.x, blockIdx.y);
}
__global__ __launch_bounds__(256) void det_pass2_kernel(const double* __restrict__ scr, int w, DetDst d) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < w) det_pass2(scr, w, d, c);
}

// member-batched: member blockIdx.z's partial table, scratch and destinations (from its Args) of the
// reduce that follows op 0 (forward of layer l: the moments of block l), 1 (head: loss, dense grads,
// block-6 backward sums) or 2 (dgrad of layer l: backward sums of block l - 1); the same passes as the
// single-model reduce, so member-batched deterministic steps equal single-model ones bitwise
__global__ __launch_bounds__(256) void det_pass1_mb_kernel(const Args* __restrict__ Am, int n, int w, long long sbase) {
  const Args& A = Am[blockIdx.z];
  det_pass1(A.det, n, w, reinterpret_cast<double*>(A.det + sbase), blockIdx.x, blockIdx.y);
}
__global__ __launch_bounds__(256) void det_pass2_mb_kernel(const Args* __restrict__ Am, int op, int l, int w,
                                                           long long sbase) {
  const Args& A = Am[blockIdx.z];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= w) return;
  DetDst d = {};
  if (op == 0) {
    d.seg[0] = {A.L[l].st, w, 1};
  } else if (op == 1) {
    d.seg[0] = {A.loss_sum, 1, 0};
    d.seg[1] = {A.g_dense_b, 1, 0};
    d.seg[2] = {A.g_dense_w, C[6], 0};
    d.seg[3] = {A.L[5].bst, 2 * C[6], 1};
  } else {
    d.seg[0] = {A.L[l - 1].bst, w, 1};
  }
  det_pass2(reinterpret_cast<const double*>(A.det + sbase), w, d, c);
}

__device__ __forceinline__ void bn_finalize_body(const Args& A, int l, int update_moving, int grads) {
  const Layer& Ly = A.L[l];
  const int Cc = (l == 0) ? C[1] : (l == 1) ? C[2] : (l == 2) ? C[3] : (l == 3) ? C[4] : (l == 4) ? C[5] : C[6];
  for (int c = threadIdx.x; c < Cc; c += blockDim.x) {
    if (update_moving) {
      for (int g = 0; g < A.groups; ++g) {  // one Keras call (= one moving update) per group
        float mu, var;
        bn_moments(A, l, g, c, mu, var);
        Ly.mmean[c] = Ly.mmean[c] * A.momentum + mu * (1.f - A.momentum);
        Ly.mvar[c] = Ly.mvar[c] * A.momentum + var * (1.f - A.momentum);
      }
    }
    if (grads) {
      Ly.gbeta[c] = (float)slot_sumd(Ly.bst + c, 2 * Cc);
      Ly.ggamma[c] = (float)slot_sumd(Ly.bst + Cc + c, 2 * Cc);
    }
  }
  if (grads && l == 5 && A.hpart != nullptr) {  // the head's slotted sums, in slot order
    for (int c = threadIdx.x; c < Cc + 2; c += blockDim.x) {
      float v = 0.f;
      for (int sl = 0; sl < kStatSlots; ++sl) v += A.hpart[sl * (Cc + 2) + c];
      if (c < Cc)
        A.g_dense_w[c] = v;
      else if (c == Cc)
        *A.loss_sum = v;
      else
        *A.g_dense_b = v;
    }
  }
}

template <bool MB>
__global__ void bn_finalize_kernel(Args A_, const Args* __restrict__ Am, int update_moving, int grads) {
  const MbPos pos = mb_pos<MB>();
  bn_finalize_body(member_args<MB>(A_, Am, pos), pos.bx, update_moving, grads);
}

// Single-device step tail (one launch instead of the reduces of blocks 2 and 1 plus the finalize): the
// finalize of block b in workgroup b < 6, then the wgrad partial reductions of block 2 (j1, the shared
// partial region) and block 1 (j0, its own region: wgrad_0 runs after wgrad_1 without a dgrad between).
__global__ __launch_bounds__(256) void step_reduce_kernel(Args A, RedJob j1, RedJob j0, int update_moving, int grads) {
  __shared__ f32x4 red[256];
  const int b = blockIdx.x;
  if (b < 6) {
    bn_finalize_body(A, b, update_moving, grads);
  } else if (b < 6 + j1.blocks) {
    wgrad_reduce_cols(j1, b - 6, j1.blocks, red);
  } else {
    wgrad_reduce_cols(j0, b - 6 - j1.blocks, j0.blocks, red);
  }
}

template __global__ void bn_finalize_kernel<false>(Args, const Args* __restrict__, int, int);
template __global__ void bn_finalize_kernel<true>(Args, const Args* __restrict__, int, int);

}  // namespace train
}  // namespace apneauq
