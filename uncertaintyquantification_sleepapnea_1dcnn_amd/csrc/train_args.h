// Shared declarations of the layer-wise training kernels (train_conv.hip) and their reductions
// (train_reduce.hip): buffer layout constants, per-layer / per-launch kernel arguments, member-batched
// placement, BN moment helpers and the parameter table.  See train_conv.hip for the design.
#pragma once
#include <type_traits>

#include "common.h"

namespace apneauq {
namespace train {

typedef short v4i16 __attribute__((ext_vector_type(4)));

constexpr int kL = 60, kSR = 64, kSlots = 2, kR = 128, kRT = 8, kHalo = 4, kRows = 136;
constexpr int kRS = 256 * 2 + 32;  // LDS row stride (bytes) of the staged activation tiles
constexpr int kThreads = 256;
constexpr int C[7] = {4, 128, 192, 224, 96, 256, 96};
constexpr int KS[6] = {7, 5, 3, 7, 9, 9};

struct Layer {
  const gbf16x8* wf;   // forward fragments  (ksteps, Cout/16, 64, 8)
  const gbf16x8* wd;   // dgrad fragments    (ksteps', Cin/16, 64, 8)
  const float* bias;
  const float* gamma;
  const float* beta;
  float* mmean;
  float* mvar;
  float* gw;           // dW (k, Cin, Cout) fp32, in the flat gradient buffer
  float* gb;
  float* ggamma;
  float* gbeta;
  __bf16* R;           // PL (rows, C) post-ReLU, pre-BN
  __bf16* dY;          // PL (rows, C) gradient wrt BN output (blocks 1..5)
  __bf16* dZ;          // PL (rows, C) gradient wrt the conv pre-activation, written by dgrad_l (l >= 1)
  double* st;          // [slots][groups][2][C] forward moment sums (sum r, sum r^2), fp64
  double* bst;         // [slots][2][C] backward sums (sum dY, sum dY * xhat), fp64: partial sums of
                       // data-parallel ranks then add exactly (a 2-rank step computes the 1-rank
                       // BN-backward coefficients bit for bit in deterministic mode)
  unsigned thr;        // dropout threshold (16-bit units) and 1/(1-p)
  float dsc;
};

struct Args {
  Layer L[6];
  const __bf16* x;     // PL (rows, 4)
  const float* y;      // labels (B)
  const float* dense_w;
  const float* dense_b;
  float* g_dense_w;
  float* g_dense_b;
  float* logits;       // (B)
  float* dlogit;       // (B)
  float* loss_sum;     // (1)
  int B;               // samples in this launch (T*N for batch-BN MC Dropout)
  int n_win;           // samples per stats group (B for training, N for MC Dropout)
  int groups;          // number of stats groups
  unsigned pass_base;  // dropout pass id of group 0
  unsigned window_offset;
  unsigned long long seed;
  int dropout;
  float inv_count;     // 1 / (samples per group * 60) — BN moment normaliser
  float inv_batch;     // 1 / global batch size — BCE mean
  float eps;
  float momentum;
  const unsigned* pass_dev;  // optional device step counter added to pass_base (HIP-graph replays)
  int st_groups;       // groups the moment buffers are allocated for (>= groups)
  float* wpart;        // wgrad partials [row group][K*Cin*Cout + Cout] (nullptr: fp32 atomics)
  float* det;          // deterministic mode (training, one stats group): per-workgroup / per-sample
                       // partial sums of the BN moments, head and dgrad statistics go here with
                       // plain stores and det_reduce_kernel adds them in a fixed order (nullptr:
                       // atomics, whose summation order varies run to run)
  int shared0;         // batch-BN MC Dropout: block 1 (no dropout before it) is computed once for the
                       // n_win windows (stats group 0, R_0 unencoded, indexed by window) and shared by
                       // every pass; block 2's staging applies block 1's dropout from the hash
  float* tab;          // single-device training: per-layer BN parameter table [6][kTabRows][256] fp32
                       // (mean, rstd, gamma*rstd, beta - mean*gamma*rstd, mean dY, mean dY*xhat), written
                       // once per step by tab_kernel; the ~512 workgroups of each backward kernel read a
                       // few KB instead of each re-summing 16 fp64 slots per channel from the device-
                       // coherent moment buffers (~100 MB per dgrad launch).  nullptr: slot sums
  float* hpart;        // training head: per-workgroup dense-weight / loss / dense-bias sums go to
                       // [kStatSlots][96 + 2] fp32 slots (workgroup % kStatSlots) that bn_finalize adds
                       // in slot order, instead of 256 workgroups' atomics on the same 98 addresses
                       // (nullptr: direct atomics)
  int bwd_self;        // dgrad / wgrad launch flag (not in the ctx): sum the backward BN rows of block l
                       // from bst[l] themselves instead of reading the table rows that wgrad_reduce's
                       // side job writes -- so a wgrad chain on a second stream (GraphedTrainStep
                       // overlap) carries no dependency back into the dgrad chain
};

template <typename T>
__device__ __forceinline__ T gld(const void* p) {
  return *(const __attribute__((address_space(1))) T*)(p);
}

// Member-batched launches (MB = true): a (gx, 1, M) grid runs M ensemble members, each member's Args
// (its own weights, activations, moments and gradients) in a device array read with scalar loads;
// MB = false takes the launch's by-value Args.  Placement is XCD-aware: workgroups are dispatched
// round-robin over the 8 XCDs in linear order, so when M divides 8 member m owns XCDs
// [m * 8/M, (m+1) * 8/M) -- its weights and activations stay in those L2s instead of 8 members'
// working sets thrashing every L2.  pos.bx is the member-local workgroup id (0 .. gx-1) the kernels
// use in place of blockIdx.x, pos.nxcd the XCDs a member spans.
struct MbPos {
  int member, bx, nxcd;
};
template <bool MB>
__device__ __forceinline__ MbPos mb_pos() {
  if constexpr (!MB) {
    return {0, (int)blockIdx.x, 8};
  } else {
    const int M = gridDim.z, gx = gridDim.x;
    if (M <= 8 && (8 % M) == 0 && ((gx * M) & 7) == 0) {
      const int lin = blockIdx.x + gx * blockIdx.z;  // dispatch order
      const int xcd = lin & 7, per = 8 / M;
      return {xcd / per, (lin >> 3) * per + xcd % per, per};
    }
    return {(int)blockIdx.z, (int)blockIdx.x, 8};
  }
}
template <bool MB>
__device__ __forceinline__ const Args& member_args(const Args& a, const Args* __restrict__ am, const MbPos& p) {
  if constexpr (MB)
    return am[p.member];
  else
    return a;
}

// R_l's sign bit = block l's dropout mask (set: dropped); |R_l| is the post-ReLU activation
__device__ __forceinline__ bool bf_dropped(__bf16 v) { return (__builtin_bit_cast(unsigned short, v) & 0x8000u) != 0; }
__device__ __forceinline__ float bf_abs(__bf16 v) {
  return __uint_as_float(((unsigned)__builtin_bit_cast(unsigned short, v) & 0x7FFFu) << 16);
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// A = dropout(BN(R)) of one packed bf16 pair of R: |r| * s + t, or 0 where the sign bit is set
// (dropped, or a pad / out-of-batch row, which the producer writes as -0.0).  7 VALU per pair:
// 2 unpacks, one v_pk_fma_f32, one v_cvt_pk_bf16_f32, v_pk_ashrrev_i16 + not + and for the masks.
__device__ __forceinline__ uint32_t decode_pair(uint32_t d, float s0, float t0, float s1, float t1) {
  const float lo = __builtin_fmaf(__uint_as_float(d << 16), s0, t0);
  const float hi = __builtin_fmaf(__uint_as_float(d & 0xFFFF0000u), s1, t1);
  const bf16x2 p = {(__bf16)lo, (__bf16)hi};
  const s16x2 sm = __builtin_bit_cast(s16x2, d) >> (s16x2){15, 15};
  return __builtin_bit_cast(uint32_t, p) & ~__builtin_bit_cast(uint32_t, sm);
}
constexpr uint32_t kNegZero2 = 0x80008000u;  // a pair of -0.0: "dropped" = decodes to A = 0

// LDS tile addressing: row-major (the transposed operand reads need no swizzle: see tr_frag)
__device__ __forceinline__ int lds_off(int r, int b, int rs) { return r * rs + b; }

__device__ __forceinline__ int row_sample(int grow) { return (grow - kHalo) >> 6; }  // may be -1 / >= B
__device__ __forceinline__ int row_time(int grow) { return (grow - kHalo) & 63; }

// BN moment sums are accumulated into kStatSlots interleaved copies (slot = workgroup % kStatSlots)
// so that the ~512 workgroups of a layer do not serialise on the same 2*C L2 atomic addresses;
// readers add the slots.  Layout per layer: st[slot][group][2][C], bst[slot][2][C].
// s_setprio 1 around the forward conv MFMAs: the co-resident workgroup's staging / copy-out VALU gets
// the leftover issue slots (-1.5 % per batch-BN chunk, profiles/batch_bn_fwd_r2.md).
constexpr bool kFwdPrio = true;

constexpr int kStatSlots = 16;
constexpr int kHeadRec = 2 + 3 * 96;  // deterministic head record per sample: loss, dlogit, dW, sum dY, sum dY xhat
// slot stride of the moment buffers: the ALLOCATED group count (a last MC-Dropout chunk may run fewer
// groups while block 1's shared moments, written by the first chunk, keep their slots)
__device__ __forceinline__ int st_stride(const Args& A, int Cc) { return A.st_groups * 2 * Cc; }
__device__ __forceinline__ float slot_sum(const float* p, int stride) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kStatSlots; ++i) s += p[i * stride];
  return s;
}
// All kStatSlots loads are issued before the first add: the training kernels run one tile per
// workgroup at batch 1024, so their per-channel prologue (2-6 of these sums per channel) is exposed
// latency -- 4 dependent round trips per sum cost dgrad 6-9 us (round 2, session 3).
__device__ __forceinline__ double slot_sumd(const double* p, int stride) {
  double v[kStatSlots];
#pragma unroll
  for (int i = 0; i < kStatSlots; ++i) v[i] = p[i * stride];
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kStatSlots; ++i) s += v[i];
  return s;
}
// stats group holding block l's moments for pass group g (block 1 is shared by all passes in shared0 mode)
__device__ __forceinline__ int stat_group(const Args& A, int l, int g) { return (l == 0 && A.shared0) ? 0 : g; }
// biased batch moments of channel c of block l, stats group g (fp64 merge, fp32 results)
__device__ __forceinline__ void bn_moments(const Args& A, int l, int g, int c, float& mu, float& var) {
  const int Cc = C[l + 1];
  const int ss = st_stride(A, Cc);
  const int gg = stat_group(A, l, g);
  const double s1 = slot_sumd(A.L[l].st + (gg * 2 + 0) * Cc + c, ss);
  const double s2 = slot_sumd(A.L[l].st + (gg * 2 + 1) * Cc + c, ss);
  const double m = s1 * (double)A.inv_count;
  mu = (float)m;
  var = (float)fmax(s2 * (double)A.inv_count - m * m, 0.0);
}

// Per-channel BN affine of block l for stats group g, into LDS: s[c], t[c], mean[c], rstd[c].
__device__ __forceinline__ void bn_affine_to_lds(const Args& A, int l, int g, float* s, float* t, float* mean,
                                                 float* rstd) {
  const int Cc = C[l + 1];
  const Layer& Ly = A.L[l];
  for (int c = threadIdx.x; c < Cc; c += kThreads) {
    float mu, var;
    bn_moments(A, l, g, c, mu, var);
    const float rs = rsqrtf(var + A.eps);
    const float sc = Ly.gamma[c] * rs;
    s[c] = sc;
    t[c] = Ly.beta[c] - mu * sc;
    if (mean) mean[c] = mu;
    if (rstd) rstd[c] = rs;
  }
}

// Per-channel batch mean and 1/sqrt(var + eps) of block l, stats group g, into LDS.
__device__ __forceinline__ void bn_stats_to_lds(const Args& A, int l, int g, float* mean, float* rstd) {
  const int Cc = C[l + 1];
  for (int c = threadIdx.x; c < Cc; c += kThreads) {
    float mu, var;
    bn_moments(A, l, g, c, mu, var);
    mean[c] = mu;
    rstd[c] = rsqrtf(var + A.eps);
  }
}

// Parameter table (Args::tab): rows of T[l][kTabRows][256]
constexpr int kTabRows = 6, kTabMean = 0, kTabRstd = 1, kTabS = 2, kTabT = 3, kTabMdy = 4, kTabMdyx = 5;
__device__ __forceinline__ const float* tab_row(const Args& A, int l, int row) {
  return A.tab + (l * kTabRows + row) * 256;
}

// Forward rows of T[l] (stats group 0) from the fp64 slots (tab_kernel).
__device__ __forceinline__ void tab_write_fwd(const Args& A, int l) {
  const int Cc = C[l + 1], c = threadIdx.x;
  if (c >= Cc) return;
  float mu, var;
  bn_moments(A, l, 0, c, mu, var);
  const float rs = rsqrtf(var + A.eps), sc = A.L[l].gamma[c] * rs;
  float* t = A.tab + l * kTabRows * 256;
  t[kTabMean * 256 + c] = mu;
  t[kTabRstd * 256 + c] = rs;
  t[kTabS * 256 + c] = sc;
  t[kTabT * 256 + c] = A.L[l].beta[c] - mu * sc;
}

// Backward rows of T[l] (mean dY, mean dY*xhat) from bst[l] (tab_kernel).
__device__ __forceinline__ void tab_write_bwd(const Args& A, int l) {
  const int Cc = C[l + 1], c = threadIdx.x;
  if (c >= Cc) return;
  float* t = A.tab + l * kTabRows * 256;
  t[kTabMdy * 256 + c] = (float)(slot_sumd(A.L[l].bst + c, 2 * Cc) * (double)A.inv_count);
  t[kTabMdyx * 256 + c] = (float)(slot_sumd(A.L[l].bst + Cc + c, 2 * Cc) * (double)A.inv_count);
}

__device__ __forceinline__ unsigned layer_sample_key(const Args& A, int l, int sample) {
  const unsigned g = (unsigned)(sample / A.n_win);
  const unsigned w = (unsigned)(sample - (int)g * A.n_win);
  const unsigned pb = A.pass_base + (A.pass_dev != nullptr ? *A.pass_dev : 0u);
  return sample_key(stream_key(A.seed, l, pb + g), A.window_offset + w);
}

// ---- reductions (train_reduce.hip)
struct TabBwd {  // backward rows of one block's parameter table entry (wgrad_reduce's side job)
  const double* bst;  // [kStatSlots][2][cc]
  float* mdy;
  float* mdyx;
  int cc;
  float inv_count;
};
// One layer's wgrad partial reduction, run as a side job of another launch (single-device steps:
// dgrad<l-1> reduces wgrad<l>'s partials for l = 2..5, step_reduce_kernel those of wgrad<1> and wgrad<0>
// next to the BN finalize) -- the same column split and summation order as wgrad_reduce_kernel's, so the gradient
// is bitwise the one the separate reduce launch computes.  part == nullptr: no job.
struct RedJob {
  const float* part;  // [rgs][kcc + cout]
  float* gw;
  float* gb;
  int rgs, kcc, cout, J, blocks;  // J threads per float4 column; blocks = the reduce launch's grid
};
// dW, db = sum over the row groups of the wgrad partials in a fixed order: deterministic, and cheaper
// than the ~K*Cin*Cout fp32 atomics per row group it replaces (25-35 us of a 70-80 us wgrad at batch
// 1024, profiles/train_step_r2.md).  Workgroup bx of nbx (256 threads) covers 256/J float4 columns at a
// time with J threads per column: thread j sums row groups j, j + J, ... (8 loads in flight), then the
// J partials are added in j order through LDS (red: 256 f32x4).  J > 1 when the row groups outnumber
// the columns' parallelism (block 1: 512 row groups of 928 float4 columns took 26 us with one thread
// per column).  The result depends on J only, not on which launch or workgroup runs a column.
__device__ __forceinline__ void wgrad_reduce_cols(const RedJob& jb, int bx, int nbx, f32x4* red) {
  const int S4 = (jb.kcc + jb.cout) >> 2;  // Cout is a multiple of 4
  const int J = jb.J, rgs = jb.rgs, kcc = jb.kcc;
  const int ncol = 256 / J;
  const int cl = threadIdx.x % ncol, j = threadIdx.x / ncol;
  const f32x4* p4 = reinterpret_cast<const f32x4*>(jb.part);
  for (int base = bx * ncol; base < S4; base += nbx * ncol) {  // workgroup-uniform
    const int e4 = base + cl;
    // 8 loads in flight per batch, the last (partial) batch predicated instead of a serial remainder
    // loop whose loads each waited for the previous add (21 row groups per thread at J = 4: 2 batches +
    // 5 dependent loads).  (16 per batch measured slower: 48.6 -> 54.7 us of reduce per step at batch 1024.)
    f32x4 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (e4 < S4) {
      int r = j;
      for (; r + 7 * J < rgs; r += 8 * J) {
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += p4[(long long)(r + q * J) * S4 + e4];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (r + q * J < rgs) acc[q] += p4[(long long)(r + q * J) * S4 + e4];
    }
    red[threadIdx.x] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __syncthreads();
    if (j == 0 && e4 < S4) {
      f32x4 s = red[cl];
      for (int q = 1; q < J; ++q) s += red[q * ncol + cl];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = 4 * e4 + i;
        if (e < kcc)
          jb.gw[e] = s[i];
        else
          jb.gb[e - kcc] = s[i];
      }
    }
    __syncthreads();
  }
}

// The table's backward rows (mean dY, mean dY*xhat) of one block from its fp64 slots.
__device__ __forceinline__ void tab_bwd_rows(const TabBwd& tb) {
  const int c = threadIdx.x;
  if (c < tb.cc) {
    tb.mdy[c] = (float)(slot_sumd(tb.bst + c, 2 * tb.cc) * (double)tb.inv_count);
    tb.mdyx[c] = (float)(slot_sumd(tb.bst + tb.cc + c, 2 * tb.cc) * (double)tb.inv_count);
  }
}

struct DetSeg {
  void* ptr;
  int cols;
  int f64;
};
struct DetDst {  // up to four destination segments (consecutive column ranges; fp64 or fp32 stores)
  DetSeg seg[4];
};
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, int rgs, int kcc, int cout, float* __restrict__ gw,
                                    float* __restrict__ gb, int J, TabBwd tb);
__global__ void wgrad_reduce_mb_kernel(const Args* __restrict__ Am, int l, int rgs, int kcc, int cout, int J, int side);
// deterministic column sums: kDetSeg row segments (pass 1, fp64 scratch [kDetSeg][w] behind the partial
// table), then the segments in order (pass 2); w <= kDetMaxW
constexpr int kDetSeg = 32, kDetMaxW = 512;
__global__ void det_pass1_kernel(const float* __restrict__ part, int n, int w, double* __restrict__ scr);
__global__ void det_pass2_kernel(const double* __restrict__ scr, int w, DetDst d);
__global__ void det_pass1_mb_kernel(const Args* __restrict__ Am, int n, int w, long long sbase);
__global__ void det_pass2_mb_kernel(const Args* __restrict__ Am, int op, int l, int w, long long sbase);
template <bool MB>
__global__ void bn_finalize_kernel(Args A_, const Args* __restrict__ Am, int update_moving, int grads);
// single-device fused step tail: BN finalize (blocks 0-5), then the partial reductions of blocks 2 and 1
__global__ void step_reduce_kernel(Args A, RedJob j1, RedJob j0, int update_moving, int grads);

}  // namespace train
}  // namespace apneauq
