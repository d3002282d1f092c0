// Layer-wise inference kernels for ANY ModelSpec (gfx950 / MI355X): the opt-in MaxPool1D variant
// (north star "Conv1D -> BN -> ReLU -> MaxPool1D -> Dropout"), other window shapes
// (the "30 s single-channel" config: L = 30, C = 1), other filter / kernel sizes.
//
// The fused whole-network kernel (fused_forward.hip) is specialised to the reference's (60, 4)
// no-pool architecture; this path trades its LDS residency for generality:
//
//   conv_block_kernel: one Conv1D(relu, same) -> BN(running) -> [MaxPool1D(2)] -> [Dropout] block as
//     an implicit GEMM on v_mfma_f32_16x16x32_bf16.  D^T[co][row] = W^T[co][k] * X^T[k][row] with
//     k = tap*Cin + ci; the weights are pre-packed A fragments (ops/fused.py:pack_conv_fragments, Cout
//     zero-padded to 16), the activations are gathered straight from global memory (16-B loads when
//     Cin % 8 == 0, so the 8 k of a lane lie in one tap; element loads otherwise).  Each lane's
//     accumulator holds one time step x 4 channels, so the epilogue -- the bias + ReLU + BN affine
//     folded into fma + med3, the 2:1 max pool as a lane-pair exchange (rows t, t^1 sit in lanes
//     l, l^1), the counter-based dropout (ops/rng.py, keyed by the pooled time step) -- runs in
//     registers and writes bf16 (N, L_out, Cout).
//   head_kernel: GAP over time + Dense(C -> 1) (+ sigmoid), one wave per sample.
//
// Rows: sample n, step t map to GEMM row n*Lp + t, Lp = L rounded up to even when pooling (pairs
// never straddle a 16-row tile).  A workgroup is 2 x 2 waves over 128 rows x 128 channels; each wave
// owns 4 row tiles x 4 channel tiles, so a k-step costs 4 activation gathers + 4 weight-fragment
// loads for 16 MFMAs (row gathers are shared through L1 by the two waves of a row half).
#include <cstdlib>

#include "common.h"

#include <type_traits>

namespace apneauq {
namespace generic {

struct ConvArgs {
  const __bf16* x;        // (N, L, Cin) bf16
  const bf16x8* wfrag;    // (nstep, Cout_pad/16, 64, 8)
  const float* epi;       // (8, Cout_pad): s, t', lo, hi, then the same x 1/(1-rate)
  __bf16* y;              // (N, Lout, Cout)
  int n, L, Lp, cin, cout, cout_pad, ksize, nstep, lout;
  int pool, dropout;
  unsigned thr;           // 16-bit dropout threshold
  int layer;              // dropout stream layer id
  int n_win;              // samples per pass (sample s: pass s / n_win, window s % n_win)
  unsigned pass_offset, window_offset;
  unsigned long long seed;
  int in_rs, in_off;      // input row addressing: sample n, step t at row n * in_rs + in_off + t
  float* stats;           // kTrain: BN moment sums (kStatSlots, 2, Cout); deterministic mode: (2 grid.x, 2, Cout),
                          // one slot per (workgroup, wave row) written with plain stores
  int det;
  long long x_rows;       // rows of the input buffer (staging bound)
  int lds_rows, lds_stride;  // conv_lds_kernel: staged rows, bytes per LDS row
};

// Epilogue modes: kInfer = bias + ReLU + BN(running) [+ pool] [+ dropout] (the folded epi rows);
// kTrain = relu(acc + bias) stored as the pre-BN activation z, with the per-channel BN moments
// (sum, sum of squares) accumulated into kStatSlots interleaved copies; kLinear = acc as is (dgrad).
enum { kInfer = 0, kTrain = 1, kLinear = 2 };
constexpr int kStatSlots = 16;

constexpr int kRT = 4, kCT = 4;  // row / channel tiles per wave; a workgroup is 2 x 2 waves

// Epilogue of one wave: acc[c][r] holds rows (rn[r], rt[r]) x channels ct*16 + 4h .. +3 per lane.
template <int MODE>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& A, f32x4 (&acc)[kCT][kRT], const int (&rn)[kRT],
                                              const int (&rt)[kRT], const bool (&rok)[kRT], int ct0, int nct,
                                              int m, int h) {
  if constexpr (MODE != kInfer) {
    // training / dgrad epilogue: no pool, no dropout; y is (N, L, Cout)
    float* st = A.stats + (long long)(A.det ? blockIdx.x * 2 + (threadIdx.x >> 7) : blockIdx.x % kStatSlots) * 2 * A.cout;
#pragma unroll
    for (int c = 0; c < kCT; ++c) {
      const int ct = ct0 + c;
      if (ct >= nct) break;  // wave-uniform
      const int co0 = ct * 16 + 4 * h;
      const bool cok = co0 < A.cout;
      float bi[4] = {0.f, 0.f, 0.f, 0.f};
      if (MODE == kTrain && cok) {
#pragma unroll
        for (int i = 0; i < 4; ++i) bi[i] = A.epi[co0 + i];
      }
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < kRT; ++r) {
        f32x4 v = acc[c][r];
        if constexpr (MODE == kTrain) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = fmaxf(v[i] + bi[i], 0.f);
            const float u = rok[r] ? v[i] : 0.f;
            s1[i] += u;
            s2[i] += u * u;
          }
        }
        if (rok[r] && cok) {
          __bf16* dst = A.y + ((long long)rn[r] * A.L + rt[r]) * A.cout + co0;
          *reinterpret_cast<bf16x4*>(dst) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
        }
      }
      if constexpr (MODE == kTrain) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          s1[i] = group16_sum(s1[i]);
          s2[i] = group16_sum(s2[i]);
        }
        if (m == 0 && cok) {
          if (A.det) {
            *reinterpret_cast<f32x4*>(st + co0) = f32x4{s1[0], s1[1], s1[2], s1[3]};
            *reinterpret_cast<f32x4*>(st + A.cout + co0) = f32x4{s2[0], s2[1], s2[2], s2[3]};
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              atomicAdd(st + co0 + i, s1[i]);
              atomicAdd(st + A.cout + co0 + i, s2[i]);
            }
          }
        }
      }
    }
    return;
  }
  // epilogue: per row tile, the lane holds row (n, t) x channels co0 .. co0+3 of each channel tile
  const float* epi = A.epi + (A.dropout ? 4 * A.cout_pad : 0);
#pragma unroll
  for (int r = 0; r < kRT; ++r) {
    const int n = rn[r], t = rt[r];
    unsigned key = 0u;
    if (A.dropout) {
      const unsigned pass = (unsigned)(n / A.n_win), win = (unsigned)(n - (int)pass * A.n_win);
      key = sample_key(stream_key(A.seed, (unsigned)A.layer, A.pass_offset + pass), A.window_offset + win);
    }
    const int tout = A.pool ? (t >> 1) : t;
    const bool store = rok[r] && (!A.pool || ((t & 1) == 0 && tout < A.lout));
#pragma unroll
    for (int c = 0; c < kCT; ++c) {
      const int ct = ct0 + c;
      if (ct >= nct) break;  // wave-uniform
      const int co0 = ct * 16 + 4 * h;
      f32x4 v = acc[c][r];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sc = epi[co0 + i], sh = epi[A.cout_pad + co0 + i];
        const float lo = epi[2 * A.cout_pad + co0 + i], hi = epi[3 * A.cout_pad + co0 + i];
        v[i] = __builtin_amdgcn_fmed3f(__builtin_fmaf(v[i], sc, sh), lo, hi);
      }
      if (A.pool) {  // MaxPool1D(2, valid) after BN: rows t and t^1 live in lanes l and l^1
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], dpp_mov<0xB1>(v[i]));  // DPP quad_perm [1,0,3,2]
      }
      if (A.dropout) {
        const unsigned b01 = dropout_bits2(key, (unsigned)tout, (unsigned)co0);
        const unsigned b23 = dropout_bits2(key, (unsigned)tout, (unsigned)co0 + 2);
        v[0] = (b01 & 0xFFFFu) >= A.thr ? v[0] : 0.f;
        v[1] = (b01 >> 16) >= A.thr ? v[1] : 0.f;
        v[2] = (b23 & 0xFFFFu) >= A.thr ? v[2] : 0.f;
        v[3] = (b23 >> 16) >= A.thr ? v[3] : 0.f;
      }
      if (store && co0 < A.cout) {
        __bf16* dst = A.y + ((long long)n * A.lout + tout) * A.cout + co0;
        *reinterpret_cast<bf16x4*>(dst) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
      }
    }
  }
}

template <bool VEC, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void conv_block_kernel(ConvArgs A) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, h = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const long long rows = (long long)A.n * A.Lp;
  const long long row_base = (long long)blockIdx.x * (2 * kRT * 16) + wr * (kRT * 16);
  const int nct = A.cout_pad / 16;
  const int ct0 = (blockIdx.y * 2 + wc) * kCT;
  if (ct0 >= nct) return;  // wave-uniform: no channel tile for this wave (no barriers below)
  const int pad = (A.ksize - 1) / 2;
  const int K = A.ksize * A.cin;

  // this lane's B rows (one per row tile): sample n, step t
  int rn[kRT], rt[kRT];
  bool rok[kRT];
#pragma unroll
  for (int r = 0; r < kRT; ++r) {
    const long long row = row_base + r * 16 + m;
    const bool ok = row < rows;
    rn[r] = ok ? (int)(row / A.Lp) : 0;
    rt[r] = ok ? (int)(row - (long long)rn[r] * A.Lp) : 0;
    rok[r] = ok && rt[r] < A.L;
  }

  f32x4 acc[kCT][kRT];
#pragma unroll
  for (int c = 0; c < kCT; ++c)
#pragma unroll
    for (int r = 0; r < kRT; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (tap, ci) of k = 32 s + 8 h, advanced incrementally (no per-step division)
  int tap = (8 * h) / A.cin, ci = 8 * h - tap * A.cin;
  // weight fragments of k-step s + 1 are loaded while step s runs (as in conv_lds_kernel)
  const gbf16x8* wf = (const gbf16x8*)A.wfrag + (long long)ct0 * 64 + lane;
  const int nc = nct - ct0 < kCT ? nct - ct0 : kCT;  // wave-uniform
  bf16x8 a[kCT];
#pragma unroll
  for (int c = 0; c < kCT; ++c) {
    if (c < nc) {
      a[c] = wf[c * 64];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[c][j] = (__bf16)0.f;
    }
  }
  for (int s = 0; s < A.nstep; ++s) {
    const int kk0 = 32 * s + 8 * h;
    // (the element-gather variant has no registers to spare for the prefetch: it loads step s here)
    bf16x8 an[kCT];
    const gbf16x8* wn = wf + (long long)(VEC ? (s + 1 < A.nstep ? s + 1 : s) : s) * nct * 64;
#pragma unroll
    for (int c = 0; c < kCT; ++c) {
      if constexpr (VEC)
        an[c] = c < nc ? wn[c * 64] : a[c];
      else if (c < nc)
        a[c] = wn[c * 64];
    }
    bf16x8 b[kRT];
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      const __bf16* xs = A.x + ((long long)rn[r] * A.in_rs + A.in_off) * A.cin;
      if constexpr (VEC) {
        const int ts = rt[r] + tap - pad;
        if (rok[r] && kk0 < K && ts >= 0 && ts < A.L) {
          b[r] = *(const gbf16x8*)(xs + (long long)ts * A.cin + ci);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) b[r][j] = (__bf16)0.f;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int kk = kk0 + j;
          const int tp = kk / A.cin, cc = kk - tp * A.cin;
          const int ts = rt[r] + tp - pad;
          b[r][j] = (rok[r] && kk < K && ts >= 0 && ts < A.L) ? xs[(long long)ts * A.cin + cc] : (__bf16)0.f;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < kCT; ++c) {
      if (c < nc) {  // wave-uniform
#pragma unroll
        for (int r = 0; r < kRT; ++r) acc[c][r] = mfma16(a[c], b[r], acc[c][r]);
      }
    }
    if constexpr (VEC) {
#pragma unroll
      for (int c = 0; c < kCT; ++c) a[c] = an[c];
      ci += 32;
      while (ci >= A.cin) {
        ci -= A.cin;
        ++tap;
      }
    }
  }

  conv_epilogue<MODE>(A, acc, rn, rt, rok, ct0, nct, m, h);
}

// LDS-staged variant (Cin % 8 == 0, host-checked LDS budget): the workgroup's input rows -- one
// contiguous range of the (row-addressed) input, 128 output rows plus the halo and any per-sample
// padding rows in between -- are staged once into LDS with coalesced 16-B loads, and the K loop
// reads B fragments with ds_read_b128 instead of one 16-B global gather per lane, row tile and
// k-step.  Taps that cross a sample boundary are masked per lane (t + tap - pad outside [0, L)).
// The row stride is padded by 16 B so the 16 rows a lane group reads fall into different banks.
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void conv_lds_kernel(ConvArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, h = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const long long rows = (long long)A.n * A.Lp;
  const long long wg_row0 = (long long)blockIdx.x * (2 * kRT * 16);
  const int pad = (A.ksize - 1) / 2;
  const int K = A.ksize * A.cin;
  // first input row the workgroup can touch: (sample, step) of its first output row, minus the halo
  const int n0 = (int)(wg_row0 / A.Lp), t0 = (int)(wg_row0 - (long long)n0 * A.Lp);
  const long long xbase = (long long)n0 * A.in_rs + A.in_off + t0 - pad;
  const int cpr = A.cin >> 3;  // 16-B chunks per row
  for (int i = threadIdx.x; i < A.lds_rows * cpr; i += 256) {
    const int lr = i / cpr, cc = i - lr * cpr;
    const long long xr = xbase + lr;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
    if (xr >= 0 && xr < A.x_rows) v = *(const gbf16x8*)(A.x + xr * A.cin + cc * 8);
    *reinterpret_cast<bf16x8*>(smem + lr * A.lds_stride + cc * 16) = v;
  }
  __syncthreads();
  const long long row_base = wg_row0 + wr * (kRT * 16);
  const int nct = A.cout_pad / 16;
  const int ct0 = (blockIdx.y * 2 + wc) * kCT;
  if (ct0 >= nct) return;  // wave-uniform, after the only barrier

  int rn[kRT], rt[kRT], lr0[kRT];
  bool rok[kRT];
#pragma unroll
  for (int r = 0; r < kRT; ++r) {
    const long long row = row_base + r * 16 + m;
    const bool ok = row < rows;
    rn[r] = ok ? (int)(row / A.Lp) : 0;
    rt[r] = ok ? (int)(row - (long long)rn[r] * A.Lp) : 0;
    rok[r] = ok && rt[r] < A.L;
    // LDS row of tap 0 (input step t - pad)
    lr0[r] = rok[r] ? (int)((long long)rn[r] * A.in_rs + A.in_off + rt[r] - pad - xbase) : 0;
    APNEAUQ_DASSERT(!rok[r] || (lr0[r] >= 0 && lr0[r] + A.ksize <= A.lds_rows));
  }

  f32x4 acc[kCT][kRT];
#pragma unroll
  for (int c = 0; c < kCT; ++c)
#pragma unroll
    for (int r = 0; r < kRT; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};
  int tap = (8 * h) / A.cin, ci = 8 * h - tap * A.cin;
  const bf16x8 zero8 = bf16x8{(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f,
                              (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
  // weight fragments are software-pipelined one k-step ahead: the global (L2) load of step s + 1
  // is in flight while the MFMAs of step s run
  const gbf16x8* wf = (const gbf16x8*)A.wfrag + (long long)ct0 * 64 + lane;
  const int nc = nct - ct0 < kCT ? nct - ct0 : kCT;  // wave-uniform
  bf16x8 a[kCT];
#pragma unroll
  for (int c = 0; c < kCT; ++c) a[c] = c < nc ? wf[c * 64] : zero8;
  for (int s = 0; s < A.nstep; ++s) {
    const bool kok = 32 * s + 8 * h < K;
    bf16x8 an[kCT];
    const gbf16x8* wn = wf + (long long)(s + 1 < A.nstep ? s + 1 : s) * nct * 64;
#pragma unroll
    for (int c = 0; c < kCT; ++c) an[c] = c < nc ? wn[c * 64] : zero8;
    bf16x8 b[kRT];
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      const int ts = rt[r] + tap - pad;
      const bool ok = rok[r] && kok && ts >= 0 && ts < A.L;
      const int lrow = ok ? lr0[r] + tap : 0;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + lrow * A.lds_stride + ci * 2);
      b[r] = ok ? v : zero8;
    }
#pragma unroll
    for (int c = 0; c < kCT; ++c) {
      if (c < nc) {  // wave-uniform
#pragma unroll
        for (int r = 0; r < kRT; ++r) acc[c][r] = mfma16(a[c], b[r], acc[c][r]);
      }
    }
#pragma unroll
    for (int c = 0; c < kCT; ++c) a[c] = an[c];
    ci += 32;
    while (ci >= A.cin) {
      ci -= A.cin;
      ++tap;
    }
  }
  conv_epilogue<MODE>(A, acc, rn, rt, rok, ct0, nct, m, h);
}

// GAP over time + Dense(C -> 1): one wave per sample, fp32 accumulation.
__global__ __launch_bounds__(256) void head_kernel(const __bf16* y, const float* w, float b, int n, int L, int C,
                                                   int out_logits, float* out) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= n) return;
  const __bf16* ys = y + (long long)s * L * C;
  float acc = 0.f;
  for (int i = lane; i < L * C; i += kWave) acc += (float)ys[i] * w[i % C];
  acc = wave_sum(acc);
  if (lane == 0) {
    const float z = acc / (float)L + b;
    out[s] = out_logits ? z : 1.0f / (1.0f + __expf(-z));
  }
}

}  // namespace generic

hipError_t launch_generic_conv(const void* x, const void* wfrag, const float* epi, void* y, int n, int L, int cin,
                               int cout, int cout_pad, int ksize, int pool, int dropout, unsigned thr, int layer,
                               int n_win, unsigned pass_offset, unsigned window_offset, unsigned long long seed,
                               hipStream_t stream, int mode, int in_rs, int in_off, float* stats, long long x_rows,
                               int det_slots) {
  generic::ConvArgs A;
  A.x = reinterpret_cast<const __bf16*>(x);
  A.wfrag = reinterpret_cast<const bf16x8*>(wfrag);
  A.epi = epi;
  A.y = reinterpret_cast<__bf16*>(y);
  A.n = n;
  A.L = L;
  A.pool = pool;
  A.Lp = pool ? (L + 1) / 2 * 2 : L;
  A.cin = cin;
  A.cout = cout;
  A.cout_pad = cout_pad;
  A.ksize = ksize;
  A.nstep = (ksize * cin + 31) / 32;
  A.lout = pool ? L / 2 : L;
  A.dropout = dropout;
  A.thr = thr;
  A.layer = layer;
  A.n_win = n_win;
  A.pass_offset = pass_offset;
  A.window_offset = window_offset;
  A.seed = seed;
  A.in_rs = in_rs > 0 ? in_rs : L;
  A.in_off = in_off;
  A.stats = stats;
  if (mode != generic::kInfer) {
    A.pool = 0;
    A.Lp = L;
    A.lout = L;
    A.dropout = 0;
  }
  const long long rows = (long long)n * A.Lp;
  if (rows == 0) return hipSuccess;
  constexpr int kRowsWG = 2 * generic::kRT * 16, kChWG = 2 * generic::kCT;  // 128 rows x 8 channel tiles
  const dim3 grid((unsigned)((rows + kRowsWG - 1) / kRowsWG), (unsigned)((cout_pad / 16 + kChWG - 1) / kChWG));
  A.det = mode == generic::kTrain && det_slots > 0;
  if (A.det && (long long)grid.x * 2 > det_slots) return hipErrorInvalidValue;  // one slot per (workgroup, wave row)
  // LDS staging when every row a workgroup can touch fits: 128 output rows span at most
  // 127 + ceil(127 / Lp) * max(0, in_rs - Lp) input rows, plus the 2 * pad halo
  const long long extra = (long long)(127 + A.Lp - 1) / A.Lp * (A.in_rs > A.Lp ? A.in_rs - A.Lp : 0);
  const long long span = 128 + extra + 2 * (long long)((ksize - 1) / 2);
  const int stride = 2 * cin + 16;
  A.x_rows = x_rows;
  A.lds_rows = (int)span;
  A.lds_stride = stride;
  const bool use_lds = cin % 8 == 0 && span * stride <= 80 * 1024 && x_rows > 0;
  if (use_lds) {
    const size_t lds = (size_t)span * stride;
    if (mode == generic::kTrain)
      hipLaunchKernelGGL(generic::conv_lds_kernel<generic::kTrain>, grid, dim3(256), lds, stream, A);
    else if (mode == generic::kLinear)
      hipLaunchKernelGGL(generic::conv_lds_kernel<generic::kLinear>, grid, dim3(256), lds, stream, A);
    else
      hipLaunchKernelGGL(generic::conv_lds_kernel<generic::kInfer>, grid, dim3(256), lds, stream, A);
    return hipGetLastError();
  }
  // direct-gather kernel: channel counts that are not a multiple of 8, or rows beyond the LDS span
  auto gather = [&](auto mode_c) {
    constexpr int M = decltype(mode_c)::value;
    if (cin % 8 == 0)
      hipLaunchKernelGGL((generic::conv_block_kernel<true, M>), grid, dim3(256), 0, stream, A);
    else
      hipLaunchKernelGGL((generic::conv_block_kernel<false, M>), grid, dim3(256), 0, stream, A);
  };
  if (mode == generic::kTrain)
    gather(std::integral_constant<int, generic::kTrain>{});
  else if (mode == generic::kLinear)
    gather(std::integral_constant<int, generic::kLinear>{});
  else
    gather(std::integral_constant<int, generic::kInfer>{});
  return hipGetLastError();
}

hipError_t launch_generic_head(const void* y, const float* w, float b, int n, int L, int C, int out_logits, float* out,
                               hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(generic::head_kernel, dim3((n + 3) / 4), dim3(256), 0, stream,
                     reinterpret_cast<const __bf16*>(y), w, b, n, L, C, out_logits, out);
  return hipGetLastError();
}

}  // namespace apneauq
