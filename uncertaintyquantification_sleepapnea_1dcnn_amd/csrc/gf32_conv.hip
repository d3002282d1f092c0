// fp32 training kernels (gfx950 / MI355X) for precision="fp32": the reference trains in fp32 (Keras
// defaults, Adam compile at /root/reference/models/cnn_baseline_train.py:100-102, fit at :210-217,
// train_deep_ensemble_cnns.py:74,158), so this path keeps every operand, activation and gradient in
// fp32 and forms the conv products on v_mfma_f32_16x16x4_f32: exact fp32 products with fp32
// accumulation (no xf32 on gfx950; the f32-input MFMA runs at the vector FP32 rate, 1/16 of bf16).
// Any ModelSpec -- the reference (60, 4) CNN, the MaxPool1D blocks, the 30 s single-channel window --
// runs here with the elementwise BN / pool / dropout / head kernels of generic_train.hip and
// generic_wgrad.hip instantiated for fp32 storage (ops/generic_train.py, precision="fp32").
//
//   conv_kernel<MODE>  implicit GEMM, D[co][row] = sum_k A[co][k] B[k][row], k = tap * Cin + ci:
//                      A = the Keras kernel read in place (forward: W[tap][ci][co]; dgrad: the flipped,
//                      transposed W[K-1-tap][co][ci]), B = input rows (zero-padded row layout); a
//                      workgroup is 2 x 2 waves over 128 rows x 128 channels, each wave 4 x 4 tiles of
//                      16 x 16; operands of k-step s + 1 are loaded while step s's 16 MFMAs run.
//                      Epilogue: kTrain = relu(acc + bias) + BN moment slots (deterministic mode: one
//                      slot per (workgroup, wave row), plain stores), kLinear = acc (dgrad).
//   wgrad_kernel       dW[tap][ci][co] = sum_r Xpad[r + tap][ci] dZpad[r][co] over a row group; every
//                      row group writes its own partial (plain stores), summed in a fixed order by the
//                      ordered reduce of generic_wgrad.hip: deterministic weight gradients.
#include "common.h"

namespace apneauq {

hipError_t launch_ordered_sum(const float* part, int nrows, long long ncols, float* out, hipStream_t st);

namespace gf32 {

constexpr int kRT = 4, kCT = 4;  // per wave: 4 row tiles x 4 channel tiles
constexpr int kStatSlots = 16;   // atomic-mode moment slots (== generic::kStatSlots)
enum { kTrain = 1, kLinear = 2 };

__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct ConvArgs {
  const float* x;     // input rows: sample n, step t at row n * in_rs + in_off + t; cin channels
  const float* w;     // Keras kernel, forward (KS, cin, cout); dgrad (KS, cout, cin) = the forward kernel
  const float* bias;  // kTrain: (cout)
  float* y;           // (N, L, cout)
  float* stats;       // kTrain: moment slots (kStatSlots or 2 grid.x, 2, cout)
  int n, L, cin, cout, ksize, in_rs, in_off, flip, det;
};

template <int MODE>
__global__ __launch_bounds__(256) void conv_kernel(ConvArgs A) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, h = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const long long rows = (long long)A.n * A.L;
  const long long row_base = (long long)blockIdx.x * 128 + wr * 64;
  const int ct0 = (blockIdx.y * 2 + wc) * kCT;  // first 16-channel tile of this wave
  const int nct = (A.cout + 15) / 16;
  if (ct0 >= nct) return;  // wave-uniform; no barriers in this kernel
  const int pad = (A.ksize - 1) / 2;
  const int K = A.ksize * A.cin;

  int rn[kRT], rt[kRT];
  bool rok[kRT];
#pragma unroll
  for (int r = 0; r < kRT; ++r) {
    const long long row = row_base + r * 16 + m;
    rok[r] = row < rows;
    rn[r] = rok[r] ? (int)(row / A.L) : 0;
    rt[r] = rok[r] ? (int)(row - (long long)rn[r] * A.L) : 0;
  }
  // A operand rows (output channels) of this lane per channel tile
  int co[kCT];
#pragma unroll
  for (int c = 0; c < kCT; ++c) co[c] = (ct0 + c) * 16 + m;

  // this lane's k = 4 s + h as (tap, ci), advanced incrementally
  int tap = h / A.cin, ci = h - (h / A.cin) * A.cin;
  auto load = [&](int kk, int tp, int cc, float (&a)[kCT], float (&b)[kRT]) {
    const bool kok = kk < K;
#pragma unroll
    for (int c = 0; c < kCT; ++c) {
      float v = 0.f;
      if (kok && co[c] < A.cout)
        v = A.flip ? A.w[((long long)(A.ksize - 1 - tp) * A.cout + co[c]) * A.cin + cc]
                   : A.w[((long long)tp * A.cin + cc) * A.cout + co[c]];
      a[c] = v;
    }
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      const int ts = rt[r] + tp - pad;
      b[r] = (kok && rok[r] && ts >= 0 && ts < A.L)
                 ? A.x[((long long)rn[r] * A.in_rs + A.in_off + ts) * A.cin + cc]
                 : 0.f;
    }
  };
  auto advance = [&](int& tp, int& cc) {
    cc += 4;
    while (cc >= A.cin) {
      cc -= A.cin;
      ++tp;
    }
  };

  f32x4 acc[kCT][kRT];
#pragma unroll
  for (int c = 0; c < kCT; ++c)
#pragma unroll
    for (int r = 0; r < kRT; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nstep = (K + 3) / 4;
  float a0[kCT], b0[kRT], a1[kCT], b1[kRT];
  load(h, tap, ci, a0, b0);
  advance(tap, ci);
  for (int s = 0; s < nstep; ++s) {
    load(4 * (s + 1) + h, tap, ci, a1, b1);  // next k-step in flight under this step's MFMAs
    advance(tap, ci);
#pragma unroll
    for (int c = 0; c < kCT; ++c)
#pragma unroll
      for (int r = 0; r < kRT; ++r) acc[c][r] = mfma4(a0[c], b0[r], acc[c][r]);
#pragma unroll
    for (int c = 0; c < kCT; ++c) a0[c] = a1[c];
#pragma unroll
    for (int r = 0; r < kRT; ++r) b0[r] = b1[r];
  }

  // epilogue: lane holds channels co0 .. co0+3 (= 16 ct + 4 h + e) of row (rn[r], rt[r])
  float* st = nullptr;
  if (MODE == kTrain)
    st = A.stats + (long long)(A.det ? blockIdx.x * 2 + wr : blockIdx.x % kStatSlots) * 2 * A.cout;
#pragma unroll
  for (int c = 0; c < kCT; ++c) {
    const int co0 = (ct0 + c) * 16 + 4 * h;
    if (ct0 + c >= nct) break;  // wave-uniform
    const bool cok = co0 < A.cout;
    f32x4 bi = f32x4{0.f, 0.f, 0.f, 0.f};
    if (MODE == kTrain && cok) bi = *reinterpret_cast<const f32x4*>(A.bias + co0);
    f32x4 s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = s1;
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      f32x4 v = acc[c][r];
      if (MODE == kTrain) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = fmaxf(v[e] + bi[e], 0.f);
          const float u = rok[r] ? v[e] : 0.f;
          s1[e] += u;
          s2[e] = __builtin_fmaf(u, u, s2[e]);
        }
      }
      if (rok[r] && cok) *reinterpret_cast<f32x4*>(A.y + ((long long)rn[r] * A.L + rt[r]) * A.cout + co0) = v;
    }
    if (MODE == kTrain) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s1[e] = group16_sum(s1[e]);
        s2[e] = group16_sum(s2[e]);
      }
      if (m == 0 && cok) {
        if (A.det) {
          *reinterpret_cast<f32x4*>(st + co0) = s1;
          *reinterpret_cast<f32x4*>(st + A.cout + co0) = s2;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            atomicAdd(st + co0 + e, s1[e]);
            atomicAdd(st + A.cout + co0 + e, s2[e]);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------- wgrad
struct WgArgs {
  const float* x;    // Xpad rows (>= R + k - 1), cin channels
  const float* dz;   // dZpad rows (R), cout channels
  float* part;       // (row groups, k, cin, cout) partials
  long long R;
  int cin, cout, k, rows_per_group;
};

// workgroup = one 16-ci tile x 4 waves of 16-co tiles x one row group; a wave holds every tap's tile
__global__ __launch_bounds__(256) void wgrad_kernel(WgArgs A) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, h = lane >> 4;
  const int ci0 = blockIdx.x * 16, co0 = (blockIdx.y * 4 + wave) * 16;
  const int rg = blockIdx.z;
  if (co0 >= A.cout) return;  // wave-uniform
  const long long r_begin = (long long)rg * A.rows_per_group;
  const long long r_end = r_begin + A.rows_per_group < A.R ? r_begin + A.rows_per_group : A.R;
  constexpr int KMAX = 15;
  f32x4 acc[KMAX];
#pragma unroll
  for (int t = 0; t < KMAX; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool aok = ci0 + m < A.cin, bok = co0 + m < A.cout;
  // D[i = ci][j = co]: A[i][k] = X[r + k + tap][ci0 + i], B[k][j] = dZ[r + k][co0 + j], k = h
  for (long long r = r_begin; r < r_end; r += 4) {
    const long long rr = r + h;
    const bool rok = rr < r_end;
    const float b = (rok && bok) ? A.dz[rr * A.cout + co0 + m] : 0.f;
#pragma unroll
    for (int t = 0; t < KMAX; ++t) {
      if (t < A.k) {  // uniform
        const float a = (rok && aok) ? A.x[(rr + t) * A.cin + ci0 + m] : 0.f;
        acc[t] = mfma4(a, b, acc[t]);
      }
    }
  }
  // D layout: lane holds rows i = 4 h + e (ci), column j = m (co)
  float* p = A.part + (long long)rg * A.k * A.cin * A.cout;
#pragma unroll
  for (int t = 0; t < KMAX; ++t) {
    if (t >= A.k) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ci = ci0 + 4 * h + e, co = co0 + m;
      if (ci < A.cin && co < A.cout) p[((long long)t * A.cin + ci) * A.cout + co] = acc[t][e];
    }
  }
}

}  // namespace gf32

hipError_t launch_gf32_conv(const float* x, const float* w, const float* bias, float* y, float* stats, int n, int L,
                            int cin, int cout, int ksize, int mode, int in_rs, int in_off, int flip, int det_slots,
                            hipStream_t st) {
  gf32::ConvArgs A{x, w, bias, y, stats, n, L, cin, cout, ksize, in_rs, in_off, flip, det_slots > 0 ? 1 : 0};
  const long long rows = (long long)n * L;
  if (rows == 0) return hipSuccess;
  const dim3 grid((unsigned)((rows + 127) / 128), (unsigned)(((cout + 15) / 16 + 7) / 8));
  if (mode == gf32::kTrain && A.det && (long long)grid.x * 2 > det_slots) return hipErrorInvalidValue;
  if (mode == gf32::kTrain)
    hipLaunchKernelGGL(gf32::conv_kernel<gf32::kTrain>, grid, dim3(256), 0, st, A);
  else
    hipLaunchKernelGGL(gf32::conv_kernel<gf32::kLinear>, grid, dim3(256), 0, st, A);
  return hipGetLastError();
}

// gw (k, cin, cout) = sum over R rows; part holds part_floats fp32 (>= one (k, cin, cout) slice)
hipError_t launch_gf32_wgrad(const float* x, const float* dz, long long R, int cin, int cout, int k, float* gw,
                             float* part, long long part_floats, hipStream_t st) {
  if (R <= 0) return hipSuccess;
  if (k < 1 || k > 15) return hipErrorInvalidValue;
  const long long wfl = (long long)k * cin * cout;
  long long groups = part_floats / wfl;
  const long long ci_t = (cin + 15) / 16, co_g = (cout + 63) / 64;
  // ~2 workgroups per CU in total, at least 256 rows per group
  long long want = (512 + ci_t * co_g - 1) / (ci_t * co_g);
  if (want > (R + 255) / 256) want = (R + 255) / 256;
  if (groups > want) groups = want;
  if (groups > 65535) groups = 65535;
  if (groups < 1) return hipErrorInvalidValue;
  long long rpg = (R + groups - 1) / groups;
  rpg = (rpg + 3) / 4 * 4;
  groups = (R + rpg - 1) / rpg;
  gf32::WgArgs A{x, dz, part, R, cin, cout, k, (int)rpg};
  hipLaunchKernelGGL(gf32::wgrad_kernel, dim3((unsigned)ci_t, (unsigned)co_g, (unsigned)groups), dim3(256), 0, st, A);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_ordered_sum(part, (int)groups, wfl, gw, st);
}

}  // namespace apneauq
