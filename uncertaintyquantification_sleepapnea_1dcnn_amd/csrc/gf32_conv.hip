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
//                      16 x 16; B staged through LDS per (tap, 32-channel) chunk, A one k-step ahead.
//                      Epilogue: kTrain = relu(acc + bias) + BN moment slots (deterministic mode: one
//                      slot per (workgroup, wave row), plain stores), kLinear = acc (dgrad).
//   wgrad_kernel       dW[tap][ci][co] = sum_r Xpad[r + tap][ci] dZpad[r][co] over a row group; every
//                      row group writes its own partial (plain stores), summed in a fixed order by the
//                      ordered reduce of generic_wgrad.hip: deterministic weight gradients.
#include "common.h"

namespace apneauq {

hipError_t launch_ordered_sum(const float* part, int nrows, long long ncols, float* out, hipStream_t st);

namespace gf32 {

constexpr int kRT = 4;  // per wave: 4 row tiles x CT channel tiles (conv_kernel template)
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

// The B operand streams through LDS in chunks of one tap x kCK input channels for the tile's 128 rows
// (each lane of the staging loads reads kCK / 4 consecutive channels of one input row: whole 128-B
// lines instead of the 64 rows-apart single floats of a direct fragment load), double-buffered with
// one barrier per chunk; row stride kBS = 34 floats: each 32-lane half of a ds_read_b32 fragment read
// (16 rows x 2 k) hits 32 distinct banks (36 was 2-way), rows 8-B aligned for ds_write_b64 staging.  The A operand (the Keras kernel's [kCK][128 co] block of the chunk) is staged beside
// it (row stride kAS = 16 mod 64 floats: conflict-free fragment reads); a direct fragment load from
// L2 one k-step ahead left the MFMAs waiting on its latency (26 % of the f32 peak).
// CT = 16-channel tiles per wave (a workgroup covers 32 CT output channels): 3 where Cout is a multiple
// of 96 (the Cout-96 / 192 blocks padded to 128 / 256 channels computed 25 % zeros), else 4.
constexpr int kCK = 32, kBS = 34;
template <int MODE, int CT>
__global__ __launch_bounds__(256, 2) void conv_kernel(ConvArgs A) {
  constexpr int kCT = CT, AW = 32 * CT;       // the workgroup's output channels
  // A chunk layout: forward [k][co] (row stride kAS = 16 mod 64: the fragment read's h rows x 16 co
  // fill the banks), dgrad (MODE kLinear, the flipped kernel, ci-contiguous in global memory) [co][k]
  // (row stride kBS like B): both staged from coalesced loads with contiguous LDS stores
  constexpr bool kFlip = MODE == kLinear;
  constexpr int kAS = (AW + 47) / 64 * 64 + 16;  // >= AW, 16 mod 64
  constexpr int kAU = kCK * AW / 256;           // A-chunk elements staged per thread
  constexpr int kASZ = kFlip ? AW * kBS : kCK * kAS;
  __shared__ float bs[2][128 * kBS];
  __shared__ float as[2][kASZ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, h = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const long long rows = (long long)A.n * A.L;
  const long long row_base = (long long)blockIdx.x * 128 + wr * 64;
  const int ct0 = (blockIdx.y * 2 + wc) * kCT;  // first 16-channel tile of this wave
  const int nct = (A.cout + 15) / 16;
  const bool active = ct0 < nct;  // wave-uniform (inactive waves still stage and pass the barriers)
  const int pad = (A.ksize - 1) / 2;

  int rn[kRT], rt[kRT];
  bool rok[kRT];
#pragma unroll
  for (int r = 0; r < kRT; ++r) {
    const long long row = row_base + r * 16 + m;
    rok[r] = row < rows;
    rn[r] = rok[r] ? (int)(row / A.L) : 0;
    rt[r] = rok[r] ? (int)(row - (long long)rn[r] * A.L) : 0;
  }
  // staging: thread i owns tile row i / 2 and channels (i % 2) * 16 .. +15 of every chunk
  const int srow = threadIdx.x >> 1, sc0 = (threadIdx.x & 1) * 16;
  const long long sgrow = (long long)blockIdx.x * 128 + srow;
  const bool s_ok = sgrow < rows;
  const int s_n = s_ok ? (int)(sgrow / A.L) : 0;
  const int s_t = s_ok ? (int)(sgrow - (long long)s_n * A.L) : 0;
  const int ncc = (A.cin + kCK - 1) / kCK;
  const int nchunk = A.ksize * ncc;
  float sv[16], sw[kAU];
  const int cob = blockIdx.y * AW;  // the workgroup's first output channel
  // A chunk element j of this thread: i = tid + 256 j = (kk, c); the forward kernel W[tap][ci][co] is
  // co-contiguous (c fastest), the dgrad kernel W[K-1-tap][co][ci] ci-contiguous (kk fastest).  The
  // element's offset from the chunk's (uniform) base and its kk do not depend on the chunk: computed
  // once (the per-chunk 64-bit index math and the divisions by AW were most of the staging VALU)
  int aoff[kAU], akk[kAU];
#pragma unroll
  for (int j = 0; j < kAU; ++j) {
    const int i = threadIdx.x + 256 * j;
    const int kk = kFlip ? (i & (kCK - 1)) : (i / AW), c = kFlip ? (i >> 5) : (i % AW);
    const bool cok = cob + c < A.cout;
    akk[j] = cok ? kk : (1 << 30);  // never valid
    aoff[j] = kFlip ? c * A.cin + kk : kk * A.cout + c;
  }
  auto load_chunk = [&](int ch) {
    const int tp = ch / ncc, ccb = (ch - tp * ncc) * kCK, cc0 = ccb + sc0;
    const int ts = s_t + tp - pad;
    const bool ok = s_ok && ts >= 0 && ts < A.L;
    const float* src = A.x + ((long long)s_n * A.in_rs + A.in_off + ts) * A.cin;
#pragma unroll
    for (int j = 0; j < 16; ++j) sv[j] = (ok && cc0 + j < A.cin) ? src[cc0 + j] : 0.f;
    const float* wb = kFlip ? A.w + ((long long)(A.ksize - 1 - tp) * A.cout + cob) * A.cin + ccb
                            : A.w + ((long long)tp * A.cin + ccb) * A.cout + cob;
    const int kmax = A.cin - ccb;
#pragma unroll
    for (int j = 0; j < kAU; ++j) sw[j] = akk[j] < kmax ? wb[aoff[j]] : 0.f;
  };
  auto store_chunk = [&](int buf) {
    float* d = &bs[buf][srow * kBS + sc0];
#pragma unroll
    for (int j = 0; j < 16; j += 2) *reinterpret_cast<f32x2*>(d + j) = f32x2{sv[j], sv[j + 1]};
#pragma unroll
    for (int j = 0; j < kAU; ++j) {
      const int i = threadIdx.x + 256 * j;
      if constexpr (kFlip)
        as[buf][(i >> 5) * kBS + (i & (kCK - 1))] = sw[j];
      else
        as[buf][(i / AW) * kAS + i % AW] = sw[j];
    }
  };

  f32x4 acc[kCT][kRT];
#pragma unroll
  for (int c = 0; c < kCT; ++c)
#pragma unroll
    for (int r = 0; r < kRT; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};
  load_chunk(0);
  store_chunk(0);
  if (nchunk > 1) load_chunk(1);
  __syncthreads();
  const int brow = wr * 64 + m;  // this lane's B rows: brow + 16 r
  const int acol = wc * 16 * CT + m;  // this lane's A columns (output channels): acol + 16 c
  for (int ch = 0; ch < nchunk; ++ch) {
    const float* b = bs[ch & 1];
    const float* a = as[ch & 1];
    // k-steps of this chunk: its channels (cin < kCK: the first layers) in groups of 4
    const int ccb = (ch % ncc) * kCK;
    const int nq = (min(kCK, A.cin - ccb) + 3) / 4;
    if (active) {
#pragma unroll
      for (int q = 0; q < kCK / 4; ++q) {
        if (q >= nq) break;  // uniform
        float aq[kCT], bq[kRT];
#pragma unroll
        for (int c = 0; c < kCT; ++c)
          aq[c] = kFlip ? a[(acol + 16 * c) * kBS + 4 * q + h] : a[(4 * q + h) * kAS + acol + 16 * c];
#pragma unroll
        for (int r = 0; r < kRT; ++r) bq[r] = b[(brow + 16 * r) * kBS + 4 * q + h];
#pragma unroll
        for (int c = 0; c < kCT; ++c)
#pragma unroll
          for (int r = 0; r < kRT; ++r) acc[c][r] = mfma4(aq[c], bq[r], acc[c][r]);
      }
    }
    // chunk ch + 1 (loaded one chunk ago) into the other buffer, whose readers (chunk ch - 1) passed
    // the previous barrier; then chunk ch + 2's loads go out under the next chunk's MFMAs
    if (ch + 1 < nchunk) store_chunk((ch + 1) & 1);
    __syncthreads();
    if (ch + 2 < nchunk) load_chunk(ch + 2);
  }
  if (!active) return;

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

// workgroup = 32 ci x 64 co x one row group (4 waves, each 16 ci x 32 co x every tap in registers).
// The row group streams through LDS in chunks of kWgRC rows (X with its k - 1 halo rows, dZ),
// double-buffered and prefetched one chunk ahead through registers, so each operand float is read from
// global memory once per workgroup; row strides 48 / 80 floats put the 4 row groups of a fragment read
// on disjoint bank quarters.
// K (taps) is a template parameter: the accumulators of every tap stay in registers (a runtime tap
// count indexed them through scratch memory).
constexpr int kWgRC = 64, kWgKMax = 15, kWgXS = 48, kWgDS = 80;
template <int K>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgArgs A) {
  constexpr int XR = kWgRC + K - 1;                 // X rows of a chunk (with the tap halo)
  constexpr int XU = (XR * 32 + 255) / 256, DU = kWgRC * 64 / 256;  // staged floats per thread
  __shared__ float xs[2][(kWgRC + kWgKMax - 1) * kWgXS];
  __shared__ float ds[2][kWgRC * kWgDS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, h = lane >> 4;
  // wave = one 16-ci tile x two 16-co tiles x every tap: per 4 rows, 2 dZ + K X fragment reads feed
  // 2 K MFMAs
  const int wci = wave & 1, wco = (wave >> 1) * 2;
  const int ci0 = blockIdx.x * 32, cog = blockIdx.y * 64;
  const int rg = blockIdx.z;
  const long long r_begin = (long long)rg * A.rows_per_group;
  const long long r_end = r_begin + A.rows_per_group < A.R ? r_begin + A.rows_per_group : A.R;
  const long long x_rows = A.R + K - 1;
  f32x4 acc[K][2];
#pragma unroll
  for (int t = 0; t < K; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // chunk staging through registers: the loads of chunk c + 1 are in flight during chunk c's MFMAs
  float px[XU], pd[DU];
  auto load = [&](long long r0) {
#pragma unroll
    for (int j = 0; j < XU; ++j) {
      const int i = threadIdx.x + 256 * j, rr = i >> 5, c = i & 31;
      const long long row = r0 + rr;
      px[j] = (i < XR * 32 && row < x_rows && row < r_end + K - 1 && ci0 + c < A.cin) ? A.x[row * A.cin + ci0 + c]
                                                                                    : 0.f;
    }
#pragma unroll
    for (int j = 0; j < DU; ++j) {
      const int i = threadIdx.x + 256 * j, rr = i >> 6, c = i & 63;
      const long long row = r0 + rr;
      pd[j] = (row < r_end && cog + c < A.cout) ? A.dz[row * A.cout + cog + c] : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < XU; ++j) {
      const int i = threadIdx.x + 256 * j;
      if (i < XR * 32) xs[buf][(i >> 5) * kWgXS + (i & 31)] = px[j];
    }
#pragma unroll
    for (int j = 0; j < DU; ++j) {
      const int i = threadIdx.x + 256 * j;
      ds[buf][(i >> 6) * kWgDS + (i & 63)] = pd[j];
    }
  };
  const bool active = cog + wco * 16 < A.cout;  // wave-uniform
  load(r_begin);
  store(0);
  if (r_begin + kWgRC < r_end) load(r_begin + kWgRC);
  __syncthreads();
  int buf = 0;
  for (long long r0 = r_begin; r0 < r_end; r0 += kWgRC, buf ^= 1) {  // workgroup-uniform
    if (active) {
      const float* xb = xs[buf] + wci * 16 + m;
      const float* db = ds[buf] + wco * 16 + m;
#pragma unroll 4
      for (int kk = 0; kk < kWgRC / 4; ++kk) {
        const int rb = 4 * kk + h;
        const float b0 = db[rb * kWgDS], b1 = db[rb * kWgDS + 16];
#pragma unroll
        for (int t = 0; t < K; ++t) {
          const float a = xb[(rb + t) * kWgXS];
          acc[t][0] = mfma4(a, b0, acc[t][0]);
          acc[t][1] = mfma4(a, b1, acc[t][1]);
        }
      }
    }
    if (r0 + kWgRC < r_end) store(buf ^ 1);  // its readers (chunk c - 1) passed the last barrier
    __syncthreads();
    if (r0 + 2 * kWgRC < r_end) load(r0 + 2 * kWgRC);
  }
  // D layout: lane holds rows i = 4 h + e (ci), column j = m (co)
  if (!active) return;
  const int ci = ci0 + wci * 16 + 4 * h;
  float* p = A.part + (long long)rg * K * A.cin * A.cout;
#pragma unroll
  for (int t = 0; t < K; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int co = cog + (wco + u) * 16 + m;
      if (co >= A.cout) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (ci + e < A.cin) p[((long long)t * A.cin + ci + e) * A.cout + co] = acc[t][u][e];
    }
}

// dispatch the runtime tap count (1 .. kWgKMax) to its wgrad_kernel<K> instantiation
template <int K>
bool launch_wgrad_k(int k, dim3 grid, const WgArgs& A, hipStream_t st) {
  if (k == K) {
    hipLaunchKernelGGL(wgrad_kernel<K>, grid, dim3(256), 0, st, A);
    return true;
  }
  if constexpr (K < kWgKMax) return launch_wgrad_k<K + 1>(k, grid, A, st);
  return false;
}

}  // namespace gf32

hipError_t launch_gf32_conv(const float* x, const float* w, const float* bias, float* y, float* stats, int n, int L,
                            int cin, int cout, int ksize, int mode, int in_rs, int in_off, int flip, int det_slots,
                            hipStream_t st) {
  gf32::ConvArgs A{x, w, bias, y, stats, n, L, cin, cout, ksize, in_rs, in_off, flip, det_slots > 0 ? 1 : 0};
  const long long rows = (long long)n * L;
  if (rows == 0) return hipSuccess;
  const int nct = (cout + 15) / 16, ct = nct % 6 == 0 ? 3 : 4;
  const dim3 grid((unsigned)((rows + 127) / 128), (unsigned)((nct + 2 * ct - 1) / (2 * ct)));
  if (mode == gf32::kTrain && A.det && (long long)grid.x * 2 > det_slots) return hipErrorInvalidValue;
  if (mode == gf32::kTrain && ct == 3)
    hipLaunchKernelGGL((gf32::conv_kernel<gf32::kTrain, 3>), grid, dim3(256), 0, st, A);
  else if (mode == gf32::kTrain)
    hipLaunchKernelGGL((gf32::conv_kernel<gf32::kTrain, 4>), grid, dim3(256), 0, st, A);
  else if (ct == 3)
    hipLaunchKernelGGL((gf32::conv_kernel<gf32::kLinear, 3>), grid, dim3(256), 0, st, A);
  else
    hipLaunchKernelGGL((gf32::conv_kernel<gf32::kLinear, 4>), grid, dim3(256), 0, st, A);
  return hipGetLastError();
}

// gw (k, cin, cout) = sum over R rows; part holds part_floats fp32 (>= one (k, cin, cout) slice)
hipError_t launch_gf32_wgrad(const float* x, const float* dz, long long R, int cin, int cout, int k, float* gw,
                             float* part, long long part_floats, hipStream_t st) {
  if (R <= 0) return hipSuccess;
  if (k < 1 || k > 15) return hipErrorInvalidValue;
  const long long wfl = (long long)k * cin * cout;
  long long groups = part_floats / wfl;
  const long long ci_t = (cin + 31) / 32, co_g = (cout + 63) / 64;
  // ~2 workgroups per CU in total (71 KB of LDS each), at least 256 rows per group
  long long want = (512 + ci_t * co_g - 1) / (ci_t * co_g);
  if (want > (R + 255) / 256) want = (R + 255) / 256;
  if (groups > want) groups = want;
  if (groups > 65535) groups = 65535;
  if (groups < 1) return hipErrorInvalidValue;
  long long rpg = (R + groups - 1) / groups;
  rpg = (rpg + gf32::kWgRC - 1) / gf32::kWgRC * gf32::kWgRC;  // whole LDS row chunks
  groups = (R + rpg - 1) / rpg;
  gf32::WgArgs A{x, dz, part, R, cin, cout, k, (int)rpg};
  const dim3 grid((unsigned)ci_t, (unsigned)co_g, (unsigned)groups);
  if (!gf32::launch_wgrad_k<1>(k, grid, A, st)) return hipErrorInvalidValue;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_ordered_sum(part, (int)groups, wfl, gw, st);
}

}  // namespace apneauq
