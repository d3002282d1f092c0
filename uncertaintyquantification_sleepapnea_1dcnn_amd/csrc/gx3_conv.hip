// fp32-faithful ("fp16x3") layer-wise conv kernels for ANY ModelSpec (gfx950 / MI355X): the precision
// path of precision="fp32" inference and train_precision="fp32" training.  The reference trains and
// infers in fp32 (Keras defaults: /root/reference/models/cnn_baseline_train.py:100-102,210-217,
// train_deep_ensemble_cnns.py:74,158, uncertainty_quantification/uq_techniques.py:22-30,
// evaluate_de_global.py:18-38 for the pooled ensemble members).
//
// Arithmetic: every operand v is prescaled by an exact power of two and split into fp16 halves
// hi = fp16(v), lo = fp16(v - hi) (22 significant bits); a product is three v_mfma_f32_16x16x32_f16
// (hi*hi + lo*hi + hi*lo, fp32 accumulate; the dropped lo*lo and the split residuals are ~2^-22
// relative, below fp32 GEMM rounding), and the epilogue undoes the prescales exactly.  Same scheme as
// the reference architecture's headline engine (x3_layers.hip); here for every shape, 3 bf16-rate
// MFMAs per 32-deep k-step instead of the eight 1/16-rate f32 MFMAs of the exact-fp32 path
// (gf32_conv.hip, kept as the oracle-grade fallback).
//
// Range safety (prescales):
//   * weights: one power of two per tensor from max|W| (wmax_kernel + pack_kernel, every step);
//   * conv inputs: one power of two per workgroup from the max over the input rows it reads (a
//     pre-pass over its samples), also published as the tensor maximum (atomicMax, optional);
//   * wgrad: one power of two per operand tensor from those published maxima (the forward conv
//     published the input's, the dgrad conv dZ's; amax_kernel covers block 1's dZ).
// The scale puts the operand's maximum in [2^13, 2^14): hi never overflows, and an element's lo
// only turns subnormal below 2^-25 of that maximum, far under fp32 rounding of the sums.
//
//   conv_kernel<MODE, CT, HALO, VEC>  implicit GEMM D[co][row] = sum_k A[co][k] B[k][row],
//     k = tap * Cin + ci (dgrad: the flipped, transposed kernel, Cin <-> Cout).  A = pre-packed hi/lo
//     fragments (global, one 16-B load per lane per half, one k-step ahead); B staged in LDS as hi/lo
//     rows.  HALO (Cin % 32 == 0, short row span): per 32-channel chunk the workgroup's input rows
//     plus the tap halo, every tap reads shifted rows of the same chunk (the conversion runs once per
//     element); else an im2col tile of 32 k per chunk.  Workgroup = 2 x 2 waves over 128 rows x 32 CT
//     channels; each wave 4 row tiles x CT channel tiles.  Epilogue kTrain: relu(acc + bias) + BN
//     moment slots (deterministic: one slot per (workgroup, wave row), plain stores); kLinear: acc.
//   wgrad_kernel<K>  dW[tap][ci][co] = sum_r Xpad[r + tap][ci] dZpad[r][co]: a workgroup = 32 ci x
//     64 co x one row group, rows streamed through LDS in 64-row chunks (hi/lo, read with the
//     transposing ds_read_b64_tr_b16), every tap's accumulators in registers; row-group partials
//     summed in a fixed order (deterministic).
#include "common.h"

namespace apneauq {

hipError_t launch_ordered_sum(const float* part, int nrows, long long ncols, float* out, hipStream_t st);

namespace gx3 {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f16x8 gf16x8;

enum { kTrain = 1, kLinear = 2 };
constexpr int kStatSlots = 16;
constexpr int kRT = 4;       // row tiles per wave
constexpr int kRowB = 160;   // LDS B row: hi 32 halfs | lo 32 halfs | 32 B pad (stride 2 mod 4 16-B slots)
constexpr int kMaxBlocks = 48;
constexpr int kMaxWG = 16;   // wmax_kernel workgroups per tensor

__device__ __forceinline__ f32x4 mfma(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// acc += A * B over one 32-deep k-step, fp16x3: small terms first
__device__ __forceinline__ f32x4 mfma3(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, f32x4 c) {
  c = mfma(al, bh, c);
  c = mfma(ah, bl, c);
  return mfma(ah, bh, c);
}

// exponent sa with max * 2^sa in [2^13, 2^14) (0 for an all-zero tensor)
__device__ __forceinline__ int prescale_exp(float mx) {
  int e = 0;
  if (mx > 0.f && mx < INFINITY) frexpf(mx, &e);
  return min(100, max(-100, 14 - e));
}

__device__ __forceinline__ void split4(const f32x4& v, float sc, f16x4& hi, f16x4& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = v[i] * sc;  // exact: sc is a power of two
    hi[i] = (_Float16)a;
    lo[i] = (_Float16)(a - (float)hi[i]);
  }
}

__device__ __forceinline__ float absmax4(const f32x4& v, float m) {
  return fmaxf(fmaxf(fmaxf(m, fabsf(v[0])), fmaxf(fabsf(v[1]), fabsf(v[2]))), fabsf(v[3]));
}

// workgroup max of a non-negative float (every thread gets it); red: >= 4 unsigned of LDS
__device__ __forceinline__ float block_max(float v, unsigned* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __float_as_uint(v);
  __syncthreads();
  float m = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, __uint_as_float(red[i]));
  __syncthreads();
  return m;
}

// ------------------------------------------------------------------------------------ weights
struct PackBlock {
  const float* w;  // (k, cin, cout) fp32
  f16x8* fwd;      // (nstep, ceil(cout/16), 2, 64) hi/lo fragments
  f16x8* dgr;      // (nstep', ceil(cin/16), 2, 64) of the flipped, transposed kernel; nullptr: none
  float* wsc;      // 2^-sw of this tensor's prescale
  int k, cin, cout;
  long long nf, nd;  // fragment elements (halfs of one of hi / lo) of each orientation
};
struct PackArgs {
  PackBlock b[kMaxBlocks];
  float* wpart;  // (nblocks, kMaxWG) partial maxima
  int nblocks;
};

__global__ __launch_bounds__(256) void wmax_kernel(PackArgs P) {
  __shared__ unsigned red[4];
  const PackBlock& B = P.b[blockIdx.y];
  const long long n4 = (long long)B.k * B.cin * B.cout / 4;  // cout % 4 == 0
  float m = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += 256LL * gridDim.x)
    m = absmax4(reinterpret_cast<const f32x4*>(B.w)[i], m);
  m = block_max(m, red);
  if (threadIdx.x == 0) P.wpart[blockIdx.y * kMaxWG + blockIdx.x] = m;
}

__global__ __launch_bounds__(256) void pack_kernel(PackArgs P) {
  const PackBlock& B = P.b[blockIdx.y];
  float mx = 0.f;
  for (int i = 0; i < kMaxWG; ++i) mx = fmaxf(mx, P.wpart[blockIdx.y * kMaxWG + i]);
  const int sw = prescale_exp(mx);
  const float sc = ldexpf(1.f, sw);
  if (blockIdx.x == 0 && threadIdx.x == 0) *B.wsc = ldexpf(1.f, -sw);
  const long long tot = B.nf + (B.dgr ? B.nd : 0);
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < tot; e += 256LL * gridDim.x) {
    const bool is_f = e < B.nf;
    const long long i = is_f ? e : e - B.nf;
    const int kin = is_f ? B.cin : B.cout;   // GEMM K channels
    const int mch = is_f ? B.cout : B.cin;   // GEMM M channels (padded to 16)
    const int j = (int)(i & 7), lane = (int)((i >> 3) & 63);
    const long long fr = i >> 9;
    const int nct = (mch + 15) / 16;
    const int ct = (int)(fr % nct), s = (int)(fr / nct);
    const int co = 16 * ct + (lane & 15);
    const int kk = 32 * s + 8 * (lane >> 4) + j;
    float v = 0.f;
    if (kk < kin * B.k && co < mch) {
      const int tap = kk / kin, ci = kk - tap * kin;
      v = is_f ? B.w[((long long)tap * B.cin + ci) * B.cout + co]
               : B.w[((long long)(B.k - 1 - tap) * B.cin + co) * B.cout + ci];
    }
    const float a = v * sc;
    const _Float16 hi = (_Float16)a;
    _Float16* out = reinterpret_cast<_Float16*>(is_f ? B.fwd : B.dgr) + fr * 1024 + (i & 511);
    out[0] = hi;
    out[512] = (_Float16)(a - (float)hi);
  }
}

// max |x| over n floats into *out (atomicMax of the fp32 bits; *out must start <= the result)
__global__ __launch_bounds__(256) void amax_kernel(const float* x, long long n, unsigned* out) {
  __shared__ unsigned red[4];
  float m = 0.f;
  const long long n4 = n / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += 256LL * gridDim.x)
    m = absmax4(reinterpret_cast<const f32x4*>(x)[i], m);
  for (long long i = n4 * 4 + blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) m = fmaxf(m, fabsf(x[i]));
  m = block_max(m, red);
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(m));
}

// ---------------------------------------------------------------------------------------- conv
struct ConvArgs {
  const float* x;       // input rows: sample n, step t at row n * in_rs + in_off + t; cin channels
  const f16x8* wfrag;   // packed hi/lo fragments (nstep, nct, 2, 64)
  const float* wsc;     // 2^-sw of the packed weights
  const float* bias;    // kTrain: (cout)
  float* y;             // (n * L, cout)
  float* stats;         // kTrain: moment slots (kStatSlots or 2 grid.x, 2, cout)
  unsigned* amax_out;   // nullable: atomicMax of the input's |x| (tensor maximum, fp32 bits)
  long long x_rows;     // rows of the input buffer
  int n, L, cin, cout, ksize, in_rs, in_off, det;
  int nstep, nct, span;  // k-steps, 16-channel tiles of cout, HALO: staged rows per chunk
  // taps that can reach a valid input row ([tap0, tap1): all of them unless L < k, where the outer taps
  // of a short sequence only ever read padding -- pooled blocks 5 / 6 at L = 3 / 1), and the k-steps
  // that hold them (IM2COL)
  int tap0, tap1, s0, s1;
};

template <bool HALO>
__host__ __device__ constexpr int b_rows(int span) { return HALO ? span : 128; }

template <int MODE, int CT, bool HALO, bool VEC>
__global__ __launch_bounds__(256, 2) void conv_kernel(ConvArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ unsigned red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, h = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const long long rows = (long long)A.n * A.L;
  const long long row0 = (long long)blockIdx.x * 128;
  const int pad = (A.ksize - 1) / 2;
  const int K = A.ksize * A.cin;
  const int span = A.span;
  const int brows = b_rows<HALO>(span);
  char* buf0 = smem;
  char* buf1 = smem + brows * kRowB;

  // ---- input prescale of this workgroup: max |x| over the samples its rows belong to
  const long long rlast = (row0 + 128 < rows ? row0 + 128 : rows) - 1;
  const int n0 = (int)(row0 / A.L), n1 = (int)(rlast / A.L);
  int sb;
  {
    float mx = 0.f;
    const int per = A.L * A.cin;
    const long long cnt = (long long)(n1 - n0 + 1) * per;
    if ((A.cin & 3) == 0) {
      for (long long i = tid; i < cnt / 4; i += 256) {
        const long long e = 4 * i;
        const int sn = (int)(e / per), rem = (int)(e - (long long)sn * per);
        const int t = rem / A.cin, c = rem - t * A.cin;
        mx = absmax4(*reinterpret_cast<const f32x4*>(A.x + ((long long)(n0 + sn) * A.in_rs + A.in_off + t) * A.cin + c), mx);
      }
    } else {
      for (long long e = tid; e < cnt; e += 256) {
        const int sn = (int)(e / per), rem = (int)(e - (long long)sn * per);
        const int t = rem / A.cin, c = rem - t * A.cin;
        mx = fmaxf(mx, fabsf(A.x[((long long)(n0 + sn) * A.in_rs + A.in_off + t) * A.cin + c]));
      }
    }
    mx = block_max(mx, red);
    if (A.amax_out != nullptr && tid == 0) atomicMax(A.amax_out, __float_as_uint(mx));
    sb = prescale_exp(mx);
  }
  const float bscale = ldexpf(1.f, sb);
  const float unscale = ldexpf(A.wsc[0], -sb);

  // ---- staging.  HALO: chunk c = input channels [32c, 32c + 32) of the rows [xbase, xbase + span);
  // IM2COL: chunk s = k in [32s, 32s + 32) of the 128 output rows (tap, ci gathered per k)
  const int t0 = (int)(row0 - (long long)n0 * A.L);
  const long long xbase = (long long)n0 * A.in_rs + A.in_off + t0 - pad;
  const int ncb = HALO ? A.cin / 32 : 0;
  const int nchunk = HALO ? ncb : A.s1 - A.s0;  // IM2COL chunk i = k-step s0 + i
  constexpr int kHU = 8;  // HALO: 16-B units per thread (span * 8 <= 256 * kHU)
  // IM2COL: thread i stages row i / 2 and k-half (i & 1) (16 k: two 8-k units when VEC)
  const int irow = tid >> 1, ikh = tid & 1;
  const long long igrow = row0 + irow;
  const bool iok = igrow < rows;
  const int in_ = iok ? (int)(igrow / A.L) : 0;
  const int it_ = iok ? (int)(igrow - (long long)in_ * A.L) : 0;
  const float* ixs = A.x + ((long long)in_ * A.in_rs + A.in_off) * A.cin;
  f32x4 sv[HALO ? kHU : 4];
  auto load_chunk = [&](int c) {
    if constexpr (HALO) {
#pragma unroll
      for (int u = 0; u < kHU; ++u) {
        const int i = tid + 256 * u, lr = i >> 3, q = i & 7;
        const long long xr = xbase + lr;
        sv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (lr < span && xr >= 0 && xr < A.x_rows)
          sv[u] = *reinterpret_cast<const f32x4*>(A.x + xr * A.cin + 32 * c + 4 * q);
      }
    } else if constexpr (VEC) {
      // two 8-k units: k0 = 32 s + 16 ikh + 8 v, all 8 in one tap (cin % 8 == 0)
      c += A.s0;
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int k0 = 32 * c + 16 * ikh + 8 * v;
        const int tap = k0 / A.cin, ci = k0 - tap * A.cin;
        const int ts = it_ + tap - pad;
        sv[2 * v] = sv[2 * v + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (iok && k0 < K && ts >= 0 && ts < A.L) {
          const float* src = ixs + (long long)ts * A.cin + ci;
          sv[2 * v] = *reinterpret_cast<const f32x4*>(src);
          sv[2 * v + 1] = *reinterpret_cast<const f32x4*>(src + 4);
        }
      }
    } else {
      c += A.s0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int kk = 32 * c + 16 * ikh + j;
        const int tap = kk / A.cin, ci = kk - tap * A.cin;
        const int ts = it_ + tap - pad;
        sv[j >> 2][j & 3] = (iok && kk < K && ts >= 0 && ts < A.L) ? ixs[(long long)ts * A.cin + ci] : 0.f;
      }
    }
  };
  auto store_chunk = [&](char* buf) {
    if constexpr (HALO) {
#pragma unroll
      for (int u = 0; u < kHU; ++u) {
        const int i = tid + 256 * u, lr = i >> 3, q = i & 7;
        if (lr < span) {
          f16x4 hi, lo;
          split4(sv[u], bscale, hi, lo);
          *reinterpret_cast<f16x4*>(buf + lr * kRowB + 8 * q) = hi;
          *reinterpret_cast<f16x4*>(buf + lr * kRowB + 64 + 8 * q) = lo;
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        f16x4 hi, lo;
        split4(sv[u], bscale, hi, lo);
        *reinterpret_cast<f16x4*>(buf + irow * kRowB + 32 * ikh + 8 * u) = hi;
        *reinterpret_cast<f16x4*>(buf + irow * kRowB + 64 + 32 * ikh + 8 * u) = lo;
      }
    }
  };

  // ---- this wave's output rows / LDS rows of tap 0
  const long long row_base = row0 + wr * 64;
  const int ct0 = (blockIdx.y * 2 + wc) * CT;
  const bool active = ct0 < A.nct;  // wave-uniform (inactive waves still stage and pass the barriers)
  int rn[kRT], rt[kRT], lrow[kRT];
  bool rok[kRT];
#pragma unroll
  for (int r = 0; r < kRT; ++r) {
    const long long row = row_base + r * 16 + m;
    rok[r] = row < rows;
    rn[r] = rok[r] ? (int)(row / A.L) : n0;
    rt[r] = rok[r] ? (int)(row - (long long)rn[r] * A.L) : 0;
    // HALO: the LDS row of tap 0 (input step t - pad); IM2COL: the local row
    lrow[r] = HALO ? (rok[r] ? (int)((long long)rn[r] * A.in_rs + A.in_off + rt[r] - pad - xbase) : 0) : wr * 64 + r * 16 + m;
    APNEAUQ_DASSERT(!HALO || !rok[r] || (lrow[r] >= 0 && lrow[r] + A.ksize <= span));
  }

  f32x4 acc[CT][kRT];
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int r = 0; r < kRT; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};
  // A fragments: step s, tile ct at wfrag + ((s * nct + ct) * 2 + half) * 64 + lane
  const int nc = A.nct - ct0 < CT ? A.nct - ct0 : CT;  // wave-uniform
  const gf16x8* wbase = (const gf16x8*)A.wfrag + (long long)(active ? ct0 : 0) * 128 + lane;
  auto a_ptr = [&](int s) { return wbase + (long long)s * A.nct * 128; };
  auto load_a = [&](const gf16x8* p, f16x8 (&xh)[CT], f16x8 (&xl)[CT]) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int cc = c < nc ? c : 0;
      xh[c] = p[cc * 128];
      xl[c] = p[cc * 128 + 64];
    }
  };
  // k-step sequence: HALO it = c * ntap + (tap - tap0) (A step tap * ncb + c); IM2COL it = s - s0
  const int ntap = A.tap1 - A.tap0;
  const int nit = HALO ? nchunk * ntap : nchunk;
  auto a_step = [&](int it) {
    if constexpr (HALO) {
      const int c = it / ntap, tap = A.tap0 + it - c * ntap;
      return tap * ncb + c;
    } else {
      return A.s0 + it;
    }
  };
  f16x8 ah[CT], al[CT];
  load_a(a_ptr(a_step(0)), ah, al);

  load_chunk(0);
  store_chunk(buf0);
  if (nchunk > 1) load_chunk(1);
  __syncthreads();
  int it = 0;
  for (int ch = 0; ch < nchunk; ++ch) {
    const char* buf = (ch & 1) ? buf1 : buf0;
    const int taps = HALO ? ntap : 1;
    for (int jj = 0; jj < taps; ++jj, ++it) {
      const int j = A.tap0 + jj;  // HALO: the tap (its rows are shifted by j)
      f16x8 nh[CT], nl[CT];
      load_a(a_ptr(a_step(it + 1 < nit ? it + 1 : it)), nh, nl);
      if (active) {
#pragma unroll
        for (int r = 0; r < kRT; ++r) {
          const char* bp = buf + (lrow[r] + (HALO ? j : 0)) * kRowB + 16 * h;
          const f16x8 bh = *reinterpret_cast<const f16x8*>(bp);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(bp + 64);
#pragma unroll
          for (int c = 0; c < CT; ++c)
            if (c < nc) acc[c][r] = mfma3(ah[c], al[c], bh, bl, acc[c][r]);  // wave-uniform
        }
      }
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        ah[c] = nh[c];
        al[c] = nl[c];
      }
    }
    // chunk ch + 1 (loaded one chunk ago) into the other buffer, whose readers (chunk ch - 1) passed
    // the previous barrier; then chunk ch + 2's loads go out under the next chunk's MFMAs
    if (ch + 1 < nchunk) store_chunk((ch & 1) ? buf0 : buf1);
    __syncthreads();
    if (ch + 2 < nchunk) load_chunk(ch + 2);
  }
  if (!active) return;

  // ---- epilogue: lane holds channels co0 .. co0+3 (= 16 ct + 4 h + e) of row (rn[r], rt[r])
  float* st = nullptr;
  if (MODE == kTrain) st = A.stats + (long long)(A.det ? blockIdx.x * 2 + wr : blockIdx.x % kStatSlots) * 2 * A.cout;
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    if (c >= nc) break;  // wave-uniform
    const int co0 = (ct0 + c) * 16 + 4 * h;
    const bool cok = co0 < A.cout;
    f32x4 bi = f32x4{0.f, 0.f, 0.f, 0.f};
    if (MODE == kTrain && cok) bi = *reinterpret_cast<const f32x4*>(A.bias + co0);
    f32x4 s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = s1;
#pragma unroll
    for (int r = 0; r < kRT; ++r) {
      f32x4 v = acc[c][r];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] *= unscale;  // exact: a power of two
        if (MODE == kTrain) {
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
  const float* x;          // Xpad rows (>= R + k - 1), cin channels
  const float* dz;         // dZpad rows (R), cout channels
  const unsigned* amax_x;  // tensor maxima (fp32 bits) of x and dz
  const unsigned* amax_dz;
  float* part;             // (row groups, k, cin, cout) partials
  long long R;
  int cin, cout, k, rows_per_group;
};

typedef short v4i16x __attribute__((ext_vector_type(4)));

// fragment of a 16x16x32 operand whose K index is the LDS row (32 rows from row_base) and whose M/N
// index is 16 columns from col0 (16-bit elements; the k-slot order of train_conv.hip tr_frag, the
// same for both operands, conflict-free on row strides that are odd multiples of 32 B)
__device__ __forceinline__ f16x8 tr_frag(const char* lds, int rs, int row_base, int col0) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const char* a0 = lds + (row_base + 4 * h + q) * rs + (col0 + 4 * p) * 2;
  const v4i16x lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16x*)a0);
  const v4i16x hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16x*)(a0 + 16 * rs));
  f16x8 r;
  const _Float16* pl = reinterpret_cast<const _Float16*>(&lo);
  const _Float16* ph = reinterpret_cast<const _Float16*>(&hi);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = pl[j];
    r[4 + j] = ph[j];
  }
  return r;
}

// workgroup = 32 ci x 64 co x one row group (4 waves, each 16 ci x 32 co x every tap in registers)
constexpr int kWgRC = 64, kWgKMax = 15;
constexpr int kWgXS = 160;  // X LDS row: 32 ci hi | 32 ci lo (128 B) -> odd multiple of 32 B
constexpr int kWgDS = 288;  // dZ LDS row: 64 co hi | 64 co lo (256 B) -> odd multiple of 32 B
template <int K>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgArgs A) {
  constexpr int XR = kWgRC + K - 1;                     // X rows of a chunk (with the tap halo)
  constexpr int XU = (XR * 8 + 255) / 256, DU = kWgRC * 16 / 256;  // 16-B units per thread
  __shared__ __attribute__((aligned(16))) char xs[2][(kWgRC + kWgKMax - 1 + 16) * kWgXS];
  __shared__ __attribute__((aligned(16))) char ds[2][kWgRC * kWgDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, h = lane >> 4;
  const int wci = wave & 1, wco = (wave >> 1) * 2;
  const int ci0 = blockIdx.x * 32, cog = blockIdx.y * 64;
  const int rg = blockIdx.z;
  const long long r_begin = (long long)rg * A.rows_per_group;
  const long long r_end = r_begin + A.rows_per_group < A.R ? r_begin + A.rows_per_group : A.R;
  const long long x_rows = A.R + K - 1;
  const int sx = prescale_exp(__uint_as_float(*A.amax_x)), sd = prescale_exp(__uint_as_float(*A.amax_dz));
  const float scx = ldexpf(1.f, sx), scd = ldexpf(1.f, sd), unscale = ldexpf(1.f, -sx - sd);
  f32x4 acc[K][2];
#pragma unroll
  for (int t = 0; t < K; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 px[XU], pd[DU];
  auto load = [&](long long r0) {
#pragma unroll
    for (int j = 0; j < XU; ++j) {
      const int i = tid + 256 * j, rr = i >> 3, q = i & 7;
      const long long row = r0 + rr;
      const int c = ci0 + 4 * q;
      px[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i < XR * 8 && row < x_rows && row < r_end + K - 1 && c < A.cin) {
        const float* src = A.x + row * A.cin + c;
        if ((A.cin & 3) == 0) {
          px[j] = *reinterpret_cast<const f32x4*>(src);
        } else {  // few input channels (the 30 s single-channel window's block 1): element loads
#pragma unroll
          for (int e = 0; e < 4; ++e) px[j][e] = c + e < A.cin ? src[e] : 0.f;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < DU; ++j) {
      const int i = tid + 256 * j, rr = i >> 4, q = i & 15;
      const long long row = r0 + rr;
      const int c = cog + 4 * q;
      pd[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (row < r_end && c < A.cout) pd[j] = *reinterpret_cast<const f32x4*>(A.dz + row * A.cout + c);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < XU; ++j) {
      const int i = tid + 256 * j, rr = i >> 3, q = i & 7;
      if (i < XR * 8) {
        f16x4 hi, lo;
        split4(px[j], scx, hi, lo);
        *reinterpret_cast<f16x4*>(xs[buf] + rr * kWgXS + 8 * q) = hi;
        *reinterpret_cast<f16x4*>(xs[buf] + rr * kWgXS + 64 + 8 * q) = lo;
      }
    }
#pragma unroll
    for (int j = 0; j < DU; ++j) {
      const int i = tid + 256 * j, rr = i >> 4, q = i & 15;
      f16x4 hi, lo;
      split4(pd[j], scd, hi, lo);
      *reinterpret_cast<f16x4*>(ds[buf] + rr * kWgDS + 8 * q) = hi;
      *reinterpret_cast<f16x4*>(ds[buf] + rr * kWgDS + 128 + 8 * q) = lo;
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
#pragma unroll
      for (int ks = 0; ks < kWgRC / 32; ++ks) {
        f16x8 bh[2], bl[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          bh[u] = tr_frag(ds[buf], kWgDS, ks * 32, (wco + u) * 16);
          bl[u] = tr_frag(ds[buf], kWgDS, ks * 32, 64 + (wco + u) * 16);
        }
#pragma unroll
        for (int t = 0; t < K; ++t) {
          const f16x8 ah = tr_frag(xs[buf], kWgXS, ks * 32 + t, wci * 16);
          const f16x8 al = tr_frag(xs[buf], kWgXS, ks * 32 + t, 32 + wci * 16);
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[t][u] = mfma3(ah, al, bh[u], bl[u], acc[t][u]);
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
        if (ci + e < A.cin) p[((long long)t * A.cin + ci + e) * A.cout + co] = acc[t][u][e] * unscale;
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

template <int MODE, int CT, bool HALO, bool VEC>
hipError_t go(const ConvArgs& A, dim3 grid, size_t lds, hipStream_t st) {
  auto k = conv_kernel<MODE, CT, HALO, VEC>;
  static size_t attr = 0;
  if (lds > 64 * 1024 && lds > attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr = lds;
  }
  hipLaunchKernelGGL(k, grid, dim3(256), lds, st, A);
  return hipGetLastError();
}

template <int MODE, int CT>
hipError_t go_mode(const ConvArgs& A, dim3 grid, bool halo, bool vec, size_t lds, hipStream_t st) {
  if (halo) return go<MODE, CT, true, true>(A, grid, lds, st);
  if (vec) return go<MODE, CT, false, true>(A, grid, lds, st);
  return go<MODE, CT, false, false>(A, grid, lds, st);
}

}  // namespace gx3

int gx3_max_blocks() { return gx3::kMaxBlocks; }

// weights of nb blocks -> hi/lo fragments (forward, + dgrad where dgr[i]) and per-tensor scales wsc[i]
// (two launches: partial maxima, then the scaled split); wpart: nb * 16 floats of scratch
hipError_t launch_gx3_pack(int nb, const float* const* w, void* const* fwd, void* const* dgr, float* const* wsc,
                           const int* k, const int* cin, const int* cout, float* wpart, hipStream_t st) {
  if (nb < 1 || nb > gx3::kMaxBlocks) return hipErrorInvalidValue;
  gx3::PackArgs P;
  P.nblocks = nb;
  P.wpart = wpart;
  long long most = 0;
  for (int i = 0; i < nb; ++i) {
    auto& B = P.b[i];
    B.w = w[i];
    B.fwd = reinterpret_cast<gx3::f16x8*>(fwd[i]);
    B.dgr = reinterpret_cast<gx3::f16x8*>(dgr[i]);
    B.wsc = wsc[i];
    B.k = k[i];
    B.cin = cin[i];
    B.cout = cout[i];
    if (cout[i] % 4 != 0) return hipErrorInvalidValue;
    B.nf = (long long)((k[i] * cin[i] + 31) / 32) * 512 * ((cout[i] + 15) / 16);
    B.nd = (long long)((k[i] * cout[i] + 31) / 32) * 512 * ((cin[i] + 15) / 16);
    const long long t = B.nf + (B.dgr ? B.nd : 0);
    most = t > most ? t : most;
  }
  hipLaunchKernelGGL(gx3::wmax_kernel, dim3(gx3::kMaxWG, nb), dim3(256), 0, st, P);
  long long gx = (most + 255) / 256;
  if (gx > 512) gx = 512;
  hipLaunchKernelGGL(gx3::pack_kernel, dim3((unsigned)gx, nb), dim3(256), 0, st, P);
  return hipGetLastError();
}

hipError_t launch_gx3_amax(const float* x, long long n, unsigned* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  long long g = (n / 4 + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(gx3::amax_kernel, dim3((unsigned)g), dim3(256), 0, st, x, n, out);
  return hipGetLastError();
}

// mode 1: y = relu(conv(x) + bias) + BN moment slots; mode 2: y = conv(x) (dgrad, flipped packed kernel)
hipError_t launch_gx3_conv(const float* x, long long x_rows, const void* wfrag, const float* wsc, const float* bias,
                           float* y, float* stats, unsigned* amax_out, int n, int L, int cin, int cout, int ksize,
                           int mode, int in_rs, int in_off, int det_slots, hipStream_t st) {
  gx3::ConvArgs A;
  A.x = x;
  A.wfrag = reinterpret_cast<const gx3::f16x8*>(wfrag);
  A.wsc = wsc;
  A.bias = bias;
  A.y = y;
  A.stats = stats;
  A.amax_out = amax_out;
  A.x_rows = x_rows;
  A.n = n;
  A.L = L;
  A.cin = cin;
  A.cout = cout;
  A.ksize = ksize;
  A.in_rs = in_rs;
  A.in_off = in_off;
  A.det = det_slots > 0 ? 1 : 0;
  A.nstep = (ksize * cin + 31) / 32;
  A.nct = (cout + 15) / 16;
  {
    const int p = (ksize - 1) / 2;
    A.tap0 = p - (L - 1) > 0 ? p - (L - 1) : 0;
    A.tap1 = p + L < ksize ? p + L : ksize;
    A.s0 = A.tap0 * cin / 32;
    A.s1 = (A.tap1 * cin + 31) / 32;
  }
  const long long rows = (long long)n * L;
  if (rows == 0) return hipSuccess;
  const int pad = (ksize - 1) / 2;
  // rows a 128-row tile can touch: 127 + ceil(127 / L) sample gaps of (in_rs - L) rows, + the halo
  const long long span = 128 + (long long)(127 + L - 1) / L * (in_rs > L ? in_rs - L : 0) + 2 * pad;
  const bool halo = cin % 32 == 0 && span * 8 <= 256 * 8;
  A.span = halo ? (int)span : 0;
  const size_t lds = (size_t)2 * (halo ? span : 128) * gx3::kRowB;
  const int ct = A.nct % 6 == 0 ? 3 : 4;
  const dim3 grid((unsigned)((rows + 127) / 128), (unsigned)((A.nct + 2 * ct - 1) / (2 * ct)));
  if (mode == gx3::kTrain && A.det && (long long)grid.x * 2 > det_slots) return hipErrorInvalidValue;
  const bool vec = cin % 8 == 0;
  if (mode == gx3::kTrain)
    return ct == 3 ? gx3::go_mode<gx3::kTrain, 3>(A, grid, halo, vec, lds, st)
                   : gx3::go_mode<gx3::kTrain, 4>(A, grid, halo, vec, lds, st);
  return ct == 3 ? gx3::go_mode<gx3::kLinear, 3>(A, grid, halo, vec, lds, st)
                 : gx3::go_mode<gx3::kLinear, 4>(A, grid, halo, vec, lds, st);
}

// gw (k, cin, cout) = sum over R rows; part holds part_floats fp32 (>= one (k, cin, cout) slice)
hipError_t launch_gx3_wgrad(const float* x, const float* dz, const unsigned* amax_x, const unsigned* amax_dz,
                            long long R, int cin, int cout, int k, float* gw, float* part, long long part_floats,
                            hipStream_t st) {
  if (R <= 0) return hipSuccess;
  if (k < 1 || k > gx3::kWgKMax || cin < 1 || cout % 4 != 0) return hipErrorInvalidValue;
  const long long wfl = (long long)k * cin * cout;
  long long groups = part_floats / wfl;
  const long long ci_t = (cin + 31) / 32, co_g = (cout + 63) / 64;
  long long want = (512 + ci_t * co_g - 1) / (ci_t * co_g);  // ~2 workgroups per CU in total
  if (want > (R + 255) / 256) want = (R + 255) / 256;         // at least 256 rows per group
  if (groups > want) groups = want;
  if (groups > 65535) groups = 65535;
  if (groups < 1) return hipErrorInvalidValue;
  long long rpg = (R + groups - 1) / groups;
  rpg = (rpg + gx3::kWgRC - 1) / gx3::kWgRC * gx3::kWgRC;  // whole LDS row chunks
  groups = (R + rpg - 1) / rpg;
  gx3::WgArgs A{x, dz, amax_x, amax_dz, part, R, cin, cout, k, (int)rpg};
  const dim3 grid((unsigned)ci_t, (unsigned)co_g, (unsigned)groups);
  if (!gx3::launch_wgrad_k<1>(k, grid, A, st)) return hipErrorInvalidValue;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_ordered_sum(part, (int)groups, wfl, gw, st);
}

}  // namespace apneauq
