// Fused whole-network inference at the reference's fp32 precision ("fp16x3" MFMA) for the
// short-sequence variants of the Alarcón 1D-CNN (gfx950 / MI355X): the pooled ensemble_cnn members
// (MaxPool1D(2) after blocks 1-5, /root/reference/models/train_deep_ensemble_cnns.py:36-66, evaluated by
// /root/reference/uncertainty_quantification/evaluate_de_global.py:18-38) and the north star's 30 s
// single-channel window.  BN on the moving statistics: Deep-Ensemble predict and standard MC Dropout
// (uq_techniques.py:22,29 with training=False BN).
//
// The bf16 kernel of the same nets (fused_tiled.hip) holds each block's input in LDS as bf16; here it is
// held as two fp16 halves, v 2^sa = hi + lo (hi = fp16(v 2^sa), lo = fp16(v 2^sa - hi)), and each
// product is formed by three v_mfma_f32_16x16x32_f16 (hi*hi + lo*hi + hi*lo, fp32 accumulate) -- the
// arithmetic of the headline engine (x3_layers.hip) and of the layer-wise kernels (gx3_conv.hip):
//
//   * weights: hi/lo fragments of W 2^sw (one exact power of two per layer, host: ops/fused.py
//     pack_blob_x3), the epilogue scale pre-multiplied by 2^-sw;
//   * activations: one power of two sa per SAMPLE and block output, chosen after the block's epilogue
//     values are known: every wave reduces the per-sample max |v| of the values it will store, the
//     barrier the in-place hand-over needs anyway publishes the wave maxima, and every lane then
//     scales by 2^sa (max |v| 2^sa in [2^13, 2^14): hi finite, lo normal) while splitting and storing.
//     A conv output row sums over its own sample's rows only, so the next block's epilogue undoes
//     2^-sa per row exactly.  The network input x (fp32) is prescaled the same way when it is staged.
//     Exponents depend on the sample's own values only: a sample's result does not depend on which
//     samples share its workgroup (sharding / chunking / pass grouping give bitwise-equal results);
//   * BN affine, clamp (ReLU folded), MaxPool, dropout, GAP, Dense and sigmoid in fp32.
//
// LDS row of a block input with c channels: [hi c x fp16 | lo c x fp16 | 16 B] = 4c + 16 bytes (c/4 + 1
// 16-B slots, odd: the ds_read_b128 lane groups of a B fragment hit distinct slots).  The doubled rows
// halve the samples per workgroup against the bf16 kernel (pooled 4, single-channel 2) so that two
// workgroups (8 waves) still share a CU.  Row tiles past the last sample (pooled block 5: 8 rows of one
// 16-row tile) read finite LDS bytes and are never stored.
#include "common.h"
#include "fused_blob.h"

namespace apneauq {
namespace tiled3 {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const f16x8 gf16x8;

using fused::C;
using fused::KS;

constexpr int kThreads = 256;  // 4 waves

__device__ __forceinline__ f32x4 mfma(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// hi = fp16(a) two at a time (v_cvt_pk_f16_f32), lo = fp16(a - hi) by one v_fma_mix per element
// (x3_layers.hip:store_chunk; bit-identical to convert / convert back / subtract / convert)
__device__ __forceinline__ void split2(float a0, float a1, unsigned& hi, unsigned& lo) {
  hi = __builtin_bit_cast(unsigned, (f16x2){(_Float16)a0, (_Float16)a1});
  unsigned l;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(hi), "v"(a0));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(hi), "v"(a1));
  lo = l;
}

// the power of two that puts a nonzero max m into [2^13, 2^14)
__device__ __forceinline__ int prescale_exp(float m) {
  int e = 0;
  if (m > 0.f && m < INFINITY) frexpf(m, &e);  // m = f 2^e, f in [0.5, 1)
  return (m > 0.f && m < INFINITY) ? min(100, max(-100, 14 - e)) : 0;
}

// one exponent per sample of the workgroup (x0 and every block output)
template <int NS>
struct SA {
  int e[NS];
};
template <int NS>
__device__ __forceinline__ int pick(const SA<NS>& s, int smp) {
  int r = s.e[0];
#pragma unroll
  for (int j = 1; j < NS; ++j) r = smp == j ? s.e[j] : r;
  return r;
}
// per-sample maxima of the 4 waves (red[wave][NS]) -> per-sample exponents
template <int NS>
__device__ __forceinline__ SA<NS> exps_from(const float* red) {
  SA<NS> o;
#pragma unroll
  for (int j = 0; j < NS; ++j)
    o.e[j] = prescale_exp(fmaxf(fmaxf(red[j], red[NS + j]), fmaxf(red[2 * NS + j], red[3 * NS + j])));
  return o;
}
template <int NS>
__device__ __forceinline__ void publish_max(float (&mxs)[NS], float* red, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const float v = wave_max(mxs[j]);
    if (lane == 0) red[wave * NS + j] = v;
  }
}

// Per-net geometry: as fused_tiled.hip (RG / NG row tiles per group / groups, WM wave rows, NF full
// channel tiles per wave, HALF shared middle tiles), one row group per block.
struct PooledNet {
  static constexpr int NS = 4, L = 60, CIN0 = 4;
  static constexpr bool IM2COL = false;  // block 1 reads 2 rows x 4 channels per lane (hi and lo) from x0
  static constexpr int X0ROWS = 64;
  static constexpr int LIN[6] = {60, 30, 15, 7, 3, 1};
  static constexpr int SIN[6] = {64, 32, 16, 12, 8, 1};
  static constexpr int OPS[6] = {64, 32, 16, 8, 2, 1};
  static constexpr int LOUT[6] = {30, 15, 7, 3, 1, 1};
  static constexpr bool POOL[6] = {true, true, true, true, true, false};
  static constexpr int T0[6] = {0, 0, 0, 0, 3, 4}, T1[6] = {7, 5, 3, 7, 7, 5};
  static constexpr int RG[6] = {16, 8, 4, 2, 1, 1};
  static constexpr int WM[6] = {1, 1, 1, 1, 1, 1}, NF[6] = {2, 3, 3, 1, 4, 2};
  static constexpr bool HALF[6] = {false, false, true, true, false, false};
};

struct Single30Net {
  static constexpr int NS = 2, L = 30, CIN0 = 1;
  static constexpr bool IM2COL = true;  // x0 row t holds x[t-3 .. t+4] (hi 16 B | lo 16 B)
  static constexpr int X0ROWS = 32;
  static constexpr int LIN[6] = {30, 30, 30, 30, 30, 30};
  static constexpr int SIN[6] = {32, 34, 34, 34, 34, 34};
  static constexpr int OPS[6] = {32, 32, 32, 32, 32, 32};
  static constexpr int LOUT[6] = {30, 30, 30, 30, 30, 30};
  static constexpr bool POOL[6] = {false, false, false, false, false, false};
  static constexpr int T0[6] = {0, 0, 0, 0, 0, 0}, T1[6] = {7, 5, 3, 7, 9, 9};
  static constexpr int RG[6] = {4, 4, 4, 4, 4, 4};
  static constexpr int WM[6] = {1, 1, 1, 1, 1, 2}, NF[6] = {2, 3, 3, 1, 4, 3};
  static constexpr bool HALF[6] = {false, false, true, true, false, false};
};

__host__ __device__ constexpr int row_bytes(int c) { return 4 * c + 16; }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <class N>
struct Lay {
  // slot row read by GEMM row o of block l at tap offset 0 (before - PAD)
  static constexpr int slot_row(int l, int o) {
    return (N::OPS[l] == N::SIN[l] || (N::OPS[5] == 1 && l == 5)) ? o : (o / N::OPS[l]) * N::SIN[l] + o % N::OPS[l];
  }
  static constexpr int max_act() {
    int m = 0;
    for (int l = 1; l < 6; ++l) m = cmax(m, N::NS * N::SIN[l] * row_bytes(C[l]));
    return m;
  }
  // zero rows in front of the first slot: the taps before row 0 that a block runs
  static constexpr int lead() {
    int m = 0;
    for (int l = 1; l < 6; ++l) m = cmax(m, cmax(0, (KS[l] - 1) / 2 - N::T0[l]) * row_bytes(C[l]));
    return (m + 15) / 16 * 16;
  }
  // bytes past max_act() that the discarded rows of the last row tile read (finite, never stored)
  static constexpr int trail() {
    int m = 0;
    for (int l = 1; l < 6; ++l) {
      const int rows = N::RG[l] * 16;
      const int last = slot_row(l, rows - 1) + N::T1[l] - 1 - (KS[l] - 1) / 2 + 1;
      m = cmax(m, last * row_bytes(C[l]) - max_act());
    }
    return (m + 15) / 16 * 16;
  }
  static constexpr int kHB = lead();
  static constexpr int kActBytes = kHB + max_act() + trail();
  static constexpr int kX0Lead = N::IM2COL ? 0 : 4;
  static constexpr int kX0RowB = N::IM2COL ? 32 : 16;  // [hi | lo]
  static constexpr int kX0Bytes = (kX0Lead + N::NS * N::X0ROWS + 8) * kX0RowB;
  static constexpr int kKeyBytes = 6 * N::NS * 4;
  static constexpr int kRedBytes = 16 * N::NS;  // [4 waves][NS] maxima
  static constexpr int kHeadBytes = 4 * N::NS * 4 + 16;
  static constexpr int kLdsBytes = kActBytes + kX0Bytes + kKeyBytes + kRedBytes + kHeadBytes;
  static_assert(kHB % 16 == 0 && kActBytes % 16 == 0 && kX0Bytes % 16 == 0, "LDS carve must stay 16-B aligned");
  static_assert(2 * kLdsBytes <= 160 * 1024, "two workgroups per CU");
};

template <class N, int L>
struct Geo {
  static constexpr int CIN = C[L], COUT = C[L + 1], K = KS[L], PAD = (KS[L] - 1) / 2;
  static constexpr bool FIRST = L == 0, HEAD = L == 5, POOL = N::POOL[L];
  static constexpr int NCT = COUT / 16;
  static constexpr int CB = FIRST ? 1 : CIN / 32;
  static constexpr int S0 = FIRST ? 0 : N::T0[L] * CB, S1 = FIRST ? 1 : N::T1[L] * CB;  // k-steps run
  static constexpr int NWC = 4 / N::WM[L];
  static constexpr int NRW = N::RG[L] / N::WM[L];
  static constexpr int SI = FIRST ? Lay<N>::kX0RowB : row_bytes(CIN);
  static constexpr int SOUT = L < 5 ? N::SIN[L + 1] : 1, SO = row_bytes(COUT);
};

template <class N, int L>
constexpr bool geometry_ok() {
  using G = Geo<N, L>;
  const bool rowhead = N::OPS[5] == 1;
  const int rows = N::RG[L] * 16;
  if (L < 5 || !rowhead) {
    // one row group covers the computed rows (at most one partly discarded row tile)
    if (rows < N::NS * N::OPS[L] || rows >= N::NS * N::OPS[L] + 16) return false;
  } else if (rows < N::NS) {
    return false;
  }
  if (N::OPS[L] > N::SIN[L] && !(L == 5 && rowhead)) return false;
  if (G::POOL && (N::OPS[L] % 2 != 0 || 2 * N::LOUT[L] > N::OPS[L] || N::SIN[L] % 2 != 0)) return false;
  if (L == 0 && (N::OPS[L] != N::SIN[L] || N::SIN[L] != N::X0ROWS)) return false;
  if (N::HALF[L] ? (N::WM[L] != 1 || G::NCT != 2 * (2 * N::NF[L] + 1) || G::NRW % 2 != 0)
                 : (G::NWC * N::NF[L] < G::NCT || N::RG[L] % N::WM[L] != 0))
    return false;
  if (L > 0 && N::LIN[L] > 1 && N::SIN[L] < N::LIN[L] + G::PAD) return false;  // zero rows = next slot's padding
  if (L < 5 && (N::LOUT[L] > G::SOUT || N::LOUT[L] > N::OPS[L])) return false;
  if (L == 5 && !rowhead && (N::OPS[5] % 16 != 0 || N::HALF[5] || G::NRW % (N::OPS[5] / 16) != 0)) return false;
  return true;
}
template <class N>
constexpr bool net_ok() {
  return geometry_ok<N, 0>() && geometry_ok<N, 1>() && geometry_ok<N, 2>() && geometry_ok<N, 3>() &&
         geometry_ok<N, 4>() && geometry_ok<N, 5>() && C[1] % 32 == 0 && C[2] % 32 == 0 && C[3] % 32 == 0 &&
         C[4] % 32 == 0 && C[5] % 32 == 0 && (N::IM2COL ? N::CIN0 * KS[0] <= 8 : N::CIN0 == 4);
}
static_assert(net_ok<PooledNet>(), "pooled geometry");
static_assert(net_ok<Single30Net>(), "single-channel geometry");

extern __shared__ __attribute__((aligned(16))) char smem[];

struct Args {
  const float* x;          // (n_win, L, CIN0) fp32, channels-last
  const uint8_t* blob;     // (n_member, kBlobBytes3) packed parameters (ops/fused.py:pack_blob_x3)
  float* out;              // (n_member, n_pass, n_win)
  long long blob_stride;
  int n_win, n_pass, n_member;
  int tiles_per_member, total_items;
  unsigned window_offset, pass_offset;
  unsigned long long seed;
  int out_logits;
  unsigned thr[6];
};

struct Ctx {
  const guint8* blob;
  unsigned thr;
};

__device__ __forceinline__ void drop4(f32x4& v, unsigned key, unsigned t, unsigned c0, unsigned thr) {
  const unsigned b01 = dropout_bits2(key, t, c0), b23 = dropout_bits2(key, t, c0 + 2);
  v[0] = (b01 & 0xFFFFu) >= thr ? v[0] : 0.f;
  v[1] = (b01 >> 16) >= thr ? v[1] : 0.f;
  v[2] = (b23 & 0xFFFFu) >= thr ? v[2] : 0.f;
  v[3] = (b23 >> 16) >= thr ? v[3] : 0.f;
}

// One block.  sa_in: the per-sample exponents of this block's LDS input; returns those of its output.
template <class N, int L, bool DROP>
__device__ __forceinline__ SA<N::NS> block(const Ctx X, const SA<N::NS> sa_in) {
  using G = Geo<N, L>;
  using Y = Lay<N>;
  constexpr int NS = N::NS, OPSL = N::OPS[L], SINL = N::SIN[L];
  char* act = smem + Y::kHB;
  const char* x0 = smem + Y::kActBytes + Y::kX0Lead * Y::kX0RowB;
  const unsigned* keys = reinterpret_cast<const unsigned*>(smem + Y::kActBytes + Y::kX0Bytes) + L * NS;
  float* red = reinterpret_cast<float*>(smem + Y::kActBytes + Y::kX0Bytes + Y::kKeyBytes);
  float* head = red + 4 * NS;
  constexpr bool HF = N::HALF[L];
  constexpr bool ROWHEAD = G::HEAD && N::OPS[5] == 1;
  constexpr int NFL = N::NF[L], NRW = G::NRW, HRT = NRW / 2;
  constexpr int NFL_A = NFL + (HF ? 1 : 0);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = lane & 15, h = lane >> 4;
  const int wc = wave % G::NWC, wr = wave / G::NWC;
  int ctf, cth = 0, rlo = wr * NRW, rhi = wr * NRW + HRT;
  if constexpr (HF) {
    const int pair = wave >> 1, odd = wave & 1;
    ctf = pair * (2 * NFL + 1) + (odd ? NFL + 1 : 0);
    cth = pair * (2 * NFL + 1) + NFL;
    rlo = odd * HRT;
    rhi = HRT - rlo;
  } else {
    ctf = wc * NFL;
  }
  auto ct_of = [&](int c) { return (HF && c == NFL) ? cth : ctf + c; };
  auto ct_ok = [&](int c) { return HF || ctf + c < G::NCT; };
  auto nrows = [&](int c) { return (HF && c == NFL) ? HRT : NRW; };
  const gf16x8* wp = reinterpret_cast<const gf16x8*>(X.blob + fused::woff3(L)) + lane;
  int ctl[NFL_A];
#pragma unroll
  for (int c = 0; c < NFL_A; ++c) ctl[c] = ct_ok(c) ? ct_of(c) : 0;
  const gfloat* epi = reinterpret_cast<const gfloat*>(X.blob + fused::eoff3(L)) + (DROP ? 4 * G::COUT : 0);

  auto rt_of = [&](int r) { return !HF ? rlo + r : r < HRT ? rlo + r : rhi + r - HRT; };
  f32x4 acc[NFL_A][NRW];
#pragma unroll
  for (int c = 0; c < NFL_A; ++c)
#pragma unroll
    for (int r = 0; r < NRW; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weight fragments of k-step s: hi at 2 (s NCT + ct), lo at the next 1-KiB fragment
  auto load_a = [&](int s, f16x8 (&ah)[NFL_A], f16x8 (&al)[NFL_A]) {
#pragma unroll
    for (int c = 0; c < NFL_A; ++c) {
      ah[c] = wp[(s * G::NCT + ctl[c]) * 128];
      al[c] = wp[(s * G::NCT + ctl[c]) * 128 + 64];
    }
  };
  const int lofs = !G::FIRST ? (m - G::PAD) * G::SI + 16 * h : N::IM2COL ? m * G::SI : (m + 2 * h - G::PAD) * G::SI;
  const char* bb_lo = (G::FIRST ? x0 : act) + rlo * 16 * G::SI + lofs;
  const char* bb_hi = (G::FIRST ? x0 : act) + rhi * 16 * G::SI + lofs;
  constexpr bool DENSE = OPSL == SINL || ROWHEAD;
  const char* bbr[NRW];
#pragma unroll
  for (int r = 0; r < NRW; ++r) {
    const int o = rt_of(r) * 16 + m;
    bbr[r] = act + ((o / OPSL) * SINL + o % OPSL - G::PAD) * G::SI + 16 * h;
  }
  // row tiles per MFMA group: >= 4 independent accumulators between dependent MFMAs
  constexpr int RB0 = NFL_A >= 4 ? 1 : NFL_A >= 2 ? 2 : 4;
  constexpr int RB = RB0 < NRW ? RB0 : NRW;
  auto step = [&](int s, const f16x8 (&ah)[NFL_A], const f16x8 (&al)[NFL_A]) {
    int soff = 0;
    if constexpr (!G::FIRST) {
      const int tap = s / G::CB, cb = s - tap * G::CB;
      soff = __builtin_amdgcn_readfirstlane(tap * G::SI + cb * 64);
    }
#pragma unroll
    for (int r0 = 0; r0 < NRW; r0 += RB) {
      f16x8 bh[RB], bl[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int r = r0 + rb < NRW ? r0 + rb : NRW - 1;
        const char* bb = !DENSE ? bbr[r]
                         : !HF  ? bb_lo + r * 16 * G::SI
                                : (r < HRT ? bb_lo : bb_hi) + (r % (HF ? HRT : 1)) * 16 * G::SI;
        if constexpr (G::FIRST && !N::IM2COL) {
          // k = tap*4 + ci: the lane's 8 k are taps 2h, 2h+1 x 4 channels = two consecutive x0 rows
          const f16x4 h0 = *reinterpret_cast<const f16x4*>(bb), h1 = *reinterpret_cast<const f16x4*>(bb + 16);
          const f16x4 l0 = *reinterpret_cast<const f16x4*>(bb + 8), l1 = *reinterpret_cast<const f16x4*>(bb + 24);
          bh[rb] = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
          bl[rb] = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
        } else if constexpr (G::FIRST) {
          // im2col row: hi 16 B | lo 16 B (lane groups h >= 1 multiply zero weights: any finite row)
          bh[rb] = *reinterpret_cast<const f16x8*>(bb);
          bl[rb] = *reinterpret_cast<const f16x8*>(bb + 16);
        } else {
          bh[rb] = *reinterpret_cast<const f16x8*>(bb + soff);
          bl[rb] = *reinterpret_cast<const f16x8*>(bb + soff + 2 * G::CIN);
        }
      }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < NFL_A; ++c)
          if (r0 + rb < NRW && ct_ok(c) && r0 + rb < nrows(c)) acc[c][r0 + rb] = mfma(ah[c], bh[rb], acc[c][r0 + rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < NFL_A; ++c)
          if (r0 + rb < NRW && ct_ok(c) && r0 + rb < nrows(c)) acc[c][r0 + rb] = mfma(al[c], bh[rb], acc[c][r0 + rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < NFL_A; ++c)
          if (r0 + rb < NRW && ct_ok(c) && r0 + rb < nrows(c)) acc[c][r0 + rb] = mfma(ah[c], bl[rb], acc[c][r0 + rb]);
    }
  };

  // K loop over k-steps [S0, S1): the fragments of step s + 1 in flight under step s's MFMAs
  constexpr int NSTEP = G::S1 - G::S0;
  {
    f16x8 ah[2][NFL_A], al[2][NFL_A];
    load_a(G::S0, ah[0], al[0]);
#pragma unroll 1
    for (int s = 0; s + 1 < NSTEP; s += 2) {
      load_a(G::S0 + s + 1, ah[1], al[1]);
      __builtin_amdgcn_sched_barrier(0);
      step(G::S0 + s, ah[0], al[0]);
      load_a(G::S0 + (s + 2 < NSTEP ? s + 2 : NSTEP - 1), ah[0], al[0]);
      __builtin_amdgcn_sched_barrier(0);
      step(G::S0 + s + 1, ah[1], al[1]);
    }
    if constexpr (NSTEP % 2 == 1) step(G::S0 + NSTEP - 1, ah[0], al[0]);
  }

  // ---- epilogue.  Phase A: bias + ReLU + BN (one fma + med3, the input's 2^-sa folded into the scale),
  // pool, dropout -> values in place in acc, and the max |v| of the values this wave stores.  Barrier
  // (every wave finished reading this block's input rows; the maxima are published).  Phase B: one
  // exponent for the block output, scale, split, store in place.
  constexpr int RPS = OPSL / 16 > 0 ? OPSL / 16 : 1;
  constexpr int NHP = (ROWHEAD || NRW < RPS) ? 1 : NRW / RPS;
  float hp[NHP];
#pragma unroll
  for (int i = 0; i < NHP; ++i) hp[i] = 0.f;
  unsigned keyr[NRW];
#pragma unroll
  for (int r = 0; r < NRW; ++r) {
    const int row = rt_of(r) * 16 + m;
    keyr[r] = DROP ? keys[ROWHEAD ? (m < NS ? m : 0) : (row / OPSL < NS ? row / OPSL : 0)] : 0u;
  }
  // the sample of row tile r of this lane; undo its input exponent (exact powers of two)
  auto smp_of = [&](int r) { return ROWHEAD ? m : (rt_of(r) * 16 + m) / OPSL; };
  // per row tile: the max |v| this lane stores (folded into per-sample maxima once, after the loop)
  float mr[NRW];
  int einr[NRW];
#pragma unroll
  for (int r = 0; r < NRW; ++r) {
    mr[r] = 0.f;
    einr[r] = -pick(sa_in, smp_of(r));
  }
  auto upd = [&](int r, bool st, float a) { mr[r] = st ? fmaxf(mr[r], a) : mr[r]; };
#pragma unroll
  for (int c = 0; c < NFL_A; ++c) {
    if (!ct_ok(c)) break;  // wave-uniform
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      if (r >= nrows(c)) break;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[c][r][i] = ldexpf(acc[c][r][i], einr[r]);
    }
  }
#pragma unroll
  for (int c = 0; c < NFL_A; ++c) {
    if (!ct_ok(c)) break;  // wave-uniform
    const int co0 = ct_of(c) * 16 + 4 * h;
    const f32x4 sc = *reinterpret_cast<const gf32x4*>(epi + co0);
    const f32x4 sh = *reinterpret_cast<const gf32x4*>(epi + G::COUT + co0);
    const f32x4 lo = *reinterpret_cast<const gf32x4*>(epi + 2 * G::COUT + co0);
    const f32x4 hi = *reinterpret_cast<const gf32x4*>(epi + 3 * G::COUT + co0);
    if constexpr (G::POOL) {
      // pool first per lane pair (rows t, t^1 = lanes m, m^1); the even lane finishes channels co0,
      // co0+1 of the pooled element, the odd lane co0+2, co0+3 (fused_tiled.hip)
      const int odd = m & 1, ch = co0 + 2 * odd;
      const float lk0 = odd ? lo[2] : lo[0], lk1 = odd ? lo[3] : lo[1];
      const float hk0 = odd ? hi[2] : hi[0], hk1 = odd ? hi[3] : hi[1];
#pragma unroll
      for (int r = 0; r < NRW; ++r) {
        if (r >= nrows(c)) break;
        f32x4 u;
#pragma unroll
        for (int i = 0; i < 4; ++i) u[i] = __builtin_fmaf(acc[c][r][i], sc[i], sh[i]);
        const float z0 = odd ? u[0] : u[2], z1 = odd ? u[1] : u[3];
        float x0v = odd ? u[2] : u[0], x1v = odd ? u[3] : u[1];
        x0v = __builtin_amdgcn_fmed3f(fmaxf(x0v, dpp_mov<0xB1>(z0)), lk0, hk0);
        x1v = __builtin_amdgcn_fmed3f(fmaxf(x1v, dpp_mov<0xB1>(z1)), lk1, hk1);
        const int row = rt_of(r) * 16 + m;
        const int smp = row / OPSL, tp = (row - smp * OPSL) >> 1;
        if constexpr (DROP) {
          const unsigned bits = dropout_bits2(keyr[r], (unsigned)tp, (unsigned)ch);
          x0v = (bits & 0xFFFFu) >= X.thr ? x0v : 0.f;
          x1v = (bits >> 16) >= X.thr ? x1v : 0.f;
        }
        const bool st = tp < N::LOUT[L] && smp < NS;
        upd(r, st, fmaxf(fabsf(x0v), fabsf(x1v)));
        acc[c][r][0] = x0v;
        acc[c][r][1] = x1v;
      }
      continue;
    }
    f32x4 dw = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (G::HEAD) dw = *reinterpret_cast<const gf32x4*>(reinterpret_cast<const gfloat*>(X.blob + fused::kDenseOff3) + co0);
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      if (r >= nrows(c)) break;
      f32x4 v = acc[c][r];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_fmed3f(__builtin_fmaf(v[i], sc[i], sh[i]), lo[i], hi[i]);
      if constexpr (ROWHEAD) {
        if constexpr (DROP) drop4(v, keyr[r], 0u, (unsigned)co0, X.thr);
        hp[0] += m < NS ? v[0] * dw[0] + v[1] * dw[1] + v[2] * dw[2] + v[3] * dw[3] : 0.f;
      } else {
        const int row = rt_of(r) * 16 + m;
        const int smp = row / OPSL, t = row - smp * OPSL;
        if constexpr (DROP) drop4(v, keyr[r], (unsigned)t, (unsigned)co0, X.thr);
        if constexpr (G::HEAD) {
          const float gsum = v[0] * dw[0] + v[1] * dw[1] + v[2] * dw[2] + v[3] * dw[3];
          hp[r / RPS] += t < N::LOUT[L] ? gsum : 0.f;
        } else {
          const bool st = t < N::LOUT[L] && smp < NS;
          const float a = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
          upd(r, st, a);
          acc[c][r] = v;
        }
      }
    }
  }
  if constexpr (!G::HEAD) {
    float mxs[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) mxs[j] = 0.f;
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      const int smp = smp_of(r);
#pragma unroll
      for (int j = 0; j < NS; ++j) mxs[j] = smp == j ? fmaxf(mxs[j], mr[r]) : mxs[j];
    }
    publish_max<NS>(mxs, red, wave, lane);
  }
  __syncthreads();  // input rows read by every wave; wave maxima visible
  SA<NS> sa_out;
#pragma unroll
  for (int j = 0; j < NS; ++j) sa_out.e[j] = 0;
  if constexpr (!G::HEAD) {
    sa_out = exps_from<NS>(red);
#pragma unroll
    for (int c = 0; c < NFL_A; ++c) {
      if (!ct_ok(c)) break;
      const int co0 = ct_of(c) * 16 + 4 * h;
#pragma unroll
      for (int r = 0; r < NRW; ++r) {
        if (r >= nrows(c)) break;
        const int row = rt_of(r) * 16 + m;
        const int smp = row / OPSL;
        if constexpr (G::POOL) {
          const int tp = (row - smp * OPSL) >> 1, ch = co0 + 2 * (m & 1);
          const int e = pick(sa_out, smp);
          unsigned hv, lv;
          split2(ldexpf(acc[c][r][0], e), ldexpf(acc[c][r][1], e), hv, lv);
          if (tp < N::LOUT[L] && smp < NS) {
            char* o = act + (smp * G::SOUT + tp) * G::SO + ch * 2;
            *reinterpret_cast<unsigned*>(o) = hv;
            *reinterpret_cast<unsigned*>(o + 2 * G::COUT) = lv;
          }
        } else {
          const int t = row - smp * OPSL;
          const int e = pick(sa_out, smp);
          uint2 hv, lv;
          split2(ldexpf(acc[c][r][0], e), ldexpf(acc[c][r][1], e), hv.x, lv.x);
          split2(ldexpf(acc[c][r][2], e), ldexpf(acc[c][r][3], e), hv.y, lv.y);
          if (t < N::LOUT[L] && smp < NS) {
            char* o = act + (smp * G::SOUT + t) * G::SO + co0 * 2;
            *reinterpret_cast<uint2*>(o) = hv;
            *reinterpret_cast<uint2*>(o + 2 * G::COUT) = lv;
          }
        }
      }
    }
    // the zero rows LOUT .. SOUT-1 of the output slots (the next block's padding), hi and lo
    constexpr int ZR = G::SOUT - N::LOUT[L], CPR = 4 * G::COUT / 16;
    if constexpr (ZR > 0)
    for (int i = threadIdx.x; i < NS * ZR * CPR; i += kThreads) {
      const int sr = i / CPR, chk = i - sr * CPR;
      const int smp = sr / ZR, tr = N::LOUT[L] + sr % ZR;
      *reinterpret_cast<f32x4*>(act + (smp * G::SOUT + tr) * G::SO + chk * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  } else if constexpr (ROWHEAD) {
    float p = hp[0];
    p += __shfl_xor(p, 16, kWave);
    p += __shfl_xor(p, 32, kWave);
    if (h == 0 && m < NS) head[wave * NS + m] = p;
  } else {
#pragma unroll
    for (int i = 0; i < NHP; ++i) {
      float p = group16_sum(hp[i]);
      p += __shfl_xor(p, 16, kWave);
      p += __shfl_xor(p, 32, kWave);
      if (lane == 0) head[(rt_of(RPS * i) / RPS) * G::NWC + wc] = p;
    }
  }
  __syncthreads();  // block output (or head partials) visible to every wave
  return sa_out;
}

template <class N, bool DROP>
__global__ __launch_bounds__(kThreads, 2) void fused_tiled_x3_kernel(Args A) {
  using Y = Lay<N>;
  constexpr int NS = N::NS;
  char* x0 = smem + Y::kActBytes;
  unsigned* keys = reinterpret_cast<unsigned*>(smem + Y::kActBytes + Y::kX0Bytes);
  float* red = reinterpret_cast<float*>(smem + Y::kActBytes + Y::kX0Bytes + Y::kKeyBytes);
  float* head = red + 4 * NS;
  // zero rows every block may read as padding (leading rows, the discarded rows' tail), once.  The rest
  // of the LDS is written before it is read by any stored row (a NaN-filled LDS gives bitwise the same
  // results: tools/debug/ft3_ab.py)
  for (int i = threadIdx.x; i < Y::kHB / 16; i += kThreads) reinterpret_cast<f32x4*>(smem)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = threadIdx.x; i < Y::trail() / 16; i += kThreads)
    reinterpret_cast<f32x4*>(smem + Y::kHB + Y::max_act())[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < Y::kX0Lead * Y::kX0RowB / 16) reinterpret_cast<f32x4*>(x0)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 8 * Y::kX0RowB / 16)
    reinterpret_cast<f32x4*>(x0 + (Y::kX0Lead + NS * N::X0ROWS) * Y::kX0RowB)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rem = nwg % 8, xcd = bid % 8;
  const int item = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + bid / 8;
  APNEAUQ_DASSERT(item < A.total_items && blockDim.x == kThreads);
  const int member = item / A.tiles_per_member;
  const int tile = item - member * A.tiles_per_member;
  const long long samples = (long long)A.n_pass * A.n_win;

  // stage x: one x0 row per thread in registers, the tile's max |x| -> one exponent, then hi / lo
  constexpr int XV = N::IM2COL ? 8 : 4;
  static_assert(NS * N::X0ROWS <= kThreads, "one x0 row per thread");
  const bool xrow = threadIdx.x < NS * N::X0ROWS;
  const int sl = threadIdx.x / N::X0ROWS, t = threadIdx.x % N::X0ROWS;
  const long long gs = (long long)tile * NS + sl;
  const bool ok = xrow && gs < samples && t < N::L;
  const float* xs = A.x + (long long)(ok ? gs % A.n_win : 0) * (N::L * N::CIN0);
  float xv[XV];
  if constexpr (N::IM2COL) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ts = t + j - (KS[0] - 1) / 2;
      xv[j] = (ok && ts >= 0 && ts < N::L && j < KS[0]) ? xs[ts] : 0.f;
    }
  } else {
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ok) v = *reinterpret_cast<const f32x4*>(xs + 4 * t);
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = v[j];
  }
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < XV; ++j) mx = fmaxf(mx, fabsf(xv[j]));
  float mxs[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) mxs[j] = xrow && sl == j ? mx : 0.f;
  publish_max<NS>(mxs, red, threadIdx.x >> 6, threadIdx.x & 63);
  // per-(block, sample) dropout keys: the same (seed, layer, pass, window) streams as every path
  if (DROP && threadIdx.x < 6 * NS) {
    const int l = threadIdx.x / NS, s2 = threadIdx.x % NS;
    const long long g2 = (long long)tile * NS + s2;
    const long long gg = g2 < samples ? g2 : 0;
    const unsigned pass = (unsigned)(gg / A.n_win), win = (unsigned)(gg % A.n_win);
    keys[threadIdx.x] = sample_key(stream_key(A.seed, (unsigned)l, A.pass_offset + pass), A.window_offset + win);
  }
  __syncthreads();
  const SA<NS> sa0 = exps_from<NS>(red);
  const int e0 = pick(sa0, sl);
  if (xrow) {
    char* row = x0 + (Y::kX0Lead + threadIdx.x) * Y::kX0RowB;
    unsigned hv[XV / 2], lv[XV / 2];
#pragma unroll
    for (int j = 0; j < XV / 2; ++j) split2(ldexpf(xv[2 * j], e0), ldexpf(xv[2 * j + 1], e0), hv[j], lv[j]);
    if constexpr (N::IM2COL) {
      *reinterpret_cast<uint4*>(row) = uint4{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<uint4*>(row + 16) = uint4{lv[0], lv[1], lv[2], lv[3]};
    } else {
      *reinterpret_cast<uint4*>(row) = uint4{hv[0], hv[1], lv[0], lv[1]};
    }
  }
  __syncthreads();

  Ctx X;
  X.blob = (const guint8*)(A.blob) + (long long)member * A.blob_stride;
  X.thr = A.thr[0];
  SA<NS> sa = block<N, 0, DROP>(X, sa0);
  X.thr = A.thr[1];
  sa = block<N, 1, DROP>(X, sa);
  X.thr = A.thr[2];
  sa = block<N, 2, DROP>(X, sa);
  X.thr = A.thr[3];
  sa = block<N, 3, DROP>(X, sa);
  X.thr = A.thr[4];
  sa = block<N, 4, DROP>(X, sa);
  X.thr = A.thr[5];
  block<N, 5, DROP>(X, sa);

  if (threadIdx.x < NS) {
    const int s2 = threadIdx.x;
    const long long g2 = (long long)tile * NS + s2;
    if (g2 < samples) {
      float logit;
      if constexpr (N::OPS[5] == 1)
        logit = head[s2] + head[NS + s2] + head[2 * NS + s2] + head[3 * NS + s2];
      else {
        constexpr int NWC5 = 4 / N::WM[5];
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NWC5; ++w) s += head[NWC5 * s2 + w];
        logit = s * (1.0f / N::L);
      }
      logit += reinterpret_cast<const gfloat*>(X.blob + fused::kDenseOff3)[C[6]];
      const int pass = (int)(g2 / A.n_win), win = (int)(g2 % A.n_win);
      A.out[((long long)member * A.n_pass + pass) * A.n_win + win] =
          A.out_logits ? logit : 1.0f / (1.0f + __expf(-logit));
    }
  }
}

template <class N>
hipError_t launch(const float* x, const uint8_t* blob, long long blob_stride, float* out, int n_win, int n_pass,
                  int n_member, unsigned window_offset, unsigned pass_offset, unsigned long long seed, int dropout,
                  int out_logits, const unsigned* thr, hipStream_t stream) {
  Args A;
  A.x = x;
  A.blob = blob;
  A.out = out;
  A.blob_stride = blob_stride;
  A.n_win = n_win;
  A.n_pass = n_pass;
  A.n_member = n_member;
  const long long samples = (long long)n_pass * n_win;
  const long long tiles = (samples + N::NS - 1) / N::NS;
  if (tiles < 1 || n_member < 1) return hipSuccess;
  if (tiles * n_member >= (1LL << 31)) return hipErrorInvalidValue;
  A.tiles_per_member = (int)tiles;
  A.total_items = (int)(tiles * n_member);
  A.window_offset = window_offset;
  A.pass_offset = pass_offset;
  A.seed = seed;
  A.out_logits = out_logits;
  for (int l = 0; l < 6; ++l) A.thr[l] = thr ? thr[l] : 0u;
  if (dropout)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(fused_tiled_x3_kernel<N, true>), dim3(A.total_items), dim3(kThreads),
                       Lay<N>::kLdsBytes, stream, A);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(fused_tiled_x3_kernel<N, false>), dim3(A.total_items), dim3(kThreads),
                       Lay<N>::kLdsBytes, stream, A);
  return hipGetLastError();
}

}  // namespace tiled3

// net 0: the pooled (60, 4) CNN; net 1: the (30, 1) single-channel CNN; fp32 input, x3 blob
hipError_t launch_fused_tiled_x3(int net, const float* x, const uint8_t* blob, long long blob_stride, float* out,
                                 int n_win, int n_pass, int n_member, unsigned window_offset, unsigned pass_offset,
                                 unsigned long long seed, int dropout, int out_logits, const unsigned* thr,
                                 hipStream_t stream) {
  if (net == 0)
    return tiled3::launch<tiled3::PooledNet>(x, blob, blob_stride, out, n_win, n_pass, n_member, window_offset,
                                             pass_offset, seed, dropout, out_logits, thr, stream);
  if (net == 1)
    return tiled3::launch<tiled3::Single30Net>(x, blob, blob_stride, out, n_win, n_pass, n_member, window_offset,
                                               pass_offset, seed, dropout, out_logits, thr, stream);
  return hipErrorInvalidValue;
}

void fused_layout_x3(int* woffs, int* eoffs, int* dense_off, int* bytes, int* lds) {
  for (int l = 0; l < 6; ++l) {
    woffs[l] = fused::woff3(l);
    eoffs[l] = fused::eoff3(l);
  }
  *dense_off = fused::kDenseOff3;
  *bytes = fused::kBlobBytes3;
  lds[0] = tiled3::Lay<tiled3::PooledNet>::kLdsBytes;
  lds[1] = tiled3::Lay<tiled3::Single30Net>::kLdsBytes;
}

}  // namespace apneauq
