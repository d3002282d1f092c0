// Fused whole-network inference of the POOLED Alarcón 1D-CNN on gfx950 (MI355X): the reference CNN
// with MaxPool1D(2, valid) after blocks 1-5 (the pooling lines commented out in
// /root/reference/models/train_deep_ensemble_cnns.py:36-66; the thesis' pooled `ensemble_cnn/`
// models, evaluate_de_global.py:18).  Sequence lengths 60 -> 30 -> 15 -> 7 -> 3 -> 1.
//
// One launch runs all six Conv1D -> ReLU -> BN(running) -> [MaxPool] -> [Dropout] blocks, GAP, Dense
// and sigmoid for every (member, pass, window) sample, like fused_forward.hip, and reads the same
// parameter blob (fused_blob.h).  What changes with pooling is the row geometry, and with it the
// design point:
//
//   * rows shrink 2x per block, so a 2-sample tile would stream the whole 1.7 MB weight set for
//     ~15 GEMM rows per block on average.  A workgroup here owns 8 samples; every weight fragment
//     feeds >= 4 row tiles (blocks 1-2 are split into row groups of 8 row tiles to bound the
//     accumulators, block 6 has one);
//   * each block's input lives in LDS in per-sample slots of SIN rows: LIN valid rows, then zero
//     rows that double as the 'same' padding of the next slot (SIN >= LIN + PAD), so the
//     implicit-GEMM conv needs no bounds checks.  LDS row = GEMM row;
//   * only the rows the pool keeps are computed where that saves row tiles (block 4: 8 of 12 slot
//     rows, block 5: 2 of 8), and taps that can never reach a valid input row are skipped: block 5
//     (3 rows, k = 9) runs taps 3..6 for its 2 kept rows, block 6 (1 row, k = 9) only the centre tap
//     -- block 6 is a dense 256 -> 96 layer, 9x fewer MFMAs than the padded conv;
//   * the epilogue pools rows t, t^1 (lanes m, m^1) with one DPP quad permute, applies the
//     counter-based dropout keyed by the pooled step (ops/rng.py, same masks as generic_conv.hip)
//     and writes bf16 in place over the block input (a barrier after the K loop; row groups
//     write only bytes no later group reads -- static_asserts below), plus the slot's zero rows;
//   * block 6 feeds Dense(96 -> 1) in fp32 (L = 1: GAP is the identity), channel-tile partials
//     combined in a fixed order (bitwise sharding invariance).
//   LDS per workgroup ~78 KiB -> 2 workgroups (8 waves) per CU.
#include "common.h"
#include "fused_blob.h"

namespace apneauq {
namespace pooled {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

using fused::C;
using fused::eoff;
using fused::kDenseOff;
using fused::KS;
using fused::woff;

constexpr int kNS = 8;          // samples per workgroup tile
constexpr int kThreads = 256;   // 4 waves
constexpr int kL = 60, kCin = 4;

// per-block geometry (block l reads slots of SIN[l] rows, LIN[l] of them valid)
constexpr int LIN[6] = {60, 30, 15, 7, 3, 1};
constexpr int SIN[6] = {64, 32, 16, 12, 8, 1};
constexpr int LOUT[6] = {30, 15, 7, 3, 1, 1};   // rows after MaxPool1D(2, valid) (block 6: no pool)
constexpr int T0[6] = {0, 0, 0, 0, 3, 4};       // taps [T0, T1) reach a valid input row of a kept output row
constexpr int T1[6] = {7, 5, 3, 7, 7, 5};
// GEMM rows computed per sample: all SIN slot rows, except where the pool keeps only a prefix --
// block 4 computes t < 8 of its 12-row slots (pool keeps t < 6), block 5 t < 2 of 8 (keeps t < 2);
// a computed row o is slot row (o / OPS) * SIN + o % OPS
constexpr int OPS[6] = {64, 32, 16, 8, 2, 1};
constexpr int RG[6] = {8, 8, 8, 4, 1, 1};       // row tiles per row group
constexpr int NG[6] = {4, 2, 1, 1, 1, 1};       // row groups
constexpr int WM[6] = {1, 1, 1, 1, 1, 1};       // wave rows (4 / WM wave columns over channel tiles)
constexpr int NF[6] = {2, 3, 3, 1, 4, 2};       // full channel tiles per wave
// HALF: Cout tiles that do not split 4 ways (224 -> 14, 96 -> 6 = 2 pairs x (2 NF + 1)) -- each wave
// pair shares its middle tile, one wave per half of the row tiles, so every weight fragment is
// requested once per workgroup and all waves issue the same MFMA count (2 wave rows loading the
// same fragments: profiles/pooled_fused_r3.md)
constexpr bool HALF[6] = {false, false, true, true, false, false};
// k-steps of weight fragments in flight ahead of the MFMAs.  Depths (3,3,2,4,3,4) and (4,4,3,6,5,6)
// measured 0.8 % and 1.9 % slower than 1 everywhere (profiles/pooled_fused_r3.md): weight latency is
// not what bounds this kernel.
constexpr int PD[6] = {1, 1, 1, 1, 1, 1};

__host__ __device__ constexpr int row_bytes(int c) { return 2 * c + 16; }  // +16 B: conflict-free rows
constexpr int kHB = 4 * row_bytes(256);                                      // leading zero rows (>= PAD rows of any block)
constexpr int act_bytes(int l) { return kNS * SIN[l] * row_bytes(C[l]); }
constexpr int max_act() {
  int m = 0;
  for (int l = 1; l < 6; ++l) m = act_bytes(l) > m ? act_bytes(l) : m;
  return m;
}
constexpr int kActBytes = kHB + max_act() + 4 * row_bytes(256);  // + trailing slack (discarded rows' taps)
constexpr int kX0Lead = 4, kX0Rows = kX0Lead + kNS * 64 + 8;
constexpr int kX0Bytes = kX0Rows * kCin * 2;
constexpr int kKeyBytes = 6 * kNS * 4;
constexpr int kHeadBytes = 4 * kNS * 4 + kNS * 4;
constexpr int kLdsBytes = kActBytes + kX0Bytes + kKeyBytes + kHeadBytes;
static_assert(kActBytes % 16 == 0 && kX0Bytes % 16 == 0, "LDS carve must stay 16-B aligned");
static_assert(2 * kLdsBytes <= 160 * 1024, "two workgroups per CU");

template <int L>
struct Geo {
  static constexpr int CIN = C[L], COUT = C[L + 1], K = KS[L], PAD = (KS[L] - 1) / 2;
  static constexpr bool FIRST = L == 0, HEAD = L == 5, POOL = L < 5;
  static constexpr int NCT = COUT / 16;
  static constexpr int CB = FIRST ? 1 : CIN / 32;
  static constexpr int S0 = FIRST ? 0 : T0[L] * CB, S1 = FIRST ? 1 : T1[L] * CB;  // k-steps run
  static constexpr int NWC = 4 / WM[L];          // wave columns
  static constexpr int NRW = RG[L] / WM[L];      // row tiles per wave per group
  static constexpr int SI = FIRST ? kCin * 2 : row_bytes(CIN);
  static constexpr int SOUT = L < 5 ? SIN[L + 1] : 1, SO = row_bytes(COUT);
  static constexpr int SPG = RG[L] * 16 / OPS[L];  // samples per row group (block 6: all 8)
};

// compile-time checks of the slot geometry and the in-place hand-over
template <int L>
constexpr bool geometry_ok() {
  using G = Geo<L>;
  if (L < 5 && RG[L] * NG[L] * 16 != kNS * OPS[L]) return false;  // row groups tile the computed rows
  if (L < 5 && (OPS[L] > SIN[L] || OPS[L] % 2 != 0 || 2 * LOUT[L] > OPS[L])) return false;  // pool pairs
  if (L == 0 && OPS[L] != SIN[L]) return false;
  if (L == 5 && RG[L] * 16 < kNS) return false;
  if (HALF[L] ? (WM[L] != 1 || G::NCT != 2 * (2 * NF[L] + 1) || RG[L] % 2 != 0)
              : (G::NWC * NF[L] < G::NCT || RG[L] % WM[L] != 0))
    return false;  // wave tiling covers the block
  if (L > 0 && L < 5 && SIN[L] < LIN[L] + G::PAD) return false;    // zero rows = next slot's padding
  if (L < 5 && (2 * LOUT[L] > SIN[L] || LOUT[L] > G::SOUT)) return false;
  // row group g's output ends before group g+1's first input row (minus the padding)
  if (L >= 1 && NG[L] > 1 &&
      G::SPG * G::SOUT * G::SO > (G::SPG * SIN[L] - G::PAD) * G::SI)
    return false;
  if (L >= 1 && kNS * SIN[L] * G::SI > max_act()) return false;
  return true;
}
static_assert(geometry_ok<0>() && geometry_ok<1>() && geometry_ok<2>() && geometry_ok<3>() && geometry_ok<4>() &&
                  geometry_ok<5>(),
              "pooled geometry");
static_assert(C[1] % 32 == 0 && C[2] % 32 == 0 && C[3] % 32 == 0 && C[4] % 32 == 0 && C[5] % 32 == 0,
              "k-steps stay inside one tap");

extern __shared__ __attribute__((aligned(16))) char smem[];

struct Args {
  const __bf16* x;         // (n_win, 60, 4) bf16, channels-last
  const uint8_t* blob;     // (n_member, kBlobBytes) packed parameters (ops/fused.py:pack_blob)
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
  int out_logits;
};

template <int L, bool DROP>
__device__ __forceinline__ void pblock(const Ctx X) {
  using G = Geo<L>;
  char* act = smem + kHB;
  const char* x0 = smem + kActBytes + kX0Lead * kCin * 2;
  const unsigned* keys = reinterpret_cast<const unsigned*>(smem + kActBytes + kX0Bytes) + L * kNS;
  float* head = reinterpret_cast<float*>(smem + kActBytes + kX0Bytes + kKeyBytes);
  constexpr bool HF = HALF[L];
  constexpr int NFL = NF[L], NRW = G::NRW, HRT = NRW / 2;
  constexpr int NFL_A = NFL + (HF ? 1 : 0);  // weight fragments per wave per k-step

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = lane & 15, h = lane >> 4;
  const int wc = wave % G::NWC, wr = wave / G::NWC;
  // channel tiles: NFL full ones from ctf (+ the pair's shared middle tile cth with HALF); local row
  // tile r < HRT is row tile rlo + r, r >= HRT is rhi + r - HRT (HALF: the odd wave of a pair
  // swaps the halves, so the shared tile always sits in local rows r < HRT, a compile-time range)
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
  auto ct_ok = [&](int c) { return HF || ctf + c < G::NCT; };  // block 6: 6 tiles over 4 x 2 (wave-uniform)
  auto nrows = [&](int c) { return (HF && c == NFL) ? HRT : NRW; };  // compile-time after unrolling
  const gbf16x8* wp = reinterpret_cast<const gbf16x8*>(X.blob + woff(L)) + lane;
  int ctl[NFL_A];  // tiles past NCT load tile 0 and skip their MFMAs
#pragma unroll
  for (int c = 0; c < NFL_A; ++c) ctl[c] = ct_ok(c) ? ct_of(c) : 0;

  const gfloat* epi = reinterpret_cast<const gfloat*>(X.blob + eoff(L)) + (DROP ? 4 * G::COUT : 0);

#pragma unroll 1
  for (int g = 0; g < NG[L]; ++g) {
    const int rg0 = g * RG[L];
    auto rt_of = [&](int r) { return rg0 + (!HF ? rlo + r : r < HRT ? rlo + r : rhi + r - HRT); };
    f32x4 acc[NFL_A][NRW];
#pragma unroll
    for (int c = 0; c < NFL_A; ++c)
#pragma unroll
      for (int r = 0; r < NRW; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto load_a = [&](int s, bf16x8 (&a)[NFL_A]) {
#pragma unroll
      for (int c = 0; c < NFL_A; ++c) a[c] = wp[(s * G::NCT + ctl[c]) * 64];
    };
    const int lofs = G::FIRST ? (m + 2 * h - G::PAD) * G::SI : (m - G::PAD) * G::SI + 16 * h;
    const char* bb_lo = (G::FIRST ? x0 : act) + (rg0 + rlo) * 16 * G::SI + lofs;
    const char* bb_hi = (G::FIRST ? x0 : act) + (rg0 + rhi) * 16 * G::SI + lofs;
    constexpr bool DENSE = OPS[L] == SIN[L];  // computed row = slot row (else one base per row tile)
    const char* bbr[NRW];
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      const int o = rt_of(r) * 16 + m;
      bbr[r] = act + ((o / OPS[L]) * SIN[L] + o % OPS[L] - G::PAD) * G::SI + 16 * h;
    }
    auto step = [&](int s, const bf16x8 (&a)[NFL_A]) {
      int soff = 0;
      if constexpr (!G::FIRST) {
        const int tap = s / G::CB, cb = s - tap * G::CB;
        soff = __builtin_amdgcn_readfirstlane(tap * G::SI + cb * 64);
      }
#pragma unroll
      for (int r = 0; r < NRW; ++r) {
        const char* bb = !DENSE ? bbr[r]
                         : !HF  ? bb_lo + r * 16 * G::SI
                                : (r < HRT ? bb_lo : bb_hi) + (r % (HF ? HRT : 1)) * 16 * G::SI;
        bf16x8 b;
        if constexpr (G::FIRST) {
          // k = tap*4 + ci: the lane's 8 k are taps 2h, 2h+1 x 4 channels = two consecutive rows
          const bf16x4 lo = *reinterpret_cast<const bf16x4*>(bb);
          const bf16x4 hi = *reinterpret_cast<const bf16x4*>(bb + 8);
          b = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else {
          b = *reinterpret_cast<const bf16x8*>(bb + soff);
        }
#pragma unroll
        for (int c = 0; c < NFL_A; ++c)
          if (ct_ok(c) && r < nrows(c)) acc[c][r] = mfma16(a[c], b, acc[c][r]);  // wave-uniform
      }
    };

    // K loop over k-steps [S0, S1): a ring of NSG register stages, the fragments of step s + PD in
    // flight under step s's MFMAs (loads past the end are clamped: vmcnt bookkeeping stays exact)
    constexpr int NSTEP = G::S1 - G::S0, PDL = PD[L] < NSTEP ? PD[L] : NSTEP, NSG = PDL + 1;
    constexpr int NFULL = NSTEP / NSG * NSG;
    bf16x8 a[NSG][NFL_A];
#pragma unroll
    for (int j = 0; j < PDL; ++j) load_a(G::S0 + j, a[j]);
#pragma unroll 1
    for (int s0 = 0; s0 < NFULL; s0 += NSG) {
#pragma unroll
      for (int j = 0; j < NSG; ++j) {
        const int s = s0 + j;
        load_a(G::S0 + (s + PDL < NSTEP ? s + PDL : NSTEP - 1), a[(j + PDL) % NSG]);
        __builtin_amdgcn_sched_barrier(0);
        step(G::S0 + s, a[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < NSTEP - NFULL; ++j) step(G::S0 + NFULL + j, a[j]);

    // ---- epilogue: bias + ReLU + BN (one fma + med3), pool, dropout; bf16 in place / dense head
    if constexpr (!G::FIRST) __syncthreads();  // every wave finished reading this group's input rows
    float hp = 0.f;                            // HEAD: this lane's share of sample m's logit
#pragma unroll
    for (int c = 0; c < NFL_A; ++c) {
      if (!ct_ok(c)) break;  // wave-uniform
      const int co0 = ct_of(c) * 16 + 4 * h;
      const f32x4 sc = *reinterpret_cast<const gf32x4*>(epi + co0);
      const f32x4 sh = *reinterpret_cast<const gf32x4*>(epi + G::COUT + co0);
      const f32x4 lo = *reinterpret_cast<const gf32x4*>(epi + 2 * G::COUT + co0);
      const f32x4 hi = *reinterpret_cast<const gf32x4*>(epi + 3 * G::COUT + co0);
      if constexpr (G::POOL) {
        // Pool first, per lane pair (rows t, t^1 = lanes m, m^1, the same 4 channels): the BN clamp is
        // monotone, so max(clamp(u_a), clamp(u_b)) == clamp(max(u_a, u_b)) exactly, u = fma(acc, s, t').
        // The even lane then finishes channels co0, co0+1 of the pooled element and the odd lane
        // co0+2, co0+3: half the clamp / dropout / convert / store work per lane.
        const int odd = m & 1, ch = co0 + 2 * odd;
        const float lk0 = odd ? lo[2] : lo[0], lk1 = odd ? lo[3] : lo[1];
        const float hk0 = odd ? hi[2] : hi[0], hk1 = odd ? hi[3] : hi[1];
#pragma unroll
        for (int r = 0; r < NRW; ++r) {
          if (r >= nrows(c)) break;
          f32x4 u;
#pragma unroll
          for (int i = 0; i < 4; ++i) u[i] = __builtin_fmaf(acc[c][r][i], sc[i], sh[i]);
          const float z0 = odd ? u[0] : u[2], z1 = odd ? u[1] : u[3];  // the partner's channels
          float x0 = odd ? u[2] : u[0], x1 = odd ? u[3] : u[1];
          x0 = __builtin_amdgcn_fmed3f(fmaxf(x0, dpp_mov<0xB1>(z0)), lk0, hk0);
          x1 = __builtin_amdgcn_fmed3f(fmaxf(x1, dpp_mov<0xB1>(z1)), lk1, hk1);
          const int row = rt_of(r) * 16 + m;
          const int smp = row / OPS[L], tp = (row - smp * OPS[L]) >> 1;
          if constexpr (DROP) {
            const unsigned bits = dropout_bits2(keys[smp], (unsigned)tp, (unsigned)ch);
            x0 = (bits & 0xFFFFu) >= X.thr ? x0 : 0.f;
            x1 = (bits >> 16) >= X.thr ? x1 : 0.f;
          }
          if (tp < LOUT[L])
            *reinterpret_cast<bf16x2*>(act + (smp * G::SOUT + tp) * G::SO + ch * 2) = bf16x2{(__bf16)x0, (__bf16)x1};
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < NRW; ++r) {  // HEAD (block 6): no pool, rows m < 8 are the samples
        f32x4 v = acc[c][r];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_fmed3f(__builtin_fmaf(v[i], sc[i], sh[i]), lo[i], hi[i]);
        if constexpr (DROP) {
          const unsigned key = keys[m < kNS ? m : 0];
          const unsigned b01 = dropout_bits2(key, 0u, (unsigned)co0);
          const unsigned b23 = dropout_bits2(key, 0u, (unsigned)co0 + 2);
          v[0] = (b01 & 0xFFFFu) >= X.thr ? v[0] : 0.f;
          v[1] = (b01 >> 16) >= X.thr ? v[1] : 0.f;
          v[2] = (b23 & 0xFFFFu) >= X.thr ? v[2] : 0.f;
          v[3] = (b23 >> 16) >= X.thr ? v[3] : 0.f;
        }
        const f32x4 dw = *reinterpret_cast<const gf32x4*>(reinterpret_cast<const gfloat*>(X.blob + kDenseOff) + co0);
        hp += m < kNS ? v[0] * dw[0] + v[1] * dw[1] + v[2] * dw[2] + v[3] * dw[3] : 0.f;
      }
    }
    if constexpr (G::HEAD) {
      hp += __shfl_xor(hp, 16, kWave);  // the 4 channel quarters of the tile (fixed order)
      hp += __shfl_xor(hp, 32, kWave);
      if (h == 0 && m < kNS) head[wave * kNS + m] = hp;
    } else {
      // the zero rows LOUT .. SOUT-1 of this group's output slots (the next block's padding)
      constexpr int ZR = G::SOUT - LOUT[L], CPR = G::COUT / 8;  // 16-B chunks per row
      for (int i = threadIdx.x; i < G::SPG * ZR * CPR; i += kThreads) {
        const int sr = i / CPR, ch = i - sr * CPR;
        const int smp = g * G::SPG + sr / ZR, tr = LOUT[L] + sr % ZR;
        *reinterpret_cast<f32x4*>(act + (smp * G::SOUT + tr) * G::SO + ch * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  __syncthreads();  // block output (or head partials) visible to every wave
}

template <bool DROP>
__global__ __launch_bounds__(kThreads, 2) void fused_pooled_kernel(Args A) {
  char* x0 = smem + kActBytes;
  unsigned* keys = reinterpret_cast<unsigned*>(smem + kActBytes + kX0Bytes);
  float* head = reinterpret_cast<float*>(smem + kActBytes + kX0Bytes + kKeyBytes);
  // zero the leading / trailing rows every block may read as padding, once
  for (int i = threadIdx.x; i < kHB / 16; i += kThreads) {
    reinterpret_cast<f32x4*>(smem)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    reinterpret_cast<f32x4*>(smem + kActBytes - 4 * row_bytes(256))[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (threadIdx.x < kX0Lead * kCin * 2 / 16)
    reinterpret_cast<f32x4*>(x0)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 8 * kCin * 2 / 16)
    reinterpret_cast<f32x4*>(x0 + (kX0Lead + kNS * 64) * kCin * 2)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};

  // XCD-aware item order (as fused_forward.hip): an XCD's workgroups take a contiguous item range
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rem = nwg % 8, xcd = bid % 8;
  const int item = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + bid / 8;
  APNEAUQ_DASSERT(item < A.total_items && blockDim.x == kThreads);
  const int member = item / A.tiles_per_member;
  const int tile = item - member * A.tiles_per_member;
  const long long samples = (long long)A.n_pass * A.n_win;

  // stage the 8 input windows: 480 B + 32 zero bytes (rows 60..63) per 512-B slot, one 16-B chunk
  // per thread
  {
    const int sl = threadIdx.x >> 5, ch = threadIdx.x & 31;
    const long long gs = (long long)tile * kNS + sl;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ch < 30 && gs < samples) {
      const int win = (int)(gs % A.n_win);
      v = reinterpret_cast<const f32x4*>(A.x + (long long)win * (kL * kCin))[ch];
    }
    reinterpret_cast<f32x4*>(x0 + (kX0Lead + sl * 64) * kCin * 2)[ch] = v;
  }
  // per-(block, sample) dropout keys: the same (seed, layer, pass, window) streams as every path
  if (DROP && threadIdx.x < 6 * kNS) {
    const int l = threadIdx.x / kNS, sl = threadIdx.x % kNS;
    const long long gs = (long long)tile * kNS + sl;
    const long long gg = gs < samples ? gs : 0;
    const unsigned pass = (unsigned)(gg / A.n_win), win = (unsigned)(gg % A.n_win);
    keys[threadIdx.x] = sample_key(stream_key(A.seed, (unsigned)l, A.pass_offset + pass), A.window_offset + win);
  }
  __syncthreads();

  Ctx X;
  X.blob = (const guint8*)(A.blob) + (long long)member * A.blob_stride;
  X.out_logits = A.out_logits;
  X.thr = A.thr[0];
  pblock<0, DROP>(X);
  X.thr = A.thr[1];
  pblock<1, DROP>(X);
  X.thr = A.thr[2];
  pblock<2, DROP>(X);
  X.thr = A.thr[3];
  pblock<3, DROP>(X);
  X.thr = A.thr[4];
  pblock<4, DROP>(X);
  X.thr = A.thr[5];
  pblock<5, DROP>(X);

  if (threadIdx.x < kNS) {
    const int sl = threadIdx.x;
    const long long gs = (long long)tile * kNS + sl;
    if (gs < samples) {
      const float logit = head[sl] + head[kNS + sl] + head[2 * kNS + sl] + head[3 * kNS + sl] +
                          reinterpret_cast<const gfloat*>(X.blob + kDenseOff)[C[6]];
      const int pass = (int)(gs / A.n_win), win = (int)(gs % A.n_win);
      A.out[((long long)member * A.n_pass + pass) * A.n_win + win] =
          A.out_logits ? logit : 1.0f / (1.0f + __expf(-logit));
    }
  }
}

}  // namespace pooled

int fused_pooled_lds_bytes() { return pooled::kLdsBytes; }

hipError_t launch_fused_pooled(const void* x, const uint8_t* blob, long long blob_stride, float* out, int n_win,
                               int n_pass, int n_member, unsigned window_offset, unsigned pass_offset,
                               unsigned long long seed, int dropout, int out_logits, const unsigned* thr,
                               hipStream_t stream) {
  pooled::Args A;
  A.x = reinterpret_cast<const __bf16*>(x);
  A.blob = blob;
  A.out = out;
  A.blob_stride = blob_stride;
  A.n_win = n_win;
  A.n_pass = n_pass;
  A.n_member = n_member;
  const long long samples = (long long)n_pass * n_win;
  const long long tiles = (samples + pooled::kNS - 1) / pooled::kNS;
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
    hipLaunchKernelGGL(pooled::fused_pooled_kernel<true>, dim3(A.total_items), dim3(pooled::kThreads),
                       pooled::kLdsBytes, stream, A);
  else
    hipLaunchKernelGGL(pooled::fused_pooled_kernel<false>, dim3(A.total_items), dim3(pooled::kThreads),
                       pooled::kLdsBytes, stream, A);
  return hipGetLastError();
}

}  // namespace apneauq
