// Fused whole-network inference with multi-sample tiles (gfx950 / MI355X) for the short-sequence
// variants of the Alarcón 1D-CNN, both with the reference's filters / kernel sizes / parameter blob
// (fused_blob.h, ops/fused.py:pack_blob):
//
//   * PooledNet: MaxPool1D(2, valid) after blocks 1-5 (the pooling lines commented out in
//     /root/reference/models/train_deep_ensemble_cnns.py:36-66; the thesis' pooled `ensemble_cnn/`
//     models, evaluate_de_global.py:18).  Sequence lengths 60 -> 30 -> 15 -> 7 -> 3 -> 1, 8 samples
//     per workgroup;
//   * Single30Net: the north star's "30 s single-channel window" (input (30, 1), no
//     pooling), 4 samples per workgroup.
//
// One launch runs all six Conv1D -> ReLU -> BN(running) -> [MaxPool] -> [Dropout] blocks, GAP, Dense
// and sigmoid for every (member, pass, window) sample, like fused_forward.hip (the (60, 4) no-pool
// CNN, 2 samples per workgroup).  Design points:
//
//   * every weight fragment feeds 8 row tiles (blocks 1-2 of the pooled net are split into row
//     groups of 8 tiles to bound the accumulators);
//   * block l's input lives in LDS in per-sample slots of SIN rows: LIN valid rows, then zero rows
//     that double as the 'same' padding of the next slot (SIN >= LIN + PAD), so the implicit-GEMM
//     conv needs no bounds checks.  A computed GEMM row o is slot row (o / OPS) * SIN + o % OPS: all
//     slot rows where OPS == SIN, else only the prefix a block needs (pooled blocks 4 / 5 compute the
//     8 of 12 / 2 of 8 rows their pool keeps; the single-channel net computes 32 rows per 34-row
//     slot, so a sample is exactly two row tiles);
//   * taps that can never reach a valid input row are skipped: pooled block 5 (3 rows, k = 9) runs
//     taps 3..6 for its 2 kept rows, block 6 (1 row, k = 9) only the centre tap -- a dense 256 -> 96
//     layer, 9x fewer MFMAs than the padded conv;
//   * the pooled epilogue pools before the BN clamp (exact: the clamp is monotone) on lane pairs
//     (rows t, t^1 = lanes m, m^1, one DPP quad permute), each lane finishing two of the four
//     channels: fold, counter-based dropout keyed by the pooled step (ops/rng.py, the masks of
//     generic_conv.hip), bf16 store in place over the block input (barrier after the K loop; row
//     groups write only bytes no later group reads -- static_asserts below), plus the slot's zero rows;
//   * block 6 feeds Dense(96 -> 1) in fp32; partials are combined in a fixed order (bitwise sharding
//     invariance).
//   LDS per workgroup ~78 KiB -> 2 workgroups (8 waves) per CU.  Measured: profiles/pooled_fused_r3.md.
#include "common.h"
#include "fused_blob.h"

namespace apneauq {
namespace tiled {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

using fused::C;
using fused::eoff;
using fused::kDenseOff;
using fused::KS;
using fused::woff;

constexpr int kThreads = 256;  // 4 waves

// Per-net geometry tables.  RG / NG: row tiles per row group / row groups; WM: wave rows (4 / WM wave
// columns over the channel tiles); NF: full channel tiles per wave; HALF: Cout tiles that do not split
// 4 ways (224 -> 14, 96 -> 6 = 2 pairs x (2 NF + 1)) -- each wave pair shares its middle tile, one
// wave per half of the row tiles, so every weight fragment is requested once per workgroup and all
// waves issue the same MFMA count.  PD: k-steps of weight fragments in flight (depths 2-6 measured
// 0.8-1.9 % slower than 1 on the pooled net: weight latency does not bound these kernels).
struct PooledNet {
  static constexpr int NS = 8, L = 60, CIN0 = 4;
  static constexpr bool IM2COL = false;  // block 1 reads 2 rows x 4 channels per lane from x0
  static constexpr int X0ROWS = 64;      // x0 slot rows per sample
  static constexpr int LIN[6] = {60, 30, 15, 7, 3, 1};
  static constexpr int SIN[6] = {64, 32, 16, 12, 8, 1};
  static constexpr int OPS[6] = {64, 32, 16, 8, 2, 1};
  static constexpr int LOUT[6] = {30, 15, 7, 3, 1, 1};  // rows stored (after the pool)
  static constexpr bool POOL[6] = {true, true, true, true, true, false};
  static constexpr int T0[6] = {0, 0, 0, 0, 3, 4}, T1[6] = {7, 5, 3, 7, 7, 5};
  static constexpr int RG[6] = {8, 8, 8, 4, 1, 1}, NG[6] = {4, 2, 1, 1, 1, 1};
  static constexpr int WM[6] = {1, 1, 1, 1, 1, 1}, NF[6] = {2, 3, 3, 1, 4, 2};
  static constexpr bool HALF[6] = {false, false, true, true, false, false};
  static constexpr int PD[6] = {1, 1, 1, 1, 1, 1};
};

struct Single30Net {
  static constexpr int NS = 4, L = 30, CIN0 = 1;
  static constexpr bool IM2COL = true;  // x0 row t holds x[t-3 .. t+4]: the 8 k of lane group h = 0
  static constexpr int X0ROWS = 32;
  static constexpr int LIN[6] = {30, 30, 30, 30, 30, 30};
  static constexpr int SIN[6] = {32, 34, 34, 34, 34, 34};
  static constexpr int OPS[6] = {32, 32, 32, 32, 32, 32};
  static constexpr int LOUT[6] = {30, 30, 30, 30, 30, 30};
  static constexpr bool POOL[6] = {false, false, false, false, false, false};
  static constexpr int T0[6] = {0, 0, 0, 0, 0, 0}, T1[6] = {7, 5, 3, 7, 9, 9};
  static constexpr int RG[6] = {8, 8, 8, 8, 8, 8}, NG[6] = {1, 1, 1, 1, 1, 1};
  static constexpr int WM[6] = {1, 1, 1, 1, 1, 2}, NF[6] = {2, 3, 3, 1, 4, 3};
  static constexpr bool HALF[6] = {false, false, true, true, false, false};
  static constexpr int PD[6] = {1, 1, 1, 1, 1, 1};
};

__host__ __device__ constexpr int row_bytes(int c) { return 2 * c + 16; }  // +16 B: conflict-free rows
constexpr int kHB = 4 * row_bytes(256);  // leading zero rows (>= PAD rows of any block)

template <class N>
struct Lay {
  static constexpr int max_act() {
    int m = 0;
    for (int l = 1; l < 6; ++l) m = N::NS * N::SIN[l] * row_bytes(C[l]) > m ? N::NS * N::SIN[l] * row_bytes(C[l]) : m;
    return m;
  }
  static constexpr int kActBytes = kHB + max_act() + 4 * row_bytes(256);  // + trailing slack (discarded rows' taps)
  static constexpr int kX0Lead = N::IM2COL ? 0 : 4;
  static constexpr int kX0RowB = N::IM2COL ? 16 : N::CIN0 * 2;
  static constexpr int kX0Bytes = (kX0Lead + N::NS * N::X0ROWS + 8) * kX0RowB;
  static constexpr int kKeyBytes = 6 * N::NS * 4;
  static constexpr int kHeadBytes = 4 * N::NS * 4 + 16;
  static constexpr int kLdsBytes = kActBytes + kX0Bytes + kKeyBytes + kHeadBytes;
  static_assert(kActBytes % 16 == 0 && kX0Bytes % 16 == 0, "LDS carve must stay 16-B aligned");
  static_assert(2 * kLdsBytes <= 160 * 1024, "two workgroups per CU");
};

template <class N, int L>
struct Geo {
  static constexpr int CIN = C[L], COUT = C[L + 1], K = KS[L], PAD = (KS[L] - 1) / 2;
  static constexpr bool FIRST = L == 0, HEAD = L == 5, POOL = N::POOL[L];
  static constexpr int NCT = COUT / 16;
  static constexpr int CB = FIRST ? 1 : CIN / 32;
  static constexpr int S0 = FIRST ? 0 : N::T0[L] * CB, S1 = FIRST ? 1 : N::T1[L] * CB;  // k-steps run
  static constexpr int NWC = 4 / N::WM[L];             // wave columns
  static constexpr int NRW = N::RG[L] / N::WM[L];      // row tiles per wave per group
  static constexpr int SI = FIRST ? Lay<N>::kX0RowB : row_bytes(CIN);
  static constexpr int SOUT = L < 5 ? N::SIN[L + 1] : 1, SO = row_bytes(COUT);
  static constexpr int SPG = N::RG[L] * 16 / N::OPS[L];  // samples per row group
};

// compile-time checks of the slot geometry and the in-place hand-over
template <class N, int L>
constexpr bool geometry_ok() {
  using G = Geo<N, L>;
  const bool rowhead = N::OPS[5] == 1;
  if (L < 5 || !rowhead) {
    if (N::RG[L] * N::NG[L] * 16 != N::NS * N::OPS[L]) return false;  // row groups tile the computed rows
  } else if (N::RG[L] * 16 < N::NS) {
    return false;
  }
  if (N::OPS[L] > N::SIN[L] && !(L == 5 && rowhead)) return false;
  if (G::POOL && (N::OPS[L] % 2 != 0 || 2 * N::LOUT[L] > N::OPS[L] || N::SIN[L] % 2 != 0)) return false;
  if (L == 0 && N::OPS[L] != N::SIN[L]) return false;
  if (L == 0 && N::SIN[L] != N::X0ROWS) return false;
  if (N::HALF[L] ? (N::WM[L] != 1 || G::NCT != 2 * (2 * N::NF[L] + 1) || G::NRW % 2 != 0)
                 : (G::NWC * N::NF[L] < G::NCT || N::RG[L] % N::WM[L] != 0))
    return false;  // wave tiling covers the block
  if (L > 0 && N::LIN[L] > 1 && N::SIN[L] < N::LIN[L] + G::PAD) return false;  // zero rows = next slot's padding
  if (L < 5 && (N::LOUT[L] > G::SOUT || N::LOUT[L] > N::OPS[L])) return false;
  // row group g's output ends before group g+1's first input row (minus the padding)
  if (L >= 1 && N::NG[L] > 1 && G::SPG * G::SOUT * G::SO > (G::SPG * N::SIN[L] - G::PAD) * G::SI) return false;
  if (L >= 1 && N::NS * N::SIN[L] * G::SI > Lay<N>::max_act()) return false;
  // GAP head: a wave's rows are whole samples (two row tiles each)
  if (L == 5 && !rowhead && (N::OPS[5] % 16 != 0 || N::NG[5] != 1 || N::HALF[5] || G::NRW % (N::OPS[5] / 16) != 0))
    return false;
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
  const __bf16* x;         // (n_win, L, CIN0) bf16, channels-last
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
};

// 32-bit dropout decisions of channels (c0 .. c0+3) at step t applied to v (fp32 selects)
__device__ __forceinline__ void drop4(f32x4& v, unsigned key, unsigned t, unsigned c0, unsigned thr) {
  const unsigned b01 = dropout_bits2(key, t, c0), b23 = dropout_bits2(key, t, c0 + 2);
  v[0] = (b01 & 0xFFFFu) >= thr ? v[0] : 0.f;
  v[1] = (b01 >> 16) >= thr ? v[1] : 0.f;
  v[2] = (b23 & 0xFFFFu) >= thr ? v[2] : 0.f;
  v[3] = (b23 >> 16) >= thr ? v[3] : 0.f;
}

template <class N, int L, bool DROP>
__device__ __forceinline__ void block(const Ctx X) {
  using G = Geo<N, L>;
  using Y = Lay<N>;
  constexpr int NS = N::NS, OPSL = N::OPS[L], SINL = N::SIN[L];
  char* act = smem + kHB;
  const char* x0 = smem + Y::kActBytes + Y::kX0Lead * Y::kX0RowB;
  const unsigned* keys = reinterpret_cast<const unsigned*>(smem + Y::kActBytes + Y::kX0Bytes) + L * NS;
  float* head = reinterpret_cast<float*>(smem + Y::kActBytes + Y::kX0Bytes + Y::kKeyBytes);
  constexpr bool HF = N::HALF[L];
  constexpr bool ROWHEAD = G::HEAD && N::OPS[5] == 1;  // block 6 of a net whose last length is 1
  constexpr int NFL = N::NF[L], NRW = G::NRW, HRT = NRW / 2;
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
  auto ct_ok = [&](int c) { return HF || ctf + c < G::NCT; };  // pooled block 6: 6 tiles over 4 x 2 (wave-uniform)
  auto nrows = [&](int c) { return (HF && c == NFL) ? HRT : NRW; };  // compile-time after unrolling
  const gbf16x8* wp = reinterpret_cast<const gbf16x8*>(X.blob + woff(L)) + lane;
  int ctl[NFL_A];  // tiles past NCT load tile 0 and skip their MFMAs
#pragma unroll
  for (int c = 0; c < NFL_A; ++c) ctl[c] = ct_ok(c) ? ct_of(c) : 0;

  const gfloat* epi = reinterpret_cast<const gfloat*>(X.blob + eoff(L)) + (DROP ? 4 * G::COUT : 0);

#pragma unroll 1
  for (int g = 0; g < N::NG[L]; ++g) {
    const int rg0 = g * N::RG[L];
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
    // B-fragment bases: x0 (block 1: 2 rows x 4 channels per lane, or the lane group's im2col row),
    // else the slot row of the computed row minus the padding, + the lane's 16-B k slice
    const int lofs = !G::FIRST ? (m - G::PAD) * G::SI + 16 * h : N::IM2COL ? m * G::SI : (m + 2 * h - G::PAD) * G::SI;
    const char* bb_lo = (G::FIRST ? x0 : act) + (rg0 + rlo) * 16 * G::SI + lofs;
    const char* bb_hi = (G::FIRST ? x0 : act) + (rg0 + rhi) * 16 * G::SI + lofs;
    constexpr bool DENSE = OPSL == SINL || ROWHEAD;  // computed row = slot row (else one base per row tile)
    const char* bbr[NRW];
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      const int o = rt_of(r) * 16 + m;
      bbr[r] = act + ((o / OPSL) * SINL + o % OPSL - G::PAD) * G::SI + 16 * h;
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
        if constexpr (G::FIRST && !N::IM2COL) {
          // k = tap*4 + ci: the lane's 8 k are taps 2h, 2h+1 x 4 channels = two consecutive rows
          const bf16x4 lo = *reinterpret_cast<const bf16x4*>(bb);
          const bf16x4 hi = *reinterpret_cast<const bf16x4*>(bb + 8);
          b = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else {
          // (im2col: lane groups h >= 1 hold k >= 8, whose weights are zero: any finite row will do)
          b = *reinterpret_cast<const bf16x8*>(bb + soff);
        }
#pragma unroll
        for (int c = 0; c < NFL_A; ++c)
          if (ct_ok(c) && r < nrows(c)) acc[c][r] = mfma16(a[c], b, acc[c][r]);  // wave-uniform
      }
    };

    // K loop over k-steps [S0, S1): a ring of NSG register stages, the fragments of step s + PD in
    // flight under step s's MFMAs (loads past the end are clamped: vmcnt bookkeeping stays exact)
    constexpr int NSTEP = G::S1 - G::S0, PDL = N::PD[L] < NSTEP ? N::PD[L] : NSTEP, NSG = PDL + 1;
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
    constexpr int RPS = OPSL / 16 > 0 ? OPSL / 16 : 1;  // GAP head: row tiles per sample
    constexpr int NHP = (ROWHEAD || NRW < RPS) ? 1 : NRW / RPS;
    float hp[NHP];  // HEAD: logit partials (ROWHEAD: of sample m; GAP: per sample of the wave)
#pragma unroll
    for (int i = 0; i < NHP; ++i) hp[i] = 0.f;
    // dropout keys of this lane's rows, read from LDS once for all channel tiles
    unsigned keyr[NRW];
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      const int row = rt_of(r) * 16 + m;
      keyr[r] = DROP ? keys[ROWHEAD ? (m < NS ? m : 0) : row / OPSL] : 0u;
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
          if (tp < N::LOUT[L])
            *reinterpret_cast<bf16x2*>(act + (smp * G::SOUT + tp) * G::SO + ch * 2) = bf16x2{(__bf16)x0v, (__bf16)x1v};
        }
        continue;
      }
      f32x4 dw = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (G::HEAD) dw = *reinterpret_cast<const gf32x4*>(reinterpret_cast<const gfloat*>(X.blob + kDenseOff) + co0);
#pragma unroll
      for (int r = 0; r < NRW; ++r) {
        if (r >= nrows(c)) break;
        f32x4 v = acc[c][r];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_fmed3f(__builtin_fmaf(v[i], sc[i], sh[i]), lo[i], hi[i]);
        if constexpr (ROWHEAD) {  // one row per sample: rows m < NS are the samples
          if constexpr (DROP) drop4(v, keyr[r], 0u, (unsigned)co0, X.thr);
          hp[0] += m < NS ? v[0] * dw[0] + v[1] * dw[1] + v[2] * dw[2] + v[3] * dw[3] : 0.f;
        } else {
          const int row = rt_of(r) * 16 + m;
          const int smp = row / OPSL, t = row - smp * OPSL;
          if constexpr (DROP) drop4(v, keyr[r], (unsigned)t, (unsigned)co0, X.thr);
          if constexpr (G::HEAD) {  // GAP: this lane's share of sample (r / RPS) of the wave's rows
            const float gsum = v[0] * dw[0] + v[1] * dw[1] + v[2] * dw[2] + v[3] * dw[3];
            hp[r / RPS] += t < N::LOUT[L] ? gsum : 0.f;
          } else if (t < N::LOUT[L]) {
            *reinterpret_cast<bf16x4*>(act + (smp * G::SOUT + t) * G::SO + co0 * 2) =
                bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
          }
        }
      }
    }
    if constexpr (ROWHEAD) {
      float p = hp[0];
      p += __shfl_xor(p, 16, kWave);  // the 4 channel quarters of the tile (fixed order)
      p += __shfl_xor(p, 32, kWave);
      if (h == 0 && m < NS) head[wave * NS + m] = p;
    } else if constexpr (G::HEAD) {
      // per sample of the wave: sum over its rows (RPS tiles x 16 lanes) and the 4 channel quarters
#pragma unroll
      for (int i = 0; i < NHP; ++i) {
        float p = group16_sum(hp[i]);
        p += __shfl_xor(p, 16, kWave);
        p += __shfl_xor(p, 32, kWave);
        if (lane == 0) head[(rt_of(RPS * i) / RPS) * G::NWC + wc] = p;  // [sample][wave column]
      }
    } else {
      // the zero rows LOUT .. SOUT-1 of this group's output slots (the next block's padding)
      constexpr int ZR = G::SOUT - N::LOUT[L], CPR = G::COUT / 8;  // 16-B chunks per row
      for (int i = threadIdx.x; i < G::SPG * ZR * CPR; i += kThreads) {
        const int sr = i / CPR, chk = i - sr * CPR;
        const int smp = g * G::SPG + sr / ZR, tr = N::LOUT[L] + sr % ZR;
        *reinterpret_cast<f32x4*>(act + (smp * G::SOUT + tr) * G::SO + chk * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  __syncthreads();  // block output (or head partials) visible to every wave
}

template <class N, bool DROP>
__global__ __launch_bounds__(kThreads, 2) void fused_tiled_kernel(Args A) {
  using Y = Lay<N>;
  constexpr int NS = N::NS;
  char* x0 = smem + Y::kActBytes;
  unsigned* keys = reinterpret_cast<unsigned*>(smem + Y::kActBytes + Y::kX0Bytes);
  float* head = reinterpret_cast<float*>(smem + Y::kActBytes + Y::kX0Bytes + Y::kKeyBytes);
  // zero the leading / trailing rows every block may read as padding, once
  for (int i = threadIdx.x; i < kHB / 16; i += kThreads) {
    reinterpret_cast<f32x4*>(smem)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    reinterpret_cast<f32x4*>(smem + Y::kActBytes - 4 * row_bytes(256))[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (threadIdx.x < Y::kX0Lead * Y::kX0RowB / 16) reinterpret_cast<f32x4*>(x0)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 8 * Y::kX0RowB / 16)
    reinterpret_cast<f32x4*>(x0 + (Y::kX0Lead + NS * N::X0ROWS) * Y::kX0RowB)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};

  // XCD-aware item order (as fused_forward.hip): an XCD's workgroups take a contiguous item range
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rem = nwg % 8, xcd = bid % 8;
  const int item = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + bid / 8;
  APNEAUQ_DASSERT(item < A.total_items && blockDim.x == kThreads);
  const int member = item / A.tiles_per_member;
  const int tile = item - member * A.tiles_per_member;
  const long long samples = (long long)A.n_pass * A.n_win;

  if constexpr (N::IM2COL) {
    // x0 row (s, t) = x[s][t-3 .. t+4] (zero outside [0, L)), one thread per row
    static_assert(NS * N::X0ROWS <= kThreads, "one x0 row per thread");
    if (threadIdx.x < NS * N::X0ROWS) {
      const int sl = threadIdx.x / N::X0ROWS, t = threadIdx.x % N::X0ROWS;
      const long long gs = (long long)tile * NS + sl;
      bf16x8 v;
      const bool ok = gs < samples && t < N::L;
      const __bf16* xs = A.x + (long long)(ok ? gs % A.n_win : 0) * N::L;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ts = t + j - (KS[0] - 1) / 2;
        v[j] = (ok && ts >= 0 && ts < N::L) ? xs[ts] : (__bf16)0.f;
      }
      *reinterpret_cast<bf16x8*>(x0 + threadIdx.x * 16) = v;
    }
  } else {
    // NS input windows: L x CIN0 bf16 + zero rows per X0ROWS-row slot, one 16-B chunk per thread
    constexpr int CPS = N::X0ROWS * N::CIN0 * 2 / 16, CVAL = N::L * N::CIN0 * 2 / 16;  // chunks per slot / valid
    static_assert(NS * CPS <= kThreads && N::L * N::CIN0 * 2 % 16 == 0, "one x0 chunk per thread");
    if (threadIdx.x < NS * CPS) {
      const int sl = threadIdx.x / CPS, chk = threadIdx.x % CPS;
      const long long gs = (long long)tile * NS + sl;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (chk < CVAL && gs < samples) {
        const int win = (int)(gs % A.n_win);
        v = reinterpret_cast<const f32x4*>(A.x + (long long)win * (N::L * N::CIN0))[chk];
      }
      reinterpret_cast<f32x4*>(x0 + (Y::kX0Lead + sl * N::X0ROWS) * Y::kX0RowB)[chk] = v;
    }
  }
  // per-(block, sample) dropout keys: the same (seed, layer, pass, window) streams as every path
  if (DROP && threadIdx.x < 6 * NS) {
    const int l = threadIdx.x / NS, sl = threadIdx.x % NS;
    const long long gs = (long long)tile * NS + sl;
    const long long gg = gs < samples ? gs : 0;
    const unsigned pass = (unsigned)(gg / A.n_win), win = (unsigned)(gg % A.n_win);
    keys[threadIdx.x] = sample_key(stream_key(A.seed, (unsigned)l, A.pass_offset + pass), A.window_offset + win);
  }
  __syncthreads();

  Ctx X;
  X.blob = (const guint8*)(A.blob) + (long long)member * A.blob_stride;
  X.thr = A.thr[0];
  block<N, 0, DROP>(X);
  X.thr = A.thr[1];
  block<N, 1, DROP>(X);
  X.thr = A.thr[2];
  block<N, 2, DROP>(X);
  X.thr = A.thr[3];
  block<N, 3, DROP>(X);
  X.thr = A.thr[4];
  block<N, 4, DROP>(X);
  X.thr = A.thr[5];
  block<N, 5, DROP>(X);

  if (threadIdx.x < NS) {
    const int sl = threadIdx.x;
    const long long gs = (long long)tile * NS + sl;
    if (gs < samples) {
      float logit;
      if constexpr (N::OPS[5] == 1)  // [wave][sample], L = 1: GAP is the identity
        logit = head[sl] + head[NS + sl] + head[2 * NS + sl] + head[3 * NS + sl];
      else {  // [sample][wave column] sums over the L rows
        constexpr int NWC5 = 4 / N::WM[5];
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NWC5; ++w) s += head[NWC5 * sl + w];
        logit = s * (1.0f / N::L);
      }
      logit += reinterpret_cast<const gfloat*>(X.blob + kDenseOff)[C[6]];
      const int pass = (int)(gs / A.n_win), win = (int)(gs % A.n_win);
      A.out[((long long)member * A.n_pass + pass) * A.n_win + win] =
          A.out_logits ? logit : 1.0f / (1.0f + __expf(-logit));
    }
  }
}

template <class N>
hipError_t launch(const void* x, const uint8_t* blob, long long blob_stride, float* out, int n_win, int n_pass,
                  int n_member, unsigned window_offset, unsigned pass_offset, unsigned long long seed, int dropout,
                  int out_logits, const unsigned* thr, hipStream_t stream) {
  Args A;
  A.x = reinterpret_cast<const __bf16*>(x);
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
    hipLaunchKernelGGL(HIP_KERNEL_NAME(fused_tiled_kernel<N, true>), dim3(A.total_items), dim3(kThreads),
                       Lay<N>::kLdsBytes, stream, A);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(fused_tiled_kernel<N, false>), dim3(A.total_items), dim3(kThreads),
                       Lay<N>::kLdsBytes, stream, A);
  return hipGetLastError();
}

}  // namespace tiled

int fused_pooled_lds_bytes() { return tiled::Lay<tiled::PooledNet>::kLdsBytes; }

// net 0: the pooled (60, 4) CNN; net 1: the (30, 1) single-channel CNN.  (The (60, 4) no-pool CNN on
// this template -- 2 samples x 64 rows, results within 2e-7 of fused_forward.hip -- ran MCD T=50 x 16384
// in 71.2 ms against 66.2 ms there: profiles/pooled_fused_r3.md.)
hipError_t launch_fused_tiled(int net, const void* x, const uint8_t* blob, long long blob_stride, float* out,
                              int n_win, int n_pass, int n_member, unsigned window_offset, unsigned pass_offset,
                              unsigned long long seed, int dropout, int out_logits, const unsigned* thr,
                              hipStream_t stream) {
  if (net == 0)
    return tiled::launch<tiled::PooledNet>(x, blob, blob_stride, out, n_win, n_pass, n_member, window_offset,
                                           pass_offset, seed, dropout, out_logits, thr, stream);
  if (net == 1)
    return tiled::launch<tiled::Single30Net>(x, blob, blob_stride, out, n_win, n_pass, n_member, window_offset,
                                             pass_offset, seed, dropout, out_logits, thr, stream);
  return hipErrorInvalidValue;
}

}  // namespace apneauq
