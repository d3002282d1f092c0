// Fused whole-network inference of the Alarcón 1D-CNN on gfx950 (MI355X).
//
// Replaces the reference's hot loops
//   * MC Dropout:    np.stack([model(x, training=True) for _ in range(T)])   (uq_techniques.py:22)
//   * Deep Ensemble: np.stack([m.predict(x) for m in models])                (uq_techniques.py:29)
// with ONE launch that runs all six Conv1D->ReLU->BN->Dropout blocks, GAP, Dense and sigmoid for
// every (member, pass, window) sample.  Activations never leave LDS; weights stream from L2.
//
// Geometry (CDNA4-first):
//   * a workgroup (4 waves, 256 threads) owns a tile of 2 samples;  each sample occupies a 64-row
//     LDS slot: 60 valid time steps + 4 zero rows.  The zero rows double as the 'same' padding
//     (halo) of the next slot, so the implicit-GEMM conv needs no bounds checks;
//   * each block is an implicit GEMM  D^T[co][row] = W^T[co][k] * X^T[k][row],  k = tap*Cin + ci,
//     on v_mfma_f32_16x16x32_bf16.  Weights are the A operand, pre-packed on the host in exact
//     fragment order (one coalesced 1 KiB load per wave per fragment); activations are the B
//     operand, read from LDS with ds_read_b128 (row stride 544 B => conflict-free lane groups);
//   * the accumulator of a lane holds one time step x 4 consecutive channels, so the epilogue
//     (bias + ReLU + BN affine + counter-based dropout + bf16 pack) writes 8 B per tile per lane,
//     in place over the block input (the whole layer output lives in registers across the barrier);
//   * block 6's epilogue feeds GAP + Dense(96->1) + sigmoid directly (fp32), never touching LDS.
//   LDS per workgroup ~75 KiB -> 2 workgroups (8 waves) per CU.
#include "common.h"
#include "fused_blob.h"

namespace apneauq {
namespace fused {

constexpr int kL = 60;                         // valid time steps per window
constexpr int kSR = 64;                        // LDS rows per sample slot
constexpr int kSlots = 2;                      // samples per workgroup tile
constexpr int kR = kSR * kSlots;               // GEMM rows per tile
constexpr int kRT = kR / 16;                   // 16-row tiles per tile
constexpr int kHalo = 4;                       // >= max (k-1)/2
constexpr int kRows = kHalo + kR + kHalo;      // LDS rows incl. leading/trailing halo
constexpr int kCin = 4;                        // input channels (SaO2, PR, THOR RES, ABDO RES)
constexpr int kRS = 256 * 2 + 32;              // activation row stride in bytes (all layers)
constexpr int kX0RS = kCin * 2;                // input row stride in bytes
constexpr int kActBytes = kRows * kRS;
constexpr int kX0Bytes = kRows * kX0RS;
constexpr int kHeadOut = 2 * 6;                // head partials: [channel tile][slot] (block 6: 6 tiles)
constexpr int kHeadBytes = (kHeadOut + 2) * 4 + 8;
constexpr int kLdsBytes = kActBytes + kX0Bytes + kHeadBytes;
constexpr int kThreads = 256;
static_assert(kActBytes % 16 == 0 && kX0Bytes % 16 == 0, "LDS carve must stay 16-B aligned");


extern __shared__ __attribute__((aligned(16))) char smem[];  // dynamic LDS, carved below

struct Args {
  const __bf16* x;         // (n_win, 60, 4) bf16, channels-last
  const uint8_t* blob;     // (n_member, kBlobBytes) packed parameters
  float* out;              // (n_member, n_pass, n_win)
  long long blob_stride;   // bytes between members
  int n_win, n_pass, n_member;
  int tiles_per_member;
  int total_items;
  int chunk;               // items per workgroup (1)
  unsigned window_offset;  // global index of window 0 (dropout sample id => sharding invariance)
  unsigned pass_offset;
  unsigned long long seed;
  int dropout;             // apply dropout masks (MC Dropout)
  int out_logits;          // 1: write logits instead of probabilities
  unsigned thr[6];         // 16-bit drop thresholds per block
  float dscale[6];         // 1/(1-rate) per block
};

// Weight-prefetch depth: 1 k-step on every block.  Measured on MI355X (same box, 3 interleaved
// reps): depth 1 everywhere 64.1-64.3 ms for MCD T=50 x 16384 windows; depths (1,2,2,3,3,3)
// 65.4-66.5 ms.  The weight stream is bound by vector-memory issue (~2.6 MB of fragments per
// 2-sample tile), not latency.
constexpr int kPD = 1;

// One Conv1D(relu) -> BN -> Dropout block as an LDS-resident implicit GEMM.
//
// Wave tiling (WM x WN = 4 waves over rows x output channels):
//   * WM = 1: every wave covers all kRT row tiles (both samples) and NF channel tiles, so no
//     weight fragment is loaded twice per workgroup.  With HALF, channel tiles that do not split
//     4 ways (Cout = 224 -> 14 tiles) are shared by wave pairs: a pair owns 2*NF+1 tiles, each wave
//     NF full ones plus half (one sample's row tiles) of the middle one, so all waves issue the same
//     MFMA count;
//   * WM = 2: a wave covers one sample (kRT/2 row tiles) and NF channel tiles; the two wave rows
//     load the same weight fragments.  Used for Cout = 96 (6 tiles), where the pair split above
//     doubles the B-operand (LDS) reads per MFMA and measured 10-19 % slower per layer
//     (profiles/fused_ablation_r1.md, v8).

// Per-block context passed by value to the block functions.
struct BlockCtx {
  const guint8* blob;  // this member's packed parameters
  unsigned skey0, skey1;  // dropout sample keys of the two slots (0 if no dropout)
  unsigned thr;
  float dsc;
  int dropout;
  int out_logits;
};

template <int LAYER, int WM, int NF, bool HALF, int PD, bool HEAD, bool DROP>
__device__ __forceinline__ void block(const BlockCtx X) {
  char* act = smem;
  const char* x0 = smem + kActBytes;
  float* head = reinterpret_cast<float*>(smem + kActBytes + kX0Bytes);
  const guint8* blob = X.blob;
  constexpr int CIN = C[LAYER], COUT = C[LAYER + 1], K = KS[LAYER];
  constexpr bool FIRST = (LAYER == 0);
  constexpr int NSTEP = ksteps(LAYER);
  constexpr int NCT = COUT / 16;
  constexpr int NW = kThreads / kWave;
  constexpr int PAD = (K - 1) / 2;
  constexpr int NA = NF + (HALF ? 1 : 0);  // weight fragments per wave per k-step
  constexpr int HRT = kRT / 2;             // row tiles of one sample (= of the shared half tile)
  constexpr int NRT = kRT / WM;            // row tiles per wave
  static_assert(WM == 1 || (WM == 2 && !HALF), "wave rows");
  static_assert(HALF ? NCT == (NW / 2) * (2 * NF + 1) : NCT == (NW / WM) * NF, "wave tiling");
  static_assert(FIRST || CIN % 32 == 0, "k-step must stay inside one tap");
  static_assert(kRT == 8 && kSR == 64 && kSlots == 2, "row-tile -> (slot, t) mapping below");
  static_assert(!HEAD || 2 * NCT <= kHeadOut, "head partials fit in LDS");

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = lane & 15, h = lane >> 4;
  // channel tiles of this wave: NF full ones from ctf, the half tile cth (local rows r < HRT);
  // local row tile r (0 .. NRT-1) is tile (r + ho) mod 8 of the workgroup.  ho is a multiple of 4
  // (one sample = 4 row tiles), so t = 16 (r mod 4) + m is compile-time in r and only the sample
  // slot of local rows r < HRT (slot 1 iff ho != 0) depends on the wave.
  int ctf, cth = 0, ho = 0;
  if constexpr (HALF) {
    const int pair = wave >> 1, odd = wave & 1;
    ctf = pair * (2 * NF + 1) + (odd ? NF + 1 : 0);
    cth = pair * (2 * NF + 1) + NF;
    ho = odd * HRT;
  } else if constexpr (WM == 2) {
    ctf = (wave % (NW / 2)) * NF;
    ho = (wave / (NW / 2)) * HRT;
  } else {
    ctf = wave * NF;
  }
  const int rt_lo = ho, rt_hi = (ho + HRT) & (kRT - 1);

  const gbf16x8* wpf = reinterpret_cast<const gbf16x8*>(blob + woff(LAYER)) + ctf * 64 + lane;
  const gbf16x8* wph = reinterpret_cast<const gbf16x8*>(blob + woff(LAYER)) + cth * 64 + lane;

  f32x4 acc[NA][NRT];
#pragma unroll
  for (int c = 0; c < NA; ++c)
#pragma unroll
    for (int r = 0; r < NRT; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};

  const char* bb_lo = act + (kHalo + rt_lo * 16 + m - PAD) * kRS + 16 * h;
  const char* bb_hi = act + (kHalo + rt_hi * 16 + m - PAD) * kRS + 16 * h;
  const char* xb_lo = x0 + (kHalo + rt_lo * 16 + m - PAD) * kX0RS + 16 * h;
  const char* xb_hi = x0 + (kHalo + rt_hi * 16 + m - PAD) * kX0RS + 16 * h;
  // B fragment (activations, LDS) of local row tile r at k-step s
  auto load_b = [&](int s, int r) -> bf16x8 {
    if constexpr (FIRST) {
      // k = tap*4 + ci: 8 consecutive k = two consecutive rows x 4 channels (16 B, 8-B aligned)
      const char* base = (r < HRT ? xb_lo : xb_hi) + (r % HRT) * 16 * kX0RS + 64 * s;
      const bf16x4 lo = *reinterpret_cast<const bf16x4*>(base);
      const bf16x4 hi = *reinterpret_cast<const bf16x4*>(base + 8);
      return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    } else {
      // lane base + uniform step offset + compile-time row-tile offset (a ds_read immediate)
      constexpr int CB = CIN / 32;
      const int tap = s / CB, cb = s - tap * CB;
      const int soff = __builtin_amdgcn_readfirstlane(tap * kRS + cb * 64);
      return *reinterpret_cast<const bf16x8*>((r < HRT ? bb_lo : bb_hi) + soff + (r % HRT) * 16 * kRS);
    }
  };
  // A fragments (weights, global/L2) of k-step s: NF full tiles, then the half tile
  auto load_a = [&](int s, bf16x8 (&a)[NA]) {
#pragma unroll
    for (int c = 0; c < NA; ++c) {
      a[c] = (c < NF ? wpf + c * 64 : wph)[s * NCT * 64];
    }
  };
  // (B fragments are read just in time: a register ring over the (k-step, row-tile) sequence
  // measured 0.5-1 % slower on MI355X — the co-resident wave already hides LDS latency.)
  auto step = [&](int s, const bf16x8 (&a)[NA]) {
#pragma unroll
    for (int r = 0; r < NRT; ++r) {
      const bf16x8 b = load_b(s, r);
#pragma unroll
      for (int c = 0; c < NF; ++c) acc[c][r] = mfma16(a[c], b, acc[c][r]);
      if constexpr (HALF) {
        if (r < HRT) acc[NF][r] = mfma16(a[NF], b, acc[NF][r]);
      }
    }
  };

  // ---- K loop.  A ring of PD+1 weight-fragment stages: the fragments of step s+PD are in flight
  // under step s's MFMAs.  Every load is unconditional (indices are clamped)
  // so hipcc's vmcnt bookkeeping stays exact; sched_barrier keeps each prefetch ahead of the MFMAs.
  constexpr int NS = PD + 1;
  bf16x8 a[NS][NA];
#pragma unroll
  for (int j = 0; j < PD; ++j) load_a(j < NSTEP ? j : NSTEP - 1, a[j]);

  constexpr int NFULL = NSTEP / NS * NS;
#pragma unroll 1
  for (int s0 = 0; s0 < NFULL; s0 += NS) {
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int s = s0 + j;
      load_a(s + PD < NSTEP ? s + PD : NSTEP - 1, a[(j + PD) % NS]);
      __builtin_amdgcn_sched_barrier(0);
      step(s, a[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < NSTEP - NFULL; ++j) step(NFULL + j, a[j]);

  // ---- epilogue: bias + ReLU + BN(running) + dropout, then bf16 in place (or GAP head).
  // relu(acc + b) * s + t == clamp(fma(acc, s, b*s + t), lo, hi) (host-folded constants, one v_fma +
  // one v_med3 per element); MC Dropout reads a second copy pre-scaled by 1/(1-rate).  Rows t >= 60
  // of a slot are the next block's zero halo: they are simply never written (zeroed at kernel start).
  const gfloat* epi = reinterpret_cast<const gfloat*>(blob + eoff(LAYER)) + (DROP ? 4 * COUT : 0);
  const bool tail_lane = m >= kL - 48;  // lanes whose row in a 48..63 row tile is a halo row
  const bool swap = ho != 0;            // local rows 0..3 belong to sample slot 1
  const unsigned key_lo = swap ? X.skey1 : X.skey0, key_hi = swap ? X.skey0 : X.skey1;
  char* ob_lo = act + (kHalo + rt_lo * 16 + m) * kRS;
  char* ob_hi = act + (kHalo + rt_hi * 16 + m) * kRS;

  if constexpr (!HEAD) __syncthreads();  // every wave has finished reading this block's input

  // HEAD: this lane's share of sum_t sum_co w[co] * y[t][co], per (channel tile, slot).  Every
  // (tile, slot) sum is formed by exactly one wave and combined in tile order, so a sample's logit
  // does not depend on the slot it occupies (bitwise sharding invariance).
  float gap[NA][kSlots];
#pragma unroll
  for (int c = 0; c < NA; ++c) gap[c][0] = gap[c][1] = 0.f;
#pragma unroll
  for (int c = 0; c < NA; ++c) {
    const int co0 = (c < NF ? ctf + c : cth) * 16 + 4 * h;
    const f32x4 sc = *reinterpret_cast<const gf32x4*>(epi + co0);
    const f32x4 sh = *reinterpret_cast<const gf32x4*>(epi + COUT + co0);
    const f32x4 lo = *reinterpret_cast<const gf32x4*>(epi + 2 * COUT + co0);
    const f32x4 hi = *reinterpret_cast<const gf32x4*>(epi + 3 * COUT + co0);
    f32x4 dw;
    if constexpr (HEAD) dw = *reinterpret_cast<const gf32x4*>(reinterpret_cast<const gfloat*>(blob + kDenseOff) + co0);
    const int nr = (HALF && c == NF) ? HRT : NRT;  // compile-time after unrolling
#pragma unroll
    for (int r = 0; r < NRT; ++r) {
      if (r >= nr) break;
      const bool tail_tile = (r % 4) == 3;  // the row tile holding t = 48..63 of its sample
      const int t = (r % 4) * 16 + m;
      f32x4 v = acc[c][r];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_fmed3f(__builtin_fmaf(v[i], sc[i], sh[i]), lo[i], hi[i]);
      if constexpr (DROP) {
        const unsigned k = r < HRT ? key_lo : key_hi;
        const unsigned b01 = dropout_bits2(k, t, co0);
        const unsigned b23 = dropout_bits2(k, t, co0 + 2);
        v[0] = (b01 & 0xFFFFu) >= X.thr ? v[0] : 0.f;
        v[1] = (b01 >> 16) >= X.thr ? v[1] : 0.f;
        v[2] = (b23 & 0xFFFFu) >= X.thr ? v[2] : 0.f;
        v[3] = (b23 >> 16) >= X.thr ? v[3] : 0.f;
        // keep the selects in fp32: otherwise LLVM folds cvt(select(x, 0)) into select(cvt(x), 0),
        // converting every element separately and re-packing the pairs with v_perm
        asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
      }
      if constexpr (HEAD) {
        const float g = v[0] * dw[0] + v[1] * dw[1] + v[2] * dw[2] + v[3] * dw[3];
        gap[c][r < HRT ? 0 : 1] += (tail_tile && tail_lane) ? 0.f : g;  // [0]: local rows 0..3
      } else {
        bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
        bf16x4* dst = reinterpret_cast<bf16x4*>((r < HRT ? ob_lo : ob_hi) + (r % HRT) * 16 * kRS + co0 * 2);
        if (!(tail_tile && tail_lane)) *dst = o;
      }
    }
  }
  if constexpr (HEAD) {
#pragma unroll
    for (int c = 0; c < NA; ++c) {
      const int ct = c < NF ? ctf + c : cth;
#pragma unroll
      for (int j = 0; j < kSlots; ++j) {
        if (((HALF && c == NF) || WM == 2) && j == 1) break;  // only local rows 0..3
        const float g = wave_sum(gap[c][j]);
        if (lane == 0) head[2 * ct + (j ^ (swap ? 1 : 0))] = g;
      }
    }
    __syncthreads();
    if (threadIdx.x < kSlots) {
      const int sl = threadIdx.x;
      float s = 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) s += head[2 * ct + sl];
      const float logit = s * (1.0f / kL) + reinterpret_cast<const gfloat*>(blob + kDenseOff)[C[6]];
      head[kHeadOut + sl] = X.out_logits ? logit : 1.0f / (1.0f + __expf(-logit));
    }
  } else {
    __syncthreads();  // block output visible before the next block reads it
  }
}

template <bool DROP>
__global__ __launch_bounds__(kThreads, 2) void fused_forward_kernel(Args A) {
  char* act = smem;
  char* x0 = smem + kActBytes;
  float* head = reinterpret_cast<float*>(x0 + kX0Bytes);

  // zero the halo rows once: leading / trailing rows of the activation and input buffers and the
  // rows t = 60..63 of every slot (the epilogues never write them)
  for (int i = threadIdx.x; i < kHalo * kRS / 16; i += kThreads) {
    reinterpret_cast<f32x4*>(act)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sl = 0; sl < kSlots; ++sl)
      reinterpret_cast<f32x4*>(act + (kHalo + sl * kSR + kL) * kRS)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (threadIdx.x < kHalo * kX0RS / 16) {
    reinterpret_cast<f32x4*>(x0)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};
    reinterpret_cast<f32x4*>(x0 + (kHalo + kR) * kX0RS)[threadIdx.x] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // XCD-aware item assignment (T1): blocks sharing an XCD get a contiguous item range, so a
  // Deep-Ensemble member's weights stay in one XCD's L2.  Bijective for any grid size.
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rem = nwg % 8, xcd = bid % 8;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + bid / 8;
  const int samples = A.n_pass * A.n_win;
  // One tile per workgroup.  (A persistent tile loop lets LICM hoist every block's address math
  // out of the loop, which blows the 256-VGPR budget; one tile per launch slot keeps it at ~206.)
  {
    const int item = wg;
    APNEAUQ_DASSERT(item < A.total_items && (int)gridDim.x == A.total_items && blockDim.x == kThreads);
    const int member = item / A.tiles_per_member;
    APNEAUQ_DASSERT(member < A.n_member);
    const int tile = item - member * A.tiles_per_member;
    const guint8* blob = (const guint8*)(A.blob) + (long long)member * A.blob_stride;
    unsigned pass[kSlots], win[kSlots];
    bool valid[kSlots];
#pragma unroll
    for (int sl = 0; sl < kSlots; ++sl) {
      const int g = tile * kSlots + sl;
      valid[sl] = g < samples;
      const int gg = valid[sl] ? g : 0;
      pass[sl] = gg / A.n_win;
      win[sl] = gg - pass[sl] * A.n_win;
      APNEAUQ_DASSERT((int)pass[sl] < A.n_pass && (int)win[sl] < A.n_win);
    }
    // stage the two input windows (480 B each) + 4 zero rows per slot into x0
    if (threadIdx.x < kSlots * 32) {
      const int sl = threadIdx.x >> 5, ch = threadIdx.x & 31;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (ch < 30 && valid[sl])
        v = reinterpret_cast<const f32x4*>(A.x + (long long)win[sl] * (kL * kCin))[ch];
      reinterpret_cast<f32x4*>(x0 + (kHalo + sl * kSR) * kX0RS)[ch] = v;
    }
    __syncthreads();
    BlockCtx X;
    X.blob = blob;
    X.out_logits = A.out_logits;
    X.skey0 = X.skey1 = 0u;
#define FUSED_CTX(L)                                                                                   \
  X.thr = A.thr[L];                                                                                      \
  X.dsc = A.dscale[L];                                                                                   \
  if (DROP) {                                                                                            \
    X.skey0 = sample_key(stream_key(A.seed, L, A.pass_offset + pass[0]), A.window_offset + win[0]);      \
    X.skey1 = sample_key(stream_key(A.seed, L, A.pass_offset + pass[1]), A.window_offset + win[1]);      \
  }
    FUSED_CTX(0) block<0, 1, 2, false, kPD, false, DROP>(X);
    FUSED_CTX(1) block<1, 1, 3, false, kPD, false, DROP>(X);
    FUSED_CTX(2) block<2, 1, 3, true, kPD, false, DROP>(X);
    FUSED_CTX(3) block<3, 2, 3, false, kPD, false, DROP>(X);
    FUSED_CTX(4) block<4, 1, 4, false, kPD, false, DROP>(X);
    FUSED_CTX(5) block<5, 2, 3, false, kPD, true, DROP>(X);
#undef FUSED_CTX
    if (threadIdx.x < kSlots && valid[threadIdx.x]) {
      const int sl = threadIdx.x;
      A.out[((long long)member * A.n_pass + pass[sl]) * A.n_win + win[sl]] = head[kHeadOut + sl];
    }
  }
}

}  // namespace fused

// ------------------------------------------------------------------------------------ host side
int fused_blob_bytes() { return fused::kBlobBytes; }
int fused_lds_bytes() { return fused::kLdsBytes; }
void fused_layout(int* woffs, int* eoffs, int* dense_off) {
  for (int l = 0; l < 6; ++l) {
    woffs[l] = fused::woff(l);
    eoffs[l] = fused::eoff(l);
  }
  *dense_off = fused::kDenseOff;
}

hipError_t launch_fused_forward(const void* x, const uint8_t* blob, long long blob_stride, float* out,
                                int n_win, int n_pass, int n_member, unsigned window_offset,
                                unsigned pass_offset, unsigned long long seed, int dropout,
                                int out_logits, const unsigned* thr, const float* dscale, int grid,
                                hipStream_t stream) {
  fused::Args A;
  A.x = reinterpret_cast<const __bf16*>(x);
  A.blob = blob;
  A.out = out;
  A.blob_stride = blob_stride;
  A.n_win = n_win;
  A.n_pass = n_pass;
  A.n_member = n_member;
  A.tiles_per_member = (n_pass * n_win + fused::kSlots - 1) / fused::kSlots;
  A.total_items = A.tiles_per_member * n_member;
  (void)grid;
  if (A.total_items < 1) return hipSuccess;
  A.chunk = 1;
  A.window_offset = window_offset;
  A.pass_offset = pass_offset;
  A.seed = seed;
  A.dropout = dropout;
  A.out_logits = out_logits;
  for (int l = 0; l < 6; ++l) {  // thresholds come from ops/rng.py so host and device agree bit-exactly
    A.thr[l] = thr ? thr[l] : 0u;
    A.dscale[l] = dscale ? dscale[l] : 1.f;
  }
  if (dropout)
    hipLaunchKernelGGL(fused::fused_forward_kernel<true>, dim3(A.total_items), dim3(fused::kThreads), fused::kLdsBytes, stream, A);
  else
    hipLaunchKernelGGL(fused::fused_forward_kernel<false>, dim3(A.total_items), dim3(fused::kThreads), fused::kLdsBytes, stream, A);
  return hipGetLastError();
}

}  // namespace apneauq
