// fp32-faithful layer-wise inference of the Alarcón 1D-CNN on gfx950 (MI355X): "fp16x3" MFMA.
//
// Replaces the reference's inference hot loops at fp32 precision (Keras runs fp32, no mixed-precision
// policy anywhere in the reference):
//   * MC Dropout  np.stack([model(x, training=True) for _ in range(T)])   (uq_techniques.py:22): BN on
//     per-pass batch statistics of the WHOLE window set, dropout on, moving averages updated;
//   * Deep Ensemble  np.stack([m.predict(x) for m in models])           (uq_techniques.py:29): BN on
//     moving statistics, no dropout;
//   * standard MC Dropout (BN on moving statistics, dropout on).
//
// Precision.  Every conv operand is split into two fp16 halves, v = hi + lo with hi = fp16(v) and
// lo = fp16(v - hi) (22 significant bits), and each product is formed by three v_mfma_f32_16x16x32_f16
// (hi*hi + hi*lo + lo*hi, fp32 accumulate): the dropped lo*lo term and the split residuals are ~2^-22
// relative, below fp32 GEMM rounding over K = 28..2304.  Weights are pre-scaled by an exact power of
// two per layer (host) so that both halves stay in the fp16 normal range; the epilogue undoes it.
// Block 1 (Cin = 4, 0.4 % of the FLOPs) runs in plain fp32 FMAs.  BN moments are fp32 per tile, fp64
// across tiles; the BN affine, dropout, GAP, Dense and sigmoid are fp32.
//
// Data flow (one launch per layer; the window set stays resident in HBM):
//   l1_kernel      R_1 = relu(conv(x) + b) fp32 (+ batch moments)           [G1][N][60][128]
//   aff_kernel     per-group BN affine of block l (batch moments or moving stats), pre-scaled by 1/(1-p)
//   layer_kernel   stage A_{l-1} = dropout(BN(R_{l-1})) as fp16 hi/lo into LDS (the mask of block l-1
//                  drawn from the counter hash here, by the loader waves), conv on MFMA,
//                  epilogue: bias + ReLU + moments, R_l stored fp32
//                  block 6: per-sample masked channel sums  S1 = sum_t keep*R,  S0 = sum_t keep
//   head_kernel    logit = b + (1/60) sum_c w_c (s_c S1_c + t_c S0_c)  (BN 6 + dropout 6 + GAP + Dense
//                  are linear per channel), p = sigmoid(logit)
//
// Layer kernel geometry (CDNA4-first):
//   * one persistent workgroup per CU (7-8 MFMA waves + 4 loader waves) walks a contiguous range of
//     tiles; a tile = S (2 or 4) samples of one group (MC-Dropout pass or ensemble member) = 64 S GEMM
//     rows, every sample a 64-row slot (60 time steps + 4 zero rows, the 'same' padding halo);
//   * the input channels stream through LDS in chunks of 32, double-buffered: while the MFMA waves
//     consume chunk c, the loader waves write chunk c+1 (BN affine + dropout + fp16 split of registers
//     loaded one chunk earlier) and issue the HBM loads of chunk c+2; one LDS-only barrier per chunk,
//     no vmcnt drain, and no HBM load ever queued in front of an MFMA wave's weight loads;
//   * LDS row = [hi 32 ch | lo 32 ch | 32 B pad] = 160 B = 10 16-B slots (stride = 2 mod 4 slots: the
//     ds_read_b128 lane groups of a 16x16x32 B fragment hit 16 distinct slots at any row offset);
//   * conv = implicit GEMM  D[co][row] = sum_{tap, ci} W[tap][ci][co] A[row + tap - pad][ci]: weights are
//     the A operand (host-packed fragments, one 1-KiB coalesced load per fragment, prefetched one k-step
//     ahead), activations the B operand (LDS).  Waves tile rows x output channels (WM x WN) per layer so
//     that each weight fragment is re-read by at most WM waves of the 256-row tile.
#include "common.h"
#include "x3_args.h"

namespace apneauq {
namespace x3 {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const f16x8 gf16x8;

// Staging waves of a layer without loader waves: the HBM loads of the next chunk are issued by MFMA
// waves 0..kStagers-1 only (one per SIMD), so that the partner wave keeps the matrix pipe busy while the
// stager's in-order vmcnt holds it at its next weight-fragment wait.
constexpr int kStagers = 4;
constexpr int kL = 60, kSR = 64, kHalo = 4;
// A chunk = CK input channels (32 or 64) of the tile's rows; LDS row: hi 2CK B | lo 2CK B | pad 32 B
// (row stride 2 mod 4 16-B slots for either CK).  Layers with few taps take 64-channel chunks: twice the
// k-steps per chunk barrier.
__host__ __device__ constexpr int row_bytes(int ck) { return 4 * ck + 32; }
// Range-safe fp16 split.  The staging splits a = s_c R + t_c (BN affine x dropout rescale, R >= 0) into
// fp16 hi + lo, which needs |a| < 65504 (hi finite) and |a| well above 2^-14 (lo normal).  Per SAMPLE
// (the rows of one window in one pass / member), |a| <= max_c |s_c| * max R + max_c |t_c| =: b, so the
// sample's activations are multiplied by the exact power of two 2^sa that puts b in [2^13, 2^14), and
// the accumulator rows of that sample by 2^-sa (a conv row sums over its own sample's rows only).  The
// prescale depends on the sample's own data and the (global) affine only: results are independent of
// sharding, chunking and grouping.  Under batch moments the bound comes free with the moments instead
// (max R_c <= sqrt(sum R_c^2), aff_kernel): one power of two per group, folded into the affine, and no
// per-sample tracking in the producer's epilogue (the moments are global, so this is invariant too).
__device__ __forceinline__ int sample_prescale(unsigned rmax_bits, const float* amax) {
  const float b = __builtin_fmaf(amax[0], __uint_as_float(rmax_bits), amax[1]);
  int e = 0;
  if (b > 0.f && b < INFINITY) frexpf(b, &e);  // b = m 2^e, m in [0.5, 1)
  return min(100, max(-100, 14 - e));
}

// per tile of S samples (S x 64 GEMM rows): LDS rows, chunk-buffer bytes, staged rows, 16-B staging units
__host__ __device__ constexpr int lds_rows(int S) { return kHalo + S * kSR + kHalo; }
__host__ __device__ constexpr int buf_bytes(int S, int ck) { return lds_rows(S) * row_bytes(ck); }
// + per-workgroup fp64 moment sums [2][COUT]
// two LDS chunk buffers, the workgroup's fp64 moment sums, and the epilogue down-scale factors of the
// two most recently staged tiles ([2][S] floats, written by the staging waves)
__host__ __device__ constexpr int lds_bytes(int S, int cout, int ck) {
  return 2 * buf_bytes(S, ck) + 2 * cout * 8 + 2 * S * 4;
}

// global-address-space load (keeps global_load_*, never flat_*)
template <typename T>
__device__ __forceinline__ T gld(const void* p) {
  return *(const __attribute__((address_space(1))) T*)(p);
}

// Thread index the optimiser cannot see through: per-iteration address math of the persistent tile
// loop is recomputed instead of being hoisted into ~100 loop-invariant VGPRs.
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

__device__ __forceinline__ f32x4 mfma(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// LDS hazard barrier: orders LDS traffic only (global loads in flight stay in flight)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// XCD-aware workgroup id (T1): blocks that share an XCD get a contiguous range.  Bijective.
__device__ __forceinline__ int xcd_wg() {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rem = nwg % 8, xcd = bid % 8;
  return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + bid / 8;
}

// Waves: WM x WN MFMA waves, plus LW loader waves (LW > 0) that do all the input staging: HBM loads of
// chunk c+2, BN affine + dropout + fp16 split of chunk c+1 into LDS.  vmcnt retires in order, so an MFMA
// wave that issued HBM loads would stall its next weight-fragment wait on them; loader waves take that
// latency instead, and wait at the chunk barrier without using issue slots.
// Register budget: the waves of WPC workgroups per CU over the 4 SIMDs, at least 2 per SIMD.
// A single workgroup of <= 4 waves per CU runs one wave per SIMD with the whole 512-register file
// (VGPR + AGPR): accumulators of twice the rows per weight fragment.
template <int NW, int WPC>
constexpr int waves_per_eu() { return NW * WPC > 8 ? (NW * WPC + 3) / 4 : NW * WPC <= 4 ? 1 : 2; }
// LW > 0: LW loader waves; LW <= 0: no loaders, MFMA waves 0 .. -LW-1 stage (LW = 0: kStagers of them)
constexpr int loaders(int lw) { return lw > 0 ? lw : 0; }
// PS: the per-sample prescale (moving statistics) is compiled in; without it (batch moments: per-group
// prescale folded into the affine) the kernel has the registers of its tracking for other uses.
template <int CIN, int COUT, int KS, int S, int WM, int WN, bool LAST, int LW, int CK, int WPC, bool PS>
__global__ __launch_bounds__((WM * WN + loaders(LW)) * 64, (waves_per_eu<WM * WN + loaders(LW), WPC>())) void layer_kernel(
    const LayerArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NWM = WM * WN, NW = NWM + loaders(LW), kThreads = NW * 64;
  constexpr int kCK = CK, kRowB = row_bytes(CK), NQ = CK / 32, kQ = CK / 4;  // 32-ch sub-chunks, quads / row
  constexpr int kS = S, kBufB = buf_bytes(S, CK), kValidRows = S * kL, kUnits = kValidRows * kQ;
  // staging waves: the LW loader waves, else MFMA waves 0..SW-1 (one per SIMD by default)
  constexpr int SW = LW > 0 ? LW : LW < 0 ? (-LW < NW ? -LW : NW) : (kStagers < NW ? kStagers : NW);
  constexpr int kSBase = LW > 0 ? NWM * 64 : 0;              // first staging thread
  constexpr int kST = SW * 64;                                // staging threads
  constexpr int kNU = (kUnits + kST - 1) / kST;              // 16-B staging units per staging thread
  static_assert(kST % kQ == 0 && (CK == 32 || CK == 64), "a staging thread keeps one channel quad");
  constexpr int NCH = CIN / kCK, NCTA = COUT / 16, NCT = NCTA / WN, NRT = 4 * S / WM, PAD = (KS - 1) / 2;
  constexpr int NSTEP = NCH * NQ * KS;  // k-steps (32 input channels x one tap) per tile
  // MFMA issue order: row tiles in groups of RG so that >= 4 accumulators rotate (dependent-issue
  // latency); B fragments double-buffered one group ahead when the accumulators leave room
  constexpr int RG = NCT >= 4                        ? 1
                     : (NCT >= 3 && NCT * NRT > 16)    ? 1
                     : NCT == 1                        ? 4
                                                       : 2;
  constexpr bool BDB = NCT * NRT <= 24 && RG < 4;
  static_assert(NRT % RG == 0, "row-tile groups");
  constexpr long long FRAG_STEP = (long long)NCTA * 128;  // f16x8 per (chunk, tap) k-step
  static_assert(CIN % kCK == 0 && COUT % 16 == 0, "channel tiling");
  static_assert(NCTA % WN == 0 && (4 * S) % WM == 0, "wave tiling");
  static_assert(NRT % 4 == 0, "whole 64-row sample slots per wave row (epilogue keys, block 6 sums)");
  double* st = reinterpret_cast<double*>(smem + 2 * kBufB);  // [2][COUT] per-workgroup moment sums
  // [tile & 1][sample of the tile]: wscale x 2^-sa, the epilogue's undo of both prescales
  float* wsc = reinterpret_cast<float*>(smem + 2 * kBufB + 2 * COUT * 8);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wm = (wave / WN) % WM;  // (loader waves: unused)
  const int ct0 = wn * NCT, rt0 = wm * NRT;
  const int m = lane & 15, h = lane >> 4;
  APNEAUQ_DASSERT(blockDim.x == kThreads);

  for (int i = tid; i < 2 * kBufB / 16; i += kThreads) reinterpret_cast<f32x4*>(smem)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = tid; i < 2 * COUT; i += kThreads) st[i] = 0.0;
  __syncthreads();

  const int wg = xcd_wg();
  const int tpg = (A.n_win + S - 1) / S;  // tiles per group at this kernel's tile size
  const int total_tiles = tpg * A.groups;
  const int t_begin = (int)((long long)wg * total_tiles / gridDim.x);
  const int t_end = (int)((long long)(wg + 1) * total_tiles / gridDim.x);
  if (t_begin >= t_end) return;  // workgroup-uniform
  const int slot = wg % kStatSlots;

  // ---- staging: staging thread i = tid - kSBase keeps the 16-B units (row ri = i/8 + kST/8 u,
  // channel quad q = i % 8) of every chunk
  const bool loader = LW > 0 && wave >= NWM;
  const bool stager = LW > 0 ? loader : wave < SW;
  // staging register set: the chunk's 16-B units + the BN affine (scale, shift) x 1/(1-p) of the
  // thread's 4 channels
  struct Stage {
    f32x4 v[kNU];
    f32x4 a, b;
  };
  Stage s0;
  // dropout keys of the current staging tile's S samples (the input's mask is drawn from the counter
  // hash of block l-1 here, at the consumer: the producer's epilogue then runs no hash at all, and the
  // loader waves' hashing overlaps the MFMA waves); recomputed when the staged tile changes
  // or the producer drew it and the input carries it in the sign bit (A.sign_in: per layer, whichever
  // side has the slack, profiles/x3_mask_side_r4.md)
  const bool hash_in = A.thr_in != 0u && !A.sign_in;
  const bool sign_in = A.thr_in != 0u && A.sign_in;
  const bool prescale = PS && A.smax_in != nullptr;
  int key_tile = -1;
  unsigned skeys[kS];
  unsigned skey_tile = 0u;  // the tile's stream key
  // prescale exponents sa of the staging tile's samples, one signed byte each (4 per register)
  static_assert(kS <= 8, "packed per-sample exponents");
  constexpr int kSP = (kS + 3) / 4;
  unsigned sa_pack[kSP];
  auto load_chunk = [&](int tile, int c, Stage& R) {
    const int tid = opaque_tid() - kSBase, q = tid % kQ;
    const int g = tile / tpg;
    const int w0 = (tile - g * tpg) * kS;
    const float* af = A.aff_in + (long long)g * A.aff_gstride + c * kCK + 4 * q;
    R.a = gld<f32x4>(af);
    R.b = gld<f32x4>(af + CIN);
#pragma unroll
    for (int u = 0; u < kNU; ++u) {
      const int ri = tid / kQ + (kST / kQ) * u;
      R.v[u] = f32x4{-0.f, -0.f, -0.f, -0.f};
      if (ri < kValidRows) {
        const int s = ri / kL, t = ri - s * kL, w = w0 + s;
        if (w < A.n_win) {
          const long long si = A.in_shared ? w : (long long)g * A.n_win + w;
          R.v[u] = gld<f32x4>(A.in + (si * kL + t) * CIN + c * kCK + 4 * q);
        }
      }
    }
  };
  auto store_chunk = [&](int tile, int c, char* buf, const Stage& R) {
    const int tid = opaque_tid() - kSBase, q = tid % kQ;
    const int g = tile / tpg;
    const int w0 = (tile - g * tpg) * kS;
    if (tile != key_tile) {  // workgroup-uniform
      const unsigned skey = stream_key(A.seed, A.layer - 1, A.pass_base + g);
      skey_tile = skey;
      const float* am = A.amax_in + (A.aff_gstride ? 2 * g : 0);
      float ws0 = A.wscale[A.p_gstride ? g : 0];
      if (A.gscale_in != nullptr) ws0 *= A.gscale_in[A.aff_gstride ? g : 0];
#pragma unroll
      for (int i = 0; i < kSP; ++i) sa_pack[i] = 0u;
#pragma unroll
      for (int s = 0; s < kS; ++s) {
        skeys[s] = sample_key(skey, A.window_offset + w0 + s);
        int sa = 0;
        if (prescale && w0 + s < A.n_win) {
          const long long si = A.in_shared ? w0 + s : (long long)g * A.n_win + w0 + s;
          sa = sample_prescale(A.smax_in[si], am);
          sa_pack[s >> 2] |= ((unsigned)sa & 0xFFu) << (8 * (s & 3));
        }
        // read by this tile's epilogue (after >= 1 barrier); the slot's previous tile (tile - 2) had its
        // epilogue before the barrier that precedes this store
        if (tid == s) wsc[(tile & 1) * kS + s] = ldexpf(ws0, -sa);
      }
      key_tile = tile;
    }
#pragma unroll
    for (int u = 0; u < kNU; ++u) {
      const int ri = tid / kQ + (kST / kQ) * u;
      if (ri >= kValidRows) continue;
      const int s = ri / kL, t = ri - s * kL, w = w0 + s;
      const f32x4 v = R.v[u];
      bool keep[4];
      if (hash_in) {
        // the sample's key: recomputed per staged unit (batch moments: block 2 -4 % over a select from
        // the tile's cached keys), or selected from the cache where the prescale needs its registers
        unsigned k;
        if constexpr (!PS) {
          k = sample_key(skey_tile, A.window_offset + w);
        } else {
          k = skeys[0];
#pragma unroll
          for (int j = 1; j < kS; ++j) k = s == j ? skeys[j] : k;
        }
        const unsigned b01 = dropout_bits2(k, t, c * kCK + 4 * q);
        const unsigned b23 = dropout_bits2(k, t, c * kCK + 4 * q + 2);
        keep[0] = (b01 & 0xFFFFu) >= A.thr_in;
        keep[1] = (b01 >> 16) >= A.thr_in;
        keep[2] = (b23 & 0xFFFFu) >= A.thr_in;
        keep[3] = (b23 >> 16) >= A.thr_in;
      } else if (sign_in) {
#pragma unroll
        for (int i = 0; i < 4; ++i) keep[i] = !__builtin_signbit(v[i]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) keep[i] = true;
      }
      const bool valid = w < A.n_win;
      // the sample's exponent: a signed byte of sa_pack (v_bfe_i32), applied exactly by v_ldexp_f32
      int sa = 0;
      if (prescale) {
        unsigned sp = sa_pack[0];
#pragma unroll
        for (int i = 1; i < kSP; ++i) sp = (s >> 2) == i ? sa_pack[i] : sp;
        sa = __builtin_amdgcn_sbfe((int)sp, 8 * (s & 3), 8);
      }
      float a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = (valid && keep[i]) ? ldexpf(__builtin_fmaf(v[i], R.a[i], R.b[i]), sa) : 0.f;
      // hi = fp16(a) two at a time (v_cvt_pk_f16_f32); lo = fp16(a - hi) in one mixed-precision FMA
      // per element, a - hi evaluated in fp32 from hi's f16 half (op_sel_hi on src0), written straight
      // into the pair's lo/hi half: 6 VALU per 4 elements instead of 16, bit-identical to the plain
      // convert/convert/subtract/convert (tools/probes/split/split_check.hip, 8.4 M pairs)
      uint2 hi, lo;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const unsigned u = __builtin_bit_cast(unsigned, (f16x2){(_Float16)a[2 * p], (_Float16)a[2 * p + 1]});
        unsigned l;
        asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(u), "v"(a[2 * p]));
        asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                     : "+v"(l)
                     : "v"(u), "v"(a[2 * p + 1]));
        (p ? hi.y : hi.x) = u;
        (p ? lo.y : lo.x) = l;
      }
      char* row = buf + (kHalo + s * kSR + t) * kRowB + 8 * q;
      *reinterpret_cast<uint2*>(row) = hi;
      *reinterpret_cast<uint2*>(row + 2 * kCK) = lo;
    }
  };

  // ---- accumulators and weight fragments
  f32x4 acc[NCT][NRT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) acc[ct][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto wbase = [&](int tile) -> const gf16x8* {
    const int g = tile / tpg;
    return (const gf16x8*)(A.wfrag) + (long long)g * A.w_gstride + ct0 * 128 + lane;
  };
  f16x8 ah[NCT], al[NCT];
  auto load_a = [&](const gf16x8* p, f16x8 (&xh)[NCT], f16x8 (&xl)[NCT]) {
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      xh[ct] = p[ct * 128];
      xl[ct] = p[ct * 128 + 64];
    }
  };

  // per-lane B-fragment base: row m of the wave's first row tile, 16-B slot h, tap offset -PAD
  const int bofs = ((rt0 * 16 + m + kHalo - PAD) * kRowB) + 16 * h;

  // conv over chunk c (k-steps c*KS .. c*KS+KS-1) from LDS buffer buf; wcur: this tile's fragments,
  // wnxt: the next tile's (prefetch across the tile boundary).  hook() runs after tap KS/2: the staging
  // waves write the NEXT chunk into the other LDS buffer there, so that VALU / LDS-write work overlaps
  // the partner wave's MFMAs instead of sitting between two barriers.
  auto compute_chunk = [&](int c, const char* buf, const gf16x8* wcur, const gf16x8* wnxt, auto&& hook) {
#pragma unroll
    for (int kk = 0; kk < NQ * KS; ++kk) {
      const int q2 = kk / KS, j = kk - q2 * KS;  // 32-channel sub-chunk, tap
      const char* bb = buf + bofs + q2 * 64;
      const int s = c * NQ * KS + kk;
      const gf16x8* np = (s + 1 < NSTEP) ? wcur + (long long)(s + 1) * FRAG_STEP : wnxt;
      // all NCT weight fragments resident, the next k-step's issued first (a full tap of MFMAs hides its
      // L2 latency); B fragments double-buffered one row tile ahead when registers allow.  The
      // sched_barriers pin that issue order (left alone, the scheduler sinks each load to its use).
      f16x8 nh[NCT], nl[NCT];
      load_a(np, nh, nl);
      __builtin_amdgcn_sched_barrier(0);
      // row tiles in groups of RG: the 3 x NCT x RG MFMAs of a group cycle through NCT x RG
      // accumulators, so a dependent MFMA follows its predecessor >= 4 issues later
      auto ldb = [&](int rt, f16x8& h_, f16x8& l_) {
        h_ = *reinterpret_cast<const f16x8*>(bb + (rt * 16 + j) * kRowB);
        l_ = *reinterpret_cast<const f16x8*>(bb + (rt * 16 + j) * kRowB + 2 * kCK);
      };
      f16x8 bh[RG], bl[RG];
#pragma unroll
      for (int r = 0; r < RG; ++r) ldb(r, bh[r], bl[r]);
#pragma unroll
      for (int rg = 0; rg < NRT; rg += RG) {
        f16x8 bh2[RG], bl2[RG];
#pragma unroll
        for (int r = 0; r < RG; ++r) {
          bh2[r] = bh[r];
          bl2[r] = bl[r];
          if (BDB && rg + RG < NRT) ldb(rg + RG + r, bh2[r], bl2[r]);
          if (!BDB) ldb(rg + r, bh[r], bl[r]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < RG; ++r)
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) acc[ct][rg + r] = mfma(ah[ct], bh[r], acc[ct][rg + r]);
#pragma unroll
        for (int r = 0; r < RG; ++r)
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) acc[ct][rg + r] = mfma(al[ct], bh[r], acc[ct][rg + r]);
#pragma unroll
        for (int r = 0; r < RG; ++r)
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) acc[ct][rg + r] = mfma(ah[ct], bl[r], acc[ct][rg + r]);
#pragma unroll
        for (int r = 0; r < RG; ++r) {
          bh[r] = bh2[r];
          bl[r] = bl2[r];
        }
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        ah[ct] = nh[ct];
        al[ct] = nl[ct];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kk == (NQ * KS) / 2) hook();
    }
  };

  // ---- epilogue of one tile: bias + ReLU, moments, block-l dropout, store / per-sample sums
  auto epilogue = [&](int tile) {
    const int lane = opaque_tid() & 63, m = lane & 15, h = lane >> 4;
    const int g = tile / tpg;
    const int w0 = (tile - g * tpg) * kS;
    // undo the weight prescale 2^sw and each sample's activation prescale 2^sa (exact powers of two;
    // the factors were put in LDS by the staging waves)
    float wsq[NRT / 4];
#pragma unroll
    for (int q = 0; q < NRT / 4; ++q) wsq[q] = wsc[(tile & 1) * kS + (rt0 >> 2) + q];
    const bool track = PS && !LAST && A.smax_out != nullptr;
    float mxs[NRT / 4];  // max of R_l per sample slot of the wave (range-safe split of the next block)
#pragma unroll
    for (int q = 0; q < NRT / 4; ++q) mxs[q] = 0.f;
    const float* bias = A.bias + (long long)g * A.p_gstride;
    // block 6 draws its output mask here (the masked per-sample sums); blocks 2..5 either store the plain
    // ReLU output (their consumer draws the mask while staging it) or, with A.sign_out, draw it here too
    const bool drop = (LAST || A.sign_out) && A.thr_out != 0u;
    // a wave's row tiles cover whole 64-row sample slots (NRT % 4 == 0): the sample of row tile rt is
    // wave-uniform, so its dropout key is computed once per sample (scalar ALU), not per (ct, rt, lane)
    unsigned skeys[NRT / 4];
    if (drop) {
      const unsigned skey = stream_key(A.seed, A.layer, A.pass_base + g);
#pragma unroll
      for (int q = 0; q < NRT / 4; ++q)
        skeys[q] = sample_key(skey, A.window_offset + w0 + (rt0 >> 2) + q);
    }
    // channel-tile outer: only one tile's 4 channels of sums are live at a time
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int co0 = (ct0 + ct) * 16 + 4 * h;
      const f32x4 b4 = gld<f32x4>(bias + co0);
      f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1, k1 = s1, k0 = s1;
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt) {
        const int s = (rt0 + rt) >> 2, t = (((rt0 + rt) & 3) << 4) + m, w = w0 + s;
        const bool valid = t < kL && w < A.n_win;
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = fmaxf(__builtin_fmaf(acc[ct][rt][e], wsq[rt >> 2], b4[e]), 0.f);
        acc[ct][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
        bool keep[4] = {true, true, true, true};
        if (drop) {
          const unsigned key = skeys[rt >> 2];
          const unsigned b01 = dropout_bits2(key, t, co0), b23 = dropout_bits2(key, t, co0 + 2);
          keep[0] = (b01 & 0xFFFFu) >= A.thr_out;
          keep[1] = (b01 >> 16) >= A.thr_out;
          keep[2] = (b23 & 0xFFFFu) >= A.thr_out;
          keep[3] = (b23 >> 16) >= A.thr_out;
        }
        if (valid) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s1[e] += r[e];
            s2[e] = __builtin_fmaf(r[e], r[e], s2[e]);
            if (!LAST) mxs[rt >> 2] = fmaxf(mxs[rt >> 2], r[e]);
            if constexpr (LAST) {
              k1[e] += keep[e] ? r[e] : 0.f;
              k0[e] += keep[e] ? 1.f : 0.f;
            }
          }
          if constexpr (!LAST) {
            const long long sample = (long long)g * A.n_win + w;
            f32x4 o = r;
            if (drop) {  // the mask travels in the sign bit (-0 for a dropped zero)
#pragma unroll
              for (int e = 0; e < 4; ++e) o[e] = keep[e] ? r[e] : __builtin_copysignf(r[e], -1.f);
            }
            *reinterpret_cast<f32x4*>(A.out + (sample * kL + t) * COUT + co0) = o;
          }
        }
        if constexpr (LAST) {
          if ((rt & 3) == 3) {  // the 4 row tiles of sample slot (rt0 + rt) / 4 are complete
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              k1[e] = group16_sum(k1[e]);
              k0[e] = group16_sum(k0[e]);
            }
            const int wl = w0 + (rt0 + rt) / 4;
            if (m == 0 && wl < A.n_win) {
              float* o = A.out + ((long long)g * A.n_win + wl) * (2 * COUT);
              *reinterpret_cast<f32x4*>(o + co0) = k1;
              *reinterpret_cast<f32x4*>(o + COUT + co0) = k0;
            }
            k1 = f32x4{0.f, 0.f, 0.f, 0.f};
            k0 = k1;
          }
        }
      }
      // reduce over the 16 rows of each lane group (lanes sharing h hold the same 4 channels)
      if (A.stats != nullptr) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = group16_sum(s1[e]), b = group16_sum(s2[e]);
          if (m == 0) {
            atomicAdd(&st[co0 + e], (double)a);
            atomicAdd(&st[COUT + co0 + e], (double)b);
          }
        }
      }
    }
    if (track) {  // per-sample maxima of R_l (R_l >= 0: fp32 bit order = value order; max is order-free)
#pragma unroll
      for (int q = 0; q < NRT / 4; ++q) {
        const float mq = wave_max(mxs[q]);
        const int w = w0 + (rt0 >> 2) + q;
        if (lane == 0 && w < A.n_win) atomicMax(A.smax_out + (long long)g * A.n_win + w, __float_as_uint(mq));
      }
    }
  };

  auto flush_stats = [&](int g) {
    __syncthreads();
    if (A.stats != nullptr) {
      double* dst = A.stats + ((long long)g * kStatSlots + slot) * 2 * COUT;
      for (int i = tid; i < 2 * COUT; i += kThreads) {
        atomicAdd(dst + i, st[i]);
        st[i] = 0.0;
      }
    }
    __syncthreads();
  };

  // ---- persistent loop over the flattened (tile, chunk) sequence, software-pipelined:
  //   iteration it: compute chunk it from buf[it & 1]; staging waves write chunk it+1 (loaded into
  //   registers one iteration earlier) into buf[(it+1) & 1] mid-way; barrier; issue the loads of it+2.
  // buf[(it+1) & 1] was last read by compute(it-1), which every wave finished before barrier(it-1).
  const int total = (t_end - t_begin) * NCH;
  auto chunk_tile = [&](int it) { return t_begin + it / NCH; };
  int g_cur = t_begin / tpg;
  if constexpr (LW > 0) {
    // Loader and MFMA waves run the same barrier sequence: one LDS barrier before the first chunk and
    // after every chunk, and the two of flush_stats at every group change and at the end.
    if (loader) {
      // chunk it+2's HBM loads are issued right after barrier(it) and land in registers during
      // compute(it+1) (two chunks of loads in flight measured no faster: profiles/x3_epilogue_ab_r3.md)
      if (stager) {
        load_chunk(t_begin, 0, s0);
        store_chunk(t_begin, 0, smem, s0);
      }
      lds_barrier();
      if (stager && total > 1) load_chunk(chunk_tile(1), 1 % NCH, s0);
#pragma unroll 1
      for (int it = 0; it < total; ++it) {
        const int tile = chunk_tile(it), c = it - (tile - t_begin) * NCH;
        if (c == 0) {
          const int g = tile / tpg;
          if (g != g_cur) {
            flush_stats(g_cur);
            g_cur = g;
          }
        }
        // chunk it+1 into the buffer compute(it-1) read (every wave passed the barrier after it)
        if (stager && it + 1 < total) store_chunk(chunk_tile(it + 1), (it + 1) % NCH, smem + ((it + 1) & 1) * kBufB, s0);
        lds_barrier();
        if (stager && it + 2 < total) load_chunk(chunk_tile(it + 2), (it + 2) % NCH, s0);
      }
      flush_stats(g_cur);
      return;
    }
    lds_barrier();
    load_a(wbase(t_begin), ah, al);
#pragma unroll 1
    for (int it = 0; it < total; ++it) {
      const int tile = chunk_tile(it), c = it - (tile - t_begin) * NCH;
      if (c == 0) {
        const int g = tile / tpg;
        if (g != g_cur) {
          flush_stats(g_cur);
          g_cur = g;
        }
      }
      const gf16x8* wcur = wbase(tile);
      const gf16x8* wnxt = wbase(tile + 1 < t_end ? tile + 1 : tile);
      compute_chunk(c, smem + (it & 1) * kBufB, wcur, wnxt, []() {});
      if (c == NCH - 1) epilogue(tile);
      lds_barrier();
    }
    flush_stats(g_cur);
    return;
  }
  if (stager) {
    load_chunk(t_begin, 0, s0);
    store_chunk(t_begin, 0, smem, s0);
  }
  lds_barrier();
  if (stager && total > 1) load_chunk(chunk_tile(1), 1 % NCH, s0);
  load_a(wbase(t_begin), ah, al);
#pragma unroll 1
  for (int it = 0; it < total; ++it) {
    const int tile = chunk_tile(it), c = it - (tile - t_begin) * NCH;
    if (c == 0) {
      const int g = tile / tpg;
      if (g != g_cur) {
        flush_stats(g_cur);
        g_cur = g;
      }
    }
    const gf16x8* wcur = wbase(tile);
    const gf16x8* wnxt = wbase(tile + 1 < t_end ? tile + 1 : tile);
    char* buf = smem + (it & 1) * kBufB;
    char* nbuf = smem + ((it + 1) & 1) * kBufB;
    compute_chunk(c, buf, wcur, wnxt, [&]() {
      if (stager && it + 1 < total) store_chunk(chunk_tile(it + 1), (it + 1) % NCH, nbuf, s0);
    });
    if (c == NCH - 1) epilogue(tile);
    lds_barrier();
    if (stager && it + 2 < total) load_chunk(chunk_tile(it + 2), (it + 2) % NCH, s0);
  }
  flush_stats(g_cur);
}

// ------------------------------------------------------------------------------- block 1 (fp32)
// R_1[g][w][t][c] = relu(b[c] + sum_{j, ci} x[w][t + j - 3][ci] W[j][ci][c]) in fp32 FMAs, 8 windows
// per 256-thread block (thread = one output channel x one half of the time steps), + batch moments.
__global__ __launch_bounds__(256) void l1_kernel(const L1Args A) {
  __shared__ float xs[kL1Win][kL + 6][4];
  __shared__ float red[2][2][128];
  __shared__ unsigned wmax[kL1Win];  // per-window max of R_1 (fp32 bits)
  const int g = blockIdx.x / A.blocks_per_group;
  const int w0 = (blockIdx.x - g * A.blocks_per_group) * kL1Win;
  const int tid = threadIdx.x, c = tid & 127, half = tid >> 7;
  for (int i = tid; i < kL1Win * (kL + 6) * 4; i += 256) {
    const int s = i / ((kL + 6) * 4), r = (i / 4) % (kL + 6), ci = i & 3;
    const int t = r - 3, w = w0 + s;
    xs[s][r][ci] = (t >= 0 && t < kL && w < A.n_win) ? A.x[((long long)w * kL + t) * 4 + ci] : 0.f;
  }
  float wr[7][4];
#pragma unroll
  for (int j = 0; j < 7; ++j)
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) wr[j][ci] = A.w[(((long long)g * 7 + j) * 4 + ci) * 128 + c];
  const float bc = A.b[g * 128 + c];
  if (tid < kL1Win) wmax[tid] = 0u;
  __syncthreads();
  float s1 = 0.f, s2 = 0.f;
  for (int s = 0; s < kL1Win; ++s) {
    const int w = w0 + s;
    if (w >= A.n_win) break;
    float* o = A.out + (((long long)g * A.n_win + w) * kL) * 128 + c;
    float mx = 0.f;
    for (int t = half * 30; t < half * 30 + 30; ++t) {
      float v = bc;
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) v = __builtin_fmaf(xs[s][t + j][ci], wr[j][ci], v);
      v = fmaxf(v, 0.f);
      o[t * 128] = v;
      s1 += v;
      s2 = __builtin_fmaf(v, v, s2);
      mx = fmaxf(mx, v);
    }
    if (A.smax != nullptr) {
      mx = wave_max(mx);
      if ((tid & 63) == 0) atomicMax(&wmax[s], __float_as_uint(mx));
    }
  }
  if (A.stats != nullptr || A.smax != nullptr) {  // block-uniform
    red[half][0][c] = s1;
    red[half][1][c] = s2;
    __syncthreads();
    if (A.stats != nullptr && tid < 128) {
      double* dst = A.stats + ((long long)g * kStatSlots + (blockIdx.x % kStatSlots)) * 2 * 128;
      atomicAdd(dst + c, (double)red[0][0][c] + (double)red[1][0][c]);
      atomicAdd(dst + 128 + c, (double)red[0][1][c] + (double)red[1][1][c]);
    }
    // every window belongs to this block alone: a plain store of its max
    if (A.smax != nullptr && tid < kL1Win && w0 + tid < A.n_win) A.smax[(long long)g * A.n_win + w0 + tid] = wmax[tid];
  }
}

// ---------------------------------------------------------------------- BN affine (+ moving update)
// aff[g][0][c] = gamma * rstd * dsc, aff[g][1][c] = (beta - mean * gamma * rstd) * dsc, where (mean, var)
// are the biased batch moments of group g (stats != nullptr) or the moving statistics.  With
// update != 0 the Keras moving averages are updated once per group in group order (one MC-Dropout
// pass after the other, the side effect of model(x, training=True)).  amax[g] = (max_c |aff scale|,
// max_c |aff shift|): the consumer's range-safe split (sample_prescale).
// Blocks 0..groups-1: group g's affine (independent); block `groups` (batch moments with the moving
// update only): the moving averages, groups in order (the recurrence is sequential; the affines use
// the batch moments, so the two never touch the same data).  One block looping over every group's
// affine and its two block reductions took ~25 us per call.
__device__ __forceinline__ void aff_moments(const AffArgs& A, int g, int c, float& mean, float& var) {
  const double* p = A.stats + (long long)g * kStatSlots * 2 * A.C + c;
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int s = 0; s < kStatSlots; ++s) {
    a += p[s * 2 * A.C];
    b += p[s * 2 * A.C + A.C];
  }
  const double mu = a * A.inv_count;
  mean = (float)mu;
  var = (float)fmax(b * A.inv_count - mu * mu, 0.0);
}

__global__ __launch_bounds__(256) void aff_kernel(const AffArgs A) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x;
  if ((int)blockIdx.x == A.groups) {  // the moving-average side effect (launched with stats + update)
    for (int c = tid; c < A.C; c += 256)
      for (int g = 0; g < A.groups; ++g) {
        const long long po = (long long)g * A.p_gstride + c;
        float mean, var;
        aff_moments(A, g, c, mean, var);
        for (int r = 0; r < A.repeat; ++r) {
          A.mmean[po] = A.mmean[po] * A.momentum + mean * (1.f - A.momentum);
          A.mvar[po] = A.mvar[po] * A.momentum + var * (1.f - A.momentum);
        }
      }
    return;
  }
  {
    const int g = blockIdx.x;
    float ms = 0.f, mt = 0.f;
    for (int c = tid; c < A.C; c += 256) {
      const long long po = (long long)g * A.p_gstride + c;
      float mean, var;
      if (A.stats != nullptr && !A.running) {
        aff_moments(A, g, c, mean, var);
      } else {
        mean = A.mmean[po];
        var = A.mvar[po];
      }
      const float sc = A.gamma[po] / sqrtf(var + A.eps);
      const float s_ = sc * A.dsc, t_ = (A.beta[po] - mean * sc) * A.dsc;
      A.aff[((long long)g * 2) * A.C + c] = s_;
      A.aff[((long long)g * 2 + 1) * A.C + c] = t_;
      if (A.gscale != nullptr) {
        // batch moments: R >= 0 gives max R_c <= sqrt(sum R_c^2) over the group's rows (of all ranks), so
        // b = max_c |s_c| sqrt(sum R_c^2) + |t_c| bounds every staged |a| of the group (with A.running the
        // affine is the moving statistics' and the sums of squares serve only this bound)
        const double* p = A.stats + (long long)g * kStatSlots * 2 * A.C + A.C + c;
        double q = 0.0;
        for (int s = 0; s < kStatSlots; ++s) q += p[s * 2 * A.C];
        ms = fmaxf(ms, __builtin_fmaf(fabsf(s_), (float)sqrt(fmax(q, 0.0)) * 1.0001f, fabsf(t_)));
      } else {
        ms = fmaxf(ms, fabsf(s_));
        mt = fmaxf(mt, fabsf(t_));
      }
    }
    if (A.gscale != nullptr) {
      // per-group power of two 2^sa putting the bound in [2^13, 2^14), folded into the affine; the layer
      // kernel multiplies its accumulators by gscale = 2^-sa
      ms = wave_max(ms);
      if ((tid & 63) == 0) red[0][tid >> 6] = ms;
      __syncthreads();
      const float bnd = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
      int e = 0;
      if (bnd > 0.f && bnd < INFINITY) frexpf(bnd, &e);
      const int sa = min(100, max(-100, 14 - e));
      for (int c = tid; c < A.C; c += 256) {
        float* af = A.aff + (long long)g * 2 * A.C + c;
        af[0] = ldexpf(af[0], sa);
        af[A.C] = ldexpf(af[A.C], sa);
      }
      if (tid == 0) A.gscale[g] = ldexpf(1.f, -sa);
      return;
    }
    if (A.amax == nullptr) return;  // kernel-uniform
    ms = wave_max(ms);
    mt = wave_max(mt);
    if ((tid & 63) == 0) {
      red[0][tid >> 6] = ms;
      red[1][tid >> 6] = mt;
    }
    __syncthreads();
    if (tid == 0) {
      A.amax[2 * g] = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
      A.amax[2 * g + 1] = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
    }
  }
}

// --------------------------------------------------------------------------------------- head
// p[g][w] = sigmoid(b + (1/60) sum_c w_c (aff_s[c] S1[c] + aff_t[c] S0[c])): one wave per sample.
__global__ __launch_bounds__(256) void head_kernel(const HeadArgs A) {
  const int lane = threadIdx.x & 63;
  const long long sidx = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sidx >= A.samples) return;
  const int g = (int)(sidx / A.n_win);
  const float* s = A.sums + sidx * 2 * A.C;
  const float* af = A.aff + (long long)g * A.aff_gstride;
  const float* dw = A.dw + (long long)g * A.p_gstride;
  float v = 0.f;
  for (int c = lane; c < A.C; c += 64) v += dw[c] * __builtin_fmaf(af[c], s[c], af[A.C + c] * s[A.C + c]);
  v = wave_sum(v);
  if (lane == 0) {
    const float logit = v * (1.0f / kL) + A.db[A.p_gstride ? g : 0];
    A.out[sidx] = A.out_logits ? logit : 1.0f / (1.0f + expf(-logit));
  }
}

// ------------------------------------------------------------------------------- launch helpers
template <int CIN, int COUT, int KS, int S, int WM, int WN, bool LAST, int LW, int CK, int WPC, bool PS>
hipError_t launch_layer(const LayerArgs& A, int grid, hipStream_t stream) {
  constexpr int lds = lds_bytes(S, COUT, CK);
  static_assert(WPC * lds <= 160 * 1024, "LDS of the workgroups sharing a CU");
  auto k = layer_kernel<CIN, COUT, KS, S, WM, WN, LAST, LW, CK, WPC, PS>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3((WM * WN + loaders(LW)) * 64), lds, stream, A);
  return hipGetLastError();
}

}  // namespace x3

// Layer table of the reference architecture (cnn_baseline_train.py:59-86), blocks 2..6:
//   <Cin, Cout, k, samples per tile, wave rows WM, wave channel groups WN, block 6, loader waves LW
//    (<= 0: no loaders, -LW MFMA waves stage) with / LWB without the per-sample prescale,
//    input channels per staged chunk CK, persistent workgroups per CU WPC>
// Each MFMA wave owns (4 S / WM) 16-row tiles x (Cout / 16 / WN) 16-channel tiles; the 64-accumulator-tile
// layers (Cout 224 / 256) run 2-sample tiles so that the next k-step's weight fragments and the B
// double-buffer fit beside the accumulators without spilling.  Loader waves (ablation table in
// profiles/x3_loader_waves.md) on every layer but block 2, whose 96-accumulator tile needs the 256-VGPR
// budget of 8 waves (loaders at 2-sample tiles: slower; at 4: 99 VGPRs spilled); its staging runs on
// MFMA waves 0..3, or on all 8 where the per-sample prescale's registers would otherwise spill.  64-channel chunks for
// blocks 3 and 6 (block 2 would spill; Cin 224 / 96 are not multiples of 64).  The Cout-96 blocks 4 and
// 6 run 4 MFMA waves of 24 accumulator tiles (WM 2 x WN 2) rather than 8 of 12: each weight fragment
// is re-read by 2 wave rows instead of 4 (their texture path was the busy one), -1.2 % MCD.
// Measurements: profiles/x3_epilogue_ab_r3.md, profiles/x3_mask_side_r4.md.
// A/B builds may substitute another table (APNEAUQ_X3_TABLE=<path.h> in csrc/build.py, tools/probes/x3_tables/):
// every entry is a complete, correct configuration, only the speed differs.
#ifdef APNEAUQ_X3_TABLE
#include APNEAUQ_X3_TABLE
#else
#define APNEAUQ_X3_LAYERS(X)                     \
  X(1, 128, 192, 5, 4, 2, 4, false, -8, 0, 32, 1) \
  X(2, 192, 224, 3, 2, 1, 7, false, 4, 4, 64, 1) \
  X(3, 224, 96, 7, 4, 2, 2, false, 4, 4, 32, 1)  \
  X(4, 96, 256, 9, 2, 1, 8, false, 4, 4, 32, 1)  \
  X(5, 256, 96, 9, 4, 2, 2, true, 4, 4, 64, 1)
#endif

int x3_lds_bytes(int layer) {
#define APNEAUQ_X3_LDS(L, CI, CO, K, S, WM, WN, LAST, LW, LWB, CK, WPC) \
  if (layer == L) return x3::lds_bytes(S, CO, CK);
  APNEAUQ_X3_LAYERS(APNEAUQ_X3_LDS)
#undef APNEAUQ_X3_LDS
  return 0;
}

int x3_tile_samples(int layer) {
#define APNEAUQ_X3_TS(L, CI, CO, K, S, WM, WN, LAST, LW, LWB, CK, WPC) \
  if (layer == L) return S;
  APNEAUQ_X3_LAYERS(APNEAUQ_X3_TS)
#undef APNEAUQ_X3_TS
  return 0;
}

int x3_wg_per_cu(int layer) {
#define APNEAUQ_X3_WPC(L, CI, CO, K, S, WM, WN, LAST, LW, LWB, CK, WPC) \
  if (layer == L) return WPC;
  APNEAUQ_X3_LAYERS(APNEAUQ_X3_WPC)
#undef APNEAUQ_X3_WPC
  return 1;
}

hipError_t x3_launch_layer(int layer, const x3::LayerArgs& A, int grid, hipStream_t stream) {
  using namespace x3;
  // the per-sample prescale variant only where it is used (moving statistics)
  const bool ps = A.smax_in != nullptr || A.smax_out != nullptr;
#define APNEAUQ_X3_LAUNCH(L, CI, CO, K, S, WM, WN, LAST, LW, LWB, CK, WPC)                                  \
  if (layer == L) {                                                                                       \
    return ps ? launch_layer<CI, CO, K, S, WM, WN, LAST, LW, CK, WPC, true>(A, grid, stream)               \
              : launch_layer<CI, CO, K, S, WM, WN, LAST, LWB, CK, WPC, false>(A, grid, stream);            \
  }
  APNEAUQ_X3_LAYERS(APNEAUQ_X3_LAUNCH)
#undef APNEAUQ_X3_LAUNCH
  return hipErrorInvalidValue;
}

hipError_t x3_launch_l1(const x3::L1Args& A, hipStream_t stream) {
  const int grid = A.groups * A.blocks_per_group;
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(x3::l1_kernel, dim3(grid), dim3(256), 0, stream, A);
  return hipGetLastError();
}

hipError_t x3_launch_aff(const x3::AffArgs& A, hipStream_t stream) {
  const int blocks = A.groups + (A.stats != nullptr && A.update ? 1 : 0);
  hipLaunchKernelGGL(x3::aff_kernel, dim3(blocks), dim3(256), 0, stream, A);
  return hipGetLastError();
}

hipError_t x3_launch_head(const x3::HeadArgs& A, hipStream_t stream) {
  if (A.samples <= 0) return hipSuccess;
  hipLaunchKernelGGL(x3::head_kernel, dim3((A.samples + 3) / 4), dim3(256), 0, stream, A);
  return hipGetLastError();
}

}  // namespace apneauq
