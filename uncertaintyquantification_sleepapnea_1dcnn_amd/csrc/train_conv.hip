// Layer-wise training kernels of the Alarcón 1D-CNN on gfx950 (MI355X): forward with batch-
// statistics BatchNorm, head (GAP + Dense + BCE + its gradient), conv dgrad / wgrad, BN finalize.
//
// Replaces the TF/cuDNN work inside model.fit (cnn_baseline_train.py:210, train_deep_ensemble_cnns.py:158;
// SURVEY K1-K8).  Keras semantics: ReLU inside the conv, BN on biased batch moments (eps 1e-3,
// momentum 0.99), inverted dropout (counter-based masks, ops/rng.py), BCE on logits, batch mean.
//
// Data layout ("padded rows", PL): an activation buffer holds 4 leading zero rows, then every
// sample as a 64-row slot (60 time steps + 4 zero rows), channels contiguous, bf16.  A workgroup
// tile = 2 samples = rows [128*tile, 128*tile + 136) — one contiguous copy including the conv halo.
//
// Per block l the buffers are R_l = relu(conv(A_{l-1}) + b) (pre-BN, bf16) and dY_l = dL/dBN-output
// (bf16).  R_l >= 0, so its sign bit is free: the producer stores the dropout mask of block l there
// (sign set = dropped; |R_l| is the activation), hashing each element's mask exactly once.  BN apply
// + dropout of block l are never materialised: the consumer of A_l (the next forward, the wgrad of
// block l+1) recomputes  A_l = [sign clear] * (|R_l| * s + t) / (1-p)  while staging into LDS (no
// hash), and the consumers of dZ_l (dgrad / wgrad of block l) recompute
//   dZ_l = [R_l > 0] * gamma * rstd * (dY_l - mean(dY_l) - xhat * mean(dY_l * xhat))
// from the per-channel sums accumulated by the producer's epilogue (moments: fp32 per-workgroup
// partials merged into fp64 slots, so batch statistics over ~10^6 rows per channel (MC Dropout with
// the whole test set as one batch) keep ~1e-7 relative precision; backward sums: fp32).  dgrad_l also
// writes its staged dZ_l rows to global memory, so wgrad_l (whose ci-blocked workgroups would each
// recompute the whole dZ tile) stages it with a plain copy.
//
// Forward and dgrad are implicit GEMMs on v_mfma_f32_16x16x32_bf16 with the weights as the A operand
// (pre-packed fragments from global/L2) and the staged activations as the B operand (LDS,
// ds_read_b128).  wgrad reduces over rows, so both operands are read with the CDNA4 transposing
// LDS read ds_read_b64_tr_b16 from row-major tiles; each workgroup sums up to 16 row tiles in
// registers and writes its output block to a per-row-group partial slot (Args::wpart), which
// wgrad_reduce_kernel adds in a fixed order (deterministic, and cheaper than fp32 atomics).
#include <algorithm>
#include <cstdlib>

#include "train_args.h"

namespace apneauq {
namespace train {

// Staging loops issue a batch of up to kStageU global loads per thread before the first LDS
// write, so a tile's staging pays the memory latency ceil(items / (256 * kStageU)) times instead of
// once per item (a plain load->use loop waits vmcnt(0) on every iteration).
constexpr int kStageU = 8;

struct bf16x16 {
  bf16x8 a, b;
};

template <int N, int UMAX = kStageU, int NT = kThreads, typename Load, typename Store>
__device__ __forceinline__ void staged_loop(Load load, Store store) {
  constexpr int IT = (N + NT - 1) / NT;
  constexpr int U = IT < UMAX ? IT : UMAX;
  using P = decltype(load(0));
  // opaque thread index: inside a tile loop (wgrad) LICM would otherwise hoist every per-item
  // index/address out of the loop and keep them live across the MFMAs (VGPR spills)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int b = 0; b < IT; b += U) {
    P v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + (b + u) * NT;
      if (b + u < IT && i < N) v[u] = load(i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + (b + u) * NT;
      if (b + u < IT && i < N) store(i, v[u]);
    }
  }
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)0.f;
  return o;
}

// 8 consecutive per-channel floats of an LDS table (c0 a multiple of 8) times a scale: two 16-B LDS
// reads issued together (element-wise reads were 8 dependent round trips per table per tile)
__device__ __forceinline__ void lds_row8(const float* tab, int c0, float scale, float (&o)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(tab + c0);
  const f32x4 b = *reinterpret_cast<const f32x4*>(tab + c0 + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = a[j] * scale;
    o[4 + j] = b[j] * scale;
  }
}

// Stage A_l (= dropout(BN(R_l))) rows [row0, row0 + NR) x channels [c0, c0 + NCW*8) of global
// PL buffer into LDS (row stride ldsrs bytes).  Pad rows and rows outside the batch become 0.
// row0 is a tile start (a multiple of 128), so the rows hold samples smp0 = row0/64 and smp0 + 1
// (plus the halo rows of the neighbours: pad rows, or rows whose outputs are discarded).
//
// Each thread owns one 8-channel chunk (cw = tid % NCW) for all its rows, so the BN affine of the
// chunk (x 1/(1-rate) when dropping) is loaded once per call instead of per 16-B item; the affine of
// the second stats group (a tile straddling an MC-Dropout pass boundary, g1 = s/t + 256) is selected
// per row only when it differs.  The dropout mask is R_l's sign bit (set by the producer), so the
// transform is  a = sign ? 0 : |r| * s + t  on the packed bf16 pairs.
template <int l, int NR, int NCW, int UMAX = kStageU, int NT = kThreads>
__device__ __forceinline__ void stage_act(const Args& A, char* lds, int ldsrs, int row0, int c0, const float* s,
                                          const float* t, int g0) {
  constexpr int Cc = C[l + 1];
  constexpr int RP = NT / NCW;  // rows per pass over the workgroup
  constexpr int NK = (NR + RP - 1) / RP;
  constexpr int U = NK < UMAX ? NK : UMAX;
  const Layer& Ly = A.L[l];
  // opaque thread index (see staged_loop): keeps the per-row addresses out of enclosing tile loops
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int cw = tid % NCW, rin = tid / NCW;
  const bool active = rin < RP;
  const int c = c0 + cw * 8;
  const int smp0 = row0 >> 6;
  const int g1 = min(smp0 + 1, A.B - 1) / A.n_win;
  const bool two = g1 != g0;  // workgroup-uniform
  const bool drop = A.dropout != 0;
  const float dsc = drop ? Ly.dsc : 1.f;
  float s0[8], t0[8], s1[8], t1[8];
  lds_row8(s, c, dsc, s0);
  lds_row8(t, c, dsc, t0);
  if (two) {  // workgroup-uniform; the tables of callers with one stats group end at s + 256
    lds_row8(s, 256 + c, dsc, s1);
    lds_row8(t, 256 + c, dsc, t1);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[j] = s0[j];
      t1[j] = t0[j];
    }
  }
  {
    // Every staged row exists in the padded buffer, and pad rows / rows past the batch / the
    // buffer's halo rows hold -0.0, which decodes to 0 like a dropped element: no per-row checks.
    auto run = [&](auto two_groups) {
#pragma unroll
      for (int b = 0; b < NK; b += U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int rc = rin + (b + u) * RP;
          if (b + u < NK && active && rc < NR) v[u] = gld<u32x4>(Ly.R + (long long)(row0 + rc) * Cc + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int rc = rin + (b + u) * RP;
          if (b + u >= NK || !active || rc >= NR) continue;
          const int r = rc;
          u32x4 o;
          if constexpr (decltype(two_groups)::value) {  // rare: a tile straddling an MC-Dropout pass boundary
            const bool hi = row_sample(row0 + r) != smp0;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              o[q] = decode_pair(v[u][q], hi ? s1[2 * q] : s0[2 * q], hi ? t1[2 * q] : t0[2 * q],
                                 hi ? s1[2 * q + 1] : s0[2 * q + 1], hi ? t1[2 * q + 1] : t0[2 * q + 1]);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = decode_pair(v[u][q], s0[2 * q], t0[2 * q], s0[2 * q + 1], t0[2 * q + 1]);
          }
          *reinterpret_cast<u32x4*>(lds + lds_off(r, cw * 16, ldsrs)) = o;
        }
      }
    };
    if (two)
      run(std::true_type{});
    else
      run(std::false_type{});
  }
}

// The forward kernels' input staging split in two phases so that a tile's global loads overlap the
// previous tile's moments and copy-out: load() issues every row load of a tile into registers (no
// wait), store() decodes A = dropout(BN(R)) from them into LDS (same transform as stage_act, all
// CIN channels, 136 rows).
//
// HASH_IN (batch-BN MC Dropout, block 2 reading the pass-shared block-1 output): R_0 holds one
// unencoded copy per WINDOW.  Branch-free: every staged row maps to a row of R_0 -- rows of the
// tile's two samples to their window's rows, all other rows (halo rows of the neighbours) to pad
// row 60, which holds -0.0 and decodes to 0 -- and block 1's dropout mask is drawn here from the
// counter hash on every row, as sign bits (pad rows stay -0.0 whatever it draws).
//
// Only the tile's 2 x 60 valid rows are loaded; the 16 halo / pad rows of the LDS tile (0-3, 64-67,
// 128-135) are written as zeros instead (no global load, no decode).
template <int l, bool HASH_IN>  // HASH_IN: may run in hash_in mode (runtime flag, workgroup-uniform)
struct ActStager {
  static constexpr int Cc = C[l + 1];
  static constexpr int NCW = Cc / 8;
  static constexpr int RP = kThreads / NCW;  // rows per pass over the workgroup
  static constexpr int NR = kSlots * kL;  // rows loaded from memory (the two samples' valid rows)
  static constexpr int NK = (NR + RP - 1) / RP;
  u32x4 v[NK];

  // LDS row of loaded row rc: the slot's time step, skipping halo and pad rows
  __device__ __forceinline__ static int lds_row(int rc) {
    const int slot = rc >= kL;
    return kHalo + slot * kSR + (rc - kL * slot);
  }

  __device__ __forceinline__ static int tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));  // opaque: keeps the per-row addresses out of the tile loop
    return t;
  }

  // every v[u] is assigned on every path (zeros where unused), so v is dead between store() and the
  // next load() -- in particular across the conv MFMAs
  // [U0, U1): the row batch to load / store (a split staging keeps fewer loads in flight)
  template <int U0 = 0, int U1 = NK>
  __device__ __forceinline__ void load(const Args& A, int row0, bool hash_in) {
    const int t = tid(), cw = t % NCW, rin = t / NCW;
#pragma unroll
    for (int u = U0; u < U1; ++u) v[u] = u32x4{0u, 0u, 0u, 0u};
    if (rin >= RP) return;
    const __bf16* R = A.L[l].R + cw * 8;
    if (HASH_IN && hash_in) {
      const int smp0 = row0 >> 6;
      const int n0 = min(smp0, A.B - 1), n1 = min(smp0 + 1, A.B - 1);
      const int g0 = n0 / A.n_win, g1 = n1 / A.n_win;
      const __bf16* src0 = R + (long long)(kHalo + (n0 - g0 * A.n_win) * kSR) * Cc;
      const __bf16* src1 = R + (long long)(kHalo + (n1 - g1 * A.n_win) * kSR) * Cc;
#pragma unroll
      for (int u = U0; u < U1; ++u) {
        const int rc = rin + u * RP;
        if (rc >= NR) continue;
        const int slot = rc >= kL;
        v[u] = gld<u32x4>((slot ? src1 : src0) + (long long)(rc - kL * slot) * Cc);
      }
    } else {
#pragma unroll
      for (int u = U0; u < U1; ++u) {
        const int rc = rin + u * RP;
        if (rc < NR)
          v[u] = gld<u32x4>(R + (long long)(row0 + lds_row(rc)) * Cc);
      }
    }
  }

  // s, t: the affine of stats group g0 (s + 256, t + 256: group g1 when the tile straddles two)
  template <int U0 = 0, int U1 = NK>
  __device__ __forceinline__ void store(const Args& A, char* lds, int row0, const float* s, const float* t,
                                        int g0, bool hash_in) const {
    const int tt_ = tid(), cw = tt_ % NCW, rin = tt_ / NCW;
    if (U0 == 0)  // the 16 halo / pad rows of the LDS tile: zeros (0-3, 64-67, 128-135)
      for (int i = tt_; i < 16 * NCW; i += kThreads) {
        const int pi = i / NCW, pr = pi < 4 ? pi : (pi < 8 ? kL + pi : 2 * kL + pi);
        *reinterpret_cast<u32x4*>(lds + pr * kRS + (i - pi * NCW) * 16) = u32x4{0u, 0u, 0u, 0u};
      }
    if (rin >= RP) return;
    const Layer& Ly = A.L[l];
    const int c = cw * 8;
    const int smp0 = row0 >> 6;
    const int g1 = min(smp0 + 1, A.B - 1) / A.n_win;
    const bool two = g1 != g0;  // workgroup-uniform
    const bool drop = A.dropout != 0;
    const float dsc = drop ? Ly.dsc : 1.f;
    float s0[8], t0[8], s1[8], t1[8];
    lds_row8(s, c, dsc, s0);
    lds_row8(t, c, dsc, t0);
    lds_row8(s, 256 + c, dsc, s1);  // second group (used only when two): unconditional, read together
    lds_row8(t, 256 + c, dsc, t1);
    unsigned key0 = 0u, key1 = 0u;
    if (HASH_IN && hash_in) {
      key0 = layer_sample_key(A, l, min(smp0, A.B - 1));
      key1 = layer_sample_key(A, l, min(smp0 + 1, A.B - 1));
    }
    const uint32_t thr2 = drop ? Ly.thr * 0x10001u : 0u;  // thr 0: nothing dropped
    auto run = [&](auto two_groups, auto hashed) {
#pragma unroll
      for (int u = U0; u < U1; ++u) {
        const int rc = rin + u * RP;
        if (rc >= NR) continue;
        const int r = lds_row(rc);
        const bool hi = rc >= kL;
        const int tstep = rc - kL * (rc >= kL);
        u32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t d = v[u][q];
          if constexpr (decltype(hashed)::value) d |= drop_signs2(dropout_bits2(hi ? key1 : key0, tstep, c + 2 * q), thr2);
          if constexpr (decltype(two_groups)::value)  // rare: a tile straddling an MC-Dropout pass boundary
            o[q] = decode_pair(d, hi ? s1[2 * q] : s0[2 * q], hi ? t1[2 * q] : t0[2 * q],
                               hi ? s1[2 * q + 1] : s0[2 * q + 1], hi ? t1[2 * q + 1] : t0[2 * q + 1]);
          else
            o[q] = decode_pair(d, s0[2 * q], t0[2 * q], s0[2 * q + 1], t0[2 * q + 1]);
        }
        *reinterpret_cast<u32x4*>(lds + r * kRS + cw * 16) = o;
      }
    };
    auto dispatch = [&](auto hashed) {
      if (two)
        run(std::true_type{}, hashed);
      else
        run(std::false_type{}, hashed);
    };
    if (HASH_IN && hash_in)
      dispatch(std::integral_constant<bool, HASH_IN>{});
    else
      dispatch(std::false_type{});
  }
};

// dZ_l rows into LDS (rows [row0, row0+NR), channels [c0, c0+NCW*8)); rows [own_lo, own_hi) are
// also written to ``gout`` (dgrad materialises dZ_l for wgrad).
//   l == 5: dY_6 = dlogit[n] * w[c] / 60 * mask6 * dsc6 (recomputed; never stored; mask6 = R_6's sign)
// As in stage_act, each thread owns one 8-channel chunk, and the BN backward
//   dz = relu'(r) * g*rstd * (dy - mean(dy) - xhat * mean(dy*xhat)),  xhat = (r - mean) * rstd
// is folded per channel into dz = relu'(r) * (al * dy + be * r + ga), evaluated from registers
// (r = |R_l|: the sign bit carries block l's dropout mask).
template <int l, int NR, int NCW>
__device__ __forceinline__ void stage_dz(const Args& A, char* lds, int ldsrs, int row0, int c0,
                                         const float* gam_rstd, const float* mean, const float* rstd, const float* mdy,
                                         const float* mdyx, __bf16* gout = nullptr,
                                         int own_lo = 0, int own_hi = 0) {
  constexpr int Cc = C[l + 1];
  constexpr int RP = kThreads / NCW;
  constexpr int NK = (NR + RP - 1) / RP;
  constexpr int U = NK < kStageU ? NK : kStageU;  // R + dY payloads in flight per thread
  const Layer& Ly = A.L[l];
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int cw = tid % NCW, rin = tid / NCW;
  const bool active = rin < RP;
  const int c = c0 + cw * 8;
  const int smp0 = (row0 >> 7) * 2;  // row0 is a tile start, or a tile start + kHalo
  float al[8], be[8], ga[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float g = gam_rstd[c + j], q = rstd[c + j] * mdyx[c + j];
    al[j] = g;
    be[j] = -g * q;
    ga[j] = g * (q * mean[c + j] - mdy[c + j]);
  }
  // block 6: dY is recomputed from dlogit, the dense weights and the dropout mask of block 6
  float dw[8] = {}, dl0 = 0.f, dl1 = 0.f;
  if constexpr (l == 5) {
    const float dsc = A.dropout ? Ly.dsc : 1.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dw[j] = A.dense_w[c + j] * dsc;
    dl0 = A.dlogit[min(smp0, A.B - 1)] * (1.0f / kL);
    dl1 = A.dlogit[min(smp0 + 1, A.B - 1)] * (1.0f / kL);
  }
  auto valid = [&](int grow) {
    const int n = row_sample(grow), tt = row_time(grow);
    return !(grow < kHalo || n >= A.B || tt >= kL);
  };
#pragma unroll
  for (int b = 0; b < NK; b += U) {
    // payload: R_l (pre-BN activation) and dY_l, both loaded in the batched first phase
    bf16x16 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = rin + (b + u) * RP;
      const int grow = row0 + r;
      if (b + u >= NK) continue;
      const bool ok = active && r < NR && valid(grow);
      q[u].a = ok ? gld<bf16x8>(Ly.R + (long long)grow * Cc + c) : zero8();
      if constexpr (l < 5) q[u].b = ok ? gld<bf16x8>(Ly.dY + (long long)grow * Cc + c) : zero8();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = rin + (b + u) * RP;
      if (b + u >= NK || !active || r >= NR) continue;
      const int grow = row0 + r;
      bf16x8 o = zero8();
      if (valid(grow)) {
        float dy[8];
        if constexpr (l == 5) {
          const bool hi = row_sample(grow) != smp0;
          const float dl = hi ? dl1 : dl0;
#pragma unroll
          for (int j = 0; j < 8; ++j) dy[j] = bf_dropped(q[u].a[j]) ? 0.f : dl * dw[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) dy[j] = (float)q[u].b[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float rr = bf_abs(q[u].a[j]);
          const float dz = __builtin_fmaf(al[j], dy[j], __builtin_fmaf(be[j], rr, ga[j]));
          o[j] = (__bf16)(rr > 0.f ? dz : 0.f);
        }
      }
      *reinterpret_cast<bf16x8*>(lds + lds_off(r, cw * 16, ldsrs)) = o;
      if (gout != nullptr && r >= own_lo && r < own_hi)
        *reinterpret_cast<bf16x8*>(gout + (long long)grow * Cc + c) = o;  // pad rows get their zeros too
    }
  }
}

// dZ_l rows [row0, row0+NR) x channels [c0, c0+NCW*8) into LDS (wgrad; dgrad materialised them)
template <int l, int NR, int NCW, int UMAX, int NT = kThreads>
__device__ __forceinline__ void stage_dz_copy(const Args& A, char* lds, int ldsrs, int row0, int c0) {
  constexpr int Cc = C[l + 1];
  const Layer& Ly = A.L[l];
  staged_loop<NR * NCW, UMAX, NT>(
      [&](int i) -> bf16x8 {
        const int rc = i / NCW, cw = i - rc * NCW;
        return gld<bf16x8>(Ly.dZ + (long long)(row0 + rc) * Cc + c0 + cw * 8);
      },
      [&](int i, const bf16x8& o) {
        const int rc = i / NCW, cw = i - rc * NCW;
        *reinterpret_cast<bf16x8*>(lds + lds_off(rc, cw * 16, ldsrs)) = o;
      });
}

// Implicit-GEMM conv tile: D^T[co][row] over the 128-row tile, weights = packed A fragments.
template <int CIN, int COUT, int K, int WM, int WN, bool FIRST>
struct Conv {
  static constexpr int NSTEP = (CIN * K + 31) / 32;
  static constexpr int NCT = COUT / 16;
  static constexpr int CT = NCT / WN;
  static constexpr int RT = kRT / WM;
  static constexpr int PAD = (K - 1) / 2;
  static_assert(NCT % WN == 0 && kRT % WM == 0 && WM * WN == 4, "wave tiling");

  template <int PD = 1, bool RING = true>
  __device__ __forceinline__ static void run(const gbf16x8* wfrag, const char* lds, int ldsrs, f32x4 (&acc)[CT][RT]) {
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    steps<0, NSTEP, PD, RING>(wfrag, lds, ldsrs, acc);
  }

  // steps [S0, S1) accumulated into acc; the wave's place in its 4-wave team is (threadIdx.x >> 6) & 3,
  // so 512-thread kernels run two teams.  PD = weight-fragment prefetch depth (k-steps in flight).
  template <int S0, int S1, int PD = 1, bool RING = true>
  __device__ __forceinline__ static void steps(const gbf16x8* wfrag, const char* lds, int ldsrs,
                                               f32x4 (&acc)[CT][RT]) {
    static_assert(S0 < S1 && PD >= 1, "step range");
    const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3;
    const int wm = wave / WN, wn = wave % WN;
    const int m = lane & 15, h = lane >> 4;
    const gbf16x8* wp = wfrag + (wn * CT) * 64 + lane;
    const int row0 = wm * RT * 16 + m;
    const char* bbase = lds + (kHalo + row0 - PAD) * ldsrs + 16 * h;
    auto load_b = [&](int s, int r) -> bf16x8 {
      if constexpr (FIRST) {
        const char* base = lds + (kHalo + row0 + r * 16 - PAD) * ldsrs + (32 * s + 8 * h) * 2;
        const bf16x4 lo = *reinterpret_cast<const bf16x4*>(base);
        const bf16x4 hi = *reinterpret_cast<const bf16x4*>(base + 8);
        return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      } else {
        // lane base + uniform step offset + compile-time row-tile offset (see fused_forward.hip)
        constexpr int CB = CIN / 32;
        const int tap = s / CB, cb = s - tap * CB;
        const int soff = __builtin_amdgcn_readfirstlane(tap * ldsrs + cb * 64);
        return *reinterpret_cast<const bf16x8*>(bbase + soff + r * 16 * ldsrs);
      }
    };
    auto load_a = [&](int s, bf16x8 (&a)[CT]) {
#pragma unroll
      for (int c = 0; c < CT; ++c) a[c] = wp[(s * NCT + c) * 64];
    };
    // Weight fragments (A, from L2) run through a ring of PD + 1 stages: step s + PD's loads are issued
    // before step s's MFMAs (the fused kernel's scheme; see FwdPD for the measured depths).
    // B fragments (activations, LDS) run through a ring of NB registers over the (step, row tile)
    // sequence: the read of fragment i + NB is issued right after the CT MFMAs of fragment i, so
    // NB - 1 LDS reads stay in flight.  RING = false reads each B fragment just in time (dgrad: one
    // tile per workgroup, two workgroups per CU, measured 5-17 % faster per layer without the ring).
    constexpr int NSA = PD + 1;
    constexpr int NB = RT < 4 ? RT : 4;  // B-fragment ring depth (2 and 8 measured equal / slower)
    static_assert(RT % NB == 0, "B ring phase restarts at every step");
    constexpr int DSN = FIRST ? 2 : 1;  // LDS reads per B fragment
    bf16x8 bq[NB];
    if constexpr (RING) {
#pragma unroll
      for (int i = 0; i < NB; ++i) bq[i] = load_b(S0, i);
    }
    // step s at position j of its group (group base sb = s - j); tail: no refills past S1
    auto step = [&](int s, const bf16x8 (&a)[CT], int j, bool tail) {
      if constexpr (!RING) {
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          const bf16x8 b = load_b(s, r);
#pragma unroll
          for (int c = 0; c < CT; ++c) acc[c][r] = mfma16(a[c], b, acc[c][r]);
        }
        return;
      }
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int i = j * RT + r;
        const bf16x8 b = bq[i % NB];
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[c][r] = mfma16(a[c], b, acc[c][r]);
        const int nx = i + NB;               // ring successor within the group
        const int sn = s - j + nx / RT;       // its step
        if (!tail || sn < S1) bq[i % NB] = load_b(sn < S1 ? sn : S1 - 1, nx % RT);  // clamped: unconditional
        __builtin_amdgcn_sched_group_barrier(0x008, CT, 0);   // the fragment's MFMAs ...
        __builtin_amdgcn_sched_group_barrier(0x100, DSN, 0);  // ... then its successor's read
      }
    };
    // unconditional (clamped) prefetch keeps hipcc's vmcnt accounting exact (see fused_forward.hip)
    bf16x8 a[NSA][CT];
#pragma unroll
    for (int j = 0; j < PD; ++j) load_a(S0 + j < S1 ? S0 + j : S1 - 1, a[j]);
    constexpr int NFULL = (S1 - S0) / NSA * NSA;
#pragma unroll 1
    for (int s0 = S0; s0 < S0 + NFULL; s0 += NSA) {
#pragma unroll
      for (int j = 0; j < NSA; ++j) {
        const int s = s0 + j;
        load_a(s + PD < S1 ? s + PD : S1 - 1, a[(j + PD) % NSA]);
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this step's MFMAs
        step(s, a[j], j, false);
      }
    }
#pragma unroll
    for (int j = 0; j < (S1 - S0) - NFULL; ++j) step(S0 + NFULL + j, a[j], j, true);
  }
};


__device__ __forceinline__ bf16x8 tr_frag(const char* lds, int ldsrs, int row_base, int col0) {
  // fragment for a 16x16x32 operand whose K index is the LDS row, 32 rows from row_base.  Lane
  // group h (16 lanes) reads 4 rows x 16 cols per ds_read_b64_tr_b16; k-slot (h, j) of the fragment
  // holds row row_base + 4h + j (j < 4, first read) or row_base + 16 + 4h + j - 4 (second read).
  // Any k-permutation is exact as long as both operands use it, and this one makes each 32-lane
  // bank group read 8 CONSECUTIVE rows: with a row stride that is an odd multiple of 32 B they fall
  // on 8 distinct 8-bank groups, conflict-free for any row_base (the natural order, rows
  // r0..r0+3 and r0+8..r0+11, is 2-way for every stride: 37-42 % conflict cycles in round 1).
  const int lane = threadIdx.x & 63;
  const int h = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int ra = row_base + 4 * h + q;
  const char* a0 = lds + lds_off(ra, (col0 + 4 * p) * 2, ldsrs);
  const char* a1 = lds + lds_off(ra + 16, (col0 + 4 * p) * 2, ldsrs);
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a1);
  // one 8 x 16-bit register quad: no per-element moves
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// Weight-fragment prefetch depth of the forward conv (k-steps in flight): depth 1 everywhere 29.8 ms
// per 16-pass x 16384-window batch-BN chunk, depth 2 30.0, per-layer (1,3,2,3,2,3) 30.4, depth 4 38.7
// (spills) -- the conv is not bound by the L2 round trip of its weight fragments
// (profiles/batch_bn_fwd_r2.md).
constexpr int kFwdPD = 1;

// Forward input staging of block l in two row batches instead of all of a tile's row loads in flight
// at once (ActStager): blocks 3 and 6 spilled 22 / 44 VGPRs with one batch; split, neither spills and
// the batch-BN MC-Dropout chunk is ~2 % faster (profiles/batch_bn_fwd_r2.md, session 3).
template <int l> struct FwdStageSplit { static constexpr bool v = l == 2 || l == 5; };
// Large training launches (more row tiles than kFwdTrainGrid workgroups: batch >= 2048, or the
// member-batched step) run the PF instantiation of the forward: kFwdTrainGrid persistent workgroups over
// contiguous tile ranges, the first FwdPF<l>::v input-row loads per thread of the NEXT tile issued before
// this tile's conv (registers each block leaves: 8 of 8 on block 2, 14 of 14 on block 4).  Batch 1024 (one
// tile per workgroup anyway) keeps the plain instantiation: the PF one measured +1 % there.
template <int l> struct FwdPF { static constexpr int v = l == 1 ? 8 : l == 3 ? 14 : 0; };
constexpr int kFwdTrainGrid = 512;

// wave tilings (WM, WN) per output-channel count
template <int COUT> struct Tiling;
template <> struct Tiling<128> { static constexpr int WM = 1, WN = 4; };
template <> struct Tiling<192> { static constexpr int WM = 1, WN = 4; };
template <> struct Tiling<224> { static constexpr int WM = 2, WN = 2; };
template <> struct Tiling<96> { static constexpr int WM = 2, WN = 2; };
template <> struct Tiling<256> { static constexpr int WM = 1, WN = 4; };

extern __shared__ __attribute__((aligned(16))) char smem[];

// Reduce per-lane partial sums over the 16 rows of a lane group and add them to a global
// per-channel accumulator (fp32 atomics; one per channel per wave row-group).
__device__ __forceinline__ void atomic_channel_sums(double* dst, int co0, const f32x4& a, bool leader) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float v = group16_sum(a[i]);
    if (leader) atomicAdd(dst + co0 + i, (double)v);
  }
}

// ------------------------------------------------------------------------------------------------
// Forward of block l:  R_l = relu(conv(A_{l-1}) + b), fwd sums of R_l per stats group.
// ------------------------------------------------------------------------------------------------
template <int l, bool MB, bool PFT = false>
__global__ __launch_bounds__(kThreads, 2) void fwd_kernel(Args A_, const Args* __restrict__ Am) {
  const MbPos pos = mb_pos<MB>();
  const Args& A = member_args<MB>(A_, Am, pos);
  constexpr int CIN = C[l], COUT = C[l + 1];
  using T = Tiling<COUT>;
  using CV = Conv<CIN, COUT, KS[l], T::WM, T::WN, l == 0>;
  char* act = smem;                                  // staged input, then staged output
  float* prm = reinterpret_cast<float*>(smem + kRows * kRS);  // [s 512 | t 512]
  constexpr int IN_RS = (l == 0) ? 8 : kRS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / T::WN, wn = wave % T::WN;
  const int m = lane & 15, h = lane >> 4;
  const Layer& Ly = A.L[l];
  // Each workgroup owns a contiguous range of tiles (so the stats group changes rarely).  The channel
  // moments of a stored tile come from the matrix cores: per 16-channel tile ct, sum_rows r^2 is the
  // diagonal of R_ct^T R_ct and sum_rows r is ones^T R_ct, 8 MFMAs over the 128 rows on operands read
  // with ds_read_b64_tr_b16 (no per-element VALU: the layer kernels are VALU-issue bound).  The lanes
  // holding a diagonal keep fp32 partials across the run of tiles of one stats group, merged (LDS
  // atomics, then fp64 global slots) only when the group changes.
  const int tiles = (A.B + 1) / 2;
  const int tpw = (tiles + gridDim.x - 1) / gridDim.x;
  const int t_begin = pos.bx * tpw;
  const int t_end = min(tiles, t_begin + tpw);
  float* lstat = prm + 1024;  // [2][COUT]: sum r, sum r^2 of the current group run
  for (int c = threadIdx.x; c < 2 * COUT; c += kThreads) lstat[c] = 0.f;
  int gcur = -1;
  double* st = Ly.st + (pos.bx % kStatSlots) * st_stride(A, COUT);
  constexpr int CW = COUT / 8;             // 16-B chunks per output row
  constexpr int RPo = kThreads / CW;       // rows per copy-out pass
  // copy-out rows: the tile's 2 x 60 valid time steps only (the R buffers are allocated filled with
  // -0.0 and their pad rows are never written)
  constexpr int kOutRows = kSlots * kL;
  constexpr int NPo = (kOutRows + RPo - 1) / RPo;
  const int ocw = threadIdx.x % CW, orin = threadIdx.x / CW;
  const bool oact = orin < RPo;
  constexpr int NCTo = COUT / 16, CPW = (NCTo + 3) / 4;  // moment channel tiles: ct = wave + 4j
  const int sn = lane & 15;
  const bool diag_lane = (lane >> 4) == (sn >> 2);        // holds D[sn][sn] of a 16x16 tile
  float ps1[CPW], ps2[CPW];
#pragma unroll
  for (int j = 0; j < CPW; ++j) ps1[j] = ps2[j] = 0.f;
  auto flush = [&]() {  // workgroup-uniform: fp32 run partials (<= ~10^4 rows / lane) merged in fp64
    if (gcur >= 0 && diag_lane) {
#pragma unroll
      for (int j = 0; j < CPW; ++j) {
        const int ct = wave + 4 * j;
        if (ct < NCTo) {
          atomicAdd(&lstat[ct * 16 + sn], ps1[j]);
          atomicAdd(&lstat[COUT + ct * 16 + sn], ps2[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < CPW; ++j) ps1[j] = ps2[j] = 0.f;
    __syncthreads();
    if (gcur >= 0 && A.det == nullptr) {
      for (int c = threadIdx.x; c < COUT; c += kThreads) {
        atomicAdd(st + (gcur * 2 + 0) * COUT + c, (double)lstat[c]);
        atomicAdd(st + (gcur * 2 + 1) * COUT + c, (double)lstat[COUT + c]);
        lstat[c] = lstat[COUT + c] = 0.f;
      }
    }
    __syncthreads();
  };
  // this block's dropout mask goes into the sign bit of R_l (not for the pass-shared block 1)
  const bool enc = A.dropout != 0 && !(l == 0 && A.shared0);
  const bool hash_in = l == 1 && A.shared0;  // workgroup-uniform
  int gaff = -1;  // stats group whose BN affine (of block l-1) is in prm
  // input staging: loads of a tile's rows, then A = dropout(BN(R)) decoded into LDS
  ActStager<(l > 0 ? l - 1 : 0), l == 1> stg;
  constexpr int NPF = !PFT || l == 0 || FwdStageSplit<l>::v ? 0
                      : (FwdPF<l>::v < decltype(stg)::NK ? FwdPF<l>::v : decltype(stg)::NK);
  if constexpr (NPF > 0) {
    if (t_begin < t_end) stg.template load<0, NPF>(A, kR * t_begin, hash_in);
  }
  for (int tile = t_begin; tile < t_end; ++tile) {
    APNEAUQ_DASSERT(2 * tile < A.B + 1 && blockDim.x == kThreads);
    const int row0 = kR * tile;                        // first staged row (global PL index)
    const int smp0 = 2 * tile;
    const int g0 = min(smp0, A.B - 1) / A.n_win, g1 = min(smp0 + 1, A.B - 1) / A.n_win;
    __syncthreads();  // previous tile's copy-out has read the LDS tile
    if constexpr (l == 0) {
      staged_loop<kRows * 8 / 16>(
          [&](int i) -> bf16x8 { return gld<bf16x8>(A.x + (long long)row0 * 4 + i * 8); },
          [&](int i, const bf16x8& v) { reinterpret_cast<bf16x8*>(act)[i] = v; });
    } else {
      if (g0 != gaff || g1 != g0) {  // (re)load the affine of block l-1 for this tile's group(s)
        bn_affine_to_lds(A, l - 1, g0, prm, prm + 512, nullptr, nullptr);
        if (g1 != g0) bn_affine_to_lds(A, l - 1, g1, prm + 256, prm + 768, nullptr, nullptr);
        gaff = (g1 == g0) ? g0 : -1;
        __syncthreads();
      }
      if constexpr (FwdStageSplit<l>::v) {  // two row batches: fewer loads in flight, no spills
        constexpr int NK = decltype(stg)::NK, H = (NK + 1) / 2;
        stg.template load<0, H>(A, row0, hash_in);
        stg.template store<0, H>(A, act, row0, prm, prm + 512, g0, hash_in);
        stg.template load<H, NK>(A, row0, hash_in);
        stg.template store<H, NK>(A, act, row0, prm, prm + 512, g0, hash_in);
      } else if constexpr (NPF > 0) {  // items [0, NPF) were loaded during the previous tile's conv
        stg.template load<NPF, decltype(stg)::NK>(A, row0, hash_in);
        stg.store(A, act, row0, prm, prm + 512, g0, hash_in);
      } else {
        stg.load(A, row0, hash_in);
        stg.store(A, act, row0, prm, prm + 512, g0, hash_in);
      }
    }
    __syncthreads();
    if constexpr (NPF > 0) {
      if (tile + 1 < t_end) stg.template load<0, NPF>(A, kR * (tile + 1), hash_in);
    }
    // epilogue of one 16 x 16 accumulator tile: bias + ReLU -> bf16 LDS tile (rows outside the batch /
    // pad rows: 0).  Only the row tiles holding t = 48..63 (pad rows on lanes m >= 12) and the batch's
    // last tile need the select.
    const bool last_tile = smp0 + 1 >= A.B;  // workgroup-uniform
    auto epi = [&](const f32x4& a4, int co0, int rtg, const f32x4& bias) {
      const int row = rtg * 16 + m;  // 0..127 within the tile (rtg wave-uniform)
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaxf(a4[i] + bias[i], 0.f);
      if ((rtg & 3) == 3 || last_tile) {
        const bool valid = (row & 63) < kL && (smp0 + (row >> 6)) < A.B;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = valid ? v[i] : 0.f;
          asm volatile("" : "+v"(v[i]));  // keep the select in fp32 (no per-element cvt + v_perm repack)
        }
      }
      bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
      *reinterpret_cast<bf16x4*>(act + row * kRS + co0 * 2) = o;
    };
    f32x4 acc[CV::CT][CV::RT];
    if constexpr (kFwdPrio) __builtin_amdgcn_s_setprio(1);
    CV::template run<kFwdPD, true>(Ly.wf, act, IN_RS, acc);
    if constexpr (kFwdPrio) __builtin_amdgcn_s_setprio(0);
    __syncthreads();  // all waves done reading the staged input; reuse it for the output tile
#pragma unroll
    for (int c = 0; c < CV::CT; ++c) {
      const int co0 = (wn * CV::CT + c) * 16 + 4 * h;
      const f32x4 bias = gld<f32x4>(Ly.bias + co0);
#pragma unroll
      for (int r = 0; r < CV::RT; ++r) epi(acc[c][r], co0, wm * CV::RT + r, bias);
    }
    __syncthreads();
    // channel moments of the stored tile (zero rows add nothing) on the matrix cores
    auto moments = [&](int sel) {  // sel: sample slot (rows 64*sel .. +64 = 32-row chunks 2sel, 2sel+1), -1: both
      {
        bf16x8 ones;
#pragma unroll
        for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
        const int si = sn & 3;
#pragma unroll
        for (int j = 0; j < CPW; ++j) {
          const int ct = wave + 4 * j;
          if (ct >= NCTo) break;  // wave-uniform
          f32x4 g = {0.f, 0.f, 0.f, 0.f}, sm = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kc = 0; kc < kR / 32; ++kc) {
            if (sel >= 0 && (kc >> 1) != sel) continue;
            const bf16x8 f = tr_frag(act, kRS, kc * 32, ct * 16);
            g = mfma16(f, f, g);       // R^T R
            sm = mfma16(ones, f, sm);  // ones^T R
          }
          const float dg = si == 0 ? g[0] : si == 1 ? g[1] : si == 2 ? g[2] : g[3];
          const float s1v = si == 0 ? sm[0] : si == 1 ? sm[1] : si == 2 ? sm[2] : sm[3];
          ps1[j] += s1v;
          ps2[j] += dg;
        }
      }
    };
    // coalesced copy-out of the 128 tile rows (16 B per thread-iteration) with this block's dropout
    // mask in the sign bits (drawn here, where no accumulators are live)
    unsigned key[kSlots] = {0u, 0u};
    if (enc) {
      key[0] = layer_sample_key(A, l, min(smp0, A.B - 1));
      key[1] = layer_sample_key(A, l, min(smp0 + 1, A.B - 1));
    }
    const uint32_t thr2 = Ly.thr * 0x10001u;
    auto copy_out = [&]() {
      // opaque row index (see staged_loop): keeps the NPo per-row addresses out of the tile loop
      int rin = orin;
      asm volatile("" : "+v"(rin));
#pragma unroll 2
      for (int k = 0; k < NPo; ++k) {
        const int rc = rin + k * RPo;
        if (!oact || rc >= kOutRows) continue;
        const int slot = rc >= kL, tt = rc - kL * slot;
        const int r = slot * kSR + tt;
        bf16x8 o = *reinterpret_cast<const bf16x8*>(act + r * kRS + ocw * 16);
        uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
        if (!(tt < kL && smp0 + slot < A.B)) {  // pad / out-of-batch rows: -0.0, decoded as A = 0
#pragma unroll
          for (int q = 0; q < 4; ++q) ow[q] = kNegZero2;
        } else if (enc) {
#pragma unroll
          for (int q = 0; q < 4; ++q) ow[q] |= drop_signs2(dropout_bits2(key[slot], tt, ocw * 8 + 2 * q), thr2);
        }
        *reinterpret_cast<bf16x8*>(Ly.R + (long long)(row0 + kHalo + r) * COUT + ocw * 8) = o;
      }
    };
    if (g0 == g1) {
      if (g0 != gcur) {
        flush();
        gcur = g0;
      }
      moments(-1);
    } else {  // a tile straddling two stats groups (MC-Dropout pass boundary): moments per slot
      flush();
      gcur = g0;
      moments(0);
      flush();
      gcur = g1;
      moments(1);
    }
    copy_out();
  }
  flush();
  if (A.det != nullptr) {  // deterministic mode (one stats group): this workgroup's moment partials
    float* dp = A.det + (long long)pos.bx * 2 * COUT;
    for (int c = threadIdx.x; c < 2 * COUT; c += kThreads) dp[c] = lstat[c];
  }
}

// Parameter table (Args::tab) of single-device training: mode 0 = the forward rows of every block
// (one workgroup per block, launched after the six forward kernels; read by the head, dgrad and wgrad),
// mode 1 = the backward rows of block l (not on the default step: the backward kernels sum bst[l]
// themselves, 2 x 16 slots per channel, which measured cheaper than one more graph node per block).
template <bool MB>
__global__ __launch_bounds__(256) void tab_kernel(Args A_, const Args* __restrict__ Am, int mode, int l) {
  const MbPos pos = mb_pos<MB>();
  const Args& A = member_args<MB>(A_, Am, pos);
  if (mode == 0)
    tab_write_fwd(A, pos.bx);
  else
    tab_write_bwd(A, l);
}

// ------------------------------------------------------------------------------------------------
// Head: A_6 = dropout(BN(R_6)) -> GAP -> Dense(96->1) -> logit, BCE, dlogit = (sigmoid - y)/B,
// dense gradients, and the backward sums of dY_6 (sum dY, sum dY * xhat) — one sample per wave,
// each lane owning channels (lane, lane + 64).
// ------------------------------------------------------------------------------------------------
template <bool MB>
__global__ __launch_bounds__(kThreads) void head_kernel(Args A_, const Args* __restrict__ Am, int backward, int spw,
                                                      int tabx) {
  const MbPos pos = mb_pos<MB>();
  const Args& A = member_args<MB>(A_, Am, pos);
  // tabx > 0: the last tabx workgroups write the forward rows of the parameter table (what a tab_kernel
  // launch did before the head), the head computes block 6's rows itself with the same arithmetic
  if (tabx > 0 && pos.bx >= (int)gridDim.x - tabx) {
    tab_write_fwd(A, pos.bx - ((int)gridDim.x - tabx));
    return;
  }
  // One sample at a time per wave, spw samples per wave (4 * spw per workgroup: fewer workgroups'
  // sums to merge at large batches).  Lane (cw, ph) = (lane % 12, lane / 12), lanes 0..59: channels
  // [8cw, 8cw+8) of rows ph, ph+5, ..., ph+55 — twelve 16-B loads per lane, all in flight at once
  // (the previous per-channel/per-row scalar loop was load-latency bound: ~50 us at any batch size).
  constexpr int Cc = C[6], NCW = Cc / 8, NPH = 5, NJ = kL / NPH;
  static_assert(NCW * NPH <= 64 && NJ * NPH == kL, "head lane map");
  float* prm = reinterpret_cast<float*>(smem);  // [mu | rs | sc | sh | w] x 96, then sums
  float* pmu = prm, *prs = prm + Cc, *psc = prm + 2 * Cc, *psh = prm + 3 * Cc, *pw = prm + 4 * Cc;
  float* dw = prm + 5 * Cc;     // dense-weight gradient sums
  float* bsum0 = dw + Cc;       // sum dY, sum dY * xhat (backward BN sums of block 6)
  float* bsum1 = bsum0 + Cc;
  float* red = bsum1 + Cc;      // per-workgroup loss / dense-bias sums: one global atomic per workgroup
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwg0 = pos.bx * 4 * spw;  // the workgroup's first sample
  const Layer& Ly = A.L[5];
  const int g_first = min(nwg0, A.B - 1) / A.n_win;
  const int g_last = min(nwg0 + 4 * spw - 1, A.B - 1) / A.n_win;
  for (int c = threadIdx.x; c < 3 * Cc + 2; c += kThreads) dw[c] = 0.f;
  auto params = [&](int g) {
    if (A.tab != nullptr && tabx == 0) {  // single-device training (one group): the forward rows of T[5]
      for (int c = threadIdx.x; c < Cc; c += kThreads) {
        pmu[c] = tab_row(A, 5, kTabMean)[c];
        prs[c] = tab_row(A, 5, kTabRstd)[c];
        psc[c] = tab_row(A, 5, kTabS)[c];
        psh[c] = tab_row(A, 5, kTabT)[c];
        pw[c] = A.dense_w[c];
      }
      return;
    }
    for (int c = threadIdx.x; c < Cc; c += kThreads) {
      float m1, var;
      bn_moments(A, 5, g, c, m1, var);
      const float r = rsqrtf(var + A.eps), sc = Ly.gamma[c] * r;  // as tab_write_fwd
      pmu[c] = m1;
      prs[c] = r;
      psc[c] = sc;
      psh[c] = Ly.beta[c] - m1 * sc;
      pw[c] = A.dense_w[c];
    }
  };
  params(g_first);
  __syncthreads();
  // (a workgroup whose samples span two stats groups — an MC-Dropout pass boundary — recomputes
  //  its per-lane parameters of the other group from the global sums directly)
  const bool mixed = g_first != g_last;
  const int cw = lane % NCW, ph = lane / NCW;
  const int c0 = cw * 8;
  const float dsc6 = A.dropout ? Ly.dsc : 1.f;
  for (int s = 0; s < spw; ++s) {  // wave-uniform
    const int n = nwg0 + s * 4 + wave;
    const bool active = n < A.B && lane < NCW * NPH;
    float mu[8], rs[8], sc[8], sh[8], w[8];
    if (active) {
      const int g = n / A.n_win;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        if (mixed && g != g_first) {
          float m1, var;
          bn_moments(A, 5, g, c, m1, var);
          rs[j] = rsqrtf(var + A.eps);
          mu[j] = m1;
          sc[j] = Ly.gamma[c] * rs[j];
          sh[j] = Ly.beta[c] - m1 * sc[j];
        } else {
          mu[j] = pmu[c];
          rs[j] = prs[c];
          sc[j] = psc[c];
          sh[j] = psh[c];
        }
        w[j] = pw[c];
      }
    }
    bf16x8 v[NJ];
    float gap[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (active) {
      const __bf16* base = Ly.R + (long long)(kHalo + n * kSR) * Cc + c0;
#pragma unroll
      for (int k = 0; k < NJ; ++k) v[k] = gld<bf16x8>(base + (long long)(ph + NPH * k) * Cc);
#pragma unroll
      for (int k = 0; k < NJ; ++k) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // block 6's dropout mask is R_6's sign bit
          const float a = bf_abs(v[k][j]) * sc[j] + sh[j];
          gap[j] += bf_dropped(v[k][j]) ? 0.f : a * dsc6;
        }
      }
    }
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) part += gap[j] * w[j];
    const float z = wave_sum(active ? part : 0.f) * (1.0f / kL) + A.dense_b[0];
    if (n < A.B && lane == 0) A.logits[n] = z;
    if (backward && n < A.B) {
      const float pz = 1.0f / (1.0f + __expf(-z));
      const float yv = A.y[n];
      const float dl = (pz - yv) * A.inv_batch;
      float* rec = A.det != nullptr ? A.det + (long long)n * kHeadRec : nullptr;  // deterministic mode
      if (lane == 0) {
        const float loss = fmaxf(z, 0.f) - z * yv + log1pf(__expf(-fabsf(z)));  // BCE on logits
        A.dlogit[n] = dl;
        if (rec != nullptr) {
          rec[0] = loss;
          rec[1] = dl;
        } else {
          atomicAdd(&red[0], loss);
          atomicAdd(&red[1], dl);
        }
      }
      if (active) {
        float b0[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, b1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < NJ; ++k) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float dy = bf_dropped(v[k][j]) ? 0.f : dl * w[j] * (1.0f / kL) * dsc6;
            const float xh = (bf_abs(v[k][j]) - mu[j]) * rs[j];
            b0[j] += dy;
            b1[j] += dy * xh;
          }
        }
        // the sample's sums over its 5 row-phase lanes (lanes cw + 12 ph), in a fixed order; then
        // one LDS atomic per channel from the ph = 0 lanes (not 5)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float sdw = 0.f, sb0 = 0.f, sb1 = 0.f;
          const float pdw = dl * gap[j] * (1.0f / kL);
#pragma unroll
          for (int q = 0; q < NPH; ++q) {
            sdw += __shfl(pdw, cw + NCW * q, kWave);
            sb0 += __shfl(b0[j], cw + NCW * q, kWave);
            sb1 += __shfl(b1[j], cw + NCW * q, kWave);
          }
          if (ph == 0) {
            if (rec != nullptr) {
              rec[2 + c0 + j] = sdw;
              rec[2 + Cc + c0 + j] = sb0;
              rec[2 + 2 * Cc + c0 + j] = sb1;
            } else {
              atomicAdd(&dw[c0 + j], sdw);
              atomicAdd(&bsum0[c0 + j], sb0);
              atomicAdd(&bsum1[c0 + j], sb1);
            }
          }
        }
      }
    }
  }
  if (backward) {
    if (A.det != nullptr) return;  // det_reduce_kernel sums the per-sample records
    __syncthreads();
    float* hp = A.hpart != nullptr ? A.hpart + (pos.bx % kStatSlots) * (Cc + 2) : nullptr;
    for (int c = threadIdx.x; c < Cc; c += kThreads) {
      if (hp != nullptr) {  // slotted: summed by bn_finalize_kernel
        if (c == 0) {
          atomicAdd(hp + Cc, red[0]);
          atomicAdd(hp + Cc + 1, red[1]);
        }
        atomicAdd(hp + c, dw[c]);
      } else {
        if (c == 0) {
          atomicAdd(A.loss_sum, red[0]);
          atomicAdd(A.g_dense_b, red[1]);
        }
        atomicAdd(A.g_dense_w + c, dw[c]);
      }
      double* bst = Ly.bst + (pos.bx % kStatSlots) * 2 * Cc;
      atomicAdd(bst + c, (double)bsum0[c]);
      atomicAdd(bst + Cc + c, (double)bsum1[c]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// dgrad of block l (l >= 1): dA_{l-1} = conv^T(dZ_l, W_l);  epilogue -> dY_{l-1} = dA * mask_{l-1}
// plus the backward sums of block l-1.
// ------------------------------------------------------------------------------------------------
// dgrad: prefetch the epilogue's R_{l-1} loads ahead of the conv (every block; block 6 has had the
// registers for it since its staging became DzStager: dgrad<5> b8192 -0.6 %, 8 members -0.5..-1.9 %)
template <int l> struct DgPre { static constexpr bool v = l >= 1 && l <= 5; };
// Persistent dgrad: a workgroup runs row tiles tile, tile + grid, ...; the first DgPF<l>::v staging items
// per thread of the NEXT tile (R_l and dY_l rows, 8 channels each) are loaded into registers before this
// tile's conv, so their latency hides under the MFMAs (the rest load at staging time, as before).
// Sized to the registers each block leaves with DgPre (tools/kernel_resources.py: no spills); trading
// DgPre for a deeper staging prefetch measured slower (profiles/train_step_r5.md).
template <int l> struct DgPF { static constexpr int v = l == 1 ? 8 : l == 2 ? 2 : l == 4 ? 12 : 0; };
// workgroups of a single-model dgrad launch: two per CU (larger batches loop over their tiles)
constexpr int kDgGrid = 512;
// Weight-fragment prefetch depth of the dgrad conv (k-steps in flight): 2 where it fits the 256-VGPR budget
// without spilling (blocks 3 / 6 spill at 2: 56 / 12 B of scratch)
template <int l> struct DgPD { static constexpr int v = (l == 1 || l == 2 || l == 4) ? 2 : 1; };

// stage_dz for dgrad (all CIN channels of 136 rows, dZ_l also written to global for wgrad) split into
// load() (the prefetched items, into registers) and store() (every item: the prefetched ones from
// registers, the rest loaded in batches there), so the next tile's loads can overlap this tile's conv.
template <int l, int NPF>
struct DzStager {
  static constexpr int Cc = C[l + 1], NCW = Cc / 8, RP = kThreads / NCW, NR = kRows;
  static constexpr int NK = (NR + RP - 1) / RP;
  static constexpr int NP = NPF < NK ? NPF : NK;
  static constexpr int U = kStageU;
  bf16x8 r[NP > 0 ? NP : 1];
  bf16x8 d[(NP > 0 && l < 5) ? NP : 1];

  __device__ __forceinline__ static int tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
  }
  __device__ __forceinline__ static bool valid(const Args& A, int grow) {
    const int n = row_sample(grow), tt = row_time(grow);
    return !(grow < kHalo || n >= A.B || tt >= kL);
  }
  __device__ __forceinline__ void load(const Args& A, int row0) {
    const int t = tid(), cw = t % NCW, rin = t / NCW;
    const bool active = rin < RP;
    const Layer& Ly = A.L[l];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int rc = rin + u * RP, grow = row0 + rc;
      const bool ok = active && rc < NR && valid(A, grow);
      r[u] = ok ? gld<bf16x8>(Ly.R + (long long)grow * Cc + cw * 8) : zero8();
      if constexpr (l < 5) d[u] = ok ? gld<bf16x8>(Ly.dY + (long long)grow * Cc + cw * 8) : zero8();
    }
  }
  // dz = relu'(r) * (al * dy + be * r + ga) per element (see stage_dz); rows [kHalo, kHalo + kR) to dZ_l too
  __device__ __forceinline__ void store(const Args& A, char* lds, int row0, const float* gam_rstd, const float* mean,
                                        const float* rstd, const float* mdy, const float* mdyx) const {
    const int t = tid(), cw = t % NCW, rin = t / NCW;
    if (rin >= RP) return;
    const Layer& Ly = A.L[l];
    const int c = cw * 8;
    const int smp0 = (row0 >> 7) * 2;
    float al[8], be[8], ga[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = gam_rstd[c + j], q = rstd[c + j] * mdyx[c + j];
      al[j] = g;
      be[j] = -g * q;
      ga[j] = g * (q * mean[c + j] - mdy[c + j]);
    }
    float dw[8] = {}, dl0 = 0.f, dl1 = 0.f;
    if constexpr (l == 5) {
      const float dsc = A.dropout ? Ly.dsc : 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) dw[j] = A.dense_w[c + j] * dsc;
      dl0 = A.dlogit[min(smp0, A.B - 1)] * (1.0f / kL);
      dl1 = A.dlogit[min(smp0 + 1, A.B - 1)] * (1.0f / kL);
    }
    auto emit = [&](int rc, const bf16x8& rv, const bf16x8& dv) {
      const int grow = row0 + rc;
      bf16x8 o = zero8();
      if (valid(A, grow)) {
        float dy[8];
        if constexpr (l == 5) {
          const float dl = row_sample(grow) != smp0 ? dl1 : dl0;
#pragma unroll
          for (int j = 0; j < 8; ++j) dy[j] = bf_dropped(rv[j]) ? 0.f : dl * dw[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) dy[j] = (float)dv[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float rr = bf_abs(rv[j]);
          const float dz = __builtin_fmaf(al[j], dy[j], __builtin_fmaf(be[j], rr, ga[j]));
          o[j] = (__bf16)(rr > 0.f ? dz : 0.f);
        }
      }
      *reinterpret_cast<bf16x8*>(lds + lds_off(rc, cw * 16, kRS)) = o;
      if (rc >= kHalo && rc < kHalo + kR)
        *reinterpret_cast<bf16x8*>(Ly.dZ + (long long)grow * Cc + c) = o;  // pad rows get their zeros too
    };
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int rc = rin + u * RP;
      if (rc >= NR) continue;
      if constexpr (l < 5)
        emit(rc, r[u], d[u]);
      else
        emit(rc, r[u], r[u]);  // block 6: dY recomputed, no payload
    }
#pragma unroll
    for (int b = NP; b < NK; b += U) {
      bf16x8 qr[U], qd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rc = rin + (b + u) * RP, grow = row0 + rc;
        if (b + u >= NK) continue;
        const bool ok = rc < NR && valid(A, grow);
        qr[u] = ok ? gld<bf16x8>(Ly.R + (long long)grow * Cc + c) : zero8();
        if constexpr (l < 5) qd[u] = ok ? gld<bf16x8>(Ly.dY + (long long)grow * Cc + c) : zero8();
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rc = rin + (b + u) * RP;
        if (b + u >= NK || rc >= NR) continue;
        if constexpr (l < 5)
          emit(rc, qr[u], qd[u]);
        else
          emit(rc, qr[u], qr[u]);
      }
    }
  }
};

template <int l, bool MB>
__global__ __launch_bounds__(kThreads, 2) void dgrad_kernel(Args A_, const Args* __restrict__ Am, RedJob rj) {
  const MbPos pos = mb_pos<MB>();
  const Args& A = member_args<MB>(A_, Am, pos);
  constexpr int CIN = C[l + 1], COUT = C[l];  // conv^T: input = dZ_l channels, output = block l-1 channels
  using T = Tiling<COUT>;
  using CV = Conv<CIN, COUT, KS[l], T::WM, T::WN, false>;
  // LDS: the staged tile + 7 x 256 per-channel floats = 79.25 KiB, so TWO workgroups fit per CU
  // (with the previous 9 x 256 floats it was 81.25 KiB and dgrad ran one workgroup per CU)
  char* act = smem;
  float* prm = reinterpret_cast<float*>(smem + kRows * kRS);
  float* gr = prm;           // gamma*rstd of block l
  float* mean = prm + 256;
  float* rstd = prm + 512;
  float* mdy = prm + 768;
  float* mdyx = prm + 1024;
  float* mean_prev = prm + 1280;  // block l-1 mean / rstd for xhat
  float* rstd_prev = prm + 1536;
  const int ntiles = (A.B + 1) / 2;
  APNEAUQ_DASSERT(blockDim.x == kThreads);
  if (A.tab != nullptr) {  // single-device training: T[l] (block 6: backward sums), T[l-1]
    const int c = threadIdx.x;
    if (c < CIN) {
      gr[c] = tab_row(A, l, kTabS)[c];
      mean[c] = tab_row(A, l, kTabMean)[c];
      rstd[c] = tab_row(A, l, kTabRstd)[c];
      if (l == 5 || A.bwd_self) {  // block 6's backward sums come from the head, no table job in between
        mdy[c] = (float)(slot_sumd(A.L[l].bst + c, 2 * CIN) * (double)A.inv_count);
        mdyx[c] = (float)(slot_sumd(A.L[l].bst + CIN + c, 2 * CIN) * (double)A.inv_count);
      } else {
        mdy[c] = tab_row(A, l, kTabMdy)[c];
        mdyx[c] = tab_row(A, l, kTabMdyx)[c];
      }
    }
    if (c < COUT) {
      mean_prev[c] = tab_row(A, l - 1, kTabMean)[c];
      rstd_prev[c] = tab_row(A, l - 1, kTabRstd)[c];
    }
  } else {
    // one channel per thread (CIN, COUT <= 256 = kThreads): block l's moments and backward sums and
    // block l-1's moments, all 96 slot loads independent (clamped indices, stores predicated)
    static_assert(CIN <= kThreads && COUT <= kThreads, "one channel per thread");
    const Layer& Ly = A.L[l];
    const int c = threadIdx.x, ci = c < CIN ? c : 0, cp = c < COUT ? c : 0;
    float mu, var, mup, varp;
    bn_moments(A, l, 0, ci, mu, var);
    const double b0 = slot_sumd(Ly.bst + ci, 2 * CIN), b1 = slot_sumd(Ly.bst + CIN + ci, 2 * CIN);
    bn_moments(A, l - 1, 0, cp, mup, varp);
    if (c < CIN) {
      const float rs = rsqrtf(var + A.eps);
      mean[c] = mu;
      rstd[c] = rs;
      gr[c] = Ly.gamma[c] * rs;
      mdy[c] = (float)(b0 * (double)A.inv_count);
      mdyx[c] = (float)(b1 * (double)A.inv_count);
    }
    if (c < COUT) {
      mean_prev[c] = mup;
      rstd_prev[c] = rsqrtf(varp + A.eps);
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / T::WN, wn = wave % T::WN;
  const int m = lane & 15, h = lane >> 4;
  const Layer& Lp = A.L[l - 1];
  DzStager<l, DgPF<l>::v> stager;
  if (DgPF<l>::v > 0 && pos.bx < ntiles) stager.load(A, kR * pos.bx);
  // blocks without a prefetch keep one tile per workgroup (a constant one-trip loop: the persistent form
  // keeps more values live and spilled block 4's dgrad)
  constexpr bool PERSIST = DgPF<l>::v > 0;
  for (int tile = pos.bx, it = 0; PERSIST ? tile < ntiles : it < 1; tile += gridDim.x, ++it) {
  const int row0 = kR * tile;
  const int smp0 = 2 * tile;
  stager.store(A, act, row0, gr, mean, rstd, mdy, mdyx);
  __syncthreads();
  // R_{l-1} at this lane's epilogue elements (|R| for xhat, sign = block l-1's dropout mask), loaded
  // before the conv so the MFMAs cover their latency (DgPre: where the registers allow)
  constexpr bool PRE = DgPre<l>::v;
  bf16x4 rpre[PRE ? CV::CT : 1][PRE ? CV::RT : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int c = 0; c < CV::CT; ++c)
#pragma unroll
      for (int r = 0; r < CV::RT; ++r) {
        const int row = wm * CV::RT * 16 + r * 16 + m;
        const bool valid = (row & 63) < kL && (smp0 + (row >> 6)) < A.B;
        const int co0 = (wn * CV::CT + c) * 16 + 4 * h;
        rpre[c][r] = valid ? gld<bf16x4>(Lp.R + (long long)(row0 + kHalo + row) * COUT + co0)
                           : bf16x4{(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
      }
  }
  if constexpr (DgPF<l>::v > 0) {
    if (tile + (int)gridDim.x < ntiles) stager.load(A, kR * (tile + gridDim.x));  // in flight during the conv
  }
  f32x4 acc[CV::CT][CV::RT];
  CV::template run<DgPD<l>::v, false>(A.L[l].wd, act, kRS, acc);  // (B ring at batch 8192: -0.6 %, batch 1024: +-0)
  __syncthreads();
  const float dscp = A.dropout ? Lp.dsc : 1.f;
#pragma unroll
  for (int c = 0; c < CV::CT; ++c) {
    const int co0 = (wn * CV::CT + c) * 16 + 4 * h;
    f32x4 b0 = {}, b1 = {};
#pragma unroll
    for (int r = 0; r < CV::RT; ++r) {
      const int row = wm * CV::RT * 16 + r * 16 + m;
      const int slot = row >> 6, tt = row & 63;
      const bool valid = tt < kL && (smp0 + slot) < A.B;
      // R_{l-1}: |R| for xhat, its sign bit = the dropout mask of block l-1
      bf16x4 rr = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
      if constexpr (PRE)
        rr = rpre[c][r];
      else if (valid)
        rr = gld<bf16x4>(Lp.R + (long long)(row0 + kHalo + row) * COUT + co0);
      f32x4 v = acc[c][r];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (!valid || bf_dropped(rr[i])) ? 0.f : v[i] * dscp;
      bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
      *reinterpret_cast<bf16x4*>(act + row * kRS + co0 * 2) = o;
      if (valid) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float q = (float)o[i];
          const float xh = (bf_abs(rr[i]) - mean_prev[co0 + i]) * rstd_prev[co0 + i];
          b0[i] += q;
          b1[i] += q * xh;
        }
      }
    }
    if (A.det != nullptr) {  // deterministic mode: this wave's row-block partial, reduced in order later
      float* dp = A.det + (long long)(tile * T::WM + wm) * 2 * COUT;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float s0 = group16_sum(b0[i]), s1 = group16_sum(b1[i]);
        if (m == 0) {
          dp[co0 + i] = s0;
          dp[COUT + co0 + i] = s1;
        }
      }
    } else {
      double* bst = Lp.bst + (tile % kStatSlots) * 2 * COUT;
      atomic_channel_sums(bst, co0, b0, m == 0);
      atomic_channel_sums(bst + COUT, co0, b1, m == 0);
    }
  }
  __syncthreads();
  constexpr int CW = COUT / 8;
  for (int i = threadIdx.x; i < kR * CW; i += kThreads) {
    const int r = i / CW, cw = i - r * CW;
    *reinterpret_cast<bf16x8*>(Lp.dY + (long long)(row0 + kHalo + r) * COUT + cw * 8) =
        *reinterpret_cast<const bf16x8*>(act + r * kRS + cw * 16);
  }
  __syncthreads();  // the next tile's staging overwrites act
  }
  // fused step (single device): wgrad<l+1>'s partials, which ran just before this launch, reduced by the
  // workgroups as they finish their tiles -- the separate reduce launch's ramp and drain are gone
  if (rj.part != nullptr) wgrad_reduce_cols(rj, pos.bx, gridDim.x, reinterpret_cast<f32x4*>(smem));
}

// ------------------------------------------------------------------------------------------------
// wgrad of block l: dW_l[tap][ci][co] = sum_rows A_{l-1}[row + tap - pad][ci] * dZ_l[row][co],
// db_l = sum_rows dZ_l.  MFMA: D[co][ci] (16x16 tiles), A-op = dZ^T, B-op = A^shift; both read
// with ds_read_b64_tr_b16 from row-major LDS tiles.  Block 1 stages an im2col (kk = tap*4+ci).
// ------------------------------------------------------------------------------------------------
template <int l> struct WgCfg;
// launch extras of a single-device fused step: the partial region's offset (wgrad<0> writes behind the
// region wgrad<1> leaves for step_reduce_kernel) and the table job (tb.bst == nullptr: none)
struct WgExt {
  long long part_off;
  TabBwd tb;
};
// CI_BLK CO_BLK WCO WCI, RTILES = 128-row tiles summed in registers per workgroup (sized so a
// batch of 1024 gives >= 256 workgroups without multiplying the output atomics needlessly)
// MINWG: the launcher lowers the row tiles per workgroup until at least this many workgroups
// exist (measured at batch 1024: blocks 2-3 prefer fewer, longer workgroups, blocks 4-6 more)
// U: dZ staging loads in flight per thread; MINB: workgroups per CU the register budget targets
// (batch-8192 probes, tools/probes/so_variants.sh: U 4 -> 8 saves 10-13 % on blocks 2, 3, 5; three
// workgroups per CU save 17 % on block 4 and spill on block 6)
// wgrad LDS tiles: the row stride is an odd multiple of 32 B (conflict-free tr_frag reads)
__host__ __device__ constexpr int wg_rs(int width_bytes) { return (width_bytes / 32) % 2 ? width_bytes : width_bytes + 32; }
// MINWG values: batch-1024 step measured with tools/probes/train_variants.sh (block 5 512 -> 768 took
// the step 0.795 -> 0.786 ms, block 2 256 -> 512 0.766-0.775 -> 0.758-0.768 ms, three interleaved rounds;
// round 4, with the straggler-free grouping: block 3 256 -> 512 batch 8192 4.20-4.22 -> 4.13-4.16 ms,
// batch 1024 / 8 members unchanged; block 4 512 -> 1024 slower)
#ifdef APNEAUQ_WG_TABLE  // A/B builds swap the complete table (tools/probes/wg_tables/)
#include APNEAUQ_WG_TABLE
#else
// WAVES: 4 (two workgroups per CU) or 8 (one per CU: the output block over twice the waves, so each
// wave holds half the accumulators and the next row tile's dZ / A rows fit in registers); PF / PFA: those
// rows (dZ / A) are loaded into registers during this tile's MFMAs and written to LDS after them.
// Blocks 2, 3, 5, 6 at 8 waves with both prefetches (tools/probes/wg_tables/w8a.h, profiles/train_step_r5.md):
// batch 1024 0.725 -> 0.687 ms, batch 8192 4.12 -> 3.94 ms, 8 members 4.21 -> 4.07 ms (two rounds each);
// block 4 keeps 4 waves (no 8-way split of its 224 x 96 block), block 1 its im2col.
template <> struct WgCfg<0> { static constexpr int CIB = 32, COB = 128, WCO = 4, WCI = 1, RTILES = 2, MINWG = 512, U = 4, MINB = 2, WAVES = 4; static constexpr bool PF = false, PFA = false; };  // im2col kk=32
template <> struct WgCfg<1> { static constexpr int CIB = 32, COB = 192, WCO = 4, WCI = 2, RTILES = 8, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<2> { static constexpr int CIB = 64, COB = 224, WCO = 2, WCI = 4, RTILES = 8, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<3> { static constexpr int CIB = 32, COB = 96, WCO = 2, WCI = 2, RTILES = 16, MINWG = 512, U = 8, MINB = 2, WAVES = 4; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<4> { static constexpr int CIB = 32, COB = 128, WCO = 4, WCI = 2, RTILES = 16, MINWG = 256, U = 8, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
template <> struct WgCfg<5> { static constexpr int CIB = 64, COB = 96, WCO = 2, WCI = 4, RTILES = 16, MINWG = 256, U = 4, MINB = 1, WAVES = 8; static constexpr bool PF = true, PFA = true; };
#endif


template <int l, bool MB>
__global__ __launch_bounds__(WgCfg<l>::WAVES * 64, WgCfg<l>::MINB) void wgrad_kernel(Args A_, const Args* __restrict__ Am,
                                                                                     WgExt ext) {
  const MbPos pos = mb_pos<MB>();
  const Args& A = member_args<MB>(A_, Am, pos);
  // fused step: the table's backward rows of block l-1 (bst[l-1] is complete: dgrad<l> ran before) for
  // dgrad<l-1> / wgrad<l-1>, the job of the separate reduce launch's extra workgroup
  if (ext.tb.bst != nullptr && blockIdx.x == 0) tab_bwd_rows(ext.tb);
  using W = WgCfg<l>;
  constexpr int NT = W::WAVES * 64;
  constexpr int CIN = C[l], COUT = C[l + 1], K = KS[l], PAD = (K - 1) / 2;
  constexpr bool FIRST = (l == 0);
  constexpr int NTAP = FIRST ? 1 : K;           // block 1: taps folded into the im2col columns
  constexpr int NCO = W::COB / 16 / W::WCO;     // co tiles per wave
  constexpr int NCI = W::CIB / 16 / W::WCI;     // ci tiles per wave
  constexpr int DZRS = wg_rs(W::COB * 2);       // LDS row strides (bytes): odd multiples of 32 B
  constexpr int ARS = wg_rs(FIRST ? 64 : W::CIB * 2);
  static_assert(W::WCO * W::WCI == W::WAVES && (W::WAVES == 4 || !(l == 0)), "one output sub-block per wave");
  static_assert((FIRST || CIN % W::CIB == 0) && COUT % W::COB == 0 && W::CIB % (16 * W::WCI) == 0 &&
                    W::COB % (16 * W::WCO) == 0,
                "wgrad blocks must tile Cin x Cout exactly (e.g. CIB 64 on Cin 224 dropped channels)");
  char* dz_lds = smem;                                   // 128 rows x COB
  char* a_lds = smem + kR * DZRS;                        // 136 rows x CIB (or 128 x 32 im2col)
  float* prm = reinterpret_cast<float*>(a_lds + kRows * ARS);
  float* gr = prm;
  float* mean = prm + 256;
  float* rstd = prm + 512;
  float* mdy = prm + 768;
  float* mdyx = prm + 1024;
  float* sp = prm + 1280;   // block l-1 affine (scale | shift) for staging A_{l-1}
  float* tp = prm + 1536;
  const int nci_blk = FIRST ? 1 : CIN / W::CIB;
  const int nco_blk = COUT / W::COB;
  // XCD-aware remap: hardware dispatch round-robins blockIdx over the 8 XCDs, so the nci*nco
  // workgroups of one row group (which stage the same dZ / A rows) would land on 8 different L2s
  // and each re-read the rows from HBM.  Contiguous logical ids per XCD keep a row group's blocks
  // on one XCD, running together, so its rows come from HBM once (bijective for any grid size).
  // (member-batched: the same remap over the XCDs the member spans)
  const int nwg = gridDim.x, bid = pos.bx, nx = pos.nxcd;
  const int xq = nwg / nx, xr = nwg % nx, xcd = bid % nx;
  const int wg = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + bid / nx;
  const int blk = wg % (nci_blk * nco_blk);
  const int rg = wg / (nci_blk * nco_blk);
  const int ci0 = (blk % nci_blk) * W::CIB, co0 = (blk / nci_blk) * W::COB;
  const bool do_bias = (ci0 == 0);
  if (A.tab != nullptr) {  // single-device training: T[l] (block 6: backward sums), T[l-1]
    const int c = threadIdx.x;
    if (c < COUT) {
      gr[c] = tab_row(A, l, kTabS)[c];
      mean[c] = tab_row(A, l, kTabMean)[c];
      rstd[c] = tab_row(A, l, kTabRstd)[c];
      if (l == 5 || A.bwd_self) {
        mdy[c] = (float)(slot_sumd(A.L[l].bst + c, 2 * COUT) * (double)A.inv_count);
        mdyx[c] = (float)(slot_sumd(A.L[l].bst + COUT + c, 2 * COUT) * (double)A.inv_count);
      } else {
        mdy[c] = tab_row(A, l, kTabMdy)[c];
        mdyx[c] = tab_row(A, l, kTabMdyx)[c];
      }
    }
    if constexpr (!FIRST) {
      if (c < CIN) {
        sp[c] = tab_row(A, l - 1, kTabS)[c];
        tp[c] = tab_row(A, l - 1, kTabT)[c];
      }
    }
  } else {
    // one channel per thread, every slot load independent (see dgrad_kernel's prologue)
    static_assert(COUT <= kThreads && CIN <= kThreads, "one channel per thread");
    const Layer& Ly = A.L[l];
    const int c = threadIdx.x, co = c < COUT ? c : 0, cp = c < CIN ? c : 0;
    float mu, var, mup = 0.f, varp = 0.f;
    bn_moments(A, l, 0, co, mu, var);
    const double b0 = slot_sumd(Ly.bst + co, 2 * COUT), b1 = slot_sumd(Ly.bst + COUT + co, 2 * COUT);
    if constexpr (!FIRST) bn_moments(A, l - 1, 0, cp, mup, varp);
    if (c < COUT) {
      const float rs = rsqrtf(var + A.eps);
      mean[c] = mu;
      rstd[c] = rs;
      gr[c] = Ly.gamma[c] * rs;
      mdy[c] = (float)(b0 * (double)A.inv_count);
      mdyx[c] = (float)(b1 * (double)A.inv_count);
    }
    if constexpr (!FIRST) {
      if (c < CIN) {
        const float sc = A.L[l - 1].gamma[c] * rsqrtf(varp + A.eps);
        sp[c] = sc;
        tp[c] = A.L[l - 1].beta[c] - mup * sc;
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wco = wave % W::WCO, wci = wave / W::WCO;
  // D[ci][co] tiles: A-op = A_shift^T (rows of D = ci), B-op = dZ (cols of D = co); K = tile rows
  f32x4 acc[NTAP][NCI][NCO];
#pragma unroll
  for (int k = 0; k < NTAP; ++k)
#pragma unroll
    for (int b = 0; b < NCI; ++b)
#pragma unroll
      for (int a = 0; a < NCO; ++a) acc[k][b][a] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias gradient on the matrix cores (a column sum of dZ = ones^T dZ): the waves of ci-block 0 with
  // wci == 0 carry NCO extra accumulators.  (Per-element LDS atomics for these sums contended on the
  // same 128-256 addresses and cost 3-4x the whole wgrad.)
  const bool bias_wave = do_bias && wci == 0;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
  f32x4 accb[NCO];
#pragma unroll
  for (int a = 0; a < NCO; ++a) accb[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntiles = (A.B + 1) / 2;
  // row tiles per workgroup: RTILES at large batches, fewer when the batch is small (the launcher
  // sizes the grid for >= ~512 workgroups)
  const int rgs = gridDim.x / (nci_blk * nco_blk);
  const int rt = (ntiles + rgs - 1) / rgs;
  const int tile0 = rg * rt, nt = min(rt, ntiles - tile0);
  // Blocks 4 and 6 (kWgPrefetch, PF below): the next tile's dZ_l and R_{l-1} rows are loaded into registers
  // before this tile's MFMAs and written to LDS (A decoded) after them, so the global-load latency
  // of a tile hides under the previous tile's matrix work instead of being paid between barriers.
  // One stats group (training): A_{l-1} = dropout(BN(R_{l-1})) with the table's single affine.
  // blocks 4 and 6 (dZ only): blocks 2 and 3 have no registers left for it (spills), and block 5
  // loses more from 2 instead of 3 workgroups per CU than the prefetch gains (wgrad<4> 276 -> 333 us
  // at batch 8192; wgrad<3>: 278 -> 243 us; profiles/train_step_r4.md)
  constexpr bool PF = W::PF;
  constexpr bool PFA = W::PFA;  // block 6: dZ only (the A rows would spill)
  constexpr int NCWD = W::COB / 8, ITD = PF ? kR * NCWD / NT : 1;
  constexpr int NCWA = W::CIB / 8, RPA = NT / NCWA, ITA = PFA ? (kRows + RPA - 1) / RPA : 1;
  static_assert(!PF || (kR * NCWD) % NT == 0, "dZ rows split evenly over the threads");
  bf16x8 pd[ITD];
  u32x4 pa[ITA];
  // the thread index is made opaque per call (see staged_loop): otherwise LICM keeps every item's
  // offset live across the tile loop (~100 VGPRs of spills)
  auto opaque_tid = [] {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
  };
  auto pf_load = [&](int tile) {
    const int ptid = opaque_tid(), cwa = ptid % NCWA, rina = ptid / NCWA;
    const int row0 = kR * tile;
    const __bf16* dz = A.L[l].dZ + (long long)(row0 + kHalo) * COUT + co0;
#pragma unroll
    for (int i = 0; i < ITD; ++i) {
      const int idx = ptid + i * NT, rc = idx / NCWD, cw = idx - rc * NCWD;
      pd[i] = gld<bf16x8>(dz + (long long)rc * COUT + cw * 8);
    }
    if constexpr (PFA) {
      const __bf16* R = A.L[l - 1].R + (long long)row0 * CIN + ci0 + cwa * 8;
#pragma unroll
      for (int j = 0; j < ITA; ++j) {
        const int rc = rina + j * RPA;
        if (rc < kRows) pa[j] = gld<u32x4>(R + (long long)rc * CIN);
      }
    }
  };
  auto pf_store = [&]() {
    const int ptid = opaque_tid(), cwa = ptid % NCWA, rina = ptid / NCWA;
#pragma unroll
    for (int i = 0; i < ITD; ++i) {
      const int idx = ptid + i * NT, rc = idx / NCWD, cw = idx - rc * NCWD;
      *reinterpret_cast<bf16x8*>(dz_lds + lds_off(rc, cw * 16, DZRS)) = pd[i];
    }
    if constexpr (PFA) {
      const float dsc = A.dropout != 0 ? A.L[l - 1].dsc : 1.f;
      float s0[8], t0[8];
      lds_row8(sp, ci0 + cwa * 8, dsc, s0);
      lds_row8(tp, ci0 + cwa * 8, dsc, t0);
#pragma unroll
      for (int j = 0; j < ITA; ++j) {
        const int rc = rina + j * RPA;
        if (rc >= kRows) continue;
        u32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = decode_pair(pa[j][q], s0[2 * q], t0[2 * q], s0[2 * q + 1], t0[2 * q + 1]);
        *reinterpret_cast<u32x4*>(a_lds + lds_off(rc, cwa * 16, ARS)) = o;
      }
    }
  };
  if constexpr (PF) {
    if (nt > 0) pf_load(tile0);
  }
  for (int it = 0; it < nt; ++it) {
    const int tile = tile0 + it;
    const int row0 = kR * tile;
    __syncthreads();
    if constexpr (PF) {
      pf_store();
      if constexpr (!PFA) stage_act<l - 1, kRows, W::CIB / 8, 4, NT>(A, a_lds, ARS, row0, ci0, sp, tp, 0);
    } else if constexpr (FIRST) {  // no dgrad for block 1: dZ_1 is recomputed here (a single ci block)
      stage_dz<l, kR, W::COB / 8>(A, dz_lds, DZRS, row0 + kHalo, co0, gr, mean, rstd, mdy, mdyx);
      // im2col of the raw input: col kk = tap*4 + ci (kk < 28), rows = tile rows; one 8-B load per
      // (row, tap) -- the 4 channels of an input row are contiguous
      for (int i = threadIdx.x; i < kR * 8; i += kThreads) {
        const int r = i >> 3, tap = i & 7;
        bf16x4 v = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
        if (tap < K) v = gld<bf16x4>(A.x + (long long)(row0 + kHalo + r + tap - PAD) * 4);
        *reinterpret_cast<bf16x4*>(a_lds + lds_off(r, tap * 8, ARS)) = v;
      }
    } else {
      stage_dz_copy<l, kR, W::COB / 8, W::U, NT>(A, dz_lds, DZRS, row0 + kHalo, co0);
      stage_act<l - 1, kRows, W::CIB / 8, 4, NT>(A, a_lds, ARS, row0, ci0, sp, tp, 0);
    }
    __syncthreads();
    if constexpr (PF) {
      if (it + 1 < nt) pf_load(tile + 1);
    }
#pragma unroll
    for (int ks = 0; ks < kR / 32; ++ks) {
      bf16x8 fb[NCO];
#pragma unroll
      for (int a = 0; a < NCO; ++a) fb[a] = tr_frag(dz_lds, DZRS, ks * 32, (wco * NCO + a) * 16);
      if (bias_wave) {  // db[co] = sum_rows dZ[row][co]: one MFMA with an all-ones A fragment
#pragma unroll
        for (int a = 0; a < NCO; ++a) accb[a] = mfma16(ones, fb[a], accb[a]);
      }
#pragma unroll
      for (int k = 0; k < NTAP; ++k) {
#pragma unroll
        for (int b = 0; b < NCI; ++b) {
          const int arow = FIRST ? ks * 32 : kHalo + ks * 32 + k - PAD;
          const bf16x8 fa = tr_frag(a_lds, ARS, arow, (wci * NCI + b) * 16);
#pragma unroll
          for (int a = 0; a < NCO; ++a) acc[k][b][a] = mfma16(fa, fb[a], acc[k][b][a]);
        }
      }
    }
  }
  // lane (m, h) holds D[ci = 4h + i][co = m] of each tile: 16 consecutive co per row -> 64-B runs
  const int m = lane & 15, h = lane >> 4;
  const Layer& Ly = A.L[l];
  float* part = A.wpart != nullptr ? A.wpart + ext.part_off + (long long)rg * (K * CIN * COUT + COUT) : nullptr;
#pragma unroll
  for (int k = 0; k < NTAP; ++k)
#pragma unroll
    for (int b = 0; b < NCI; ++b)
#pragma unroll
      for (int a = 0; a < NCO; ++a) {
        const int co = co0 + (wco * NCO + a) * 16 + m;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rowi = (wci * NCI + b) * 16 + 4 * h + i;  // ci (or kk for block 1)
          int e;  // element of dW (k, Cin, Cout)
          if constexpr (FIRST) {
            const int tap = rowi >> 2, ci = rowi & 3;
            if (tap >= K) continue;
            e = (tap * CIN + ci) * COUT + co;
          } else {
            e = (k * CIN + ci0 + rowi) * COUT + co;
          }
          if (part != nullptr)
            part[e] = acc[k][b][a][i];  // this row group's exclusive slot: summed in order by wgrad_reduce
          else
            atomicAdd(Ly.gw + e, acc[k][b][a][i]);
        }
      }
  if (bias_wave && h == 0) {  // row 0 of each ones^T dZ tile: lanes 0-15 hold its 16 column sums
#pragma unroll
    for (int a = 0; a < NCO; ++a) {
      const int co = co0 + (wco * NCO + a) * 16 + m;
      if (part != nullptr)
        part[K * CIN * COUT + co] = accb[a][0];
      else
        atomicAdd(Ly.gb + co, accb[a][0]);
    }
  }
}

}  // namespace train

// ------------------------------------------------------------------------------------------------ host
using train::Args;

constexpr int lds_fwd() { return train::kRows * train::kRS + (1024 + 2 * 256) * 4; }  // tile + affine + lstat
constexpr int lds_dgrad() { return train::kRows * train::kRS + 1792 * 4; }
static_assert(2 * lds_dgrad() <= 160 * 1024, "dgrad must fit two workgroups per CU");
template <int l>
constexpr int lds_wgrad() {
  return train::kR * train::wg_rs(train::WgCfg<l>::COB * 2) +
         train::kRows * train::wg_rs(l == 0 ? 64 : train::WgCfg<l>::CIB * 2) + 1792 * 4;
}
template <int l>
constexpr bool wg_lds_fits() {
  return train::WgCfg<l>::WAVES == 8 ? lds_wgrad<l>() <= 160 * 1024 : 2 * lds_wgrad<l>() <= 160 * 1024;
}
static_assert(wg_lds_fits<0>() && wg_lds_fits<1>() && wg_lds_fits<2>() && wg_lds_fits<3>() && wg_lds_fits<4>() &&
                  wg_lds_fits<5>(),
              "wgrad tiles must fit two 4-wave (or one 8-wave) workgroups per CU");

int train_args_size() { return (int)sizeof(Args); }

int train_layer_size() { return (int)sizeof(train::Layer); }

__global__ void bump_counters_kernel(int* c, int n) {
  if (threadIdx.x < n) c[threadIdx.x] += 1;
}

hipError_t train_bump_counters(int* c, int n, hipStream_t st) {
  hipLaunchKernelGGL(bump_counters_kernel, dim3(1), dim3(64), 0, st, c, n);
  return hipGetLastError();
}

// Dropout stream keys of one training step computed on the device from the step counter c[0]
// (keys[l] = stream_key(seed, l, pass_base + c[0])): a graph replay reads no host-written key array.
__global__ void stream_keys_kernel(unsigned* keys, const int* c, int n, unsigned long long seed, unsigned pass_base) {
  if (threadIdx.x < n) keys[threadIdx.x] = stream_key(seed, threadIdx.x, pass_base + (unsigned)c[0]);
}

hipError_t train_stream_keys(unsigned* keys, const int* c, int n, unsigned long long seed, unsigned pass_base,
                             hipStream_t st) {
  hipLaunchKernelGGL(stream_keys_kernel, dim3(1), dim3(64), 0, st, keys, c, n, seed, pass_base);
  return hipGetLastError();
}

static long long det_scratch_base(int B);
// A.det's partial table (n rows of w) -> d, through the fp64 segment scratch behind the table
static hipError_t det_reduce(const Args& A, int n, int w, train::DetDst d, hipStream_t st) {
  if (w > train::kDetMaxW) return hipErrorInvalidValue;
  double* scr = reinterpret_cast<double*>(A.det + det_scratch_base(A.B));
  hipLaunchKernelGGL(train::det_pass1_kernel, dim3((w + 63) / 64, train::kDetSeg), dim3(256), 0, st, A.det, n, w, scr);
  hipLaunchKernelGGL(train::det_pass2_kernel, dim3((w + 255) / 256), dim3(256), 0, st, scr, w, d);
  return hipGetLastError();
}

static train::DetDst det_dst(void* p0, int c0, int f0, void* p1 = nullptr, int c1 = 0, void* p2 = nullptr, int c2 = 0,
                             void* p3 = nullptr, int c3 = 0, int f3 = 0) {
  train::DetDst d;
  d.seg[0] = {p0, c0, f0};
  d.seg[1] = {p1, c1, 0};
  d.seg[2] = {p2, c2, 0};
  d.seg[3] = {p3, c3, f3};
  return d;
}

// Persistent forward: workgroups per CU (2 are resident at a time), each over a contiguous tile range.
// Batch-BN MC Dropout (409,600 tiles per layer launch) measured 8 / 16 / 32 / 64 per CU: MCD phase
// 91.9 / 91.1-91.4 / 91.0-91.4 / 90.5-90.9 ms (tools/probes/so_bench1.sh, one box), and 64 / 128 / 256
// on another: 90.8-90.9 / 91.2-91.8 / 91.9-92.1 ms: shorter ranges
// balance the launch tail.  Batches of <= 16384 tiles (training) get one tile per workgroup anyway.
constexpr int kFwdWgPerCu = 64;
static int fwd_grid(int B) { return std::min((B + 1) / 2, 256 * kFwdWgPerCu); }
// floats of the partial table (fwd / head / dgrad reuse it), then the fp64 scratch of the two-pass reduce
static long long det_scratch_base(int B) {
  const int tiles = (B + 1) / 2;
  const long long t = std::max({(long long)fwd_grid(B) * 2 * 256, (long long)B * train::kHeadRec,
                                (long long)tiles * 2 * 2 * 256});
  return (t + 3) / 4 * 4;  // 16-B aligned scratch
}
int train_det_floats(int B) { return (int)(det_scratch_base(B) + 2LL * train::kDetSeg * train::kDetMaxW); }

// Kernel launches shared by the single-model path (MB = false: by-value Args, Am = nullptr, M = 1)
// and the member-batched path (MB = true: gridDim.z = M members, Args from the device array Am).
template <bool MB>
static hipError_t fwd_launch(const Args& A, const Args* Am, int M, int l, int grid, hipStream_t st, bool pf = false) {
  const dim3 g(grid, 1, M);
  switch (l) {
    case 0: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<0, MB>), g, dim3(256), lds_fwd(), st, A, Am); break;
    case 1:
      if (pf)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<1, MB, true>), g, dim3(256), lds_fwd(), st, A, Am);
      else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<1, MB>), g, dim3(256), lds_fwd(), st, A, Am);
      break;
    case 2: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<2, MB>), g, dim3(256), lds_fwd(), st, A, Am); break;
    case 3:
      if (pf)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<3, MB, true>), g, dim3(256), lds_fwd(), st, A, Am);
      else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<3, MB>), g, dim3(256), lds_fwd(), st, A, Am);
      break;
    case 4: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<4, MB>), g, dim3(256), lds_fwd(), st, A, Am); break;
    case 5: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::fwd_kernel<5, MB>), g, dim3(256), lds_fwd(), st, A, Am); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// the PF forward (FwdPF) for a training launch of M members x B samples: persistent workgroups, only
// when the tiles outnumber kFwdTrainGrid (never in deterministic mode: its moment partials are per
// workgroup of the fwd_grid layout, which the member-batched step must share with the single one)
static bool fwd_pf(const Args& A, int M, int l) {
  const bool has = (l == 1 && train::FwdPF<1>::v > 0) || (l == 3 && train::FwdPF<3>::v > 0);
  return has && A.det == nullptr && A.groups == 1 && !A.shared0 && (long long)((A.B + 1) / 2) * M > train::kFwdTrainGrid;
}

template <bool MB>
static hipError_t dgrad_launch(const Args& A, const Args* Am, int M, int l, hipStream_t st,
                               const train::RedJob& rj = train::RedJob{}) {
  // persistent blocks (DgPF > 0): at most kDgGrid workgroups over all members, each looping over its
  // member's tiles; the others one workgroup per tile
  const int tiles = (A.B + 1) / 2;
  const bool persist = (l == 1 && train::DgPF<1>::v > 0) || (l == 2 && train::DgPF<2>::v > 0) ||
                       (l == 3 && train::DgPF<3>::v > 0) || (l == 4 && train::DgPF<4>::v > 0) ||
                       (l == 5 && train::DgPF<5>::v > 0);
  const dim3 g(persist ? std::max(1, std::min(tiles, train::kDgGrid / std::max(1, M))) : tiles, 1, M);
  switch (l) {
    case 1: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::dgrad_kernel<1, MB>), g, dim3(256), lds_dgrad(), st, A, Am, rj); break;
    case 2: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::dgrad_kernel<2, MB>), g, dim3(256), lds_dgrad(), st, A, Am, rj); break;
    case 3: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::dgrad_kernel<3, MB>), g, dim3(256), lds_dgrad(), st, A, Am, rj); break;
    case 4: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::dgrad_kernel<4, MB>), g, dim3(256), lds_dgrad(), st, A, Am, rj); break;
    case 5: hipLaunchKernelGGL(HIP_KERNEL_NAME(train::dgrad_kernel<5, MB>), g, dim3(256), lds_dgrad(), st, A, Am, rj); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t train_launch_fwd(const Args& A, int l, hipStream_t st) {
  const int grid = fwd_grid(A.B);
  if (A.det != nullptr) {  // deterministic training: single-team kernel, ordered moment reduction
    if (A.groups != 1 || A.shared0) return hipErrorInvalidValue;
    const hipError_t e = fwd_launch<false>(A, nullptr, 1, l, grid, st);
    if (e != hipSuccess) return e;
    const int cc = train::C[l + 1];
    return det_reduce(A, grid, 2 * cc, det_dst(A.L[l].st, 2 * cc, 1), st);
  }
  // persistent forward: each workgroup over a contiguous tile range
  if (fwd_pf(A, 1, l)) return fwd_launch<false>(A, nullptr, 1, l, train::kFwdTrainGrid, st, true);
  return fwd_launch<false>(A, nullptr, 1, l, grid, st);
}

hipError_t train_launch_tab(const Args& A, int mode, int l, hipStream_t st) {
  if (A.tab == nullptr) return hipSuccess;  // no table (multi-rank / deterministic / MC-Dropout ctx)
  if (l < 0 || l >= 6) return hipErrorInvalidValue;
  hipLaunchKernelGGL(train::tab_kernel<false>, dim3(mode == 0 ? 6 : 1), dim3(256), 0, st, A, nullptr, mode, l);
  return hipGetLastError();
}

// training head samples per wave: 1 while that leaves <= 512 workgroups, else up to 4 (batch 8192:
// 512 workgroups instead of 2048, a quarter of the per-workgroup global sums onto the same 16 slots);
// the forward-only head (MC Dropout, no sums) keeps one sample per wave
static int head_spw(int B, int M, int backward) {
  int spw = 1;
  while (backward && spw < 4 && (long long)B * M > 512LL * 4 * spw) spw *= 2;
  return spw;
}

hipError_t train_launch_head(const Args& A, int backward, hipStream_t st, bool with_tab) {
  const int spw = head_spw(A.B, 1, backward);
  const int tabx = (with_tab && A.tab != nullptr) ? 6 : 0;  // + the table's forward rows, one workgroup per block
  hipLaunchKernelGGL(train::head_kernel<false>, dim3((A.B + 4 * spw - 1) / (4 * spw) + tabx), dim3(256),
                     (8 * train::C[6] + 2) * 4, st, A, nullptr, backward, spw, tabx);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess || !backward || A.det == nullptr) return e;
  constexpr int cc = train::C[6];  // per-sample records: loss, dlogit, dW, sum dY, sum dY xhat
  return det_reduce(A, A.B, train::kHeadRec,
                    det_dst(A.loss_sum, 1, 0, A.g_dense_b, 1, A.g_dense_w, cc, A.L[5].bst, 2 * cc, 1), st);
}

static bool fused_ok(const Args& A);
static train::RedJob red_job_rt(const Args& A, int l, const float* part);
// fused (l <= 4): the launch also reduces wgrad<l+1>'s partials, which the previous launch wrote
hipError_t train_launch_dgrad(const Args& A, int l, hipStream_t st, bool fused) {
  if (fused && (!fused_ok(A) || l > 4)) return hipErrorInvalidValue;
  const hipError_t e =
      dgrad_launch<false>(A, nullptr, 1, l, st, fused ? red_job_rt(A, l + 1, A.wpart) : train::RedJob{});
  if (e != hipSuccess || A.det == nullptr) return e;
  const int tiles = (A.B + 1) / 2;
  static constexpr int wm[6] = {0, train::Tiling<train::C[1]>::WM, train::Tiling<train::C[2]>::WM,
                                train::Tiling<train::C[3]>::WM, train::Tiling<train::C[4]>::WM,
                                train::Tiling<train::C[5]>::WM};
  const int cc = train::C[l];  // block l's backward sums (of BN l-1's output) per (tile, wave row block)
  return det_reduce(A, tiles * wm[l], 2 * cc, det_dst(A.L[l - 1].bst, 2 * cc, 1), st);
}

template <int l>
static int wg_rgs(int B, int M = 1) {
  using W = train::WgCfg<l>;
  const int nci = (l == 0) ? 1 : train::C[l] / W::CIB;
  const int nco = train::C[l + 1] / W::COB;
  const int tiles = (B + 1) / 2;
  // ~MINWG workgroups (over all M members of a member-batched launch) while tiles remain, at most RTILES
  // row tiles each up to 2048 samples per launch; beyond, up to 64: fewer row groups, so fewer partial
  // slots to write and reduce (batch 8192: step 4.74 -> 4.52 ms; the small-batch caps were tuned at
  // batch 1024, where block 3 prefers more, shorter workgroups)
  const int nblk = nci * nco;
  const int cap = tiles * M > 1024 ? std::max(W::RTILES, 64) : W::RTILES;
  int rt = std::max(1, std::min(cap, (tiles * M * nblk + W::MINWG - 1) / W::MINWG));
  // no straggler round: rounding the row groups up could leave a few workgroups past MINWG (one
  // CU-slot's worth), which then run as a second round of their own -- block 4 at batch 1024 / 8192:
  // 518 workgroups on 512 slots, 244 us at batch 8192 vs 178 us with 448
  while (rt < cap && (long long)M * nblk * ((tiles + rt - 1) / rt) > W::MINWG) ++rt;
  return (tiles + rt - 1) / rt;
}

template <int l>
static long long wg_part_floats(int B) {
  return (long long)wg_rgs<l>(B) * (train::KS[l] * train::C[l] * train::C[l + 1] + train::C[l + 1]);
}

// The reduction of wgrad<l>'s partials (row grouping of an M-member launch) at part.
template <int l>
static train::RedJob red_job(const Args& A, int M, const float* part) {
  const int rgs = wg_rgs<l>(A.B, M);
  const int kcc = train::KS[l] * train::C[l] * train::C[l + 1];
  const int s4 = (kcc + train::C[l + 1]) / 4;
  // threads per column: enough columns x row-group splits to fill ~1024 workgroups' worth of lanes, at
  // least 8 row groups per thread (one batch of 8 loads in flight).  Block 1 (928 float4 columns, 512
  // row groups at batch 1024): J 16 -> 64, 58 -> 232 workgroups, one load batch per thread instead of 4
  int J = 1;
  while (J < 64 && rgs >= 8 * (2 * J) && (long long)s4 * J < 256LL * 1024) J *= 2;
  const int blocks = std::min(2048, (s4 * J + 255) / 256);
  return {part, A.L[l].gw, A.L[l].gb, rgs, kcc, train::C[l + 1], J, blocks};
}
static train::RedJob red_job_rt(const Args& A, int l, const float* part) {
  switch (l) {
    case 0: return red_job<0>(A, 1, part);
    case 1: return red_job<1>(A, 1, part);
    case 2: return red_job<2>(A, 1, part);
    case 3: return red_job<3>(A, 1, part);
    case 4: return red_job<4>(A, 1, part);
    default: return red_job<5>(A, 1, part);
  }
}
// floats of the partial region wgrad<1..5> share, and of wgrad<0>'s own region behind it (fused step)
static long long wg_main_floats(int B) {
  return std::max({wg_part_floats<1>(B), wg_part_floats<2>(B), wg_part_floats<3>(B), wg_part_floats<4>(B),
                   wg_part_floats<5>(B)});
}

// fused: the single-device step whose reductions run inside other launches (train_launch_dgrad /
// train_launch_finalize with fused set): no reduce launch here; the table job in workgroup 0; wgrad<0>'s
// partials behind the shared region
template <int l, bool MB>
static void wg_launch(const Args& A, const Args* Am, int M, hipStream_t st, bool fused = false) {
  using W = train::WgCfg<l>;
  const int nci = (l == 0) ? 1 : train::C[l] / W::CIB;
  const int nco = train::C[l + 1] / W::COB;
  // deterministic mode: the single-model row grouping (M = 1), so a member-batched step sums every
  // gradient in the same order as the member's own step
  const int rgs = wg_rgs<l>(A.B, A.det != nullptr ? 1 : M);
  // the table's backward rows of block l-1 (bst[l-1] is complete after dgrad<l>, which ran before this
  // wgrad) for dgrad<l-1> / wgrad<l-1>: the reduce launch's extra workgroup, or (fused) wgrad's workgroup 0
  const bool side = A.tab != nullptr && l >= 1 && !A.bwd_self;
  train::TabBwd tb = {};
  if constexpr (l >= 1) {
    if (side) {
      tb.bst = A.L[l - 1].bst;
      tb.cc = train::C[l];
      tb.mdy = A.tab + ((l - 1) * train::kTabRows + train::kTabMdy) * 256;
      tb.mdyx = A.tab + ((l - 1) * train::kTabRows + train::kTabMdyx) * 256;
      tb.inv_count = A.inv_count;
    }
  }
  train::WgExt ext = {};
  if (fused) {
    ext.part_off = (l == 0) ? wg_main_floats(A.B) : 0;
    ext.tb = tb;
  }
  hipLaunchKernelGGL(HIP_KERNEL_NAME(train::wgrad_kernel<l, MB>), dim3(nci * nco * rgs, 1, M), dim3(W::WAVES * 64), lds_wgrad<l>(),
                     st, A, Am, ext);
  if (A.wpart != nullptr && !fused) {
    const train::RedJob rj = red_job<l>(A, A.det != nullptr ? 1 : M, A.wpart);
    const int J = rj.J, blocks = rj.blocks, kcc = rj.kcc;
    if constexpr (MB) {
      hipLaunchKernelGGL(train::wgrad_reduce_mb_kernel, dim3(blocks + (side ? 1 : 0), 1, M), dim3(256), 0, st, Am, l,
                         rgs, kcc, train::C[l + 1], J, side ? 1 : 0);
    } else {
      hipLaunchKernelGGL(train::wgrad_reduce_kernel, dim3(blocks, side ? 2 : 1), dim3(256), 0, st, A.wpart, rgs, kcc,
                         train::C[l + 1], A.L[l].gw, A.L[l].gb, J, tb);
    }
  }
}

// Partial floats a workspace of batch capacity B needs: the shared region plus wgrad<0>'s region of the
// fused step, for EVERY batch n <= B (a partial last batch runs the row grouping of its own size, which
// is not monotone in n: the row-tile cap changes at 2048 samples)
long long train_wgrad_part_floats(int B) {
  long long mx = 0;
  for (int n = 2; n < B + 2; n += 2) {  // the grouping depends on the tile count (n + 1) / 2 only
    const int b = std::min(n, B);
    mx = std::max(mx, wg_main_floats(b) + wg_part_floats<0>(b));
  }
  return mx;
}

template <bool MB>
static hipError_t wgrad_launch(const Args& A, const Args* Am, int M, int l, hipStream_t st, bool fused = false) {
  switch (l) {
    case 0: wg_launch<0, MB>(A, Am, M, st, fused); break;
    case 1: wg_launch<1, MB>(A, Am, M, st, fused); break;
    case 2: wg_launch<2, MB>(A, Am, M, st, fused); break;
    case 3: wg_launch<3, MB>(A, Am, M, st, fused); break;
    case 4: wg_launch<4, MB>(A, Am, M, st, fused); break;
    case 5: wg_launch<5, MB>(A, Am, M, st, fused); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// The fused single-device step (Python: train_ops.FUSED_REDUCE): atomic mode with the parameter table and
// wgrad partials, backward BN rows from the table.
static bool fused_ok(const Args& A) {
  return A.tab != nullptr && A.det == nullptr && A.wpart != nullptr && A.groups == 1 && !A.bwd_self;
}

hipError_t train_launch_wgrad(const Args& A, int l, hipStream_t st, bool fused) {
  if (A.groups != 1) return hipErrorInvalidValue;  // training: one stats group (the staging's single affine)
  if (fused && !fused_ok(A)) return hipErrorInvalidValue;
  return wgrad_launch<false>(A, nullptr, 1, l, st, fused);
}

// fused: BN finalize and the reductions of wgrad<1> / wgrad<0>'s partials in one launch
hipError_t train_launch_finalize(const Args& A, int update_moving, int grads, hipStream_t st, bool fused) {
  if (!fused) {
    hipLaunchKernelGGL(train::bn_finalize_kernel<false>, dim3(6), dim3(256), 0, st, A, nullptr, update_moving, grads);
    return hipGetLastError();
  }
  if (!fused_ok(A)) return hipErrorInvalidValue;
  const train::RedJob j1 = red_job<1>(A, 1, A.wpart), j0 = red_job<0>(A, 1, A.wpart + wg_main_floats(A.B));
  hipLaunchKernelGGL(train::step_reduce_kernel, dim3(6 + j1.blocks + j0.blocks), dim3(256), 0, st, A, j1, j0,
                     update_moving, grads);
  return hipGetLastError();
}

// Member-batched training step ops (one launch for M ensemble members of identical batch size):
// A0 = member 0's Args (host copy: sizes and flags, identical for every member), Am = the device array of
// all M members' Args.  op: 0 fwd(layer) | 1 head(flag = backward) | 2 dgrad(layer) | 3 wgrad(layer)
// | 4 finalize(layer = update_moving, flag = grads) | 5 forward rows of the parameter table.
// Single-device training only (no shared block 1).  Deterministic mode (every member with partial
// tables, A0.det set): each reduction is followed by the two det passes over all members.
static hipError_t det_reduce_mb(const Args& A0, const Args* Am, int M, int op, int l, int n, int w, hipStream_t st) {
  if (w > train::kDetMaxW) return hipErrorInvalidValue;
  const long long sb = det_scratch_base(A0.B);
  hipLaunchKernelGGL(train::det_pass1_mb_kernel, dim3((w + 63) / 64, train::kDetSeg, M), dim3(256), 0, st, Am, n, w, sb);
  hipLaunchKernelGGL(train::det_pass2_mb_kernel, dim3((w + 255) / 256, 1, M), dim3(256), 0, st, Am, op, l, w, sb);
  return hipGetLastError();
}

hipError_t train_launch_mb(const Args& A0, const Args* Am, int M, int op, int layer, int flag, hipStream_t st) {
  if (M < 1 || M > 65535 || Am == nullptr || A0.shared0 || A0.groups != 1) return hipErrorInvalidValue;
  const bool det = A0.det != nullptr;
  if (det && A0.tab != nullptr) return hipErrorInvalidValue;
  switch (op) {
    case 0: {
      if (fwd_pf(A0, M, layer))
        return fwd_launch<true>(A0, Am, M, layer, std::max(1, train::kFwdTrainGrid / M), st, true);
      const hipError_t e = fwd_launch<true>(A0, Am, M, layer, fwd_grid(A0.B), st);
      if (e != hipSuccess || !det) return e;
      return det_reduce_mb(A0, Am, M, 0, layer, fwd_grid(A0.B), 2 * train::C[layer + 1], st);
    }
    case 1: {
      const int spw = head_spw(A0.B, M, flag);
      hipLaunchKernelGGL(train::head_kernel<true>, dim3((A0.B + 4 * spw - 1) / (4 * spw), 1, M), dim3(256),
                         (8 * train::C[6] + 2) * 4, st, A0, Am, flag, spw, 0);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess || !det || !flag) return e;
      return det_reduce_mb(A0, Am, M, 1, 0, A0.B, train::kHeadRec, st);
    }
    case 2: {
      const hipError_t e = dgrad_launch<true>(A0, Am, M, layer, st);
      if (e != hipSuccess || !det) return e;
      static constexpr int wm[6] = {0, train::Tiling<train::C[1]>::WM, train::Tiling<train::C[2]>::WM,
                                    train::Tiling<train::C[3]>::WM, train::Tiling<train::C[4]>::WM,
                                    train::Tiling<train::C[5]>::WM};
      return det_reduce_mb(A0, Am, M, 2, layer, ((A0.B + 1) / 2) * wm[layer], 2 * train::C[layer], st);
    }
    case 3: return wgrad_launch<true>(A0, Am, M, layer, st);
    case 4:
      hipLaunchKernelGGL(train::bn_finalize_kernel<true>, dim3(6, 1, M), dim3(256), 0, st, A0, Am, layer, flag);
      return hipGetLastError();
    case 5:
      if (A0.tab == nullptr) return hipSuccess;
      hipLaunchKernelGGL(train::tab_kernel<true>, dim3(6, 1, M), dim3(256), 0, st, A0, Am, 0, 0);
      return hipGetLastError();
    default: return hipErrorInvalidValue;
  }
}

}  // namespace apneauq
