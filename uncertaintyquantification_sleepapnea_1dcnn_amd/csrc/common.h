// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of apneauq.
//
// Written directly against CDNA4: 64-lane wavefronts, bf16 MFMA (v_mfma_f32_16x16x32_bf16),
// 160 KiB LDS per CU.  No CUDA shims, no dual-platform paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Bounds-checked debug builds (APNEAUQ_DEBUG=1, see build.py): device asserts on the launch
// geometry and index invariants every kernel relies on.  Compiled out otherwise.
#ifdef APNEAUQ_DEBUG
#include <cassert>
#define APNEAUQ_DASSERT(x) assert(x)
#else
#define APNEAUQ_DASSERT(x) ((void)0)
#endif

namespace apneauq {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Explicit global-address-space views (keep loads as global_load_*, never flat_*).
typedef __attribute__((address_space(1))) const bf16x8 gbf16x8;
typedef __attribute__((address_space(1))) const f32x4 gf32x4;
typedef __attribute__((address_space(1))) const float gfloat;
typedef __attribute__((address_space(1))) const uint8_t guint8;

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------------
// Counter-based dropout RNG -- bit-identical to ops/rng.py (see its docstring for the definition)
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ uint32_t stream_key(uint64_t seed, uint32_t layer, uint32_t pass) {
  uint32_t k = mix32((uint32_t)(seed & 0xFFFFFFFFu) ^ 0x68BC21EBu);
  k = mix32(k ^ (uint32_t)(seed >> 32));
  k = mix32(k ^ (layer * 0x9E3779B9u));
  k = mix32(k ^ pass);
  return k;
}

__host__ __device__ __forceinline__ uint32_t sample_key(uint32_t skey, uint32_t sample) {
  return mix32(skey ^ mix32(sample + 0x2545F491u));
}

// 16-bit uniforms of channels (c, c+1), c even, at time step t.
__device__ __forceinline__ uint32_t dropout_bits2(uint32_t skey, uint32_t t, uint32_t c_even) {
  return mix32(skey ^ ((t << 9) | (c_even >> 1)));
}

// Dropout decisions of a dropout_bits2 pair as bf16 sign bits: bit 15 set iff the low 16-bit uniform
// is < thr, bit 31 iff the high one is (thr2 = thr * 0x10001).  Three packed VALU ops:
// sat(thr - u) is nonzero iff u < thr, and sat(that + 0x7FFF) then has its top bit set.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t drop_signs2(uint32_t h, uint32_t thr2) {
  const u16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, thr2), __builtin_bit_cast(u16x2, h));
  const u16x2 t = __builtin_elementwise_add_sat(d, (u16x2){0x7FFF, 0x7FFF});
  return __builtin_bit_cast(uint32_t, t) & 0x80008000u;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Sum over the 16 lanes of a 16-lane group (lanes sharing lane>>4 = one DPP row), every lane gets
// the sum: two quad permutes and two row rotations as v_add_f32_dpp on the VALU.  (__shfl_xor lowers
// to ds_swizzle / ds_bpermute: four dependent LDS round trips per sum; the x3 batch-BN MC Dropout
// epilogues ran 2.3 % faster with DPP, profiles/x3_epilogue_ab_r3.md.)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float group16_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x124>(v);  // row_ror 4
  v += dpp_mov<0x128>(v);  // row_ror 8
  return v;
}

// Max over the 16 lanes of a 16-lane group, every lane gets it (DPP as group16_sum).
__device__ __forceinline__ float group16_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x124>(v));
  v = fmaxf(v, dpp_mov<0x128>(v));
  return v;
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

}  // namespace apneauq
