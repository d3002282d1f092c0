// VALU issue-rate probe (gfx950): cycles per wave-instruction of 32-bit integer ops used by the
// dropout hash, measured with 8 independent chains per lane and 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void probe(unsigned* out, unsigned seed) {
  unsigned x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) x[i] = x[i] * 0x7feb352du;                       // v_mul_lo_u32
      if constexpr (OP == 1) x[i] = __umul24(x[i], 0x7feb35u) ; // v_mul_u32_u24 (signed i24 ok)
      if constexpr (OP == 2) x[i] = x[i] ^ (x[i] >> 15);                      // shift + xor
      if constexpr (OP == 3) x[i] = (unsigned)(((unsigned long long)(x[i] & 0xFFFFFFu) * 0x7feb35ull) >> 32);
      if constexpr (OP == 4) x[i] = x[i] + 0x9e3779b9u;                       // v_add_u32
#if defined(HAVE_PRNG)
      if constexpr (OP == 5) x[i] = __builtin_amdgcn_prng_b32(x[i]);
#endif
      asm volatile("" : "+v"(x[i]));
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
float run(unsigned* d, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  probe<OP><<<blocks, 256>>>(d, 1);
  hipEventRecord(a);
  probe<OP><<<blocks, 256>>>(d, 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  int blocks = 256 * 8;  // 8 WGs x 4 waves per CU = 8 waves per SIMD
  unsigned* d;
  hipMalloc(&d, blocks * 256 * 4);
  const double waves_per_simd = blocks * 4.0 / (256 * 4);
  const double ops = (double)kIters * 8 * waves_per_simd;  // wave-instructions per SIMD (per op kind)
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const char* names[] = {"mul_lo_u32", "mul_u32_u24", "lshr+xor", "mul_hi_u32_u24", "add_u32", "prng_b32"};
  float t[6] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks), 0.f};
#if defined(HAVE_PRNG)
  t[5] = run<5>(d, blocks);
#endif
  for (int i = 0; i < 6; ++i)
    if (t[i] > 0) printf("%-16s %8.3f ms  %6.2f ns per wave-op per SIMD  (%.2f cycles at %.0f MHz)\n", names[i], t[i],
                         t[i] * 1e6 / ops, t[i] * 1e6 / ops * clk_khz / 1e6, clk_khz / 1e3);
  return 0;
}
