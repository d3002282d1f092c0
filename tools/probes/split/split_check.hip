// Bit-identity check of the fp16 hi/lo split: plain C (cvt, cvt back, sub, cvt) vs v_cvt_pk_f16_f32 +
// v_fma_mix{lo,hi}_f16 (tools/probes/split; run on the GPU box: hipcc -O3 --offload-arch=gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* a, unsigned* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const float a0 = a[2 * i], a1 = a[2 * i + 1];
  _Float16 h0 = (_Float16)a0, h1 = (_Float16)a1;
  _Float16 l0 = (_Float16)(a0 - (float)h0), l1 = (_Float16)(a1 - (float)h1);
  f16x2 hp = (f16x2){(_Float16)a0, (_Float16)a1};
  unsigned u = __builtin_bit_cast(unsigned, hp), l;
  asm volatile("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(u), "v"(a0));
  asm volatile("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(u), "v"(a1));
  const unsigned ref_h = __builtin_bit_cast(unsigned, (f16x2){h0, h1});
  const unsigned ref_l = __builtin_bit_cast(unsigned, (f16x2){l0, l1});
  out[i] = (ref_h != u) | ((ref_l != l) << 1);
}
int main() {
  const int n = 1 << 24;
  float* h = (float*)malloc(n * 4);
  unsigned s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    unsigned bits = s;
    if (i % 4 == 0) bits = (bits & 0x807FFFFFu) | ((100u + (bits >> 24) % 60u) << 23);  // |v| in [2^-27, 2^33)
    float v;
    memcpy(&v, &bits, 4);
    if (!(v == v) || __builtin_isinf(v)) v = 1.f;
    h[i] = (i % 4 == 1) ? (float)(s % 20000) - 10000.f + (float)(s >> 20) * 1e-4f : v;
  }
  float* d;
  unsigned* o;
  hipMalloc(&d, n * 4);
  hipMalloc(&o, n * 2);
  hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 2 / 256), dim3(256), 0, 0, d, o, n);
  unsigned* r = (unsigned*)malloc(n * 2);
  hipMemcpy(r, o, n * 2, hipMemcpyDeviceToHost);
  long bad_h = 0, bad_l = 0;
  for (int i = 0; i < n / 2; ++i) {
    bad_h += r[i] & 1;
    bad_l += (r[i] >> 1) & 1;
  }
  printf("pairs %d  hi mismatches %ld  lo mismatches %ld\n", n / 2, bad_h, bad_l);
  return (bad_h || bad_l) ? 1 : 0;
}
