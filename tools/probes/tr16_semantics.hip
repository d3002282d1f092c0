#include <hip/hip_runtime.h>
typedef short v4i16 __attribute__((ext_vector_type(4)));
// verify tr16 semantics: lds holds [row][16 cols] of value row*100+col
__global__ void k(v4i16* out) {
  __shared__ short lds[64*16];
  for (int i = threadIdx.x; i < 64*16; i += 64) lds[i] = (i/16)*100 + (i%16);
  __syncthreads();
  int lane = threadIdx.x, g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  // group g reads rows [4g, 4g+4)
  const short* a = lds + (4*g + q) * 16 + 4*p;
  out[lane] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a);
}
int main() {
  v4i16* d; hipMalloc(&d, 64*8); hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
  v4i16 h[64]; hipMemcpy(h, d, 64*8, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 5) printf("lane %d: %d %d %d %d\n", l, h[l][0], h[l][1], h[l][2], h[l][3]);
  return 0;
}
