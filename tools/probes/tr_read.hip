// Probe of ds_read_b64_tr_b16 semantics on gfx950: LDS holds a 16x32 tile of
// 16-bit values v = row*100 + col; each lane supplies &tile[q][4p] (+ group
// offsets) and we print what it receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ short t[16][32];
  for (int i = threadIdx.x; i < 16 * 32; i += 64) t[i / 32][i % 32] = (i / 32) * 100 + (i % 32);
  __syncthreads();
  const int g = threadIdx.x / 16, j = threadIdx.x % 16, q = j / 4, p = j % 4;
  // group g: rows 4*(g/2).. , columns 16*(g%2)..
  const short* a = &t[4 * (g / 2) + q][16 * (g % 2) + 4 * p];
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a));
  for (int e = 0; e < 4; ++e) out[threadIdx.x * 4 + e] = v[e];
}
int main() {
  short* d;
  hipMalloc(&d, 64 * 4 * 2);
  k<<<1, 64>>>(d);
  short h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  return 0;
}
