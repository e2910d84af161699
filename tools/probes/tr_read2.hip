// ds_read_b64_tr_b16 with the attention tile layout: [32][72] bf16-sized cells,
// value = row*100 + col; lane address = &t[4hf + (j>>2)][16gh + 4(j&3)].
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out, int variant) {
  __shared__ __attribute__((aligned(16))) short t[32][72];
  for (int i = threadIdx.x; i < 32 * 72; i += 64) t[i / 72][i % 72] = (i / 72) * 100 + (i % 72);
  __syncthreads();
  const int lane = threadIdx.x, j = lane & 15, hf = lane >> 5, gh = (lane >> 4) & 1;
  const short* a = &t[4 * hf + (j >> 2)][16 * gh + 4 * (j & 3)];
  typedef __attribute__((address_space(3))) s4 ls4;
  s4 v;
  if (variant == 0) {
    v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls4*)(a));
  } else {
    // explicit LDS offset arithmetic instead of a flat->LDS pointer cast
    const unsigned off = ((4 * hf + (j >> 2)) * 72 + 16 * gh + 4 * (j & 3)) * 2;
    v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls4*)((__attribute__((address_space(3))) char*)(t) + off));
  }
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}
int main() {
  short* d;
  (void)hipMalloc(&d, 64 * 4 * 2);
  short h[256];
  for (int variant = 0; variant < 2; ++variant) {
    k<<<1, 64>>>(d, variant);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("variant %d\n", variant);
    for (int l = 0; l < 64; l += 1) printf("lane %2d: %5d %5d %5d %5d\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  }
  return 0;
}
