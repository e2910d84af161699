// Semantics probe of ds_read_b64_tr_b16 (gfx950): LDS holds a [16 rows][64 cols]
// u16 image with value row*64+col; lane 4q+p of each 16-lane group g supplies
// the address of row 4g+q, columns 4p..4p+3 (+ a per-group column offset
// 16g).  Prints what each lane receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short v4i16 __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ short lds[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = i;
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int row = 4 * g + q, col = 16 * g + 4 * p;
  v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(lds + row * 64 + col));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}
int main() {
  short* d;
  hipMalloc(&d, 256 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256];
  hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int lane = 0; lane < 64; ++lane) {
    const int g = lane >> 4, i = lane & 15;
    printf("lane %2d:", lane);
    for (int e = 0; e < 4; ++e) {
      printf(" (%d,%d)", h[lane * 4 + e] / 64, h[lane * 4 + e] % 64);
      // expectation from the guide: lane i of group g gets column 16g+i of rows 4g..4g+3
      if (h[lane * 4 + e] != (4 * g + e) * 64 + 16 * g + i) ++bad;
    }
    printf("\n");
  }
  printf("mismatches vs expectation: %d\n", bad);
  return 0;
}
