// probe: what ds_read_b64_tr_b8 returns per lane (LDS byte i = i & 255 over 512 bytes, lane address lane * 8)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(int* out) {
  __shared__ unsigned char s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = (unsigned char)(i & 255);
  __syncthreads();
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(s + threadIdx.x * 8));
  out[threadIdx.x * 2] = v[0];
  out[threadIdx.x * 2 + 1] = v[1];
}
int main() {
  int* d;
  int h[128];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int b = 0; b < 8; ++b) printf(" %3d", (h[2 * l + b / 4] >> (8 * (b % 4))) & 255);
    printf("\n");
  }
  return 0;
}
