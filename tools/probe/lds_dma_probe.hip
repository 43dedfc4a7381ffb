// Probe: does LDS-DMA (buffer_load ... lds / global_load_lds) reach LDS byte offsets >= 64 KiB?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(64) void probe(const uint32_t* src, uint32_t* out, int mode) {
  __shared__ __attribute__((aligned(16))) uint4 smem[9216];  // 144 KiB
  for (int i = threadIdx.x; i < 9216; i += 64) smem[i] = make_uint4(0xdead, 0xdead, 0xdead, 0xdead);
  __syncthreads();
  const int lane = threadIdx.x;
  // write 1 KiB at each of offsets 0, 32K, 64K, 96K, 128K
  for (int k = 0; k < 5; ++k) {
    uint4* dst = smem + k * 2048;  // 32 KiB steps
    if (mode == 0) {
      auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 1 << 20, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16,
                                               (uint32_t)((k * 64 + lane) * 16), 0, 0, 0);
    } else {
      __builtin_amdgcn_global_load_lds((const void*)(src + (k * 64 + lane) * 4),
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  }
  __syncthreads();
  for (int k = 0; k < 5; ++k) out[k * 64 + lane] = smem[k * 2048 + lane].x;
}

int main() {
  uint32_t *src, *out;
  hipMalloc(&src, 1 << 20);
  hipMalloc(&out, 4096);
  uint32_t h[5 * 64 * 4];
  for (int i = 0; i < 5 * 64 * 4; ++i) h[i] = i;
  hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out, mode);
    uint32_t o[320];
    hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
    printf("mode %d (%s):", mode, mode ? "global_load_lds" : "buffer_load lds");
    for (int k = 0; k < 5; ++k) {
      int bad = 0;
      for (int l = 0; l < 64; ++l) bad += o[k * 64 + l] != (uint32_t)((k * 64 + l) * 4);
      printf("  [%d KiB] %s (lane0=%#x)", k * 32, bad ? "WRONG" : "ok", o[k * 64]);
    }
    printf("\n");
  }
  return 0;
}
