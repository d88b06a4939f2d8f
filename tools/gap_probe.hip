// Probe: the gap between dependent kernels on one stream (rocprofv3 --kernel-trace), for the
// BR stream's pattern: a one-workgroup kernel with 150 KB of LDS (the chain) alternating
// with a 150-workgroup kernel (the targets).  Variants: the chain's LDS (150 KB / 16 KB),
// the chain's run time (spin ~100 us / none).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void k_chainlike(float* out, int spin) {
  extern __shared__ float sm[];
  sm[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  float x = sm[(threadIdx.x + 1) & 255];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) x = x * 0.999f + 1.f;
  if (threadIdx.x == 0) out[blockIdx.x] = x;
}
__global__ void k_targetslike(float* out) {
  __shared__ float sw[2400];
  for (int i = threadIdx.x; i < 2400; i += 256) sw[i] = (float)i;
  __syncthreads();
  float acc = 0.f;
  for (int k = 0; k < 64; ++k) acc += sw[(threadIdx.x * 7 + k * 33) % 2400];
  out[1024 + blockIdx.x * 256 + threadIdx.x] = acc;
}
int main(int argc, char** argv) {
  float* out;
  if (hipMalloc(&out, 1 << 22) != hipSuccess) return 1;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  const int lds_big = 150 * 1024, lds_small = 16 * 1024;
  if (hipFuncSetAttribute((const void*)k_chainlike, hipFuncAttributeMaxDynamicSharedMemorySize, lds_big) != hipSuccess) return 1;
  for (int variant = 0; variant < 4; ++variant) {
    const int lds = (variant & 1) ? lds_small : lds_big;
    const int spin = (variant & 2) ? 0 : 10000;          // 100 us at 100 MHz
    for (int it = 0; it < 200; ++it) {
      hipLaunchKernelGGL(k_chainlike, dim3(1), dim3(256), lds, s, out, spin);
      hipLaunchKernelGGL(k_targetslike, dim3(150), dim3(256), 0, s, out);
    }
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    printf("variant %d done (lds %d, spin %d)\n", variant, lds, spin);
  }
  return 0;
}
