// Probe: does hipExtLaunchKernel(..., hipExtAnyOrderLaunch) let a kernel start before the
// previous kernel on the same stream completes?  k_wait (launched first) polls a flag that
// k_set (launched second, any-order) raises.  Any-order honoured: k_wait ends within micro-
// seconds; ignored: k_wait gives up after its bounded spin (0.2 s) and k_set runs after it.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
typedef __attribute__((address_space(1))) unsigned gu32;
__global__ void k_wait(unsigned* flag, unsigned long long* out) {
  if (threadIdx.x) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (__hip_atomic_load((gu32*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
    __builtin_amdgcn_s_sleep(2);
    t = __builtin_amdgcn_s_memrealtime();
    if (t - t0 > 20000000ull) break;     // 0.2 s at 100 MHz
  }
  out[0] = t - t0;
}
__global__ void k_set(unsigned* flag) {
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
int main() {
  unsigned* flag; unsigned long long* out;
  hipMalloc(&flag, 4); hipMalloc(&out, 8);
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int mode = 0; mode < 2; ++mode) {
    hipMemset(flag, 0, 4); hipMemset(out, 0, 8); hipDeviceSynchronize();
    hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, flag, out);
    void* args[] = {&flag};
    hipError_t e = hipExtLaunchKernel((const void*)k_set, dim3(1), dim3(64), args, 0, s, nullptr, nullptr,
                                      mode ? hipExtAnyOrderLaunch : 0);
    hipStreamSynchronize(s);
    unsigned long long h = 0; hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    printf("mode %s: launch %s, k_wait spun %.3f ms\n", mode ? "any-order" : "ordered", hipGetErrorString(e), h / 1e5);
  }
  return 0;
}
