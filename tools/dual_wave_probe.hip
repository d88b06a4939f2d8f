// Probe: VALU issue rate of one wave per SIMD against two waves per SIMD (one workgroup on one
// CU, 4 or 8 waves).  Each wave runs `iters` x 16 independent instructions of one kind (asm,
// 8 registers, no dependences inside a group of 8); the kernel reports shader cycles per
// instruction per wave (s_memtime around the loop, wave 0) -- if two waves on a SIMD each keep
// the one-wave rate, the SIMD's VALU capacity is not what bounds a one-wave-per-SIMD chain.
//   hipcc --offload-arch=gfx950 -O3 tools/dual_wave_probe.hip -o tools/bin/dual_wave_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define BODY8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)

template <int KIND>
__global__ void __launch_bounds__(512) k_probe(int iters, float seed, unsigned long long* out, float* sink) {
  float r0 = seed + threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
        r6 = r0 + 6, r7 = r0 + 7;
  const float a = seed * 0.5f, b = seed * 0.25f;
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i) {
#define R(k) r##k
    if constexpr (KIND == 0) {   // v_fma_f32
#define I(k) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(R(k)) : "v"(a), "v"(b));
      BODY8(I) BODY8(I)
#undef I
    } else if constexpr (KIND == 1) {   // v_dot2_f32_bf16
#define I(k) asm volatile("v_dot2_f32_bf16 %0, %1, %2, %0" : "+v"(R(k)) : "v"(a), "v"(b));
      BODY8(I) BODY8(I)
#undef I
    } else if constexpr (KIND == 2) {   // v_cvt_pk_bf16_f32
#define I(k) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "+v"(R(k)) : "v"(a), "v"(b));
      BODY8(I) BODY8(I)
#undef I
    } else if constexpr (KIND == 3) {   // v_fmac_f32_dpp row_newbcast
#define I(k) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(R(k)) : "v"(a), "v"(b));
      BODY8(I) BODY8(I)
#undef I
    } else if constexpr (KIND == 4) {   // v_pk_fma_f32 (two values per instruction)
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 p0 = {r0, r1}, p1 = {r2, r3}, p2 = {r4, r5}, p3 = {r6, r7};
      const f2 A = {a, b};
#define I(k) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(p##k) : "v"(A));
      I(0) I(1) I(2) I(3) I(0) I(1) I(2) I(3) I(0) I(1) I(2) I(3) I(0) I(1) I(2) I(3)
#undef I
      r0 = p0.x + p1.x + p2.x + p3.x;
      r1 = p0.y + p1.y + p2.y + p3.y;
    } else if constexpr (KIND == 5) {   // v_permlane32_swap (pairs)
#define I(k) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(r0), "+v"(r1)); \
             asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(r2), "+v"(r3));
      BODY8(I)
#undef I
    } else {                            // v_add_f32_dpp row_ror:8 (the tot32 sums)
#define I(k) asm volatile("v_add_f32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(R(k)) : "v"(a));
      BODY8(I) BODY8(I)
#undef I
    }
#undef R
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if ((threadIdx.x & 63) == 0) out[threadIdx.x >> 6] = t1 - t0;
  sink[threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}

int main() {
  unsigned long long* out;
  float* sink;
  hipMalloc(&out, 8 * 8);
  hipMalloc(&sink, 512 * 4);
  const char* names[] = {"v_fma_f32", "v_dot2_f32_bf16", "v_cvt_pk_bf16_f32", "v_fmac_f32_dpp",
                         "v_pk_fma_f32", "v_permlane32_swap", "v_add_f32_dpp"};
  const int iters = 4000;
  for (int kind = 0; kind < 7; ++kind) {
    for (int threads : {256, 512}) {
      auto run = [&]() {
        switch (kind) {
          case 0: k_probe<0><<<1, threads>>>(iters, 1.f, out, sink); break;
          case 1: k_probe<1><<<1, threads>>>(iters, 1.f, out, sink); break;
          case 2: k_probe<2><<<1, threads>>>(iters, 1.f, out, sink); break;
          case 3: k_probe<3><<<1, threads>>>(iters, 1.f, out, sink); break;
          case 4: k_probe<4><<<1, threads>>>(iters, 1.f, out, sink); break;
          case 5: k_probe<5><<<1, threads>>>(iters, 1.f, out, sink); break;
          default: k_probe<6><<<1, threads>>>(iters, 1.f, out, sink); break;
        }
      };
      run();
      hipDeviceSynchronize();
      run();
      hipDeviceSynchronize();
      unsigned long long c[8] = {};
      hipMemcpy(c, out, 8 * 8, hipMemcpyDeviceToHost);
      double mx = 0;
      for (int w = 0; w < threads / 64; ++w) mx = c[w] > mx ? c[w] : mx;
      printf("%-20s waves/SIMD %d: %.2f cycles per instruction per wave (slowest wave)\n", names[kind],
             threads / 256, mx / (iters * 16.0));
    }
  }
  return 0;
}
