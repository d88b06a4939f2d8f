// Probe: is v_mfma_f32_16x16x4_f32 bitwise a sequential fmaf chain over k (k = 0 first, from
// C)?  If so, the SGD chain's per-sample dh = fma(x2, W2_2, fma(x0, W2_0, x1 * W2_1)) can be one
// MFMA with K slots (x1, x0, x2, 0) and C = -0 (a product keeps its sign of zero).
// Also times a dependent pair of them (latency) on one wave.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_f32_probe.hip -o tools/bin/mfma_f32_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));

// A[16][4], B[4][16], C[16][16] -> D[16][16]; one wave
__global__ void k_probe(const float* A, const float* B, const float* Cm, float* D, long long* cyc) {
  const int l = threadIdx.x, g = l >> 4, c = l & 15;
  const float a = A[c * 4 + g];               // lane (g, c): A[row c][k g]
  const float b = B[g * 16 + c];              //              B[k g][col c]
  floatx4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = Cm[(4 * g + r) * 16 + c];   // D[4g + r][c]
  const long long t0 = clock64();
  floatx4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  floatx4 e = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d, 0, 0, 0);   // dependent
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  const float keep = e[0] + e[1] + e[2] + e[3];
  const long long t1 = clock64();
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + c] = d[r];
  if (l == 0) cyc[0] = t1 - t0 + (keep == 12345.f ? 1 : 0);
}

// v_mfma_f32_4x4x1_16b_f32: 16 blocks of 4 lanes; lane l supplies a = A[l], b = B[l]; expected
// D[l][r] = fma(A[4 (l / 4) + r], B[l], C[l][r]) (block l / 4: row r, column l % 4).  Then a
// chain of three (the dh form), and the ds_swizzle bitmask pattern and 0x13 / or 4 that moves
// lane 16 g' + (c & 3) (+ 4) to lane 16 g' + c.
__global__ void k_probe4(const float* A, const float* B, const float* Cm, float* D, int* sw, long long* cyc) {
  const int l = threadIdx.x;
  floatx4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = Cm[l * 4 + r];
  const long long t0 = clock64();
  floatx4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], acc, 0, 0, 0);
  floatx4 e = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], d, 0, 0, 0);
  e = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], e, 0, 0, 0);
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  const float keep = e[0] + e[1] + e[2] + e[3];
  const long long t1 = clock64();
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = d[r];
  sw[l] = __builtin_amdgcn_ds_swizzle(l, 0x13);
  sw[64 + l] = __builtin_amdgcn_ds_swizzle(l, 0x13 | (4 << 5));
  if (l == 0) cyc[0] = t1 - t0 + (keep == 12345.f ? 1 : 0);
}

static float rnd(std::mt19937& g, int mode) {
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  switch (mode) {
    case 0: return u(g);
    case 1: return u(g) * std::ldexp(1.f, (int)(g() % 40) - 20);
    case 2: { int k = g() % 6; return k == 0 ? 0.f : k == 1 ? -0.f : u(g) * 1e-3f; }
    default: return std::ldexp(u(g), (int)(g() % 200) - 100);
  }
}

int main() {
  float *A, *B, *Cm, *D;
  long long* cyc;
  hipMalloc(&A, 64 * 4); hipMalloc(&B, 64 * 4); hipMalloc(&Cm, 256 * 4); hipMalloc(&D, 256 * 4);
  hipMalloc(&cyc, 8);
  std::mt19937 gen(7);
  std::vector<float> a(64), b(64), c(256), d(256);
  long long mism[6] = {0, 0, 0, 0, 0, 0}, total = 0, lat = 0;
  const int orders[6][4] = {{0, 1, 2, 3}, {3, 2, 1, 0}, {1, 0, 3, 2}, {0, 2, 1, 3}, {2, 3, 0, 1}, {0, 1, 3, 2}};
  for (int it = 0; it < 4000; ++it) {
    const int mode = it % 4;
    for (auto& x : a) x = rnd(gen, mode);
    for (auto& x : b) x = rnd(gen, mode);
    for (auto& x : c) x = (it % 3 == 0) ? -0.f : rnd(gen, mode);
    hipMemcpy(A, a.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(B, b.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(Cm, c.data(), 1024, hipMemcpyHostToDevice);
    k_probe<<<1, 64>>>(A, B, Cm, D, cyc);
    hipMemcpy(d.data(), D, 1024, hipMemcpyDeviceToHost);
    long long cy;
    hipMemcpy(&cy, cyc, 8, hipMemcpyDeviceToHost);
    lat += cy;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        ++total;
        for (int o = 0; o < 6; ++o) {
          float acc = c[i * 16 + j];
          for (int q = 0; q < 4; ++q) {
            const int k = orders[o][q];
            acc = std::fmaf(a[i * 4 + k], b[k * 16 + j], acc);
          }
          uint32_t x, y;
          std::memcpy(&x, &acc, 4);
          std::memcpy(&y, &d[i * 16 + j], 4);
          if (x != y) ++mism[o];
        }
      }
  }
  // 4x4x1
  int* SW;
  hipMalloc(&SW, 128 * 4);
  long long m4 = 0, m4t = 0, t4 = 0, lat4 = 0;
  std::vector<float> a4(64), b4(64), c4(256), d4(256);
  for (int it = 0; it < 2000; ++it) {
    const int mode = it % 4;
    for (auto& x : a4) x = rnd(gen, mode);
    for (auto& x : b4) x = rnd(gen, mode);
    for (auto& x : c4) x = (it % 3 == 0) ? -0.f : rnd(gen, mode);
    hipMemcpy(A, a4.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(B, b4.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(Cm, c4.data(), 1024, hipMemcpyHostToDevice);
    k_probe4<<<1, 64>>>(A, B, Cm, D, SW, cyc);
    hipMemcpy(d4.data(), D, 1024, hipMemcpyDeviceToHost);
    long long cy;
    hipMemcpy(&cy, cyc, 8, hipMemcpyDeviceToHost);
    lat4 += cy;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        ++t4;
        const float x = std::fmaf(a4[4 * (l / 4) + r], b4[l], c4[l * 4 + r]);     // row r, col l % 4
        const float y = std::fmaf(a4[l], b4[4 * (l / 4) + r], c4[l * 4 + r]);     // transposed
        uint32_t u, v, w;
        std::memcpy(&u, &x, 4); std::memcpy(&v, &y, 4); std::memcpy(&w, &d4[l * 4 + r], 4);
        if (u != w) ++m4;
        if (v != w) ++m4t;
      }
  }
  int sw[128];
  hipMemcpy(sw, SW, 512, hipMemcpyDeviceToHost);
  int swbad = 0;
  for (int l = 0; l < 64; ++l) {
    const int base = (l & ~31) | (l & 16);
    if (sw[l] != (base | (l & 3))) ++swbad;
    if (sw[64 + l] != (base | 4 | (l & 3))) ++swbad;
  }
  printf("4x4x1 f32: %lld elements, mismatches vs fmaf(A[blk row r], B[lane], C) %lld, transposed %lld; "
         "3 dependent + 16 nop states: %.1f cycles; swizzle mismatches %d\n", t4, m4, m4t, (double)lat4 / 2000, swbad);
  printf("elements %lld; bitwise mismatches vs fmaf chains in k order 0123 %lld, 3210 %lld, 1032 %lld, "
         "0213 %lld, 2301 %lld, 0132 %lld\n", total, mism[0], mism[1], mism[2], mism[3], mism[4], mism[5]);
  printf("two dependent 16x16x4 f32 MFMAs + 36 nop states + 4 adds: %.1f cycles (clock64) on average\n",
         (double)lat / 4000);
  return 0;
}
