// Microbenchmark of the learner's SGD chain kernels (k_chain, k_chain2, k_chain3) on synthetic minibatch
// rows: microseconds per SGD step, and with -DNFSP_CHAIN_STAMPS the per-phase cycle
// split of wave 0..3 (s_memtime).  Not part of libnfsp.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -I<pkg>/csrc tools/bench_chain.hip
#include <stdio.h>
#include <stdlib.h>
#include <math.h>

#include <random>
#include <vector>

#include "../neural-ficititious-self-play-in-imperfect-information-games_amd/csrc/learner.hip"

// the host helpers learner.hip's nfsp_engine_update references (unused here)
namespace nfsp {
int fail(int code, const std::string&) { return code; }
int hip_fail(hipError_t, const char*) { return NFSP_EHIP; }
namespace eng {
hipEvent_t take_event(nfsp_engine*) { return nullptr; }
}
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int U = argc > 1 ? atoi(argv[1]) : 200;
  const int relu = argc > 2 ? atoi(argv[2]) : 1;
  const int B = 128, E = 2;
  std::mt19937 rng(7);
  std::vector<FitRow> fit((size_t)U * E * B);
  for (auto& r : fit) {
    uint32_t x = 1u << (24 + rng() % 3);
    for (int k = 0; k < 6; ++k) if (rng() & 1) x |= 1u << (rng() % 24);
    r.x = x;
    r.t0 = (rng() % 1000) / 500.f; r.t1 = (rng() % 1000) / 500.f; r.t2 = (rng() % 1000) / 500.f;
  }
  std::vector<float> w(nn::NP);
  // continuous weights: a grid of values makes exact-zero ReLU inputs likely, where the
  // derivative flips with the summation order
  std::uniform_real_distribution<float> ud(-0.2f, 0.2f);
  for (auto& v : w) v = ud(rng);
  // bit-transposed minibatch masks (the prep kernels' xt) and the per-update BR lr table
  std::vector<uint32_t> xt(fit.size(), 0);
  for (size_t blk = 0; blk < fit.size() / 32; ++blk)
    for (int k = 0; k < 32; ++k)
      for (int i = 0; i < 30; ++i)
        if ((fit[blk * 32 + k].x >> i) & 1u) xt[blk * 32 + i] |= 1u << k;
  std::vector<float> lrt(U);
  for (int u = 0; u < U; ++u) lrt[u] = (float)(0.05 / (1.0 + 0.003 * sqrt((double)(2 * u))));
  uint32_t* dxt; float* dlr;
  CK(hipMalloc(&dxt, xt.size() * 4));
  CK(hipMalloc(&dlr, lrt.size() * 4));
  CK(hipMemcpy(dxt, xt.data(), xt.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlr, lrt.data(), lrt.size() * 4, hipMemcpyHostToDevice));
  FitRow* dfit; float* dw; unsigned long long* dst;
  CK(hipMalloc(&dfit, fit.size() * sizeof(FitRow)));
  CK(hipMalloc(&dw, w.size() * 4));
  CK(hipMalloc(&dst, 80 * 8));
  CK(hipMemset(dst, 0, 80 * 8));
  CK(hipMemcpy(dfit, fit.data(), fit.size() * sizeof(FitRow), hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  ChainArgs C{};
  C.w[0] = dw; C.sync_to[0] = nullptr; C.fit = dfit; C.active = nullptr; C.umax = U;
  C.u0[0] = 0; C.u1[0] = U; C.agents[0] = 0; C.B = B; C.E = E; C.relu = relu;
  C.lr_fixed = 0.1f; C.lr0 = 0.05; C.it0[0] = 0; C.stamps = dst;
  C.xt = dxt; C.lr_tab = dlr;
  const int variant = argc > 3 ? atoi(argv[3]) : 2;
  if (variant == 0) {   // agreement: k_chain2 (f32 MFMA) vs k_chain3 (split bf16 MFMA)
    std::vector<float> out[2];
    for (int k = 0; k < 2; ++k) {
      CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
      if (k == 0 && relu) k_chain2<1><<<1, 256, sizeof(Chain2Smem)>>>(C);
      else if (k == 0) k_chain2<0><<<1, 256, sizeof(Chain2Smem)>>>(C);
      else if (relu) k_chain3<1><<<1, 256, sizeof(Chain3Smem)>>>(C);
      else k_chain3<0><<<1, 256, sizeof(Chain3Smem)>>>(C);
      CK(hipDeviceSynchronize());
      out[k].resize(nn::NP);
      CK(hipMemcpy(out[k].data(), dw, nn::NP * 4, hipMemcpyDeviceToHost));
    }
    double md = 0, mc = 0, ma = 0;
    int at = -1;
    for (int i = 0; i < nn::NP; ++i) {
      const double d = fabs((double)out[0][i] - out[1][i]);
      if (d > md) { md = d; at = i; }
      mc = fmax(mc, fabs((double)out[1][i] - w[i]));
      ma = fmax(ma, fabs((double)out[1][i]));
    }
    printf("compare relu=%d updates=%d: max|chain2 - chain3| = %.3g at %d (max |change| %.3g, max |w| %.3g)\n",
           relu, U, md, at, mc, ma);
    return md <= 1e-5 * (1.0 + U) ? 0 : 3;
  }
  CK(hipFuncSetAttribute((const void*)k_chain, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ChainSmem)));
  auto launch = [&]() {
    if (variant == 3 && relu) k_chain3<1><<<1, 256, sizeof(Chain3Smem)>>>(C);
    else if (variant == 3) k_chain3<0><<<1, 256, sizeof(Chain3Smem)>>>(C);
    else if (variant == 2 && relu) k_chain2<1><<<1, 256, sizeof(Chain2Smem)>>>(C);
    else if (variant == 2) k_chain2<0><<<1, 256, sizeof(Chain2Smem)>>>(C);
    else k_chain<<<1, 256, sizeof(ChainSmem)>>>(C);
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  launch();   // warm
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dst, 0, 80 * 8));
  CK(hipEventRecord(a));
  launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  const int steps = U * E * (B / 32);
  std::vector<float> wout(nn::NP);
  CK(hipMemcpy(wout.data(), dw, wout.size() * 4, hipMemcpyDeviceToHost));
  double cs = 0; for (float v : wout) cs += v;
  printf("variant=%d checksum=%.9g ", variant, cs);
  printf("relu=%d updates=%d sgd_steps=%d  %.3f ms  %.3f us/step  %.2f us/update\n", relu, U, steps, ms,
         ms * 1e3 / steps, ms * 1e3 / U);
  std::vector<unsigned long long> st(80);
  CK(hipMemcpy(st.data(), dst, 80 * 8, hipMemcpyDeviceToHost));
  const char* names1[10] = {"rows", "lr+prefetch", "fwd", "reduce24", "loss", "backward", "barrier1",
                            "update", "barrier2", "-"};
  const char* names2[10] = {"rows+masks", "fwd-mfma", "layer2+po", "barrier", "loss+gb2", "bwd-valu",
                            "mfma-dW1+upd", "-", "-", "-"};
  const char* names3[10] = {"fwd-mfma", "layer2+po", "barrier", "loss+gb2", "bwd+dW1", "update+ops",
                            "-", "-", "-", "-"};
  const char** names = variant == 3 ? names3 : variant == 2 ? names2 : names1;
  for (int wv = 0; wv < 4; ++wv) {
    unsigned long long tot = 0;
    for (int k = 0; k < 9; ++k) tot += st[wv * 10 + k];
    if (!tot) continue;
    printf("wave %d cycles/step:", wv);
    for (int k = 0; k < 9; ++k) printf(" %s=%.0f", names[k], (double)st[wv * 10 + k] / steps);
    printf("  total=%.0f\n", (double)tot / steps);
  }
  return 0;
}
