// Microbenchmark of the learner's SGD chain kernel (k_chain) on synthetic minibatch
// rows: microseconds per SGD step, and with -DNFSP_CHAIN_STAMPS the per-phase cycle
// split of wave 0..3 (s_memtime).  Not part of libnfsp.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -I<pkg>/csrc tools/bench_chain.hip
#include <stdio.h>
#include <stdlib.h>

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
  for (auto& v : w) v = ((int)(rng() % 2001) - 1000) / 5000.f;
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
  const int variant = argc > 3 ? atoi(argv[3]) : 2;
  CK(hipFuncSetAttribute((const void*)k_chain, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ChainSmem)));
  auto launch = [&]() {
    if (variant == 2 && relu) k_chain2<1><<<1, 256, sizeof(Chain2Smem)>>>(C);
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
  const char** names = variant == 2 ? names2 : names1;
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
