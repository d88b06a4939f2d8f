// Microbenchmark of the learner's SGD chain (learner.hip k_chain3) on synthetic step
// records: microseconds per SGD step, and with -DNFSP_CHAIN_STAMPS the per-phase cycle
// split of waves 0..3 (s_memtime).  Mode "compare" checks k_chain3 against the previous
// f32-MFMA chain (tools/chain_ref.hip) from the same start.  Not part of libnfsp.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize \
//         -fno-honor-nans -falign-loops=64 -mllvm -amdgpu-sched-strategy=max-ilp \
//         [-mllvm -amdgpu-use-amdgpu-trackers] -Iinclude -I<pkg>/csrc tools/bench_chain.hip
//   (one binary, one set of flags: build() gives the BR chain the trackers, the AR chain not)
//   ./bench_chain <updates> <relu 0|1> [time|compare] [blocks 1|2] [layer-2 weight scale]
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../neural-ficititious-self-play-in-imperfect-information-games_amd/csrc/learner.hip"
#include "../neural-ficititious-self-play-in-imperfect-information-games_amd/csrc/chain_ar.hip"
#include "chain_ref.hip"
#include "chain8_probe.h"

// the host helpers learner.hip's nfsp_engine_update references (unused here)
namespace nfsp {
int fail(int code, const std::string&) { return code; }
int hip_fail(hipError_t, const char*) { return NFSP_EHIP; }
namespace eng {
hipEvent_t take_event(nfsp_engine*) { return nullptr; }
int engine_create(nfsp_ctx*, const nfsp_engine_cfg*, bool, nfsp_engine**) { return NFSP_EINVAL; }
int group_rollout_table(nfsp_engine* const*, int, void**) { return NFSP_EINVAL; }
int group_rollout_launch(nfsp_engine* const*, int, const void*, int) { return NFSP_EINVAL; }
int group_snap_launch(nfsp_engine* const*, int, const void*, int) { return NFSP_EINVAL; }
int group_snap_part_launch(nfsp_engine* const*, int, const void*, int, int, hipStream_t) { return NFSP_EINVAL; }
int exchange_enqueue(nfsp_engine*, hipStream_t) { return NFSP_EINVAL; }
int rollout_launch_with(nfsp_engine*, const float*, const double*) { return NFSP_EINVAL; }
}
}
namespace nfsp { namespace chain {
int launch_chain_br_linear(const ChainArgs&, int, bool, bool, hipStream_t) { return NFSP_EINVAL; }
} }
extern "C" int nfsp_engine_destroy(nfsp_engine*) { return NFSP_OK; }
extern "C" int nfsp_engine_get_timings(nfsp_engine*, double*, int64_t*) { return NFSP_OK; }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

static uint4 bits8_host(uint32_t x, int g) {
  const uint32_t n0 = (x >> (4 * g)) & 0xFu, n1 = (x >> (16 + 4 * g)) & 0xFu;
  auto pr = [](uint32_t n) { return (n & 1u) * 0x3F80u + ((n >> 1) & 1u) * 0x3F800000u; };
  return make_uint4(pr(n0), pr(n0 >> 2), pr(n1), pr(n1 >> 2));
}

int main(int argc, char** argv) {
  const int U = argc > 1 ? atoi(argv[1]) : 200;
  const int relu = argc > 2 ? atoi(argv[2]) : 1;
  const bool compare = argc > 3 && !strcmp(argv[3], "compare");
  const int nblk = argc > 4 ? atoi(argv[4]) : 1;     // concurrent chains (as the AR launch: 2;
                                                      // > 2: the engine-group instantiation)
  const bool distinct = getenv("DISTINCT_RECS") && atoi(getenv("DISTINCT_RECS"));  // > 2 chains:
                                                      // each its own copy of the records (HBM)
  const float wscale = argc > 5 ? (float)atof(argv[5]) : 1.f;   // e.g. 60: saturated softmax,
                                                                // exercises the CE clip
  const int B = 128, E = 2, NMB = B / 32;
  std::mt19937 rng(7);
  std::vector<chainref::FitRow> fit((size_t)U * E * B);
  for (auto& r : fit) {
    uint32_t x = 1u << (24 + rng() % 3);
    for (int k = 0; k < 6; ++k) if (rng() & 1) x |= 1u << (rng() % 24);
    r.x = x;
    r.t0 = (rng() % 1000) / 500.f; r.t1 = (rng() % 1000) / 500.f; r.t2 = (rng() % 1000) / 500.f;
  }
  // continuous weights: a grid of values makes exact-zero ReLU inputs likely, where the
  // derivative flips with the summation order
  std::vector<float> w(nn::NP);
  std::uniform_real_distribution<float> ud(-0.2f, 0.2f);
  for (auto& v : w) v = ud(rng);
  for (int i = nn::OW2; i < nn::NP; ++i) w[i] *= wscale;
  // step records, as k_br_targets / k_ar_prep emit them
  // step records as k_br_targets / k_ar_prep emit them (emit_recs): the swizzled fa image,
  // targets (AR: / batch) and the lr per sample
  const size_t nrec = (size_t)U * E * NMB;
  std::vector<StepRec> rec(nrec);
  for (size_t st = 0; st < nrec; ++st) {
    const int u = (int)(st / (E * NMB));
    const float lr = relu ? (float)(0.05 / (1.0 + 0.003 * sqrt((double)(2 * u)))) : 0.1f;
    for (int k = 0; k < 32; ++k) {
      const auto& r = fit[st * 32 + k];
      const uint32_t xb = r.x | CHAIN_BIAS_BIT;      // the bias input
      for (int g = 0; g < 4; ++g) rec[st].fa[g][fa_slot(g, k)] = bits8_host(xb, g);
      const float ts = relu ? 1.f : 1.f / 32.f;
      rec[st].tg[k] = make_float4(r.t0 * ts, r.t1 * ts, r.t2 * ts, lr);
    }
  }
  const void* rec_host = rec.data();
  const size_t rec_bytes = nrec * sizeof(StepRec);
  chainref::FitRow* dfit; char* drec; float* dw; unsigned long long* dst;
  CK(hipMalloc(&dfit, fit.size() * sizeof(chainref::FitRow)));
  CK(hipMalloc(&drec, rec_bytes));
  CK(hipMalloc(&dw, w.size() * 4));
  CK(hipMalloc(&dst, 80 * 8));
  CK(hipMemset(dst, 0, 80 * 8));
  CK(hipMemcpy(dfit, fit.data(), fit.size() * sizeof(chainref::FitRow), hipMemcpyHostToDevice));
  CK(hipMemcpy(drec, rec_host, rec_bytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  float* dw2;
  CK(hipMalloc(&dw2, w.size() * 4));
  CK(hipMemcpy(dw2, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  ChainArgs C{};
  C.job[0].w = dw; C.job[0].rec = reinterpret_cast<const StepRec*>(drec); C.job[0].u0 = 0; C.job[0].u1 = U; C.B = B; C.E = E; C.stamps = dst;
  C.job[1] = C.job[0];
  C.job[1].w = dw2;                                  // second chain: same records, own weights
  chainref::RefArgs R{};
  R.w[0] = dw; R.fit = dfit; R.umax = U; R.u0[0] = 0; R.u1[0] = U; R.B = B; R.E = E;
  R.lr_fixed = 0.1f; R.lr0 = 0.05;
  CK(hipFuncSetAttribute((const void*)k_chain3<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN_LDS));
  CK(hipFuncSetAttribute((const void*)k_chain3<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN_LDS));
  // engine-group form: a device job table, one workgroup per chain, own weights each
  ChainJob* djobs = nullptr;
  if (nblk > 2) {
    std::vector<ChainJob> jobs(nblk, C.job[0]);
    float* wall; char* rall = drec;
    CK(hipMalloc(&wall, (size_t)nblk * w.size() * 4));
    if (distinct) CK(hipMalloc(&rall, (size_t)nblk * rec_bytes));
    for (int k = 0; k < nblk; ++k) {
      CK(hipMemcpy(wall + (size_t)k * w.size(), w.data(), w.size() * 4, hipMemcpyHostToDevice));
      if (distinct) CK(hipMemcpy(rall + (size_t)k * rec_bytes, rec_host, rec_bytes, hipMemcpyHostToDevice));
      jobs[k].w = wall + (size_t)k * w.size();
      jobs[k].rec = reinterpret_cast<const StepRec*>(rall + (distinct ? (size_t)k * rec_bytes : 0));
    }
    CK(hipMalloc(&djobs, sizeof(ChainJob) * nblk));
    CK(hipMemcpy(djobs, jobs.data(), sizeof(ChainJob) * nblk, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void*)k_chain3<0, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN_LDS));
    CK(hipFuncSetAttribute((const void*)k_chain3<1, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN_LDS));
  }
  const int lds = getenv("CHAIN_LDS_BYTES") ? atoi(getenv("CHAIN_LDS_BYTES")) : CHAIN_LDS;
  // CHAIN8=1: the 8-wave sample-split chain (chain8.h) instead of k_chain3
  const bool c8 = getenv("CHAIN8") && atoi(getenv("CHAIN8"));
  for (const void* f : {(const void*)k_chain8<0, 0, 0>, (const void*)k_chain8<1, 0, 0>,
                        (const void*)k_chain8<0, 0, 1>, (const void*)k_chain8<1, 0, 1>})
    CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN_LDS));
  ChainArgs CT = C;
  CT.jobs = djobs;
  auto launch3 = [&]() {
    if (c8) {
      if (nblk > 2) {
        if (relu) k_chain8<1, 0, 1><<<nblk, 512, CHAIN_LDS>>>(CT);
        else k_chain8<0, 0, 1><<<nblk, 512, CHAIN_LDS>>>(CT);
      } else if (relu) k_chain8<1, 0><<<nblk, 512, CHAIN_LDS>>>(C);
      else k_chain8<0, 0><<<nblk, 512, CHAIN_LDS>>>(C);
      return;
    }
    if (nblk > 2) {
      if (relu) k_chain3<1, 0, 1><<<nblk, 256, lds>>>(CT);
      else k_chain3<0, 0, 1><<<nblk, 256, lds>>>(CT);
    } else if (relu) k_chain3<1, 0><<<nblk, 256, CHAIN_LDS>>>(C);
    else k_chain3<0, 0><<<nblk, 256, CHAIN_LDS>>>(C);
  };
  if (compare) {
    std::vector<float> out[2];
    for (int k = 0; k < 2; ++k) {
      CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
      if (k == 0 && relu) chainref::ref_chain2<1><<<1, 256, sizeof(chainref::Chain2Smem)>>>(R);
      else if (k == 0) chainref::ref_chain2<0><<<1, 256, sizeof(chainref::Chain2Smem)>>>(R);
      else launch3();
      CK(hipDeviceSynchronize());
      out[k].resize(nn::NP);
      CK(hipMemcpy(out[k].data(), dw, nn::NP * 4, hipMemcpyDeviceToHost));
    }
    double md = 0, mc = 0;
    int at = -1;
    for (int i = 0; i < nn::NP; ++i) {
      const double d = fabs((double)out[0][i] - out[1][i]);
      if (d > md) { md = d; at = i; }
      mc = fmax(mc, fabs((double)out[1][i] - w[i]));
    }
    printf("compare relu=%d updates=%d: max|ref - chain3| = %.3g at %d (max |change| %.3g)\n", relu, U, md, at, mc);
    return md <= 1e-6 * (1.0 + U) ? 0 : 3;
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  launch3();   // warm
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dst, 0, 80 * 8));
  CK(hipEventRecord(a));
  launch3();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  const int steps = U * E * NMB;
  std::vector<float> wout(nn::NP);
  CK(hipMemcpy(wout.data(), dw, wout.size() * 4, hipMemcpyDeviceToHost));
  double cs = 0; for (float v : wout) cs += v;
  unsigned long long hsh = 1469598103934665603ull;     // FNV-1a over the weights' bits
  for (float v : wout) { uint32_t u; memcpy(&u, &v, 4); hsh = (hsh ^ u) * 1099511628211ull; }
  printf("%s blocks=%d checksum=%.9g hash=%016llx relu=%d updates=%d sgd_steps=%d  %.3f ms  %.3f us/step  %.2f us/update\n",
         c8 ? "k_chain8" : "k_chain3", nblk, cs, hsh, relu, U, steps, ms, ms * 1e3 / steps, ms * 1e3 / U);
  std::vector<unsigned long long> st(80);
  CK(hipMemcpy(st.data(), dst, 80 * 8, hipMemcpyDeviceToHost));
  const char* names3[6] = {"fwd-mfma", "layer2+po", "barrier", "loss+gb2", "bwd+dW1", "update+load"};
  const char* names8[7] = {"split+zh", "layer2+po", "B1", "loss", "bwd+dW1+xch", "B2", "update"};
  const int nph = c8 ? 7 : 6, nwv = c8 ? 8 : 4;
  for (int wv = 0; wv < nwv; ++wv) {
    unsigned long long tot = 0;
    for (int k = 0; k < nph; ++k) tot += st[wv * 10 + k];
    if (!tot) continue;
    printf("wave %d cycles/step:", wv);
    for (int k = 0; k < nph; ++k) printf(" %s=%.0f", c8 ? names8[k] : names3[k], (double)st[wv * 10 + k] / steps);
    printf("  total=%.0f kernel=%.0f\n", (double)tot / steps, (double)st[wv * 10 + 8] / steps);
  }
  return 0;
}
