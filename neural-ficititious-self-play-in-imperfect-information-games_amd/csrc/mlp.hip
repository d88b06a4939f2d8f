// Network kernels of libnfsp: batched predict, Keras-semantics SGD fit (Huber / CE) and
// the DQN target construction.  Reference: agent/agent.py:90-116 (heads),
// agent/agent.py:209-264 (updates).  Oracle: oracle/nn_oracle.py.
//
// The fit kernel is one 256-thread workgroup that keeps the whole 2,179-parameter net,
// the minibatch and every activation in LDS for all epochs x minibatches: an update
// is ONE launch with no HBM traffic beyond reading its 128 samples once.
#include "nfsp_internal.h"
#include "nn_device.h"

namespace {

using nfsp::nn::H;
using nfsp::nn::MAXB;
using nfsp::nn::NP;
using nfsp::nn::OB1;
using nfsp::nn::OB2;
using nfsp::nn::OW1;
using nfsp::nn::OW2;

// ---------------------------------------------------------------------------
// predict: one row per lane, weights staged in LDS, dense fixed-order sums
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_mlp_forward(const float* __restrict__ w, int act,
                                                     const float* __restrict__ x,
                                                     float* __restrict__ y, int64_t B) {
#pragma clang fp contract(off)
  __shared__ float sw[NP];
  for (int i = threadIdx.x; i < NP; i += blockDim.x) sw[i] = w[i];
  __syncthreads();
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  float xi[nfsp::OBS];
#pragma unroll
  for (int i = 0; i < nfsp::OBS; ++i) xi[i] = x[row * nfsp::OBS + i];
  float o0 = 0.f, o1 = 0.f, o2 = 0.f;
  for (int j = 0; j < H; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < nfsp::OBS; ++i) acc = acc + xi[i] * sw[OW1 + i * H + j];
    float hj = acc + sw[OB1 + j];
    hj = hj > 0.f ? hj : 0.f;
    o0 = o0 + hj * sw[OW2 + j * 3 + 0];
    o1 = o1 + hj * sw[OW2 + j * 3 + 1];
    o2 = o2 + hj * sw[OW2 + j * 3 + 2];
  }
  o0 = o0 + sw[OB2 + 0];
  o1 = o1 + sw[OB2 + 1];
  o2 = o2 + sw[OB2 + 2];
  if (act == NFSP_ACT_RELU) {
    y[row * 3 + 0] = o0 > 0.f ? o0 : 0.f;
    y[row * 3 + 1] = o1 > 0.f ? o1 : 0.f;
    y[row * 3 + 2] = o2 > 0.f ? o2 : 0.f;
  } else {
    const float m = fmaxf(fmaxf(o0, o1), o2);
    const float e0 = expf(o0 - m), e1 = expf(o1 - m), e2 = expf(o2 - m);
    const float s = (e0 + e1) + e2;
    y[row * 3 + 0] = e0 / s;
    y[row * 3 + 1] = e1 / s;
    y[row * 3 + 2] = e2 / s;
  }
}

// ---------------------------------------------------------------------------
// fit: epochs x (n / bs) SGD steps in one workgroup (nn_device.h sgd_step).  Gradient
// formulas follow oracle/nn_oracle.py MLP.grads exactly; summation orders differ, so
// parity is within tolerance, not bitwise.
// ---------------------------------------------------------------------------
struct FitSmem {
  float w[NP];
  float x[MAXB][nfsp::OBS];
  float t[MAXB][nfsp::NA];
  nfsp::nn::StepScratch sc;
};

__global__ void __launch_bounds__(256) k_mlp_fit(float* __restrict__ w, int act,
                                                 const float* __restrict__ x,
                                                 const float* __restrict__ t, int n,
                                                 const int32_t* __restrict__ perm, int epochs,
                                                 int bs, float lr) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FitSmem& sm = *reinterpret_cast<FitSmem*>(smem_raw);
  for (int i = threadIdx.x; i < NP; i += blockDim.x) sm.w[i] = w[i];
  __syncthreads();
  for (int ep = 0; ep < epochs; ++ep) {
    for (int b0 = 0; b0 < n; b0 += bs) {
      const int m = min(bs, n - b0);
      for (int e = threadIdx.x; e < m * nfsp::OBS; e += blockDim.x) {
        const int b = e / nfsp::OBS, i = e - b * nfsp::OBS;
        sm.x[b][i] = x[(int64_t)perm[ep * n + b0 + b] * nfsp::OBS + i];
      }
      for (int e = threadIdx.x; e < m * nfsp::NA; e += blockDim.x) {
        const int b = e / nfsp::NA, k = e - b * nfsp::NA;
        sm.t[b][k] = t[(int64_t)perm[ep * n + b0 + b] * nfsp::NA + k];
      }
      __syncthreads();
      nfsp::nn::sgd_step(sm.w, &sm.x[0][0], &sm.t[0][0], nullptr, m, act, lr, sm.sc);
    }
  }
  for (int i = threadIdx.x; i < NP; i += blockDim.x) w[i] = sm.w[i];
}

// ---------------------------------------------------------------------------
// DQN targets (agent/agent.py:219-241): one row per lane, then lane 0 applies the
// sequential overwrite and the exploitability mean.
// ---------------------------------------------------------------------------
constexpr int MAXT = 1024;

__global__ void __launch_bounds__(256) k_br_targets(const float* __restrict__ tw,
                                                    const float* __restrict__ s,
                                                    const float* __restrict__ a,
                                                    const float* __restrict__ r,
                                                    const float* __restrict__ s2,
                                                    const uint8_t* __restrict__ t, int n,
                                                    double gamma, unsigned quirks,
                                                    float* __restrict__ out,
                                                    double* __restrict__ expl) {
  __shared__ float sw[NP];
  __shared__ float tgt[MAXT][3];
  __shared__ double val[MAXT];
  __shared__ unsigned char amax[MAXT];
  for (int i = threadIdx.x; i < NP; i += blockDim.x) sw[i] = tw[i];
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    float q[3], qn[3];
    nfsp::nn::forward_relu_row(sw, s + (int64_t)k * nfsp::OBS, q);
    nfsp::nn::forward_relu_row(sw, s2 + (int64_t)k * nfsp::OBS, qn);
    tgt[k][0] = q[0]; tgt[k][1] = q[1]; tgt[k][2] = q[2];
    const float qmax = fmaxf(fmaxf(qn[0], qn[1]), qn[2]);
    const bool terminal = !(quirks & NFSP_QUIRK_TERMINAL_BOOTSTRAP) && t[k];
    val[k] = terminal ? (double)r[k] : (double)r[k] + gamma * (double)qmax;
    amax[k] = (unsigned char)nfsp::argmax3(a[3 * k], a[3 * k + 1], a[3 * k + 2]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = 0.0;
    for (int k = 0; k < n; ++k) acc += (double)fmaxf(fmaxf(tgt[k][0], tgt[k][1]), tgt[k][2]);
    *expl = n > 0 ? acc / n : 0.0;
    for (int k = 0; k < n; ++k) {
      const int row = (quirks & NFSP_QUIRK_ROW0_TARGET) ? 0 : k;
      tgt[row][amax[k]] = (float)val[k];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n * 3; e += blockDim.x) out[e] = tgt[e / 3][e % 3];
}

}  // namespace

extern "C" int nfsp_mlp_forward(nfsp_ctx* c, const float* w, int hidden, int act, const float* x,
                                float* y, int64_t B) {
  NFSP_REQUIRE(c && w && x && y, "null argument");
  NFSP_REQUIRE(hidden == H, "only hidden == 64 is built");
  NFSP_REQUIRE(act == NFSP_ACT_RELU || act == NFSP_ACT_SOFTMAX, "bad act");
  if (B <= 0) return NFSP_OK;
  k_mlp_forward<<<nfsp_blocks(B, 256), 256, 0, c->stream>>>(w, act, x, y, B);
  NFSP_LAUNCHED("k_mlp_forward");
  return NFSP_OK;
}

extern "C" int nfsp_mlp_fit(nfsp_ctx* c, float* w, int hidden, int act, const float* x,
                            const float* t, int n, const int32_t* perm, int epochs, int bs,
                            float lr) {
  NFSP_REQUIRE(c && w && x && t && perm, "null argument");
  NFSP_REQUIRE(hidden == H, "only hidden == 64 is built");
  NFSP_REQUIRE(act == NFSP_ACT_RELU || act == NFSP_ACT_SOFTMAX, "bad act");
  NFSP_REQUIRE(bs >= 1 && bs <= MAXB, "batch_size must be in [1, 64]");
  NFSP_REQUIRE(n >= 0 && epochs >= 0, "bad sizes");
  if (n == 0 || epochs == 0) return NFSP_OK;
  k_mlp_fit<<<1, 256, sizeof(FitSmem), c->stream>>>(w, act, x, t, n, perm, epochs, bs, lr);
  NFSP_LAUNCHED("k_mlp_fit");
  return NFSP_OK;
}

extern "C" int nfsp_br_targets(nfsp_ctx* c, const float* tw, int hidden, const float* s,
                               const float* a, const float* r, const float* s2, const uint8_t* t,
                               int n, double gamma, unsigned quirks, float* out, double* expl) {
  NFSP_REQUIRE(c && tw && s && a && r && s2 && t && out && expl, "null argument");
  NFSP_REQUIRE(hidden == H, "only hidden == 64 is built");
  NFSP_REQUIRE(n >= 0 && n <= MAXT, "n must be in [0, 1024]");
  k_br_targets<<<1, 256, 0, c->stream>>>(tw, s, a, r, s2, t, n, gamma, quirks, out, expl);
  NFSP_LAUNCHED("k_br_targets");
  return NFSP_OK;
}
