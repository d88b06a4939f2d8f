// Network kernels of libnfsp: batched predict, Keras-semantics SGD fit (Huber / CE) and
// the DQN target construction.  Reference: agent/agent.py:90-116 (heads),
// agent/agent.py:209-264 (updates).  Oracle: oracle/nn_oracle.py.
//
// The fit kernel is one 256-thread workgroup that keeps the whole 2,179-parameter net,
// the minibatch and every activation in LDS for all epochs x minibatches: an update
// is ONE launch with no HBM traffic beyond reading its 128 samples once.
#include "nfsp_internal.h"

namespace {

constexpr int H = 64;                         // config [Agent] HiddenLayer
constexpr int NP = nfsp::OBS * H + H + H * nfsp::NA + nfsp::NA;   // 2,179
constexpr int OW1 = 0, OB1 = nfsp::OBS * H, OW2 = OB1 + H, OB2 = OW2 + H * nfsp::NA;
constexpr int MAXB = 64;                      // largest fit minibatch

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
// fit: epochs x (n / bs) SGD steps in one workgroup.  Gradients follow
// oracle/nn_oracle.py MLP.grads exactly in formula (summation orders differ:
// parity is within tolerance, not bitwise).
// ---------------------------------------------------------------------------
struct FitSmem {
  float w[NP];
  float x[MAXB][nfsp::OBS];
  float t[MAXB][nfsp::NA];
  float z1[MAXB][H + 1];       // +1: break the 64-float row stride for column reads
  float o[MAXB][nfsp::NA];
  float dz2[MAXB][nfsp::NA];
  float dz1[MAXB][H + 1];
};

__device__ inline void fit_step(FitSmem& sm, int m, int act, float lr) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x;
  // layer 1 (dense, fixed order like predict)
  for (int e = tid; e < m * H; e += blockDim.x) {
    const int b = e / H, j = e - b * H;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < nfsp::OBS; ++i) acc = acc + sm.x[b][i] * sm.w[OW1 + i * H + j];
    sm.z1[b][j] = acc + sm.w[OB1 + j];
  }
  __syncthreads();
  // layer 2, one (row, output) per lane, sequential over the hidden units
  for (int e = tid; e < m * nfsp::NA; e += blockDim.x) {
    const int b = e / nfsp::NA, k = e - b * nfsp::NA;
    float acc = 0.f;
    for (int j = 0; j < H; ++j) {
      const float z = sm.z1[b][j];
      acc = acc + (z > 0.f ? z : 0.f) * sm.w[OW2 + j * 3 + k];
    }
    sm.o[b][k] = acc + sm.w[OB2 + k];
  }
  __syncthreads();
  // dL/dz2 per row
  for (int b = tid; b < m; b += blockDim.x) {
    const float z0 = sm.o[b][0], z1 = sm.o[b][1], z2 = sm.o[b][2];
    float d0, d1, d2;
    if (act == NFSP_ACT_RELU) {
      // Huber, mean over the 3 outputs and the batch; output relu
      const float inv = 1.0f / (float)(3 * m);
      const float zs[3] = {z0, z1, z2};
      float dd[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float y = zs[k] > 0.f ? zs[k] : 0.f;
        const float e = sm.t[b][k] - y;
        const float g = fabsf(e) > 1.0f ? (e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f)) : e;
        dd[k] = zs[k] > 0.f ? (-g * inv) : 0.f;
      }
      d0 = dd[0]; d1 = dd[1]; d2 = dd[2];
    } else {
      // softmax -> x / sum(x) -> clip(eps, 1-eps) -> -sum(t log p), mean over the batch
      const float m_ = fmaxf(fmaxf(z0, z1), z2);
      const float e0 = expf(z0 - m_), e1 = expf(z1 - m_), e2 = expf(z2 - m_);
      const float s = (e0 + e1) + e2;
      const float y[3] = {e0 / s, e1 / s, e2 / s};
      const float S = (y[0] + y[1]) + y[2];
      const float eps = 1e-7f, hi = 1.0f - 1e-7f;
      float dp[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float p = y[k] / S;
        const float pc = fminf(fmaxf(p, eps), hi);
        const float msk = (p >= eps && p <= hi) ? 1.f : 0.f;
        dp[k] = (-sm.t[b][k] / pc) * msk / (float)m;
      }
      const float dpy = (dp[0] * y[0] + dp[1] * y[1]) + dp[2] * y[2];
      float dy[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) dy[k] = dp[k] / S - dpy / (S * S);
      const float dyy = (dy[0] * y[0] + dy[1] * y[1]) + dy[2] * y[2];
      d0 = y[0] * (dy[0] - dyy);
      d1 = y[1] * (dy[1] - dyy);
      d2 = y[2] * (dy[2] - dyy);
    }
    sm.dz2[b][0] = d0; sm.dz2[b][1] = d1; sm.dz2[b][2] = d2;
  }
  __syncthreads();
  // dz1 = (dz2 W2^T) * relu'(z1)   (reads W2 before it is updated)
  for (int e = tid; e < m * H; e += blockDim.x) {
    const int b = e / H, j = e - b * H;
    const float dh = (sm.dz2[b][0] * sm.w[OW2 + j * 3 + 0] + sm.dz2[b][1] * sm.w[OW2 + j * 3 + 1]) +
                     sm.dz2[b][2] * sm.w[OW2 + j * 3 + 2];
    sm.dz1[b][j] = sm.z1[b][j] > 0.f ? dh : 0.f;
  }
  // gW2 / gb2 (kept in registers until W2 readers are done)
  float g2 = 0.f;
  int w2i = -1;
  if (tid < H * nfsp::NA + nfsp::NA) {
    if (tid < H * nfsp::NA) {
      const int j = tid / 3, k = tid - j * 3;
      for (int b = 0; b < m; ++b) {
        const float z = sm.z1[b][j];
        g2 = g2 + (z > 0.f ? z : 0.f) * sm.dz2[b][k];
      }
      w2i = OW2 + tid;
    } else {
      const int k = tid - H * nfsp::NA;
      for (int b = 0; b < m; ++b) g2 = g2 + sm.dz2[b][k];
      w2i = OB2 + k;
    }
  }
  __syncthreads();
  if (w2i >= 0) sm.w[w2i] = sm.w[w2i] - lr * g2;
  // gW1 = x^T dz1, gb1 = sum dz1; each lane owns its W1 entries
  for (int e = tid; e < nfsp::OBS * H + H; e += blockDim.x) {
    float g = 0.f;
    if (e < nfsp::OBS * H) {
      const int i = e / H, j = e - i * H;
      for (int b = 0; b < m; ++b) g = g + sm.x[b][i] * sm.dz1[b][j];
    } else {
      const int j = e - nfsp::OBS * H;
      for (int b = 0; b < m; ++b) g = g + sm.dz1[b][j];
    }
    sm.w[e] = sm.w[e] - lr * g;
  }
  __syncthreads();
}

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
      fit_step(sm, m, act, lr);
    }
  }
  for (int i = threadIdx.x; i < NP; i += blockDim.x) w[i] = sm.w[i];
}

// ---------------------------------------------------------------------------
// DQN targets (agent/agent.py:219-241): one row per lane, then lane 0 applies the
// sequential overwrite and the exploitability mean.
// ---------------------------------------------------------------------------
__device__ inline void fwd_row_relu(const float* sw, const float* xrow, float out[3]) {
#pragma clang fp contract(off)
  float o0 = 0.f, o1 = 0.f, o2 = 0.f;
  for (int j = 0; j < H; ++j) {
    float acc = 0.f;
    for (int i = 0; i < nfsp::OBS; ++i) acc = acc + xrow[i] * sw[OW1 + i * H + j];
    float hj = acc + sw[OB1 + j];
    hj = hj > 0.f ? hj : 0.f;
    o0 = o0 + hj * sw[OW2 + j * 3 + 0];
    o1 = o1 + hj * sw[OW2 + j * 3 + 1];
    o2 = o2 + hj * sw[OW2 + j * 3 + 2];
  }
  o0 = o0 + sw[OB2 + 0];
  o1 = o1 + sw[OB2 + 1];
  o2 = o2 + sw[OB2 + 2];
  out[0] = o0 > 0.f ? o0 : 0.f;
  out[1] = o1 > 0.f ? o1 : 0.f;
  out[2] = o2 > 0.f ? o2 : 0.f;
}

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
    fwd_row_relu(sw, s + (int64_t)k * nfsp::OBS, q);
    fwd_row_relu(sw, s2 + (int64_t)k * nfsp::OBS, qn);
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
