// Workgroup-level network routines shared by the fit API (mlp.hip) and the on-device
// learner (engine.hip): one Keras SGD step of a 30 -> 64 -> 3 head, whole net in LDS.
// Formulas = oracle/nn_oracle.py MLP.grads (Huber for the ReLU head, Keras/TF
// categorical cross-entropy for the softmax head); reference: agent/agent.py:90-116,
// 243, 261.
#pragma once
#include "nfsp_device.h"

namespace nfsp {
namespace nn {

constexpr int H = 64;                                            // [Agent] HiddenLayer
constexpr int NP = OBS * H + H + H * NA + NA;                   // 2,179 parameters
constexpr int OW1 = 0, OB1 = OBS * H, OW2 = OB1 + H, OB2 = OW2 + H * NA;
constexpr int MAXB = 64;                                         // largest minibatch

struct StepScratch {
  float z1[MAXB][H + 1];       // +1 breaks the 64-float stride of column walks
  float o[MAXB][NA];
  float dz2[MAXB][NA];
  float dz1[MAXB][H + 1];
};

// One SGD step on the minibatch rows sel[0..m) of x (row stride OBS) / t (stride NA),
// both in LDS (sel == nullptr: rows 0..m-1).  Must be called by the whole workgroup.
__device__ inline void sgd_step(float* w, const float* x, const float* t, const int* sel, int m,
                                int act, float lr, StepScratch& sc) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < m * H; e += nt) {
    const int b = e / H, j = e - b * H;
    const float* xr = x + (sel ? sel[b] : b) * OBS;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < OBS; ++i) acc = acc + xr[i] * w[OW1 + i * H + j];
    sc.z1[b][j] = acc + w[OB1 + j];
  }
  __syncthreads();
  for (int e = tid; e < m * NA; e += nt) {
    const int b = e / NA, k = e - b * NA;
    float acc = 0.f;
    for (int j = 0; j < H; ++j) {
      const float z = sc.z1[b][j];
      acc = acc + (z > 0.f ? z : 0.f) * w[OW2 + j * NA + k];
    }
    sc.o[b][k] = acc + w[OB2 + k];
  }
  __syncthreads();
  for (int b = tid; b < m; b += nt) {
    const float* tr = t + (sel ? sel[b] : b) * NA;
    const float z[3] = {sc.o[b][0], sc.o[b][1], sc.o[b][2]};
    float d[3];
    if (act == 0) {
      const float inv = 1.0f / (float)(3 * m);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float y = z[k] > 0.f ? z[k] : 0.f;
        const float e = tr[k] - y;
        const float g = fabsf(e) > 1.0f ? (e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f)) : e;
        d[k] = z[k] > 0.f ? (-g * inv) : 0.f;
      }
    } else {
      const float mx = fmaxf(fmaxf(z[0], z[1]), z[2]);
      const float e0 = expf(z[0] - mx), e1 = expf(z[1] - mx), e2 = expf(z[2] - mx);
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
        dp[k] = (-tr[k] / pc) * msk / (float)m;
      }
      const float dpy = (dp[0] * y[0] + dp[1] * y[1]) + dp[2] * y[2];
      float dy[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) dy[k] = dp[k] / S - dpy / (S * S);
      const float dyy = (dy[0] * y[0] + dy[1] * y[1]) + dy[2] * y[2];
#pragma unroll
      for (int k = 0; k < 3; ++k) d[k] = y[k] * (dy[k] - dyy);
    }
    sc.dz2[b][0] = d[0]; sc.dz2[b][1] = d[1]; sc.dz2[b][2] = d[2];
  }
  __syncthreads();
  for (int e = tid; e < m * H; e += nt) {
    const int b = e / H, j = e - b * H;
    const float dh = (sc.dz2[b][0] * w[OW2 + j * 3 + 0] + sc.dz2[b][1] * w[OW2 + j * 3 + 1]) +
                     sc.dz2[b][2] * w[OW2 + j * 3 + 2];
    sc.dz1[b][j] = sc.z1[b][j] > 0.f ? dh : 0.f;
  }
  float g2 = 0.f;
  int w2i = -1;
  for (int e = tid; e < H * NA + NA; e += nt) {   // nt >= 195: one entry per lane
    if (e < H * NA) {
      const int j = e / 3, k = e - j * 3;
      for (int b = 0; b < m; ++b) {
        const float z = sc.z1[b][j];
        g2 = g2 + (z > 0.f ? z : 0.f) * sc.dz2[b][k];
      }
      w2i = OW2 + e;
    } else {
      const int k = e - H * NA;
      for (int b = 0; b < m; ++b) g2 = g2 + sc.dz2[b][k];
      w2i = OB2 + k;
    }
  }
  __syncthreads();
  if (w2i >= 0) w[w2i] = w[w2i] - lr * g2;
  for (int e = tid; e < OBS * H + H; e += nt) {
    float g = 0.f;
    if (e < OBS * H) {
      const int i = e / H, j = e - i * H;
      for (int b = 0; b < m; ++b) g = g + x[(sel ? sel[b] : b) * OBS + i] * sc.dz1[b][j];
    } else {
      const int j = e - OBS * H;
      for (int b = 0; b < m; ++b) g = g + sc.dz1[b][j];
    }
    w[e] = w[e] - lr * g;
  }
  __syncthreads();
}

// Q_target forward of one row (ReLU head), fixed order as in predict.
__device__ inline void forward_relu_row(const float* w, const float* xr, float out[3]) {
#pragma clang fp contract(off)
  float o0 = 0.f, o1 = 0.f, o2 = 0.f;
  for (int j = 0; j < H; ++j) {
    float acc = 0.f;
    for (int i = 0; i < OBS; ++i) acc = acc + xr[i] * w[OW1 + i * H + j];
    float hj = acc + w[OB1 + j];
    hj = hj > 0.f ? hj : 0.f;
    o0 = o0 + hj * w[OW2 + j * 3 + 0];
    o1 = o1 + hj * w[OW2 + j * 3 + 1];
    o2 = o2 + hj * w[OW2 + j * 3 + 2];
  }
  o0 = o0 + w[OB2 + 0];
  o1 = o1 + w[OB2 + 1];
  o2 = o2 + w[OB2 + 2];
  out[0] = o0 > 0.f ? o0 : 0.f;
  out[1] = o1 > 0.f ? o1 : 0.f;
  out[2] = o2 > 0.f ? o2 : 0.f;
}

}  // namespace nn
}  // namespace nfsp
