// Reference SGD chain for tools/bench_chain.hip's agreement check: the previous
// production kernel (hidden split over 4 waves, layer-1 forward and dW1 as chained
// v_mfma_f32_16x16x4_f32, exact f32), reading plain fit rows.  Not part of libnfsp.
// Included by bench_chain.hip after learner.hip (uses its dpp / permlane helpers).
namespace chainref {

struct __attribute__((aligned(16))) FitRow {   // observation bits + 3 fit targets
  uint32_t x;
  float t0, t1, t2;
};

struct RefArgs {
  float* w[2];
  float* sync_to[2];
  const FitRow* fit;              // [umax][E][B]
  const uint8_t* active;
  int64_t umax;
  int64_t u0[2], u1[2];
  int agents[2];
  int B, E;
  float lr_fixed;                 // AR lr
  double lr0;                     // BR: lr_u = lr0 / (1 + 0.003 sqrt(it0 + 2u))
  int64_t it0[2];
  unsigned long long* stamps;
};

__device__ inline int64_t next_active(const RefArgs& C, int64_t slot0, int64_t u, int64_t u1) {
  if (C.active)
    while (u < u1 && !C.active[slot0 + u]) ++u;
  return u;
}

struct Chain2Smem {
  float po[2][4][32][4];
  uint32_t xm[4][32];
  float4 dm[4][32];
};

template <int RELU>
__global__ void __launch_bounds__(256) ref_chain2(RefArgs C) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Chain2Smem& sm = *reinterpret_cast<Chain2Smem*>(smem_raw);
  const int a = C.agents[blockIdx.x];
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = tid & 63;
  const int g = l >> 4, c = l & 15;
  const int hid = 16 * w + c;
  float* gw = C.w[blockIdx.x];
  float wr[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int i = 16 * (kk >> 2) + 4 * g + (kk & 3);
    wr[kk] = i < nfsp::OBS ? gw[nn::OW1 + i * nn::H + hid] : 0.f;
  }
  float b1 = gw[nn::OB1 + hid];
  float W2_0 = gw[nn::OW2 + 3 * hid + 0], W2_1 = gw[nn::OW2 + 3 * hid + 1], W2_2 = gw[nn::OW2 + 3 * hid + 2];
  float b2_0 = gw[nn::OB2 + 0], b2_1 = gw[nn::OB2 + 1], b2_2 = gw[nn::OB2 + 2];
  const int nmb = C.B / CHAIN_MB;
  const float inv3m = 1.0f / (float)(3 * CHAIN_MB);
  const float invm = 1.0f / (float)CHAIN_MB;
  const int64_t slot0 = (int64_t)a * C.umax;
  const int64_t u1 = C.u1[blockIdx.x];
  int64_t u = next_active(C, slot0, C.u0[blockIdx.x], u1);
  int e = 0, s = 0, buf = 0;
  uint4 pf = make_uint4(0, 0, 0, 0);          // row of sample (l & 31), one step ahead
  auto issue = [&](int64_t uu, int ee, int ss) {
    const uint4* rows = reinterpret_cast<const uint4*>(C.fit + ((slot0 + uu) * C.E + ee) * C.B +
                                                       ss * CHAIN_MB);
    pf = rows[l & 31];
  };
  if (u < u1) issue(u, e, s);
  float lr = 0.f;
#ifdef NFSP_CHAIN_STAMPS
  unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_last = 0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
  while (u < u1) {
    const uint32_t myx = pf.x;
    const float tt0 = __uint_as_float(pf.y), tt1 = __uint_as_float(pf.z), tt2 = __uint_as_float(pf.w);
    if (l < 32) sm.xm[w][l] = myx;
    if (e == 0 && s == 0)
      lr = RELU ? (float)(C.lr0 / (1.0 + 0.003 * sqrt((double)(C.it0[blockIdx.x] + 2 * u)))) : C.lr_fixed;
    int64_t nu = u;
    int ne = e, ns = s + 1;
    if (ns == nmb) {
      ns = 0;
      if (++ne == C.E) {
        ne = 0;
        nu = next_active(C, slot0, u + 1, u1);
      }
    }
    if (nu < u1) issue(nu, ne, ns);
    const uint32_t xa0 = sm.xm[w][c], xa1 = sm.xm[w][16 + c];
    uint32_t xs[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) xs[kk] = sm.xm[w][16 * (kk >> 2) + 4 * g + (kk & 3)];
    CHAIN_STAMP(0);
    // ---- forward layer 1 on the matrix cores
    floatx4 z0 = {}, z1 = {};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int i = 16 * (kk >> 2) + 4 * g + (kk & 3);
      const float a0 = ((xa0 >> i) & 1u) ? 1.f : 0.f;
      const float a1 = ((xa1 >> i) & 1u) ? 1.f : 0.f;
      z0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, wr[kk], z0, 0, 0, 0);
      z1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, wr[kk], z1, 0, 0, 0);
    }
    float zz[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      zz[r] = z0[r] + b1;          // sample 4g + r
      zz[4 + r] = z1[r] + b1;      // sample 16 + 4g + r
    }
    CHAIN_STAMP(1);
    // ---- layer 2, partial over this wave's 16 hidden units: sum over the row's 16 lanes
    float v[24];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float h = zz[q] > 0.f ? zz[q] : 0.f;
      v[3 * q + 0] = h * W2_0;
      v[3 * q + 1] = h * W2_1;
      v[3 * q + 2] = h * W2_2;
    }
    float hs[12];
    const bool up = c & 8;
#pragma unroll
    for (int i = 0; i < 12; ++i) {      // halve with lane ^ 8, then full sums inside 8 lanes
      const float keep = up ? v[i + 12] : v[i];
      const float send = up ? v[i] : v[i + 12];
      float x = keep + dpp_f(send, 0x128);
      x = x + dpp_f(x, 0xB1);
      x = x + dpp_f(x, 0x4E);
      hs[i] = x + dpp_f(x, 0x141);
    }
    if (c == 0 || c == 8) {             // lane c = 0: samples 4g + r; c = 8: 16 + 4g + r
      const int sb = (c ? 16 : 0) + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float4*>(&sm.po[buf][w][sb + r][0]) =
            make_float4(hs[3 * r + 0], hs[3 * r + 1], hs[3 * r + 2], 0.f);
    }
    CHAIN_STAMP(2);
    __syncthreads();
    CHAIN_STAMP(3);
    // ---- output + loss of sample (l & 31), every wave redundantly (identical results)
    float d0, d1, d2;
    {
      const int sm_i = l & 31;
      const float4 p0 = *reinterpret_cast<const float4*>(&sm.po[buf][0][sm_i][0]);
      const float4 p1 = *reinterpret_cast<const float4*>(&sm.po[buf][1][sm_i][0]);
      const float4 p2 = *reinterpret_cast<const float4*>(&sm.po[buf][2][sm_i][0]);
      const float4 p3 = *reinterpret_cast<const float4*>(&sm.po[buf][3][sm_i][0]);
      const float o0 = (((p0.x + p1.x) + p2.x) + p3.x) + b2_0;
      const float o1 = (((p0.y + p1.y) + p2.y) + p3.y) + b2_1;
      const float o2 = (((p0.z + p1.z) + p2.z) + p3.z) + b2_2;
      if (RELU) {
        const float oz[3] = {o0, o1, o2}, tt[3] = {tt0, tt1, tt2};
        float dd[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float y = oz[k] > 0.f ? oz[k] : 0.f;
          const float ee = tt[k] - y;
          const float gg = fabsf(ee) > 1.0f ? (ee > 0.f ? 1.f : (ee < 0.f ? -1.f : 0.f)) : ee;
          dd[k] = oz[k] > 0.f ? (-gg * inv3m) : 0.f;
        }
        d0 = dd[0]; d1 = dd[1]; d2 = dd[2];
      } else {
        const float mx = fmaxf(fmaxf(o0, o1), o2);
        const float e0 = expf(o0 - mx), e1 = expf(o1 - mx), e2 = expf(o2 - mx);
        const float ssum = (e0 + e1) + e2;
        const float y[3] = {e0 / ssum, e1 / ssum, e2 / ssum};
        const float S = (y[0] + y[1]) + y[2];
        const float eps = 1e-7f, hi = 1.0f - 1e-7f;
        const float tt[3] = {tt0, tt1, tt2};
        float dp[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float p = y[k] / S;
          const float pc = fminf(fmaxf(p, eps), hi);
          const float msk = (p >= eps && p <= hi) ? 1.f : 0.f;
          dp[k] = (-tt[k] / pc) * msk * invm;
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
    }
    if (l < 32) sm.dm[w][l] = make_float4(d0, d1, d2, 0.f);
    // gb2 = sum over the 32 samples (lanes 32..63 mirror 0..31)
    float gb2[3] = {d0, d1, d2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float x = gb2[k];
      x = x + dpp_any(x, 0x128);
      x = x + dpp_any(x, 0x124);
      x = x + dpp_any(x, 0x122);
      x = x + dpp_any(x, 0x121);
      gb2[k] = sum_x16(x);
    }
    CHAIN_STAMP(4);
    // ---- backward: dZ1 in the forward's accumulator layout, layer-2 / bias gradients
    float dz[8];
    float g2_0 = 0.f, g2_1 = 0.f, g2_2 = 0.f, gb1 = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 dd = sm.dm[w][16 * (q >> 2) + 4 * g + (q & 3)];
      const float h = zz[q] > 0.f ? zz[q] : 0.f;
      g2_0 += h * dd.x;
      g2_1 += h * dd.y;
      g2_2 += h * dd.z;
      const float dh = (dd.x * W2_0 + dd.y * W2_1) + dd.z * W2_2;
      dz[q] = zz[q] > 0.f ? dh : 0.f;
      gb1 += dz[q];
    }
    g2_0 = sum_x16(sum_x32(g2_0));
    g2_1 = sum_x16(sum_x32(g2_1));
    g2_2 = sum_x16(sum_x32(g2_2));
    gb1 = sum_x16(sum_x32(gb1));
    CHAIN_STAMP(5);
    // dW1[i][hid] = sum_s x_s[i] dZ1[s][hid]: k-step kk = samples s(kk >> 2, g, kk & 3)
    floatx4 gA = {}, gB = {};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const float a0 = ((xs[kk] >> c) & 1u) ? 1.f : 0.f;          // input c
      const float a1 = ((xs[kk] >> (16 + c)) & 1u) ? 1.f : 0.f;   // input 16 + c
      gA = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, dz[kk], gA, 0, 0, 0);
      gB = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, dz[kk], gB, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      wr[r] = wr[r] - lr * gA[r];          // input 4g + r
      wr[4 + r] = wr[4 + r] - lr * gB[r];  // input 16 + 4g + r
    }
    W2_0 = W2_0 - lr * g2_0;
    W2_1 = W2_1 - lr * g2_1;
    W2_2 = W2_2 - lr * g2_2;
    b1 = b1 - lr * gb1;
    b2_0 = b2_0 - lr * gb2[0];
    b2_1 = b2_1 - lr * gb2[1];
    b2_2 = b2_2 - lr * gb2[2];
    CHAIN_STAMP(6);
    buf ^= 1;
    u = nu;
    e = ne;
    s = ns;
  }
#ifdef NFSP_CHAIN_STAMPS
  if (C.stamps && l == 0)
    for (int k = 0; k < 10; ++k) C.stamps[(blockIdx.x * 4 + w) * 10 + k] = st_acc[k];
#endif
  float* dsts[2] = {gw, C.sync_to[blockIdx.x]};
  for (int k = 0; k < 2; ++k) {
    float* dst = dsts[k];
    if (!dst) continue;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int i = 16 * (kk >> 2) + 4 * g + (kk & 3);
      if (i < nfsp::OBS) dst[nn::OW1 + i * nn::H + hid] = wr[kk];
    }
    if (g == 0) {
      dst[nn::OB1 + hid] = b1;
      dst[nn::OW2 + 3 * hid + 0] = W2_0;
      dst[nn::OW2 + 3 * hid + 1] = W2_1;
      dst[nn::OW2 + 3 * hid + 2] = W2_2;
    }
    if (w == 0 && l == 0) {
      dst[nn::OB2 + 0] = b2_0;
      dst[nn::OB2 + 1] = b2_1;
      dst[nn::OB2 + 2] = b2_2;
    }
  }
}


}  // namespace chainref
