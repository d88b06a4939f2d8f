// k_chain8: the SGD chain with the minibatch split over two waves per SIMD (round 6) -- a
// measured experiment, NOT part of libnfsp (tools/bench_chain.hip CHAIN8=1).  Result
// (profiles/r06/chain8_*.log): correct (200 updates within 1.2e-7 BR / 2.7e-5 AR of the f32
// reference chain) but SLOWER: 1.016 / 1.091 us per SGD step against k_chain3's 0.719 / 0.758.
// Its stamps show why: the younger wave of each SIMD pair runs every phase about as long as a
// k_chain3 wave runs the whole (double) phase, and the older wave waits 250-420 cycles at each
// barrier for it -- the SIMD's instruction issue, not one wave's, is the bound, and the pair
// issues ~1.2x k_chain3's instructions per step (the duplicated W split and loss, the
// exchange).  DESIGN.md Appendix A.0.
// Reference: agent/agent.py:241-264 (model.fit(batch_size=32, epochs=2) of the BR Q-net and
// the AR policy net), the same step records and job tables as k_chain3 (chain3.h).
//
// Why: k_chain3's step is ~300 instructions issued in order by ONE wave per SIMD, and a wave
// alone issues a plain VALU instruction every ~4 cycles while the SIMD could take one every 2
// (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'); the step was issue-bound at
// 0.72 / 0.76 us (BR / AR).  Here the 8 waves of a chain workgroup are (w, h): hidden slice
// 16w .. 16w + 15 as before, and h = the half of the 32-sample minibatch whose layer 2, loss,
// backward and dW1 the wave computes.  Waves w and w + 4 share SIMD w and each issue about
// half of what one k_chain3 wave does per step (the W split stays duplicated).  Per step:
//   * layer 1: Z1^T (hidden-major, 3 v_mfma_f32_16x16x32_bf16 over the exact 3-term split of
//     W1) and Z1 (sample-major) for the wave's 16 samples only;
//   * layer 2 partial sums over the slice, reduced over the 4 lane rows by two permlane32 and
//     one permlane16 swap, into po[w][sample] (LDS); barrier B1;
//   * the loss of the wave's 16 samples (4 lanes each), the backward of its samples, and the
//     partial dW1 = X^T dZ1 over them (K = 16: v_mfma_f32_16x16x16_bf16, X^T by
//     ds_read_b64_tr_b16 from the record's bf16 image);
//   * the two halves' partial dW1, dW2 and db2 meet through LDS (barrier B2); both waves of a
//     pair add own + partner's (a + b == b + a bit for bit, so their W copies stay identical)
//     and update W1 (registers), W2 / b2 (wave-private LDS).
// The 32-sample sums are therefore added as two 16-sample halves: not k_chain3's order (not
// bit-identical to it); every product is still exact (0/1 inputs, exact bf16 splits) and every
// sum f32.  Parity: the learner tests' written tolerances.
#pragma once
#include "../neural-ficititious-self-play-in-imperfect-information-games_amd/csrc/chain3.h"

namespace nfsp {
namespace chain {

struct Chain8Smem {
  float4 po[4][32];          // layer-2 partial outputs: [hidden slice][sample] (x, y, z used)
  float4 w2t[8][64];         // wave-private: W2[16 w + r][0..2] in rows 0..15
  float b2s[8][4];           // wave-private: b2
  float4 xch[8][3][64];      // the halves' exchange: [wave][dW1 tile 0 | tile 1 | (V, U, loss)][lane]
  StepRec ring[4];           // step records t .. t + 2 (slot t & 3), an eighth per wave
  uint4 rec_sink[64];
  float4 psink[64];          // po stores of the lane rows that hold a duplicate
};
constexpr int REC_EIGHTH = REC_CHUNKS / 8;                  // 20 chunks of 16 B per wave
static_assert(REC_CHUNKS % 8 == 0, "record chunking");
constexpr int CHAIN8_LDS = (int)((sizeof(Chain8Smem) + 1023) & ~size_t(1023));
static_assert(CHAIN8_LDS <= CHAIN_LDS, "chain8 LDS");

typedef short short4x __attribute__((ext_vector_type(4)));
// v_mfma_f32_16x16x16_bf16, three chained terms: Z = A.lo + A.mid + A.hi (exact products)
__device__ inline floatx4 mfma16x3(short4x a, short4x bhi, short4x bmid, short4x blo) {
  floatx4 z = {};
  z = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, blo, z, 0, 0, 0);
  z = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bmid, z, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bhi, z, 0, 0, 0);
}

// The exact three-term bf16 split of 4 f32 values (split3's construction on one pair group:
// a - hi(a) = dot((hi(a), hi(b)), (-1, 0)) + a, exact).  DOT results are read >= 3 wait
// states after they are written (s_nop 2 where the order does not space them); the string
// ends with s_nop 1 for the MFMAs that read the terms.
__device__ inline void split3x4(const float (&v)[4], short4x& hi, short4x& mid, short4x& lo, SplitK K) {
  uint32_t h0, h1, m0, m1, o0, o1;
  float r0, r1, r2, r3;
  asm volatile(
      "v_cvt_pk_bf16_f32 %0, %10, %11\n\t"
      "v_cvt_pk_bf16_f32 %1, %12, %13\n\t"
      "v_dot2_f32_bf16 %6, %0, %14, %10\n\t"
      "v_dot2_f32_bf16 %7, %0, %15, %11\n\t"
      "v_dot2_f32_bf16 %8, %1, %14, %12\n\t"
      "v_dot2_f32_bf16 %9, %1, %15, %13\n\t"
      "s_nop 2\n\t"
      "v_cvt_pk_bf16_f32 %2, %6, %7\n\t"
      "v_cvt_pk_bf16_f32 %3, %8, %9\n\t"
      "v_dot2_f32_bf16 %6, %2, %14, %6\n\t"
      "v_dot2_f32_bf16 %7, %2, %15, %7\n\t"
      "v_dot2_f32_bf16 %8, %3, %14, %8\n\t"
      "v_dot2_f32_bf16 %9, %3, %15, %9\n\t"
      "s_nop 2\n\t"
      "v_cvt_pk_bf16_f32 %4, %6, %7\n\t"
      "v_cvt_pk_bf16_f32 %5, %8, %9\n\t"
      "s_nop 1"
      : "=&v"(h0), "=&v"(h1), "=&v"(m0), "=&v"(m1), "=&v"(o0), "=&v"(o1), "=&v"(r0), "=&v"(r1), "=&v"(r2),
        "=&v"(r3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(K.cl), "v"(K.ch));
  hi = __builtin_bit_cast(short4x, make_uint2(h0, h1));
  mid = __builtin_bit_cast(short4x, make_uint2(m0, m1));
  lo = __builtin_bit_cast(short4x, make_uint2(o0, o1));
}

// 4 bf16 of a transposed operand: one ds_read_b64_tr_b16 (rows lo .. lo + 3 of a 16-bit
// image in LDS).  The whole wave must be active.
__device__ inline short4x tr4(const char* p) {
  return __builtin_bit_cast(short4x, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)p));
}

// RELU / LOSS / TABLE as k_chain3's.
template <int RELU, int LOSS, int TABLE = 0>
__global__ void __launch_bounds__(512) k_chain8(ChainArgs C) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Chain8Smem& sm = *reinterpret_cast<Chain8Smem*>(smem_raw);
  const ChainJob J = TABLE ? C.jobs[blockIdx.x] : C.job[blockIdx.x];
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);    // wave 0..7 (SIMD wv & 3)
  const int w = wv & 3, h = wv >> 2;                          // hidden slice, sample half
  const int l = tid & 63;
  const int g = l >> 4, c = l & 15;
  const int hid = 16 * w + c;
  // this lane's loss sample: lane j of row g holds sample 16h + 4g + (j & 3) -- the sample
  // backward slot j & 3 of the row's lanes needs (row_newbcast:j for j < 4)
  const int ls = 16 * h + 4 * g + (c & 3);
  float* gw = J.w;
  float wr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int i = 16 * (j >> 2) + 4 * g + (j & 3);
    wr[j] = i < nfsp::OBS ? gw[nn::OW1 + i * nn::H + hid] : i == CHAIN_BIAS_IN ? gw[nn::OB1 + hid] : 0.f;
  }
  float W2_0 = gw[nn::OW2 + 3 * hid + 0], W2_1 = gw[nn::OW2 + 3 * hid + 1], W2_2 = gw[nn::OW2 + 3 * hid + 2];
  float b2_0 = gw[nn::OB2 + 0], b2_1 = gw[nn::OB2 + 1], b2_2 = gw[nn::OB2 + 2];
  const int nmb = C.B / CHAIN_MB;
  const int spu = C.E * nmb;                   // SGD steps per update
  const float inv3m = 1.0f / (float)(3 * CHAIN_MB);
  const float invm = 1.0f / (float)CHAIN_MB;
  const int64_t u1 = J.u1;
  int64_t u0 = J.u0;
  if (J.active) {          // AR: skip the inactive prefix (M_SL <= batch; monotone in u)
    while (u0 < u1) {
      const int64_t q = u0 + l;
      const unsigned long long m = __ballot(q < u1 && J.active[q]);
      if (m) { u0 += __builtin_ctzll(m); break; }
      u0 += 64;
    }
    if (u0 > u1) u0 = u1;
  }
  const int T1 = (int)(u1 * spu);
  int t = (int)(u0 * spu);
  // this wave's eighth of record p (clamped) into a register, then into ring slot p & 3
  const bool in_q = l < REC_EIGHTH;
  const int la = in_q ? l : REC_EIGHTH - 1;
  const int T1c = T1 > 0 ? T1 : 1;
  const auto rrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<StepRec*>(J.rec), 0,
                                                       (int)((size_t)T1c * sizeof(StepRec)), 0x00020000);
  const int va_off = (REC_EIGHTH * wv + la) * 16;
  auto issue = [&](int p, uint4& va) {
    const int pc = p < T1 ? p : T1 - 1;
    va = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rrsrc, va_off, pc * (int)sizeof(StepRec), 0));
  };
  auto stash_slot = [&](int slot, const uint4& va) {
    uint4* dst = reinterpret_cast<uint4*>(&sm.ring[slot]) + REC_EIGHTH * wv;
    *(in_q ? dst + l : &sm.rec_sink[l]) = va;
  };
  // X^T of this half (the dW1 operand, K = samples 16h + 4g .. + 3): lane c of group g gets
  // input c (tile 0) / 16 + c (tile 1, +8 B) of those samples (chain3.h tr_off, +256 B per half)
  const int tr_off = 512 * (c & 3) + 16 * fa_slot(c & 3, 4 * g + (c >> 2)) + 256 * h;
  const int fsw = 12 * (g & 1);                // fa_slot(g, .) of this lane row
  const SplitK SK = split_consts();
  // W2 / b2 ownership after the reductions (each total sits in one lane row):
  //   row 0: W2[c][0]   row 1: W2[c][2]   row 2: W2[c][1]   row 3: b2[0]      (V)
  //   rows 0, 1: b2[1]   rows 2, 3: b2[2]                                      (U)
  float* const own1 = g == 3 ? &sm.b2s[wv][0] : reinterpret_cast<float*>(&sm.w2t[wv][c]) + (g == 0 ? 0 : g == 1 ? 2 : 1);
  float* const own2 = &sm.b2s[wv][g < 2 ? 1 : 2];
  // layer-2 store target: row 0 output 0, row 2 output 1, rows 1 / 3 output 2 (row 3: a copy)
  float* const po_dst = g == 3 ? reinterpret_cast<float*>(&sm.psink[l])
                               : reinterpret_cast<float*>(&sm.po[w][16 * h + c]) + (g == 0 ? 0 : g == 2 ? 1 : 2);
  const int pw = wv ^ 4;                       // the partner wave (same slice, other half)
  float loss_acc = 0.f;
#ifdef NFSP_CHAIN_STAMPS
  unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_last = 0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
  const unsigned long long st_t0 = st_last;
#endif
  auto step = [&](auto PHC) {
    constexpr int PH = decltype(PHC)::value;
    const int slot = PH >= 0 ? PH : (t & 3);
    uint4 va;
    issue(t + 2, va);
    const StepRec& R = sm.ring[slot];
    const bf16x8 fa = __builtin_bit_cast(bf16x8, R.fa[g][(16 * h + c) ^ fsw]);
    const char* const rtr = reinterpret_cast<const char*>(&R.fa[0][0]) + tr_off;
    // ---- layer 1, both orientations, this half's samples
    bf16x8 whi, wmid, wlo;
    split3(wr, whi, wmid, wlo, SK);
    float W2h[4][3];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const floatx4 q = lds4(&sm.w2t[wv][4 * g + r]);
      W2h[r][0] = q[0]; W2h[r][1] = q[1]; W2h[r][2] = q[2];
    }
    const floatx4 w2c = lds4(&sm.w2t[wv][c]);     // W2 of this lane's hidden unit (backward)
    const float W2_0 = w2c[0], W2_1 = w2c[1], W2_2 = w2c[2];
    const floatx4 b2v = lds4(&sm.b2s[wv][0]);
    const floatx4 zh = mfma3t(whi, wmid, wlo, fa);      // Z1^T: hidden 16w + 4g + r, sample 16h + c
    __builtin_amdgcn_sched_barrier(0);
    CHAIN_STAMP(0);
    // ---- layer 2 partial over the slice (the wave's 16 hidden units)
    float p[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float hr = fmaxf(zh[r], 0.f);               // b1 is W1's row 30 (CHAIN_BIAS_IN)
#pragma unroll
      for (int k = 0; k < 3; ++k) p[k] = p[k] + hr * W2h[r][k];
    }
    {   // rows g, g ^ 2 (one swap for outputs 0 / 1: lanes 0-31 get output 0, 32-63 output 1),
        // then rows g, g ^ 1 (outputs 0 / 1 against 2)
      const auto r01 = __builtin_amdgcn_permlane32_swap(__float_as_uint(p[0]), __float_as_uint(p[1]), false, false);
      const float q01 = __uint_as_float(r01[0]) + __uint_as_float(r01[1]);
      const float q2 = sum_x32(p[2]);
      const auto z = __builtin_amdgcn_permlane16_swap(__float_as_uint(q01), __float_as_uint(q2), false, false);
      *po_dst = __uint_as_float(z[0]) + __uint_as_float(z[1]);
    }
    const floatx4 zs = mfma3(fa, whi, wmid, wlo);       // Z1: sample 16h + 4g + r, hidden 16w + c
    const float4 tg = R.tg[ls];
    CHAIN_STAMP(1);
    __syncthreads();                                    // B1: the partial outputs
    CHAIN_STAMP(2);
    const short4x ba0 = tr4(rtr), ba1 = tr4(rtr + 8);
    // ---- output + loss of sample ls (the half's 4 waves redundantly, identical results)
    float d0, d1, d2;
    float Ls = 0.f;
    {
      const floatx4 a0 = lds4(&sm.po[0][ls]);
      const floatx4 a1 = lds4(&sm.po[1][ls]);
      const floatx4 a2 = lds4(&sm.po[2][ls]);
      const floatx4 a3 = lds4(&sm.po[3][ls]);
      const float o0 = (((a0[0] + a1[0]) + a2[0]) + a3[0]) + b2v[0];
      const float o1 = (((a0[1] + a1[1]) + a2[1]) + a3[1]) + b2v[1];
      const float o2 = (((a0[2] + a1[2]) + a2[2]) + a3[2]) + b2v[2];
      const float tt[3] = {tg.x, tg.y, tg.z};
      const float oz[3] = {o0, o1, o2};
      if (RELU) {          // Huber on ReLU outputs (RELU 2: linear outputs), mean over 3 x batch
        float dd[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float ee = tt[k] - (RELU >= 2 ? oz[k] : fmaxf(oz[k], 0.f));
          const float gg = RELU == 3 ? ee * 2.0f : __builtin_amdgcn_fmed3f(ee, -1.f, 1.f);
          dd[k] = (RELU >= 2 || oz[k] > 0.f) ? gg * -inv3m : 0.f;
          if (LOSS) {      // huber_loss with py2's 1 / 2 == 0 (RELU 3: e^2), mean over 3
            Ls += RELU == 3 ? ee * ee : (fabsf(ee) > 1.0f ? fabsf(ee) : 0.5f * ee * ee);
          }
        }
        d0 = dd[0]; d1 = dd[1]; d2 = dd[2];
        if (LOSS) Ls *= 1.0f / 3.0f;
      } else {
        // Keras categorical cross-entropy on the softmax: d_k = (y_k T_M - [k in M] t_k) / batch
        // (chain3.h k_chain3 for the derivation; AR records carry t / batch)
        const float mx = fmaxf(fmaxf(o0, o1), o2);
        const float L2E = 1.44269504088896341f, mxl = mx * L2E;
        const float e0 = __builtin_amdgcn_exp2f(__builtin_fmaf(o0, L2E, -mxl));
        const float e1 = __builtin_amdgcn_exp2f(__builtin_fmaf(o1, L2E, -mxl));
        const float e2 = __builtin_amdgcn_exp2f(__builtin_fmaf(o2, L2E, -mxl));
        const float rs = __builtin_amdgcn_rcpf((e0 + e1) + e2);
        const float y0 = e0 * rs, y1 = e1 * rs, y2 = e2 * rs;
        const float eps = 1e-7f, hi = 1.0f - 1e-7f;
        const float m0 = __builtin_amdgcn_fmed3f(y0, eps, hi) == y0 ? tt[0] : 0.f;
        const float m1 = __builtin_amdgcn_fmed3f(y1, eps, hi) == y1 ? tt[1] : 0.f;
        const float m2 = __builtin_amdgcn_fmed3f(y2, eps, hi) == y2 ? tt[2] : 0.f;
        const float k = (m0 + m1) + m2;
        d0 = y0 * k - m0;
        d1 = y1 * k - m1;
        d2 = y2 * k - m2;
        if (LOSS) {
          const float yy[3] = {y0, y1, y2};
          for (int q = 0; q < 3; ++q)
            Ls -= (tt[q] * (float)CHAIN_MB) * __logf(fminf(fmaxf(yy[q], 1e-7f), 1.0f - 1e-7f));
        }
      }
    }
    CHAIN_STAMP(3);
    // ---- backward, sample-major: samples 16h + 4g + r, hidden 16w + c
    float dz[4];
    float g2_0, g2_1, g2_2;
    {
      const float zz[4] = {zs[0], zs[1], zs[2], zs[3]};
      float dh[4];
#define NFSP_BWD8(J) dh[J] = bwd_dpp<J>(g2_0, g2_1, g2_2, d0, d1, d2, fmaxf(zz[J], 0.f), W2_0, W2_1, W2_2)
      NFSP_BWD8(0); NFSP_BWD8(1); NFSP_BWD8(2); NFSP_BWD8(3);
#undef NFSP_BWD8
#pragma unroll
      for (int j = 0; j < 4; ++j) dz[j] = zz[j] > 0.f ? dh[j] : 0.f;
    }
    short4x dhi, dmid, dlo;
    split3x4(dz, dhi, dmid, dlo, SK);
    // partial dW1 over this half: [16 t + 4g + r][16w + c] (row 30: gb1)
    const floatx4 gA = mfma16x3(ba0, dhi, dmid, dlo);
    const floatx4 gB = mfma16x3(ba1, dhi, dmid, dlo);
    // the half's db2: each row's 4 samples (lanes j & 3; the row's quads are copies), then the
    // rows through the transposes below
    auto quad = [](float x) { x = x + dpp_bc<0xB1>(x); return x + dpp_bc<0x4E>(x); };
    const float S0 = quad(d0), S1 = quad(d1), S2 = quad(d2);
    float V, U;
    {   // (g2_0, g2_1, g2_2, S0) over the 4 rows: row 0 g2_0, row 1 g2_2, row 2 g2_1, row 3 db2[0]
      const auto ab = __builtin_amdgcn_permlane32_swap(__float_as_uint(g2_0), __float_as_uint(g2_1), false, false);
      const float tab = __uint_as_float(ab[0]) + __uint_as_float(ab[1]);
      const auto cd = __builtin_amdgcn_permlane32_swap(__float_as_uint(g2_2), __float_as_uint(S0), false, false);
      const float tcd = __uint_as_float(cd[0]) + __uint_as_float(cd[1]);
      const auto z = __builtin_amdgcn_permlane16_swap(__float_as_uint(tab), __float_as_uint(tcd), false, false);
      V = __uint_as_float(z[0]) + __uint_as_float(z[1]);
      // (S1, S2): rows 0 / 1 db2[1], rows 2 / 3 db2[2]
      const auto e = __builtin_amdgcn_permlane32_swap(__float_as_uint(S1), __float_as_uint(S2), false, false);
      U = sum_x16(__uint_as_float(e[0]) + __uint_as_float(e[1]));
    }
    float LsH = 0.f;
    if (LOSS) LsH = sum_x16(sum_x32(quad(Ls)));          // the half's 16 samples' losses
    sm.xch[wv][0][l] = make_float4(gA[0], gA[1], gA[2], gA[3]);
    sm.xch[wv][1][l] = make_float4(gB[0], gB[1], gB[2], gB[3]);
    sm.xch[wv][2][l] = make_float4(V, U, LsH, 0.f);
    CHAIN_STAMP(4);
    __syncthreads();                                    // B2: the halves meet
    CHAIN_STAMP(5);
    const floatx4 pA = lds4(&sm.xch[pw][0][l]);
    const floatx4 pB = lds4(&sm.xch[pw][1][l]);
    const floatx4 pv = lds4(&sm.xch[pw][2][l]);
    const float lr = tg.w;
    {
      const float Vt = V + pv[0], Ut = U + pv[1];       // own + partner: the pair adds alike
      const float v1 = *own1, v2 = *own2;
      *own1 = v1 - lr * Vt;
      *own2 = v2 - lr * Ut;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      wr[r] = wr[r] - lr * (gA[r] + pA[r]);
      wr[4 + r] = wr[4 + r] - lr * (gB[r] + pB[r]);
    }
    if (LOSS && wv == 0 && l == 0) {      // Keras' epoch mean of the minibatch losses
      const float x = LsH + pv[2];
      const int in_u = t % spu;
      loss_acc += x * invm;
      if (in_u % nmb == nmb - 1) {
        const int64_t uu = t / spu, ee = in_u / nmb;
        J.loss_out[uu * C.E + ee] = loss_acc / (float)nmb;
        loss_acc = 0.f;
      }
    }
    stash_slot(PH >= 0 ? ((PH + 2) & 3) : ((t + 2) & 3), va);
    CHAIN_STAMP(6);
  };
  if (t < T1) {
    {
      uint4 va;
      issue(t, va);
      stash_slot(t & 3, va);
      issue(t + 1, va);
      stash_slot((t + 1) & 3, va);
    }
    sm.w2t[wv][l] = make_float4(W2_0, W2_1, W2_2, 0.f);
    if (l < 3) sm.b2s[wv][l] = l == 0 ? b2_0 : l == 1 ? b2_1 : b2_2;
    __syncthreads();
    __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): drain the prologue's loads
    if (spu % 4 == 0) {
      for (; t < T1; ++t) {
        step(std::integral_constant<int, 0>{});
        ++t;
        step(std::integral_constant<int, 1>{});
        ++t;
        step(std::integral_constant<int, 2>{});
        ++t;
        step(std::integral_constant<int, 3>{});
      }
    } else {
      for (; t < T1; ++t) step(std::integral_constant<int, -1>{});
    }
  }
#ifdef NFSP_CHAIN_STAMPS
  if (l == 0 && C.stamps && blockIdx.x == 0) {
    unsigned long long t_end;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_end)::"memory");
    st_acc[8] = t_end - st_t0;
    st_acc[9] = (unsigned long long)(T1 - (int)(u0 * spu));
    for (int k = 0; k < 10; ++k) C.stamps[wv * 10 + k] = st_acc[k];
  }
#endif
  if (t > (int)(u0 * spu)) {             // the loop ran: W2 / b2 as the last step left them
    const float4 fw = sm.w2t[wv][c];
    W2_0 = fw.x; W2_1 = fw.y; W2_2 = fw.z;
    b2_0 = sm.b2s[wv][0]; b2_1 = sm.b2s[wv][1]; b2_2 = sm.b2s[wv][2];
  }
  if (h) return;                         // the pair's copies are identical: half 0 writes
  float* dsts[3] = {gw, J.sync_to, J.snap_to};
  for (int k = 0; k < 3; ++k) {
    float* dst = dsts[k];
    if (!dst) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = 16 * (j >> 2) + 4 * g + (j & 3);
      if (i < nfsp::OBS) dst[nn::OW1 + i * nn::H + hid] = wr[j];
      else if (i == CHAIN_BIAS_IN) dst[nn::OB1 + hid] = wr[j];
    }
    if (g == 0) {
      dst[nn::OW2 + 3 * hid + 0] = W2_0;
      dst[nn::OW2 + 3 * hid + 1] = W2_1;
      dst[nn::OW2 + 3 * hid + 2] = W2_2;
    }
    if (wv == 0 && l == 0) {
      dst[nn::OB2 + 0] = b2_0;
      dst[nn::OB2 + 1] = b2_1;
      dst[nn::OB2 + 2] = b2_2;
    }
  }
}

// Launch k_chain8<RELU, loss_log, C.jobs != null> on `s` (512 threads, CHAIN_LDS bytes: a CU
// to itself, as k_chain3's one-engine launches), setting the LDS attribute once per device.
template <int RELU>
int launch_chain8(const ChainArgs& C, int blocks, bool loss_log, hipStream_t s, std::atomic<uint64_t>& attr) {
  const int rc = set_chain_lds(attr, (const void*)k_chain8<RELU, 0, 0>, (const void*)k_chain8<RELU, 1, 0>,
                               (const void*)k_chain8<RELU, 0, 1>, (const void*)k_chain8<RELU, 1, 1>);
  if (rc != NFSP_OK) return rc;
  if (C.jobs) {
    if (loss_log) k_chain8<RELU, 1, 1><<<blocks, 512, CHAIN_LDS, s>>>(C);
    else k_chain8<RELU, 0, 1><<<blocks, 512, CHAIN_LDS, s>>>(C);
  } else {
    if (loss_log) k_chain8<RELU, 1, 0><<<blocks, 512, CHAIN_LDS, s>>>(C);
    else k_chain8<RELU, 0, 0><<<blocks, 512, CHAIN_LDS, s>>>(C);
  }
  NFSP_LAUNCHED("k_chain8");
  return NFSP_OK;
}

}  // namespace chain
}  // namespace nfsp
