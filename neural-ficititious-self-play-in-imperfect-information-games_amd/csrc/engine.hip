// The batched NFSP self-play engine: the fused rollout kernel, the deterministic
// commit of its records into the agents' memories, and the on-device learner.
// Declarations and the semantics contract: include/nfsp.h (nfsp_engine_*).
//
// Data path of one nfsp_engine_step (all on the ctx stream, no host sync):
//   k_rollout   one lane = one env: deal, eta draws, main.train's D/L/D scheduler, every
//               Agent.play (observe -> RL record, act with the AR net or eps-greedy BR
//               net -> env.step -> SL record).  Networks of both agents in LDS.  Records
//               go to lane-major staging ([slot][lane], so a wave's stores coalesce).
//   k_scan1/2   exclusive prefix over lanes of the 4 per-lane record counts -> canonical
//               insert order (lane, then play order) independent of scheduling.
//   k_commit    RL records -> each agent's circular M_RL log (fp32 reference layout);
//               SL records -> the agent's pending list with their RL stream position.
//   k_learner   4 workgroups (agent x {AR, BR}): update_strategy once per
//               inserts_per_update RL inserts, each a sampled minibatch, the DQN targets,
//               epochs x minibatch SGD (nn_device.h), and the reference schedules; the
//               AR workgroup applies the reservoir inserts in stream order in between.
#include <math.h>

#include <vector>

#include "nfsp_internal.h"
#include "nn_device.h"

using nfsp::Hand;
using nfsp::u32x4;
namespace nn = nfsp::nn;

namespace {

constexpr int MAXREC = 6;          // records of one kind per lane per hand (<= 6 decisions)
constexpr int W1S = 65;            // padded LDS row stride of W1: row i of lane A and row
                                   // i' of lane B hit banks (i + j), (i' + j) mod 32
constexpr int NET_LDS = nfsp::OBS * W1S + nn::H + nn::H * nfsp::NA + nfsp::NA;   // 2,209
constexpr int LB1 = nfsp::OBS * W1S, LW2 = LB1 + nn::H, LB2 = LW2 + nn::H * nfsp::NA;
constexpr int MAX_LEARN_BATCH = 128;

// Philox counter word x: rollout uses the lane id (< 2^24); learner streams use 0x8?......
constexpr uint32_t TAG_SAMPLE = 0x81000000u, TAG_PERM = 0x82000000u, TAG_RES = 0x83000000u;

struct EngineDev {
  int64_t rl_total[2], sl_total[2], sl_count[2];
  int64_t last_rl[2], last_sl[2];
  int64_t iteration[2], target_count[2], target_syncs[2];
  int64_t br_updates[2], ar_updates[2];
  int64_t hands, rollouts;
  unsigned long long actions[2][3];
  long long reward_half[2];
  double epsilon[2], temp[2], expl[2];
  float lr_br[2];
};

struct Staging {
  uint32_t* rl_s2;     // [MAXREC][N] observation after (bits)
  uint32_t* rl_meta;   // [MAXREC][N] r (int8 half units) | t << 8 | player << 9
  uint32_t* rl_s;      // [MAXREC][N] s at observation time (no-alias mode)
  float* rl_a;         // [MAXREC][3][N]
  uint32_t* sl_x;      // [MAXREC][N]
  float* sl_a;         // [MAXREC][3][N]
  uint32_t* sl_meta;   // [MAXREC][N] player | lane-local RL count << 8
  uint32_t* fin_s;     // [2][N] env.s[p] at hand end (alias mode)
  float* fin_a;        // [2][3][N] env.last_action[p] at hand end
  uint32_t* counts;    // [N] rl0 | rl1 << 4 | sl0 << 8 | sl1 << 12
  unsigned long long* local;   // [N] packed 4 x 16-bit exclusive prefix within the block
  uint4* block_sum;    // [nblk]
  uint4* block_base;   // [nblk]
};

struct Memories {
  // M_RL: circular logs, agent-major [2][log_cap][...]
  float *rl_s, *rl_a, *rl_r, *rl_s2;
  uint8_t* rl_t;
  int64_t log_cap;
  // M_SL: reservoirs [2][sl_cap][...]
  float *sl_s, *sl_a;
  int64_t sl_cap;
  // pending SL records of the last rollout [2][4N]
  uint32_t* pend_x;
  float* pend_a;
  int64_t* pend_pos;
  int64_t pend_cap;
  // learner debug: last update's rows / perms per (agent, role)
  int64_t* dbg_rows;    // [4][batch]
  int32_t* dbg_perms;   // [4][epochs][batch]
};

__device__ inline void fwd_lds(const float* __restrict__ sw, uint32_t x, int act, float y[3]) {
#pragma clang fp contract(off)
  int rows[9];
  int nb = 0;
  uint32_t b = x;
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    rows[u] = 0;
    if (b) {
      rows[u] = __builtin_ctz(b) * W1S;
      b &= b - 1;
      nb = u + 1;
    }
  }
  float o0 = 0.f, o1 = 0.f, o2 = 0.f;
  for (int j = 0; j < nn::H; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 9; ++u)
      if (u < nb) acc = acc + sw[rows[u] + j];
    if (b) {   // > 9 set bits: impossible for Leduc observations, kept exact anyway
      uint32_t rest = b;
      while (rest) {
        const int i = __builtin_ctz(rest);
        rest &= rest - 1;
        acc = acc + sw[i * W1S + j];
      }
    }
    float h = acc + sw[LB1 + j];
    h = h > 0.f ? h : 0.f;
    o0 = o0 + h * sw[LW2 + 3 * j + 0];
    o1 = o1 + h * sw[LW2 + 3 * j + 1];
    o2 = o2 + h * sw[LW2 + 3 * j + 2];
  }
  o0 = o0 + sw[LB2 + 0];
  o1 = o1 + sw[LB2 + 1];
  o2 = o2 + sw[LB2 + 2];
  if (act == NFSP_ACT_RELU) {
    y[0] = o0 > 0.f ? o0 : 0.f;
    y[1] = o1 > 0.f ? o1 : 0.f;
    y[2] = o2 > 0.f ? o2 : 0.f;
  } else {
    const float m = fmaxf(fmaxf(o0, o1), o2);
    const float e0 = expf(o0 - m), e1 = expf(o1 - m), e2 = expf(o2 - m);
    const float s = (e0 + e1) + e2;
    y[0] = e0 / s; y[1] = e1 / s; y[2] = e2 / s;
  }
}

// ---------------------------------------------------------------------------
// k_rollout
// ---------------------------------------------------------------------------
struct RolloutArgs {
  int N;
  uint32_t k0, k1;
  uint32_t g_lo, g_hi;      // hand index of this rollout (per lane)
  float eta;
  unsigned quirks;
  const float* w;           // [2][3][NP]
  EngineDev* st;
  Staging S;
};

__global__ void __launch_bounds__(256) k_rollout(RolloutArgs A) {
  __shared__ __attribute__((aligned(16))) float sw[4 * NET_LDS];
  __shared__ unsigned s_act[2][3];
  __shared__ int s_rew[2];
  const int tid = threadIdx.x;
  // stage AR0, BR0, AR1, BR1 (padded W1 rows)
  for (int e = tid; e < 4 * nn::NP; e += blockDim.x) {
    const int net = e / nn::NP, q = e - net * nn::NP;
    const int agent = net >> 1, kind = net & 1;
    const float v = A.w[(agent * 3 + kind) * nn::NP + q];
    int d;
    if (q < nn::OB1) d = (q / nn::H) * W1S + (q % nn::H);
    else d = LB1 + (q - nn::OB1);
    sw[net * NET_LDS + d] = v;
  }
  if (tid < 6) s_act[tid / 3][tid % 3] = 0;
  if (tid < 2) s_rew[tid] = 0;
  __syncthreads();

  const int L = blockIdx.x * blockDim.x + tid;
  if (L < A.N) {
    const int N = A.N;
    const double eps0 = A.st->epsilon[0], eps1 = A.st->epsilon[1];
    const int dealer = (int)((L + A.g_lo) & 1u);
    const int lhand = 1 - dealer;
    uint8_t r0, r1, rp;
    {
      const u32x4 u = nfsp::philox4x32({(uint32_t)L, A.g_lo, A.g_hi, 0u}, A.k0, A.k1);
      nfsp::deal_from_draws(nfsp::below(u.x, 6), nfsp::below(u.y, 5), nfsp::below(u.z, 4), r0, r1, rp);
    }
    // eta draws, dealer first (main.py:36-45): 'a' (AR) iff random() > eta
    int polBR[2];
    {
      const u32x4 u = nfsp::philox4x32({(uint32_t)L, A.g_lo, A.g_hi, 1u}, A.k0, A.k1);
      polBR[dealer] = !(nfsp::u01(u.x) > A.eta);
      polBR[lhand] = !(nfsp::u01(u.y) > A.eta);
    }
    Hand h;
    nfsp::hand_reset(h, dealer, r0, r1, rp);
    const bool alias = (A.quirks & NFSP_QUIRK_ALIAS_RL) != 0;
    int nrl = 0, nsl = 0, nrlp[2] = {0, 0}, nslp[2] = {0, 0};
    int dec = 0;
    uint64_t act_pack = 0;       // 6 x 8-bit action counters (agent*3 + action)
    int rew_half[2] = {0, 0};
    // main.train scheduler (main.py:55-67) as phases of one while-iteration
    int phase = 0, rnd0 = 0;
    bool dT = false, lT = false, first = true;
    for (;;) {
      int who = -1;
      bool initial = false;
      while (!(dT && lT)) {
        if (phase == 0) {
          phase = 1;
          rnd0 = h.rnd;
          if (!dT) { who = dealer; initial = first; first = false; break; }
        } else if (phase == 1) {
          phase = 2;
          if (!lT) { who = lhand; break; }
        } else {
          phase = 0;
          if (rnd0 == h.rnd && !dT) { who = dealer; break; }
        }
      }
      if (who < 0) break;
      const int p = who;
      bool t = false;
      bool acted = false;
      // ---- Agent.play (agent/agent.py:130-156) ----
      if (!initial) {
        t = h.term != 0;
        const float r = t ? h.rew[p] : 0.f;
        const double asum = ((double)h.la[p][0] + (double)h.la[p][1]) + (double)h.la[p][2];
        if (asum != 0.0) {        // np.average(a) != 0 -> remember_for_rl
          const int k = nrl++;
          nrlp[p]++;
          const int rh = (int)(r * 2.0f);
          A.S.rl_s2[k * N + L] = nfsp::hand_obs(h, p);
          A.S.rl_meta[k * N + L] = ((uint32_t)rh & 0xFFu) | ((t ? 1u : 0u) << 8) | ((uint32_t)p << 9);
          if (!alias) {
            A.S.rl_s[k * N + L] = h.s[p];
            A.S.rl_a[(k * 3 + 0) * N + L] = h.la[p][0];
            A.S.rl_a[(k * 3 + 1) * N + L] = h.la[p][1];
            A.S.rl_a[(k * 3 + 2) * N + L] = h.la[p][2];
          }
        }
        if (t) rew_half[p] += (int)(r * 2.0f);
      }
      if (!t) {
        const uint32_t x = nfsp::hand_obs(h, p);
        float y[3];
        if (!polBR[p]) {
          fwd_lds(sw + (p * 2 + 0) * NET_LDS, x, NFSP_ACT_SOFTMAX, y);
        } else {
          const u32x4 u = nfsp::philox4x32({(uint32_t)L, A.g_lo, A.g_hi, 2u + (uint32_t)dec}, A.k0, A.k1);
          dec++;
          if ((double)nfsp::u01(u.x) > (p ? eps1 : eps0)) {
            fwd_lds(sw + (p * 2 + 1) * NET_LDS, x, NFSP_ACT_RELU, y);
          } else {                 // np.random.rand(1, 1, 3)
            y[0] = nfsp::u01(u.y); y[1] = nfsp::u01(u.z); y[2] = nfsp::u01(u.w);
          }
        }
        nfsp::hand_step(h, p, y[0], y[1], y[2]);
        acted = true;
        if (polBR[p]) {           // remember_best_response(s2, a_t)
          const int k = nsl++;
          nslp[p]++;
          A.S.sl_x[k * N + L] = x;
          A.S.sl_a[(k * 3 + 0) * N + L] = y[0];
          A.S.sl_a[(k * 3 + 1) * N + L] = y[1];
          A.S.sl_a[(k * 3 + 2) * N + L] = y[2];
          A.S.sl_meta[k * N + L] = (uint32_t)p | ((uint32_t)nrlp[p] << 8);
        }
        act_pack += 1ull << (8 * (p * 3 + nfsp::argmax3(y[0], y[1], y[2])));
      }
      (void)acted;
      if (p == dealer) dT = t; else lT = t;
    }
    A.S.fin_s[0 * N + L] = h.s[0];
    A.S.fin_s[1 * N + L] = h.s[1];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int c = 0; c < 3; ++c) A.S.fin_a[(q * 3 + c) * N + L] = h.la[q][c];
    A.S.counts[L] = (uint32_t)nrlp[0] | ((uint32_t)nrlp[1] << 4) | ((uint32_t)nslp[0] << 8) |
                    ((uint32_t)nslp[1] << 12);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const unsigned v = (unsigned)((act_pack >> (8 * q)) & 0xFFu);
      if (v) atomicAdd(&s_act[q / 3][q % 3], v);
    }
    if (rew_half[0]) atomicAdd(&s_rew[0], rew_half[0]);
    if (rew_half[1]) atomicAdd(&s_rew[1], rew_half[1]);
  }
  __syncthreads();
  if (tid < 6 && s_act[tid / 3][tid % 3])
    atomicAdd(&A.st->actions[tid / 3][tid % 3], (unsigned long long)s_act[tid / 3][tid % 3]);
  if (tid < 2 && s_rew[tid]) atomicAdd((unsigned long long*)&A.st->reward_half[tid],
                                       (unsigned long long)(long long)s_rew[tid]);
}

// ---------------------------------------------------------------------------
// scan of the 4 per-lane counts (canonical insert order)
// ---------------------------------------------------------------------------
__device__ inline unsigned long long unpack_counts(uint32_t c) {
  return (unsigned long long)(c & 15u) | ((unsigned long long)((c >> 4) & 15u) << 16) |
         ((unsigned long long)((c >> 8) & 15u) << 32) | ((unsigned long long)((c >> 12) & 15u) << 48);
}

__global__ void __launch_bounds__(256) k_scan1(const uint32_t* __restrict__ counts, int N,
                                               unsigned long long* __restrict__ local,
                                               uint4* __restrict__ block_sum) {
  __shared__ unsigned long long wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int L = blockIdx.x * 256 + tid;
  const unsigned long long v = L < N ? unpack_counts(counts[L]) : 0ull;
  // inclusive wave scan (fields never carry: block totals <= 256 * 4)
  unsigned long long x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  unsigned long long pre = 0;
  for (int k = 0; k < wv; ++k) pre += wsum[k];
  if (L < N) local[L] = pre + x - v;
  if (tid == 255) {
    const unsigned long long tot = pre + x;
    block_sum[blockIdx.x] = make_uint4((uint32_t)(tot & 0xFFFF), (uint32_t)((tot >> 16) & 0xFFFF),
                                       (uint32_t)((tot >> 32) & 0xFFFF), (uint32_t)(tot >> 48));
  }
}

__global__ void __launch_bounds__(1024) k_scan2(const uint4* __restrict__ block_sum, int nblk,
                                                uint4* __restrict__ block_base, EngineDev* st) {
  __shared__ uint4 part[1024];
  __shared__ uint4 carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = make_uint4(0, 0, 0, 0);
  __syncthreads();
  for (int c0 = 0; c0 < nblk; c0 += 1024) {
    const int i = c0 + tid;
    const uint4 v = i < nblk ? block_sum[i] : make_uint4(0, 0, 0, 0);
    part[tid] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      uint4 y = make_uint4(0, 0, 0, 0);
      if (tid >= d) y = part[tid - d];
      __syncthreads();
      if (tid >= d) {
        uint4 p = part[tid];
        p.x += y.x; p.y += y.y; p.z += y.z; p.w += y.w;
        part[tid] = p;
      }
      __syncthreads();
    }
    const uint4 inc = part[tid];
    const uint4 cb = carry;
    if (i < nblk)
      block_base[i] = make_uint4(cb.x + inc.x - v.x, cb.y + inc.y - v.y, cb.z + inc.z - v.z,
                                 cb.w + inc.w - v.w);
    __syncthreads();
    if (tid == 1023) carry = make_uint4(cb.x + inc.x, cb.y + inc.y, cb.z + inc.z, cb.w + inc.w);
    __syncthreads();
  }
  if (tid == 0) {
    st->last_rl[0] = carry.x;
    st->last_rl[1] = carry.y;
    st->last_sl[0] = carry.z;
    st->last_sl[1] = carry.w;
  }
}

// ---------------------------------------------------------------------------
// k_commit: staging -> M_RL logs (fp32 rows) and the pending SL lists
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_commit(int N, unsigned quirks, Staging S, Memories M,
                                                const EngineDev* __restrict__ st) {
  const int L = blockIdx.x * blockDim.x + threadIdx.x;
  if (L >= N) return;
  const uint32_t cnt = S.counts[L];
  const unsigned long long loc = S.local[L];
  const uint4 bb = S.block_base[L >> 8];
  const int64_t off_rl[2] = {(int64_t)bb.x + (int64_t)(loc & 0xFFFF),
                             (int64_t)bb.y + (int64_t)((loc >> 16) & 0xFFFF)};
  const int64_t off_sl[2] = {(int64_t)bb.z + (int64_t)((loc >> 32) & 0xFFFF),
                             (int64_t)bb.w + (int64_t)(loc >> 48)};
  const int nrl = (int)(cnt & 15u) + (int)((cnt >> 4) & 15u);
  const int nsl = (int)((cnt >> 8) & 15u) + (int)((cnt >> 12) & 15u);
  const bool alias = (quirks & NFSP_QUIRK_ALIAS_RL) != 0;
  int seen[2] = {0, 0};
  for (int k = 0; k < nrl; ++k) {
    const uint32_t meta = S.rl_meta[k * N + L];
    const int p = (meta >> 9) & 1;
    const int64_t pos = st->rl_total[p] + off_rl[p] + seen[p]++;
    const int64_t row = (int64_t)p * M.log_cap + pos % M.log_cap;
    const uint32_t sb = alias ? S.fin_s[p * N + L] : S.rl_s[k * N + L];
    const uint32_t s2b = S.rl_s2[k * N + L];
    float* srow = M.rl_s + row * nfsp::OBS;
    float* s2row = M.rl_s2 + row * nfsp::OBS;
#pragma unroll
    for (int f = 0; f < nfsp::OBS; ++f) {
      srow[f] = (float)((sb >> f) & 1u);
      s2row[f] = (float)((s2b >> f) & 1u);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c)
      M.rl_a[row * 3 + c] = alias ? S.fin_a[(p * 3 + c) * N + L] : S.rl_a[(k * 3 + c) * N + L];
    M.rl_r[row] = (float)(int8_t)(meta & 0xFFu) * 0.5f;
    M.rl_t[row] = (uint8_t)((meta >> 8) & 1u);
  }
  int sseen[2] = {0, 0};
  for (int k = 0; k < nsl; ++k) {
    const uint32_t meta = S.sl_meta[k * N + L];
    const int p = meta & 1;
    const int64_t li = (int64_t)p * M.pend_cap + off_sl[p] + sseen[p]++;
    M.pend_x[li] = S.sl_x[k * N + L];
#pragma unroll
    for (int c = 0; c < 3; ++c) M.pend_a[li * 3 + c] = S.sl_a[(k * 3 + c) * N + L];
    M.pend_pos[li] = st->rl_total[p] + off_rl[p] + (int64_t)(meta >> 8);
  }
}

// ---------------------------------------------------------------------------
// k_learner
// ---------------------------------------------------------------------------
struct LearnArgs {
  Memories M;
  EngineDev* st;
  float* w;                 // [2][3][NP]
  uint32_t k0, k1;
  int batch, per_update, target_every, epochs, fit_batch;
  float lr_br0, lr_ar;
  double gamma;
  unsigned quirks;
  int64_t rl_cap;
};

struct LearnSmem {
  float w[nn::NP];
  float tw[nn::NP];                         // target net (BR role)
  float x[MAX_LEARN_BATCH][nfsp::OBS];
  float t[MAX_LEARN_BATCH][nfsp::NA];
  uint32_t s2b[MAX_LEARN_BATCH];
  float a[MAX_LEARN_BATCH][nfsp::NA];
  float r[MAX_LEARN_BATCH];
  uint8_t term[MAX_LEARN_BATCH];
  int64_t cand[MAX_LEARN_BATCH];
  uint32_t key[MAX_LEARN_BATCH];
  int perm[4][MAX_LEARN_BATCH];
  double vmax[MAX_LEARN_BATCH];
  int flag;
  nn::StepScratch sc;
};

// `batch` distinct uniform rows of [lo, lo + win): parallel draw, redraw duplicates.
__device__ void sample_rows(LearnSmem& sm, int batch, int64_t lo, int64_t win, uint32_t stream,
                            uint32_t m_lo, uint32_t m_hi, uint32_t k0, uint32_t k1) {
  const int b = threadIdx.x;
  uint32_t attempt = 0;
  bool redraw = b < batch;
  for (;;) {
    if (redraw) {
      const u32x4 u = nfsp::philox4x32({stream, m_lo, m_hi, (attempt << 8) | (uint32_t)b}, k0, k1);
      const uint64_t r64 = ((uint64_t)u.x << 32) | u.y;
      sm.cand[b] = lo + (int64_t)(r64 % (uint64_t)win);
      attempt++;
    }
    __syncthreads();
    bool dup = false;
    if (b < batch)
      for (int k = 0; k < b; ++k) dup |= sm.cand[k] == sm.cand[b];
    redraw = dup;
    if (!__syncthreads_or(dup)) break;
  }
}

// epochs random permutations of [0, batch): rank of a unique random key
__device__ void draw_perms(LearnSmem& sm, int batch, int epochs, uint32_t stream, uint32_t m_lo,
                           uint32_t m_hi, uint32_t k0, uint32_t k1) {
  const int b = threadIdx.x;
  for (int e = 0; e < epochs; ++e) {
    if (b < batch) {
      const u32x4 u = nfsp::philox4x32({stream, m_lo, m_hi, ((uint32_t)e << 8) | (uint32_t)b}, k0, k1);
      sm.key[b] = (u.x & ~0xFFu) | (uint32_t)b;      // unique
    }
    __syncthreads();
    if (b < batch) {
      int rank = 0;
      for (int k = 0; k < batch; ++k) rank += sm.key[k] < sm.key[b];
      sm.perm[e][rank] = b;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_learner(LearnArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  LearnSmem& sm = *reinterpret_cast<LearnSmem*>(smem_raw);
  const int agent = blockIdx.x >> 1, role = blockIdx.x & 1;   // role 0 = AR, 1 = BR
  const int tid = threadIdx.x;
  EngineDev* st = A.st;
  const Memories& M = A.M;
  float* gw = A.w + (agent * 3 + (role ? 1 : 0)) * nn::NP;
  float* gtw = A.w + (agent * 3 + 2) * nn::NP;
  for (int i = tid; i < nn::NP; i += blockDim.x) {
    sm.w[i] = gw[i];
    if (role) sm.tw[i] = gtw[i];
  }
  const int64_t P0 = st->rl_total[agent];
  const int64_t n_rl = st->last_rl[agent];
  const int64_t c = A.per_update;
  const int64_t m_first = P0 / c + 1, m_last = (P0 + n_rl) / c;
  const int B = A.batch;
  const int dbg = agent * 2 + role;
  __syncthreads();

  if (role == 1) {
    // ---------------- update_best_response_network (agent/agent.py:209-253) ----------
    int64_t iteration = st->iteration[agent], tcount = st->target_count[agent];
    int64_t syncs = st->target_syncs[agent], nupd = st->br_updates[agent];
    double eps = st->epsilon[agent], temp = st->temp[agent], expl = st->expl[agent];
    float lr = st->lr_br[agent];
    for (int64_t m = m_first; m <= m_last; ++m) {
      const int64_t pm = m * c;
      const int64_t win = pm < A.rl_cap ? pm : A.rl_cap;
      if (win <= B) continue;                         // size() > minibatch_size
      iteration += 1;
      sample_rows(sm, B, pm - win, win, TAG_SAMPLE | (uint32_t)dbg, (uint32_t)m,
                  (uint32_t)(m >> 32), A.k0, A.k1);
      // gather the minibatch (rows of the agent's log)
      for (int e = tid; e < B * 32; e += blockDim.x) {
        const int b = e >> 5, f = e & 31;
        const int64_t row = (int64_t)agent * M.log_cap + sm.cand[b] % M.log_cap;
        if (f < nfsp::OBS) sm.x[b][f] = M.rl_s[row * nfsp::OBS + f];
        else if (f == 30) sm.r[b] = M.rl_r[row];
        else sm.term[b] = M.rl_t[row];
      }
      for (int e = tid; e < B * 3; e += blockDim.x)
        sm.a[e / 3][e % 3] = M.rl_a[((int64_t)agent * M.log_cap + sm.cand[e / 3] % M.log_cap) * 3 + e % 3];
      if (tid < B) {
        const int64_t row = (int64_t)agent * M.log_cap + sm.cand[tid] % M.log_cap;
        uint32_t bits = 0;
        for (int f = 0; f < nfsp::OBS; ++f) bits |= (M.rl_s2[row * nfsp::OBS + f] != 0.f ? 1u : 0u) << f;
        sm.s2b[tid] = bits;
      }
      __syncthreads();
      // targets with the target net (agent/agent.py:219-238)
      if (tid < B) {
        float q[3], qn[3], xs2[nfsp::OBS];
        for (int f = 0; f < nfsp::OBS; ++f) xs2[f] = (float)((sm.s2b[tid] >> f) & 1u);
        nn::forward_relu_row(sm.tw, sm.x[tid], q);
        nn::forward_relu_row(sm.tw, xs2, qn);
        sm.t[tid][0] = q[0]; sm.t[tid][1] = q[1]; sm.t[tid][2] = q[2];
        const float qmax = fmaxf(fmaxf(qn[0], qn[1]), qn[2]);
        const bool terminal = !(A.quirks & NFSP_QUIRK_TERMINAL_BOOTSTRAP) && sm.term[tid];
        sm.vmax[tid] = terminal ? (double)sm.r[tid] : (double)sm.r[tid] + A.gamma * (double)qmax;
      }
      __syncthreads();
      if (tid == 0) {
        double acc = 0.0;
        for (int k = 0; k < B; ++k) acc += (double)fmaxf(fmaxf(sm.t[k][0], sm.t[k][1]), sm.t[k][2]);
        expl = acc / B;
        for (int k = 0; k < B; ++k) {
          const int row = (A.quirks & NFSP_QUIRK_ROW0_TARGET) ? 0 : k;
          sm.t[row][nfsp::argmax3(sm.a[k][0], sm.a[k][1], sm.a[k][2])] = (float)sm.vmax[k];
        }
      }
      draw_perms(sm, B, A.epochs, TAG_PERM | (uint32_t)dbg, (uint32_t)m, (uint32_t)(m >> 32), A.k0, A.k1);
      for (int e = 0; e < A.epochs; ++e)
        for (int b0 = 0; b0 < B; b0 += A.fit_batch)
          nn::sgd_step(sm.w, &sm.x[0][0], &sm.t[0][0], &sm.perm[e][b0], min(A.fit_batch, B - b0),
                       NFSP_ACT_RELU, lr, sm.sc);
      // schedules (agent/agent.py:245-253, 266-273)
      iteration += 1;
      temp = 1.0 / (1.0 + 0.02 * sqrt((double)iteration));
      if (tcount % A.target_every == 0) {
        for (int i = tid; i < nn::NP; i += blockDim.x) sm.tw[i] = sm.w[i];
        syncs++;
      }
      tcount++;
      lr = (float)(A.lr_br0 / (1.0 + 0.003 * sqrt((double)iteration)));
      eps = eps / (double)iteration;
      nupd++;
      if (tid < B) {
        A.M.dbg_rows[dbg * B + tid] = sm.cand[tid];
        for (int e = 0; e < A.epochs; ++e) A.M.dbg_perms[(dbg * A.epochs + e) * B + tid] = sm.perm[e][tid];
      }
      __syncthreads();
    }
    for (int i = tid; i < nn::NP; i += blockDim.x) {
      gw[i] = sm.w[i];
      gtw[i] = sm.tw[i];
    }
    if (tid == 0) {
      st->iteration[agent] = iteration;
      st->target_count[agent] = tcount;
      st->target_syncs[agent] = syncs;
      st->br_updates[agent] = nupd;
      st->epsilon[agent] = eps;
      st->temp[agent] = temp;
      st->expl[agent] = expl;
      st->lr_br[agent] = lr;
      st->rl_total[agent] = P0 + n_rl;
    }
  } else {
    // ---------------- update_avg_response_network (agent/agent.py:255-264) ----------
    int64_t sl_total = st->sl_total[agent], sl_count = st->sl_count[agent];
    int64_t nupd = st->ar_updates[agent];
    const int64_t n_sl = st->last_sl[agent];
    const int64_t* pend_pos = M.pend_pos + (int64_t)agent * M.pend_cap;
    const uint32_t* pend_x = M.pend_x + (int64_t)agent * M.pend_cap;
    const float* pend_a = M.pend_a + (int64_t)agent * M.pend_cap * 3;
    float* res_s = M.sl_s + (int64_t)agent * M.sl_cap * nfsp::OBS;
    float* res_a = M.sl_a + (int64_t)agent * M.sl_cap * 3;
    int64_t cur = 0;
    // reservoir inserts (utils/ReservoirBuffer.py:18-28) in stream order; every lane
    // computes the slot, lane f writes field f, so a later insert to the same slot lands
    // after the earlier one in that lane's program order (no barrier needed).
    auto apply_until = [&](int64_t limit_pos, bool all) {
      while (cur < n_sl && (all || pend_pos[cur] <= limit_pos)) {
        int64_t slot;
        if (sl_count < M.sl_cap) {
          slot = sl_count++;
        } else {
          const u32x4 u = nfsp::philox4x32({TAG_RES | (uint32_t)agent, (uint32_t)sl_total,
                                            (uint32_t)(sl_total >> 32), 0u}, A.k0, A.k1);
          const uint64_t r64 = ((uint64_t)u.x << 32) | u.y;
          const int64_t j = 1 + (int64_t)(r64 % (uint64_t)M.sl_cap);     // randrange(1, N+1)
          slot = j < M.sl_cap ? j : -1;
        }
        sl_total++;
        if (slot >= 0) {
          if (tid < nfsp::OBS) res_s[slot * nfsp::OBS + tid] = (float)((pend_x[cur] >> tid) & 1u);
          else if (tid < nfsp::OBS + 3) res_a[slot * 3 + tid - nfsp::OBS] = pend_a[cur * 3 + tid - nfsp::OBS];
        }
        cur++;
      }
    };
    for (int64_t m = m_first; m <= m_last; ++m) {
      const int64_t pm = m * c;
      apply_until(pm, false);
      if (sl_count <= B) continue;
      __threadfence_block();
      __syncthreads();
      sample_rows(sm, B, 0, sl_count, TAG_SAMPLE | (uint32_t)dbg, (uint32_t)m, (uint32_t)(m >> 32),
                  A.k0, A.k1);
      __threadfence();   // the reservoir rows just written by this block's lanes
      __syncthreads();
      for (int e = tid; e < B * 33; e += blockDim.x) {
        const int b = e / 33, f = e - b * 33;
        const int64_t row = sm.cand[b];
        if (f < nfsp::OBS) sm.x[b][f] = res_s[row * nfsp::OBS + f];
        else sm.t[b][f - nfsp::OBS] = res_a[row * 3 + f - nfsp::OBS];
      }
      __syncthreads();
      draw_perms(sm, B, A.epochs, TAG_PERM | (uint32_t)dbg, (uint32_t)m, (uint32_t)(m >> 32), A.k0, A.k1);
      for (int e = 0; e < A.epochs; ++e)
        for (int b0 = 0; b0 < B; b0 += A.fit_batch)
          nn::sgd_step(sm.w, &sm.x[0][0], &sm.t[0][0], &sm.perm[e][b0], min(A.fit_batch, B - b0),
                       NFSP_ACT_SOFTMAX, A.lr_ar, sm.sc);
      nupd++;
      if (tid < B) {
        A.M.dbg_rows[dbg * B + tid] = sm.cand[tid];
        for (int e = 0; e < A.epochs; ++e) A.M.dbg_perms[(dbg * A.epochs + e) * B + tid] = sm.perm[e][tid];
      }
      __syncthreads();
    }
    apply_until(0, true);
    for (int i = tid; i < nn::NP; i += blockDim.x) gw[i] = sm.w[i];
    if (tid == 0) {
      st->sl_total[agent] = sl_total;
      st->sl_count[agent] = sl_count;
      st->ar_updates[agent] = nupd;
    }
  }
}

__global__ void k_finish_rollout(EngineDev* st, int64_t N) {
  if (threadIdx.x == 0) {
    st->hands += N;
    st->rollouts += 1;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct nfsp_engine {
  nfsp_ctx* ctx = nullptr;
  nfsp_engine_cfg cfg{};
  int N = 0;
  int nblk = 0;
  uint64_t rollouts = 0;
  bool pending_update = false;
  float* w = nullptr;
  EngineDev* st = nullptr;
  Staging S{};
  Memories M{};
  std::vector<void*> allocs;
  // optional per-kernel timing: (kernel id, start, stop) event triples on the ctx stream
  bool timing = false;
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> marks;
};

enum { KT_ROLLOUT = 0, KT_SCAN = 1, KT_COMMIT = 2, KT_LEARNER = 3, KT_N = 4 };

static hipEvent_t eng_event(nfsp_engine* e) {
  if (!e->pool.empty()) {
    hipEvent_t ev = e->pool.back();
    e->pool.pop_back();
    return ev;
  }
  hipEvent_t ev = nullptr;
  (void)hipEventCreate(&ev);
  return ev;
}

// RAII bracket: records start/stop events around one kernel launch when timing is on
struct KTimer {
  nfsp_engine* e;
  int id;
  hipEvent_t a = nullptr, b = nullptr;
  KTimer(nfsp_engine* e_, int id_) : e(e_), id(id_) {
    if (e->timing) {
      a = eng_event(e);
      (void)hipEventRecord(a, e->ctx->stream);
    }
  }
  ~KTimer() {
    if (e->timing) {
      b = eng_event(e);
      (void)hipEventRecord(b, e->ctx->stream);
      e->marks.push_back({id, {a, b}});
    }
  }
};

static int eng_alloc(nfsp_engine* e, void** p, size_t bytes) {
  hipError_t r = hipMalloc(p, bytes);
  if (r != hipSuccess) return nfsp::hip_fail(r, "nfsp_engine_create: hipMalloc");
  e->allocs.push_back(*p);
  r = hipMemsetAsync(*p, 0, bytes, e->ctx->stream);
  if (r != hipSuccess) return nfsp::hip_fail(r, "nfsp_engine_create: hipMemset");
  return NFSP_OK;
}

#define EALLOC(ptr, bytes)                                                    \
  do {                                                                        \
    int _rc = eng_alloc(e, (void**)&(ptr), (size_t)(bytes));                  \
    if (_rc != NFSP_OK) { nfsp_engine_destroy(e); return _rc; }               \
  } while (0)

extern "C" int nfsp_engine_default_cfg(nfsp_engine_cfg* c) {
  NFSP_REQUIRE(c, "null argument");
  c->n_lanes = 65536;
  c->hidden = 64;
  c->rl_capacity = 40000;
  c->sl_capacity = 40000;
  c->batch = 128;
  c->inserts_per_update = 128;
  c->target_every = 150;
  c->epochs = 2;
  c->fit_batch = 32;
  c->quirks = NFSP_QUIRKS_REFERENCE;
  c->eta = 0.1f;
  c->lr_br = 0.05f;
  c->lr_ar = 0.1f;
  c->gamma = 0.95;
  c->epsilon = 0.06;
  c->seed = 1234;
  return NFSP_OK;
}

extern "C" int nfsp_engine_destroy(nfsp_engine* e) {
  if (!e) return NFSP_OK;
  if (e->ctx) (void)hipStreamSynchronize(e->ctx->stream);
  for (void* p : e->allocs) (void)hipFree(p);
  for (auto& m : e->marks) {
    e->pool.push_back(m.second.first);
    e->pool.push_back(m.second.second);
  }
  for (hipEvent_t ev : e->pool) (void)hipEventDestroy(ev);
  delete e;
  return NFSP_OK;
}

extern "C" int nfsp_engine_create(nfsp_ctx* ctx, const nfsp_engine_cfg* cfg, nfsp_engine** out) {
  NFSP_REQUIRE(ctx && cfg && out, "null argument");
  NFSP_REQUIRE(cfg->hidden == nn::H, "only hidden == 64 is built");
  NFSP_REQUIRE(cfg->n_lanes > 0 && cfg->n_lanes < (1 << 24), "n_lanes must be in [1, 2^24)");
  NFSP_REQUIRE(cfg->batch >= 1 && cfg->batch <= MAX_LEARN_BATCH, "batch must be in [1, 128]");
  NFSP_REQUIRE(cfg->fit_batch >= 1 && cfg->fit_batch <= nn::MAXB, "fit_batch must be in [1, 64]");
  NFSP_REQUIRE(cfg->epochs >= 0 && cfg->epochs <= 4, "epochs must be in [0, 4]");
  NFSP_REQUIRE(cfg->rl_capacity > cfg->batch && cfg->sl_capacity > cfg->batch,
               "capacities must exceed the batch");
  NFSP_REQUIRE(cfg->sl_capacity < (1ll << 40) && cfg->rl_capacity < (1ll << 40), "capacity too large");
  NFSP_REQUIRE(cfg->inserts_per_update >= 1 && cfg->target_every >= 1, "bad cadence");
  *out = nullptr;
  nfsp_engine* e = new nfsp_engine();
  e->ctx = ctx;
  e->cfg = *cfg;
  e->N = cfg->n_lanes;
  e->nblk = (e->N + 255) / 256;
  const int64_t N = e->N;
  EALLOC(e->w, sizeof(float) * 6 * nn::NP);
  EALLOC(e->st, sizeof(EngineDev));
  EALLOC(e->S.rl_s2, 4 * MAXREC * N);
  EALLOC(e->S.rl_meta, 4 * MAXREC * N);
  EALLOC(e->S.rl_s, 4 * MAXREC * N);
  EALLOC(e->S.rl_a, 4 * 3 * MAXREC * N);
  EALLOC(e->S.sl_x, 4 * MAXREC * N);
  EALLOC(e->S.sl_a, 4 * 3 * MAXREC * N);
  EALLOC(e->S.sl_meta, 4 * MAXREC * N);
  EALLOC(e->S.fin_s, 4 * 2 * N);
  EALLOC(e->S.fin_a, 4 * 6 * N);
  EALLOC(e->S.counts, 4 * N);
  EALLOC(e->S.local, 8 * N);
  EALLOC(e->S.block_sum, sizeof(uint4) * e->nblk);
  EALLOC(e->S.block_base, sizeof(uint4) * e->nblk);
  // an agent makes <= 4 decisions per hand: <= 4 RL and <= 4 SL records per lane
  e->M.log_cap = cfg->rl_capacity + 4 * N;
  e->M.sl_cap = cfg->sl_capacity;
  e->M.pend_cap = 4 * N;
  const int64_t lc = 2 * e->M.log_cap, sc = 2 * e->M.sl_cap, pc = 2 * e->M.pend_cap;
  EALLOC(e->M.rl_s, 4 * nfsp::OBS * lc);
  EALLOC(e->M.rl_s2, 4 * nfsp::OBS * lc);
  EALLOC(e->M.rl_a, 4 * 3 * lc);
  EALLOC(e->M.rl_r, 4 * lc);
  EALLOC(e->M.rl_t, lc);
  EALLOC(e->M.sl_s, 4 * nfsp::OBS * sc);
  EALLOC(e->M.sl_a, 4 * 3 * sc);
  EALLOC(e->M.pend_x, 4 * pc);
  EALLOC(e->M.pend_a, 4 * 3 * pc);
  EALLOC(e->M.pend_pos, 8 * pc);
  EALLOC(e->M.dbg_rows, 8 * 4 * cfg->batch);
  EALLOC(e->M.dbg_perms, 4 * 4 * 4 * cfg->batch);
  EngineDev h{};
  for (int a = 0; a < 2; ++a) {
    h.epsilon[a] = cfg->epsilon;
    h.temp[a] = 1.0;
    h.lr_br[a] = cfg->lr_br;
  }
  hipError_t r = hipMemcpyAsync(e->st, &h, sizeof(h), hipMemcpyHostToDevice, ctx->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(ctx->stream);
  if (r != hipSuccess) {
    nfsp_engine_destroy(e);
    return nfsp::hip_fail(r, "nfsp_engine_create: init state");
  }
  *out = e;
  return NFSP_OK;
}

extern "C" int nfsp_engine_weights(nfsp_engine* e, int agent, int net, float** dev_w) {
  NFSP_REQUIRE(e && dev_w, "null argument");
  NFSP_REQUIRE((agent == 0 || agent == 1) && net >= 0 && net <= 2, "bad agent/net");
  *dev_w = e->w + (agent * 3 + net) * nn::NP;
  return NFSP_OK;
}

extern "C" int nfsp_rollout(nfsp_engine* e) {
  NFSP_REQUIRE(e, "null argument");
  NFSP_REQUIRE(!e->pending_update, "nfsp_engine_update must consume the previous rollout first");
  hipStream_t s = e->ctx->stream;
  RolloutArgs A;
  A.N = e->N;
  A.k0 = (uint32_t)e->cfg.seed;
  A.k1 = (uint32_t)(e->cfg.seed >> 32);
  A.g_lo = (uint32_t)e->rollouts;
  A.g_hi = (uint32_t)(e->rollouts >> 32);
  A.eta = e->cfg.eta;
  A.quirks = e->cfg.quirks;
  A.w = e->w;
  A.st = e->st;
  A.S = e->S;
  {
    KTimer kt(e, KT_ROLLOUT);
    k_rollout<<<e->nblk, 256, 0, s>>>(A);
  }
  NFSP_LAUNCHED("k_rollout");
  {
    KTimer kt(e, KT_SCAN);
    k_scan1<<<e->nblk, 256, 0, s>>>(e->S.counts, e->N, e->S.local, e->S.block_sum);
    k_scan2<<<1, 1024, 0, s>>>(e->S.block_sum, e->nblk, e->S.block_base, e->st);
  }
  NFSP_LAUNCHED("k_scan");
  {
    KTimer kt(e, KT_COMMIT);
    k_commit<<<e->nblk, 256, 0, s>>>(e->N, e->cfg.quirks, e->S, e->M, e->st);
  }
  NFSP_LAUNCHED("k_commit");
  k_finish_rollout<<<1, 64, 0, s>>>(e->st, e->N);
  NFSP_LAUNCHED("k_finish_rollout");
  e->rollouts++;
  e->pending_update = true;
  return NFSP_OK;
}

extern "C" int nfsp_engine_update(nfsp_engine* e) {
  NFSP_REQUIRE(e, "null argument");
  if (!e->pending_update) return NFSP_OK;
  LearnArgs A;
  A.M = e->M;
  A.st = e->st;
  A.w = e->w;
  A.k0 = (uint32_t)e->cfg.seed;
  A.k1 = (uint32_t)(e->cfg.seed >> 32);
  A.batch = e->cfg.batch;
  A.per_update = e->cfg.inserts_per_update;
  A.target_every = e->cfg.target_every;
  A.epochs = e->cfg.epochs;
  A.fit_batch = e->cfg.fit_batch;
  A.lr_br0 = e->cfg.lr_br;
  A.lr_ar = e->cfg.lr_ar;
  A.gamma = e->cfg.gamma;
  A.quirks = e->cfg.quirks;
  A.rl_cap = e->cfg.rl_capacity;
  static bool attr_set = false;
  if (!attr_set) {
    NFSP_HIP(hipFuncSetAttribute((const void*)k_learner, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)sizeof(LearnSmem)));
    attr_set = true;
  }
  {
    KTimer kt(e, KT_LEARNER);
    k_learner<<<4, 256, sizeof(LearnSmem), e->ctx->stream>>>(A);
  }
  NFSP_LAUNCHED("k_learner");
  e->pending_update = false;
  return NFSP_OK;
}

extern "C" int nfsp_engine_step(nfsp_engine* e) {
  int rc = nfsp_rollout(e);
  if (rc != NFSP_OK) return rc;
  return nfsp_engine_update(e);
}

extern "C" int nfsp_engine_get_stats(nfsp_engine* e, nfsp_engine_stats* out) {
  NFSP_REQUIRE(e && out, "null argument");
  EngineDev h;
  NFSP_HIP(hipMemcpyAsync(&h, e->st, sizeof(h), hipMemcpyDeviceToHost, e->ctx->stream));
  NFSP_HIP(hipStreamSynchronize(e->ctx->stream));
  *out = nfsp_engine_stats{};
  out->hands = h.hands;
  out->rollouts = h.rollouts;
  for (int a = 0; a < 2; ++a) {
    // before nfsp_engine_update has consumed a rollout its inserts are already in M_RL
    const int64_t rl_total = h.rl_total[a] + (e->pending_update ? h.last_rl[a] : 0);
    out->rl_total[a] = rl_total;
    out->sl_total[a] = h.sl_total[a];
    out->rl_size[a] = rl_total < e->cfg.rl_capacity ? rl_total : e->cfg.rl_capacity;
    out->sl_size[a] = h.sl_count[a];
    out->last_rl[a] = h.last_rl[a];
    out->last_sl[a] = h.last_sl[a];
    out->br_updates[a] = h.br_updates[a];
    out->ar_updates[a] = h.ar_updates[a];
    out->iteration[a] = h.iteration[a];
    out->target_syncs[a] = h.target_syncs[a];
    for (int k = 0; k < 3; ++k) out->actions[a][k] = (int64_t)h.actions[a][k];
    out->reward[a] = 0.5 * (double)h.reward_half[a];
    out->epsilon[a] = h.epsilon[a];
    out->temp[a] = h.temp[a];
    out->lr_br[a] = h.lr_br[a];
    out->exploitability[a] = h.expl[a];
  }
  return NFSP_OK;
}

extern "C" int nfsp_engine_memories(nfsp_engine* e, int agent, nfsp_records* rl, int64_t* log_cap,
                                    nfsp_records* sl, uint32_t** px, float** pa, int64_t** ppos) {
  NFSP_REQUIRE(e && (agent == 0 || agent == 1), "bad argument");
  const int64_t lo = (int64_t)agent * e->M.log_cap;
  if (rl) {
    rl->s = e->M.rl_s + lo * nfsp::OBS;
    rl->a = e->M.rl_a + lo * 3;
    rl->r = e->M.rl_r + lo;
    rl->s2 = e->M.rl_s2 + lo * nfsp::OBS;
    rl->t = e->M.rl_t + lo;
    rl->cap = e->M.log_cap;
  }
  if (log_cap) *log_cap = e->M.log_cap;
  const int64_t so = (int64_t)agent * e->M.sl_cap;
  if (sl) {
    sl->s = e->M.sl_s + so * nfsp::OBS;
    sl->a = e->M.sl_a + so * 3;
    sl->r = nullptr;
    sl->s2 = nullptr;
    sl->t = nullptr;
    sl->cap = e->M.sl_cap;
  }
  const int64_t po = (int64_t)agent * e->M.pend_cap;
  if (px) *px = e->M.pend_x + po;
  if (pa) *pa = e->M.pend_a + po * 3;
  if (ppos) *ppos = e->M.pend_pos + po;
  return NFSP_OK;
}

extern "C" int nfsp_engine_last_update(nfsp_engine* e, int agent, int role, int64_t** rows,
                                       int32_t** perms) {
  NFSP_REQUIRE(e && (agent == 0 || agent == 1) && (role == 0 || role == 1), "bad argument");
  const int d = agent * 2 + role;
  if (rows) *rows = e->M.dbg_rows + d * e->cfg.batch;
  if (perms) *perms = e->M.dbg_perms + d * e->cfg.epochs * e->cfg.batch;
  return NFSP_OK;
}

extern "C" int nfsp_engine_set_timing(nfsp_engine* e, int on) {
  NFSP_REQUIRE(e, "null argument");
  e->timing = on != 0;
  return NFSP_OK;
}

extern "C" int nfsp_engine_get_timings(nfsp_engine* e, double* ms, int64_t* launches) {
  NFSP_REQUIRE(e && ms && launches, "null argument");
  NFSP_HIP(hipStreamSynchronize(e->ctx->stream));
  for (int k = 0; k < KT_N; ++k) { ms[k] = 0.0; launches[k] = 0; }
  for (auto& m : e->marks) {
    float t = 0.f;
    NFSP_HIP(hipEventElapsedTime(&t, m.second.first, m.second.second));
    ms[m.first] += t;
    launches[m.first] += 1;
    e->pool.push_back(m.second.first);
    e->pool.push_back(m.second.second);
  }
  e->marks.clear();
  return NFSP_OK;
}
