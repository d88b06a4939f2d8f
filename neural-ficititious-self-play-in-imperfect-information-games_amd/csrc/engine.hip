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

#include <cmath>
#include <utility>
#include <vector>

#include "engine_internal.h"

using nfsp::Hand;
using nfsp::u32x4;
namespace nn = nfsp::nn;
using namespace nfsp::eng;

namespace {

// ---------------------------------------------------------------------------
// k_rollout
// ---------------------------------------------------------------------------
struct RolloutArgs {
  int N;                    // lanes of this rollout (one slice)
  uint32_t lane0;           // global id of the slice's first lane (cfg.slices)
  uint32_t k0, k1;
  uint32_t g_lo, g_hi;      // hand index of this rollout (per lane)
  float eta;
  unsigned quirks;
  int game;                 // nfsp::GAME_LEDUC | GAME_KUHN
  int eps_by_value;         // 1: eps_v (the host's schedule mirror); 0: st->epsilon (groups)
  double eps_v[2];
  const float* w;           // [2][3][NP]: the acting nets (the engine's, or a snapshot)
  EngineDev* st;
  Staging S;
};

// One replica's rollout / commit arguments in an engine group's device table.
struct GroupRollout {
  RolloutArgs A;
  Memories M;
  int nblk;
  float* snap;          // slice_lag 2: the replica's snapshots [2][2][3][NP] (else null)
  double* snap_eps;     //   and their epsilons [2][2], on device
};

__device__ __forceinline__ void rollout_body(const RolloutArgs& A, int bx) {
  __shared__ __attribute__((aligned(16))) float sw[4 * NET_LDS];
  __shared__ unsigned s_act[2][3];
  __shared__ int s_rew[2];
  const int tid = threadIdx.x;
  // stage AR0, BR0, AR1, BR1 (fwd_lds layout: padded W1 rows, {b1, W2} per hidden unit)
  for (int e = tid; e < 4 * nn::NP; e += blockDim.x) {
    const int net = e / nn::NP, q = e - net * nn::NP;
    const int agent = net >> 1, kind = net & 1;
    sw[net * NET_LDS + net_lds_index(q)] = A.w[(agent * 3 + kind) * nn::NP + q];
  }
  for (int e = tid; e < 4 * nn::H; e += blockDim.x) sw[(e / nn::H) * NET_LDS + ZROW + e % nn::H] = 0.f;
  if (tid < 6) s_act[tid / 3][tid % 3] = 0;
  if (tid < 2) s_rew[tid] = 0;
  __syncthreads();

  const int L = bx * blockDim.x + tid;     // staging index (lane within the slice)
  if (L < A.N) {
    const int N = A.N;
    const uint32_t LG = A.lane0 + (uint32_t)L;   // global lane id: Philox counters, dealer
    const double eps0 = A.eps_by_value ? A.eps_v[0] : A.st->epsilon[0];
    const double eps1 = A.eps_by_value ? A.eps_v[1] : A.st->epsilon[1];
    const int dealer = (int)((LG + A.g_lo) & 1u);
    const int lhand = 1 - dealer;
    uint8_t r0, r1, rp = 0;
    {
      const u32x4 u = nfsp::philox4x32({LG, A.g_lo, A.g_hi, 0u}, A.k0, A.k1);
      if (A.game == nfsp::GAME_KUHN)
        nfsp::deal_kuhn(nfsp::below(u.x, 3), nfsp::below(u.y, 2), r0, r1);
      else
        nfsp::deal_from_draws(nfsp::below(u.x, 6), nfsp::below(u.y, 5), nfsp::below(u.z, 4), r0, r1, rp);
    }
    // eta draws, dealer first (main.py:36-45): 'a' (AR) iff random() > eta
    int polBR[2];
    {
      const u32x4 u = nfsp::philox4x32({LG, A.g_lo, A.g_hi, 1u}, A.k0, A.k1);
      polBR[dealer] = !(nfsp::u01(u.x) > A.eta);
      polBR[lhand] = !(nfsp::u01(u.y) > A.eta);
    }
    Hand h;
    nfsp::hand_reset(h, dealer, r0, r1, rp, A.game);
    const bool alias = (A.quirks & NFSP_QUIRK_ALIAS_RL) != 0;
    int nrl = 0, nsl = 0, nrlp[2] = {0, 0}, nslp[2] = {0, 0};
    int dec = 0, dec_ar = 0;
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
        // one forward for the whole wave: the net (AR or BR of seat p) is a per-lane LDS
        // base, so lanes acting with different nets share the instructions instead of the
        // wave running an AR and a BR forward one after the other
        const bool br = polBR[p] != 0;
        bool fwd = true;
        u32x4 ub{};
        if (br) {                  // act_best_response's eps draw (agent/agent.py:124-128)
          ub = nfsp::philox4x32({LG, A.g_lo, A.g_hi, 2u + (uint32_t)dec}, A.k0, A.k1);
          dec++;
          fwd = (double)nfsp::u01(ub.x) > (p ? eps1 : eps0);
        }
        if (fwd) {
          fwd_lds(sw + (p * 2 + (br ? 1 : 0)) * NET_LDS, x, br ? br_act(A.quirks) : NFSP_ACT_SOFTMAX, y);
        } else {                   // np.random.rand(1, 1, 3)
          y[0] = nfsp::u01(ub.y); y[1] = nfsp::u01(ub.z); y[2] = nfsp::u01(ub.w);
        }
        if (!br && (A.quirks & NFSP_EXT_SAMPLE_AR)) {   // sample the average policy (textbook NFSP)
          const u32x4 u = nfsp::philox4x32({LG, A.g_lo, A.g_hi, 0x80000000u + (uint32_t)dec_ar},
                                           A.k0, A.k1);
          dec_ar++;
          const float r = nfsp::u01(u.x);
          const int v = r < y[0] ? 0 : (r < y[0] + y[1] ? 1 : 2);
          y[0] = v == 0 ? 1.f : 0.f; y[1] = v == 1 ? 1.f : 0.f; y[2] = v == 2 ? 1.f : 0.f;
        }
        nfsp::hand_step(h, p, y[0], y[1], y[2]);
        acted = true;
        if (polBR[p]) {           // remember_best_response(s2, a_t)
          const int k = nsl++;
          nslp[p]++;
          A.S.sl_x[k * N + L] = x;
          if (A.quirks & NFSP_EXT_SL_ONEHOT) {   // the action taken (textbook NFSP)
            const int v = nfsp::argmax3(y[0], y[1], y[2]);
            A.S.sl_a[(k * 3 + 0) * N + L] = v == 0 ? 1.f : 0.f;
            A.S.sl_a[(k * 3 + 1) * N + L] = v == 1 ? 1.f : 0.f;
            A.S.sl_a[(k * 3 + 2) * N + L] = v == 2 ? 1.f : 0.f;
          } else {
            A.S.sl_a[(k * 3 + 0) * N + L] = y[0];
            A.S.sl_a[(k * 3 + 1) * N + L] = y[1];
            A.S.sl_a[(k * 3 + 2) * N + L] = y[2];
          }
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

// One engine's rollout runs 512-lane workgroups (8 waves): a 65,536-lane slice then takes
// 128 CUs instead of all 256.  Each rollout workgroup holds 38 KB of LDS (the four nets), so a
// CU running one cannot take a chain workgroup (150 KB, chain3.h CHAIN_LDS); with every CU
// holding one, a BR chain launched during the rollout waited for it to drain (~86 us, once
// per slice on agent 0's BR stream: 1.3 ms per C3 step).
constexpr int ROLLOUT_WG = 512;
__global__ void __launch_bounds__(ROLLOUT_WG) k_rollout(RolloutArgs A) { rollout_body(A, blockIdx.x); }

// engine groups: blockIdx.y = replica (the rollout index is the same for every replica)
// par >= 0 (slice_lag 2): the replica acts with its snapshot `par` and that snapshot's epsilon
__global__ void __launch_bounds__(256) k_rollout_g(const GroupRollout* __restrict__ tab, uint32_t g_lo,
                                                   uint32_t g_hi, uint32_t lane0, int par) {
  const GroupRollout& T = tab[blockIdx.y];
  RolloutArgs A = T.A;
  A.g_lo = g_lo;
  A.g_hi = g_hi;
  A.lane0 = lane0;
  if (par >= 0) {
    A.w = T.snap + (size_t)par * 6 * nn::NP;
    A.eps_by_value = 1;
    A.eps_v[0] = T.snap_eps[2 * par + 0];
    A.eps_v[1] = T.snap_eps[2 * par + 1];
  }
  rollout_body(A, blockIdx.x);
}

// slice_lag 2 in a group: replica blockIdx.y's nets and epsilon -> its snapshot `par` (-1: both
// parities, a step's start), after the slice's learner (and exchange) on the same stream
__global__ void __launch_bounds__(256) k_group_snap(const GroupRollout* __restrict__ tab, int par) {
  const GroupRollout& T = tab[blockIdx.y];
  const int p0 = par < 0 ? 0 : par, p1 = par < 0 ? 1 : par;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 6 * nn::NP; i += gridDim.x * blockDim.x) {
    const float v = T.A.w[i];
    for (int p = p0; p <= p1; ++p) T.snap[(size_t)p * 6 * nn::NP + i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2)
    for (int p = p0; p <= p1; ++p) T.snap_eps[2 * p + threadIdx.x] = T.A.st->epsilon[threadIdx.x];
}

// The same for a pipelined group step (nfsp_group_step, slice_lag 2): the nets of one learner
// stream only, on that stream right after its chains -- part 0: both agents' AR nets (after
// the AR chains and the exchange); part 1: the BR and target nets and the epsilons (after the
// BR chains and their k_finalize).  Together the two write what k_group_snap writes.
__global__ void __launch_bounds__(256) k_group_snap_part(const GroupRollout* __restrict__ tab, int par, int part) {
  const GroupRollout& T = tab[blockIdx.y];
  float* const dst = T.snap + (size_t)par * 6 * nn::NP;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 6 * nn::NP; i += gridDim.x * blockDim.x) {
    const int net = (i / nn::NP) % 3;            // [agent][AR, BR, target][NP]
    if ((net == 0) == (part == 0)) dst[i] = T.A.w[i];
  }
  if (part == 1 && blockIdx.x == 0 && threadIdx.x < 2) T.snap_eps[2 * par + threadIdx.x] = T.A.st->epsilon[threadIdx.x];
}

// ---------------------------------------------------------------------------
// scan of the 4 per-lane counts (canonical insert order)
// ---------------------------------------------------------------------------
__device__ inline unsigned long long unpack_counts(uint32_t c) {
  return (unsigned long long)(c & 15u) | ((unsigned long long)((c >> 4) & 15u) << 16) |
         ((unsigned long long)((c >> 8) & 15u) << 32) | ((unsigned long long)((c >> 12) & 15u) << 48);
}

__device__ __forceinline__ void scan1_body(const uint32_t* __restrict__ counts, int N,
                                           unsigned long long* __restrict__ local,
                                           uint4* __restrict__ block_sum, int bx) {
  __shared__ unsigned long long wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int L = bx * 256 + tid;
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
    block_sum[bx] = make_uint4((uint32_t)(tot & 0xFFFF), (uint32_t)((tot >> 16) & 0xFFFF),
                               (uint32_t)((tot >> 32) & 0xFFFF), (uint32_t)(tot >> 48));
  }
}

__global__ void __launch_bounds__(256) k_scan1(const uint32_t* __restrict__ counts, int N,
                                               unsigned long long* __restrict__ local,
                                               uint4* __restrict__ block_sum) {
  scan1_body(counts, N, local, block_sum, blockIdx.x);
}

__global__ void __launch_bounds__(256) k_scan1_g(const GroupRollout* __restrict__ tab) {
  const RolloutArgs& A = tab[blockIdx.y].A;
  scan1_body(A.S.counts, A.N, A.S.local, A.S.block_sum, blockIdx.x);
}

__device__ __forceinline__ void scan2_body(const uint4* __restrict__ block_sum, int nblk,
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

__global__ void __launch_bounds__(1024) k_scan2(const uint4* __restrict__ block_sum, int nblk,
                                                uint4* __restrict__ block_base, EngineDev* st) {
  scan2_body(block_sum, nblk, block_base, st);
}

__global__ void __launch_bounds__(1024) k_scan2_g(const GroupRollout* __restrict__ tab) {   // block = replica
  const GroupRollout& T = tab[blockIdx.x];
  scan2_body(T.A.S.block_sum, T.nblk, T.A.S.block_base, T.A.st);
}

// ---------------------------------------------------------------------------
// k_commit: staging -> M_RL logs (fp32 rows) and the pending SL lists
// ---------------------------------------------------------------------------
__device__ __forceinline__ void commit_body(int N, unsigned quirks, const Staging& S, const Memories& M,
                                            const EngineDev* __restrict__ st, int bx) {
  const int L = bx * blockDim.x + threadIdx.x;
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
    float a[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) a[c] = alias ? S.fin_a[(p * 3 + c) * N + L] : S.rl_a[(k * 3 + c) * N + L];
    RlRec rec;
    rec.s = alias ? S.fin_s[p * N + L] : S.rl_s[k * N + L];
    rec.s2 = S.rl_s2[k * N + L];
    rec.meta = (uint32_t)nfsp::argmax3(a[0], a[1], a[2]) | (meta & 0x100u) | ((meta & 0xFFu) << 16);
    rec.a0 = a[0]; rec.a1 = a[1]; rec.a2 = a[2];
    rec.pad[0] = rec.pad[1] = 0;
    M.rl[row] = rec;
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

__global__ void __launch_bounds__(256) k_commit(int N, unsigned quirks, Staging S, Memories M,
                                                const EngineDev* __restrict__ st) {
  commit_body(N, quirks, S, M, st, blockIdx.x);
}

__global__ void __launch_bounds__(256) k_commit_g(const GroupRollout* __restrict__ tab) {
  const GroupRollout& T = tab[blockIdx.y];
  commit_body(T.A.N, T.A.quirks, T.A.S, T.M, T.A.st, blockIdx.x);
}

// the reference's fp32 tuple layout (utils/replay_buffer.py:53-57) of agent a's memories
__global__ void __launch_bounds__(256) k_export_mem(Memories M, int a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M.log_cap) {
    const int64_t row = (int64_t)a * M.log_cap + i;
    const RlRec r = M.rl[row];
#pragma unroll
    for (int f = 0; f < nfsp::OBS; ++f) {
      M.ex_rl_s[row * nfsp::OBS + f] = (float)((r.s >> f) & 1u);
      M.ex_rl_s2[row * nfsp::OBS + f] = (float)((r.s2 >> f) & 1u);
    }
    M.ex_rl_a[row * 3 + 0] = r.a0;
    M.ex_rl_a[row * 3 + 1] = r.a1;
    M.ex_rl_a[row * 3 + 2] = r.a2;
    M.ex_rl_r[row] = (float)(int8_t)((r.meta >> 16) & 0xFFu) * 0.5f;
    M.ex_rl_t[row] = (uint8_t)((r.meta >> 8) & 1u);
  }
  if (i < M.sl_cap) {
    const int64_t row = (int64_t)a * M.sl_cap + i;
    const SlRec r = M.sl[row];
#pragma unroll
    for (int f = 0; f < nfsp::OBS; ++f) M.ex_sl_s[row * nfsp::OBS + f] = (float)((r.x >> f) & 1u);
    M.ex_sl_a[row * 3 + 0] = r.a0;
    M.ex_sl_a[row * 3 + 1] = r.a1;
    M.ex_sl_a[row * 3 + 2] = r.a2;
  }
}

__global__ void k_finish_rollout(EngineDev* st, int64_t N) {
  if (threadIdx.x == 0) {
    st->hands += N;
    st->rollouts += 1;
  }
}

__global__ void k_finish_rollout_g(const GroupRollout* __restrict__ tab, int R) {
  for (int r = threadIdx.x; r < R; r += blockDim.x) {   // R may exceed the block
    EngineDev* st = tab[r].A.st;
    st->hands += tab[r].A.N;
    st->rollouts += 1;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace nfsp {
namespace eng {
hipEvent_t take_event(nfsp_engine* e) {
  if (!e->pool.empty()) {
    hipEvent_t ev = e->pool.back();
    e->pool.pop_back();
    return ev;
  }
  hipEvent_t ev = nullptr;
  (void)hipEventCreate(&ev);
  return ev;
}
}  // namespace eng
}  // namespace nfsp

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
  c->slices = 1;
  c->slice_lag = 1;
  const char* ls = getenv("NFSP_LEARNER_SERIAL");
  c->sched = ls && atoi(ls) ? NFSP_SCHED_LEARNER_SERIAL : 0u;
  return NFSP_OK;
}

extern "C" int nfsp_engine_destroy(nfsp_engine* e) {
  if (!e) return NFSP_OK;
  // every stream the engine enqueues on: an update that failed midway may have left a chain
  // running on a side stream without its join into the ctx stream
  if (e->ctx) (void)hipStreamSynchronize(e->ctx->stream);
  for (hipStream_t st : {e->s_br[0], e->s_br[1], e->s_ar})
    if (st) (void)hipStreamSynchronize(st);
  for (void* p : e->allocs) (void)hipFree(p);
  for (auto& pe : e->snap_ev)
    for (hipEvent_t ev : pe)
      if (ev) (void)hipEventDestroy(ev);
  for (auto& m : e->marks) {
    e->pool.push_back(m.second.first);
    e->pool.push_back(m.second.second);
  }
  for (hipEvent_t ev : e->pool) (void)hipEventDestroy(ev);
  for (hipStream_t st : {e->s_br[0], e->s_br[1], e->s_ar})
    if (st) (void)hipStreamDestroy(st);
  delete e;
  return NFSP_OK;
}

namespace nfsp {
namespace eng {
// own_streams: the engine's own AR / BR chain streams (nfsp_engine_update); a replica of an
// engine group has none (the group launches its chains)
int engine_create(nfsp_ctx* ctx, const nfsp_engine_cfg* cfg, bool own_streams, nfsp_engine** out) {
  NFSP_REQUIRE(ctx && cfg && out, "null argument");
  NFSP_REQUIRE(cfg->hidden == nn::H, "only hidden == 64 is built");
  NFSP_REQUIRE(cfg->n_lanes > 0 && cfg->n_lanes < (1 << 24), "n_lanes must be in [1, 2^24)");
  NFSP_REQUIRE(cfg->slices >= 1 && cfg->n_lanes % cfg->slices == 0,
               "slices must be >= 1 and divide n_lanes");
  NFSP_REQUIRE(cfg->slice_lag == 1 || cfg->slice_lag == 2, "slice_lag must be 1 or 2");
  NFSP_REQUIRE(cfg->fit_batch == CHAIN_MB, "the SGD chains are built for fit_batch == 32");
  NFSP_REQUIRE(cfg->batch >= CHAIN_MB && cfg->batch <= MAX_BATCH && cfg->batch % CHAIN_MB == 0,
               "batch must be 32, 64, 96 or 128");
  NFSP_REQUIRE(cfg->epochs >= 1 && cfg->epochs <= 4, "epochs must be in [1, 4]");
  NFSP_REQUIRE(cfg->rl_capacity > cfg->batch && cfg->sl_capacity > cfg->batch,
               "capacities must exceed the batch");
  // reservoir slots are int32 in the learner (LearnBufs::res_slot)
  NFSP_REQUIRE(cfg->sl_capacity < (1ll << 31), "sl_capacity must be < 2^31");
  NFSP_REQUIRE(cfg->rl_capacity < (1ll << 40), "rl_capacity too large");
  NFSP_REQUIRE(cfg->inserts_per_update >= 1 && cfg->target_every >= 1, "bad cadence");
  NFSP_REQUIRE((cfg->quirks & ~(NFSP_QUIRKS_REFERENCE | NFSP_TEXTBOOK_MSE)) == 0,
               "unknown bits in quirks (NFSP_QUIRK_* | NFSP_EXT_*)");
  NFSP_REQUIRE(!(cfg->quirks & NFSP_EXT_MSE_Q) || (cfg->quirks & NFSP_EXT_LINEAR_Q),
               "NFSP_EXT_MSE_Q requires NFSP_EXT_LINEAR_Q");
  // the chains read an agent's step records through a buffer descriptor with 32-bit offsets
  // (k_chain3): [umax][epochs][batch / 32] records of one learner call must stay below 2 GiB
  NFSP_REQUIRE((4 * (int64_t)(cfg->n_lanes / cfg->slices) / cfg->inserts_per_update + 2) * cfg->epochs *
                       (cfg->batch / CHAIN_MB) * (int64_t)sizeof(StepRec) < (1ll << 31),
               "one slice's step records exceed 2 GiB: use more slices (or more inserts per update)");
  *out = nullptr;
  nfsp_engine* e = new nfsp_engine();
  e->ctx = ctx;
  e->cfg = *cfg;
  e->slices = cfg->slices;
  e->N = cfg->n_lanes / cfg->slices;     // lanes per rollout: staging and learner bounds
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
  EALLOC(e->M.rl, sizeof(RlRec) * lc);
  EALLOC(e->M.sl, sizeof(SlRec) * sc);
  EALLOC(e->M.pend_x, 4 * pc);
  EALLOC(e->M.pend_a, 4 * 3 * pc);
  EALLOC(e->M.pend_pos, 8 * pc);
  EALLOC(e->M.dbg_rows, 8 * 4 * cfg->batch);
  EALLOC(e->M.dbg_perms, 4 * 4 * 4 * cfg->batch);
  // learner: <= 4N RL inserts per agent per rollout -> <= 4N / c + 2 update triggers
  // (cfg.slice_lag 2: two sets, slice parity; the reservoir lists are shared -- only the
  // ctx stream's prep kernels use them, in slice order)
  e->slice_lag = cfg->slice_lag;
  for (int k = 0; k < (e->slice_lag == 2 ? 2 : 1); ++k) {   // (group replicas too: pipelined groups)
    LearnBufs& L = e->LBs[k];
    L.umax = 4 * N / cfg->inserts_per_update + 2;
    const int64_t ub = 2 * L.umax * cfg->batch, ueb = ub * cfg->epochs;
    EALLOC(L.br_rows, sizeof(BrRow) * ub);
    EALLOC(L.br_perm, ueb);
    EALLOC(L.br_expl, sizeof(double) * 2 * L.umax);
    EALLOC(L.br_rec, sizeof(StepRec) * (ueb / CHAIN_MB));
    EALLOC(L.ar_rec, sizeof(StepRec) * (ueb / CHAIN_MB));
    EALLOC(L.ar_active, 2 * L.umax);
    EALLOC(L.br_loss, 4 * 2 * L.umax * cfg->epochs);
    EALLOC(L.ar_loss, 4 * 2 * L.umax * cfg->epochs);
    if (k == 0) {
      EALLOC(L.res_head, sizeof(unsigned long long) * sc);
      EALLOC(L.res_next, 4 * pc);
      EALLOC(L.res_slot, 4 * pc);
    } else {
      L.res_head = e->LBs[0].res_head;
      L.res_next = e->LBs[0].res_next;
      L.res_slot = e->LBs[0].res_slot;
    }
  }
  e->LB = e->LBs[0];
  if (e->slice_lag == 2) {
    EALLOC(e->snap, sizeof(float) * 2 * 6 * nn::NP);
    if (!own_streams) EALLOC(e->snap_eps_dev, sizeof(double) * 4);   // a group replica
    for (auto& pe : e->snap_ev)
      for (hipEvent_t& ev : pe) {
        const hipError_t er = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (er != hipSuccess) {
          nfsp_engine_destroy(e);
          return nfsp::hip_fail(er, "nfsp_engine_create: hipEventCreate");
        }
      }
  }
  for (hipStream_t* st : {&e->s_br[0], &e->s_br[1], &e->s_ar}) {
    if (!own_streams) break;
    hipError_t sr = hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    if (sr != hipSuccess) {
      nfsp_engine_destroy(e);
      return nfsp::hip_fail(sr, "nfsp_engine_create: hipStreamCreate");
    }
  }
  EngineDev h{};
  for (int a = 0; a < 2; ++a) {
    h.epsilon[a] = cfg->epsilon;
    h.temp[a] = 1.0;
    h.lr_br[a] = cfg->lr_br;
    e->hs.epsilon[a] = cfg->epsilon;
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
}  // namespace eng
}  // namespace nfsp

extern "C" int nfsp_engine_create(nfsp_ctx* ctx, const nfsp_engine_cfg* cfg, nfsp_engine** out) {
  return nfsp::eng::engine_create(ctx, cfg, true, out);
}

extern "C" int nfsp_engine_weights(nfsp_engine* e, int agent, int net, float** dev_w) {
  NFSP_REQUIRE(e && dev_w, "null argument");
  NFSP_REQUIRE((agent == 0 || agent == 1) && net >= 0 && net <= 2, "bad agent/net");
  *dev_w = e->w + (agent * 3 + net) * nn::NP;
  return NFSP_OK;
}

namespace nfsp {
namespace eng {
static RolloutArgs rollout_args(const nfsp_engine* e) {
  RolloutArgs A;
  A.N = e->N;
  A.eps_by_value = 0;               // groups: each replica's st->epsilon (static table)
  A.eps_v[0] = A.eps_v[1] = 0.0;
  // the next rollout plays slice rollouts % slices; a lane's hand index is its hand count
  const uint64_t hand = e->rollouts / (uint64_t)e->slices;
  A.lane0 = (uint32_t)((e->rollouts % (uint64_t)e->slices) * (uint64_t)e->N);
  A.k0 = (uint32_t)e->cfg.seed;
  A.k1 = (uint32_t)(e->cfg.seed >> 32);
  A.g_lo = (uint32_t)hand;
  A.g_hi = (uint32_t)(hand >> 32);
  A.eta = e->cfg.eta;
  A.quirks = e->cfg.quirks;
  A.game = e->ctx->game;
  A.w = e->w;
  A.st = e->st;
  A.S = e->S;
  return A;
}

int rollout_launch(nfsp_engine* e) { return rollout_launch_with(e, e->w, e->hs.epsilon); }

int rollout_launch_with(nfsp_engine* e, const float* w, const double eps[2]) {
  NFSP_REQUIRE(!e->pending_update, "nfsp_engine_update must consume the previous rollout first");
  hipStream_t s = e->ctx->stream;
  RolloutArgs A = rollout_args(e);
  A.w = w;
  A.eps_by_value = 1;               // the schedule as the host computed it (= st->epsilon)
  A.eps_v[0] = eps[0];
  A.eps_v[1] = eps[1];
  {
    KTimer kt(e, KT_ROLLOUT);
    k_rollout<<<(e->N + ROLLOUT_WG - 1) / ROLLOUT_WG, ROLLOUT_WG, 0, s>>>(A);
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

int group_rollout_table(nfsp_engine* const* eng, int R, void** d_tab) {
  std::vector<GroupRollout> h(R);
  for (int r = 0; r < R; ++r) {
    NFSP_REQUIRE(eng[r]->N == eng[0]->N && eng[r]->slices == eng[0]->slices,
                 "group replicas differ in n_lanes or slices");
    h[r].A = rollout_args(eng[r]);
    h[r].M = eng[r]->M;
    h[r].nblk = eng[r]->nblk;
    h[r].snap = eng[r]->snap;
    h[r].snap_eps = eng[r]->snap_eps_dev;
  }
  NFSP_HIP(hipMalloc(d_tab, sizeof(GroupRollout) * R));
  NFSP_HIP(hipMemcpy(*d_tab, h.data(), sizeof(GroupRollout) * R, hipMemcpyHostToDevice));
  return NFSP_OK;
}

// every replica's rollout in one launch per kernel (blockIdx.y = replica); the marks are
// kept on replica 0
int group_rollout_launch(nfsp_engine* const* eng, int R, const void* d_tab, int par) {
  nfsp_engine* e0 = eng[0];
  for (int r = 0; r < R; ++r)
    NFSP_REQUIRE(!eng[r]->pending_update && eng[r]->rollouts == e0->rollouts,
                 "group replicas out of step");
  hipStream_t s = e0->ctx->stream;
  const GroupRollout* tab = static_cast<const GroupRollout*>(d_tab);
  {
    KTimer kt(e0, KT_ROLLOUT);
    const RolloutArgs A0 = rollout_args(e0);   // slice and hand index, the same for every replica
    k_rollout_g<<<dim3(e0->nblk, R), 256, 0, s>>>(tab, A0.g_lo, A0.g_hi, A0.lane0, par);
  }
  NFSP_LAUNCHED("k_rollout_g");
  {
    KTimer kt(e0, KT_SCAN);
    k_scan1_g<<<dim3(e0->nblk, R), 256, 0, s>>>(tab);
    k_scan2_g<<<R, 1024, 0, s>>>(tab);
  }
  NFSP_LAUNCHED("k_scan_g");
  {
    KTimer kt(e0, KT_COMMIT);
    k_commit_g<<<dim3(e0->nblk, R), 256, 0, s>>>(tab);
  }
  NFSP_LAUNCHED("k_commit_g");
  k_finish_rollout_g<<<1, 256, 0, s>>>(tab, R);
  NFSP_LAUNCHED("k_finish_rollout_g");
  for (int r = 0; r < R; ++r) {
    eng[r]->rollouts++;
    eng[r]->pending_update = true;
  }
  return NFSP_OK;
}

int group_snap_part_launch(nfsp_engine* const* eng, int R, const void* d_tab, int par, int part, hipStream_t s,
                           int r0) {
  k_group_snap_part<<<dim3(nfsp_blocks(6 * nn::NP, 256), R), 256, 0, s>>>(
      static_cast<const GroupRollout*>(d_tab) + r0, par, part);
  NFSP_LAUNCHED("k_group_snap_part");
  return NFSP_OK;
}

int group_snap_launch(nfsp_engine* const* eng, int R, const void* d_tab, int par) {
  for (int r = 0; r < R; ++r)
    NFSP_REQUIRE(eng[r]->snap && eng[r]->snap_eps_dev, "group replica without snapshots (slice_lag 1)");
  k_group_snap<<<dim3(nfsp_blocks(6 * nn::NP, 256), R), 256, 0, eng[0]->ctx->stream>>>(
      static_cast<const GroupRollout*>(d_tab), par);
  NFSP_LAUNCHED("k_group_snap");
  return NFSP_OK;
}
}  // namespace eng
}  // namespace nfsp

extern "C" int nfsp_rollout_with(nfsp_engine* e, const float* dev_w, const double* eps) {
  NFSP_REQUIRE(e && dev_w && eps, "null argument");
  NFSP_REQUIRE(e->s_ar, "a replica of an engine group is stepped by nfsp_group_step");
  const double ev[2] = {eps[0], eps[1]};
  return nfsp::eng::rollout_launch_with(e, dev_w, ev);
}

extern "C" int nfsp_rollout(nfsp_engine* e) {
  NFSP_REQUIRE(e, "null argument");
  NFSP_REQUIRE(e->s_ar, "a replica of an engine group is stepped by nfsp_group_step");
  return nfsp::eng::rollout_launch(e);
}

// one hand on every lane: each slice's rollout, then the learner on its inserts
extern "C" int nfsp_engine_step(nfsp_engine* e) {
  NFSP_REQUIRE(e, "null argument");
  if (e->slice_lag == 2 && e->slices > 1 && e->s_ar) return nfsp::eng::step_pipelined(e);
  for (int k = 0; k < e->slices; ++k) {
    int rc = nfsp_rollout(e);
    if (rc != NFSP_OK) return rc;
    if ((rc = nfsp_engine_update(e)) != NFSP_OK) return rc;
  }
  return NFSP_OK;
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
    // before nfsp_engine_update has consumed a rollout its inserts are already made: the
    // RL ones are in M_RL, the SL ones wait in the pending list
    const int64_t rl_total = h.rl_total[a] + (e->pending_update ? h.last_rl[a] : 0);
    out->rl_total[a] = rl_total;
    out->sl_total[a] = h.sl_total[a] + (e->pending_update ? h.last_sl[a] : 0);
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
  Memories& M = e->M;
  if ((rl || sl) && !M.ex_sl_a) {      // the fp32 reference-layout views, on first use
    // (resumable: a failed allocation leaves the export unusable until a later call
    // completes the set -- ex_sl_a, the last one, is the "all allocated" mark)
    const int64_t lc = 2 * M.log_cap, sc = 2 * M.sl_cap;
    for (auto pr : {std::make_pair((void**)&M.ex_rl_s, 4 * nfsp::OBS * lc), std::make_pair((void**)&M.ex_rl_s2, 4 * nfsp::OBS * lc),
                    std::make_pair((void**)&M.ex_rl_a, 4 * 3 * lc), std::make_pair((void**)&M.ex_rl_r, 4 * lc),
                    std::make_pair((void**)&M.ex_rl_t, lc), std::make_pair((void**)&M.ex_sl_s, 4 * nfsp::OBS * sc),
                    std::make_pair((void**)&M.ex_sl_a, 4 * 3 * sc)}) {
      if (*pr.first) continue;
      NFSP_HIP(hipMalloc(pr.first, (size_t)pr.second));
      e->allocs.push_back(*pr.first);
    }
  }
  const int64_t lo = (int64_t)agent * M.log_cap;
  const int64_t so = (int64_t)agent * M.sl_cap;
  if (rl || sl) {
    const int64_t n = M.log_cap > M.sl_cap ? M.log_cap : M.sl_cap;
    k_export_mem<<<(unsigned)nfsp_blocks(n, 256), 256, 0, e->ctx->stream>>>(M, agent);
    NFSP_LAUNCHED("k_export_mem");
  }
  if (rl) {
    rl->s = M.ex_rl_s + lo * nfsp::OBS;
    rl->a = M.ex_rl_a + lo * 3;
    rl->r = M.ex_rl_r + lo;
    rl->s2 = M.ex_rl_s2 + lo * nfsp::OBS;
    rl->t = M.ex_rl_t + lo;
    rl->cap = M.log_cap;
  }
  if (log_cap) *log_cap = M.log_cap;
  if (sl) {
    sl->s = M.ex_sl_s + so * nfsp::OBS;
    sl->a = M.ex_sl_a + so * 3;
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

extern "C" int nfsp_engine_lane_counts(nfsp_engine* e, uint32_t** counts) {
  NFSP_REQUIRE(e && counts, "null argument");
  *counts = e->S.counts;
  return NFSP_OK;
}

extern "C" int nfsp_engine_set_timing(nfsp_engine* e, int on) {
  NFSP_REQUIRE(e, "null argument");
  e->timing = on != 0;
  return NFSP_OK;
}

extern "C" int nfsp_engine_set_loss_log(nfsp_engine* e, int on) {
  NFSP_REQUIRE(e, "null argument");
  e->log_loss = on != 0;
  return NFSP_OK;
}

extern "C" int nfsp_engine_losses(nfsp_engine* e, double* out) {
  NFSP_REQUIRE(e && out, "null argument");
  NFSP_REQUIRE(e->log_loss, "the loss log is off (nfsp_engine_set_loss_log)");
  NFSP_HIP(hipStreamSynchronize(e->ctx->stream));
  const int E = e->cfg.epochs;
  for (int a = 0; a < 2; ++a)
    for (int n = 0; n < 2; ++n) {                 // n: 0 = AR (avg_strategy_model), 1 = BR
      const int64_t U = n ? e->last_Ubr[a] : e->last_U[a];
      const float* src = (n ? e->LB.br_loss : e->LB.ar_loss) + (int64_t)a * e->LB.umax * E;
      std::vector<float> h((size_t)(U * E));
      if (U > 0) NFSP_HIP(hipMemcpy(h.data(), src, sizeof(float) * U * E, hipMemcpyDeviceToHost));
      double sum = 0.0, last = NAN;
      int64_t cnt = 0;
      for (int64_t q = 0; q < U * E; ++q)
        if (!std::isnan(h[q])) { sum += h[q]; cnt++; last = h[q]; }
      out[(a * 2 + n) * 2 + 0] = cnt ? sum / (double)cnt : NAN;
      out[(a * 2 + n) * 2 + 1] = last;
    }
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
