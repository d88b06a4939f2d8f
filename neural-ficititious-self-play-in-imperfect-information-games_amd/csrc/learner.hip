// The engine's learner (nfsp_engine_update): update_strategy at the reference cadence
// for the RL/SL inserts of the last rollout.  Reference: agent/agent.py:192-273.
//
// An update's inputs (sampled rows, fit permutations, reservoir contents at that moment,
// DQN targets) do not depend on the weights being trained, except the targets on the
// target net, which only changes every TargetModelUpdateRate BR updates.  So all of it
// is produced by wide parallel kernels, and the only sequential work -- the SGD steps
// themselves -- runs in one workgroup per (agent, net) with the whole net resident:
//
//   k_br_prep       [all BR updates]  sample 128 M_RL rows in the window the reference
//                                     would see, gather (s, s2, argmax a, r, t), perms
//   k_ar_slots      [all SL inserts]  reservoir slot of every insert (Philox), per-slot
//                                     insert lists (so any past moment can be read back)
//   k_ar_prep       [all AR updates]  M_SL size at the trigger, sample 128 slots, read the
//                                     slot contents AS OF the trigger, perms -> fit rows
//   k_res_apply     [all SL inserts]  final reservoir contents (last writer per slot)
//   k_br_targets    [a segment]       Q_target forwards, TD values, proxy, row-0 quirk
//   k_chain3<BR/AR> [1 WG per agent]  epochs x minibatch SGD, whole net in registers
// BR chains are cut into segments at target-sync points; the two agents' BR chains and
// the AR chains run on separate streams.
#include <math.h>
#include <stdlib.h>

#include "engine_internal.h"

using nfsp::u32x4;
namespace nn = nfsp::nn;
using namespace nfsp::eng;

namespace {

struct AgentPlan {
  int64_t P0;          // agent's RL inserts before the last rollout
  int64_t m_first;     // first trigger index (trigger m at RL stream position m * c)
  int64_t U;           // triggers in the last rollout
  int64_t m_br0;       // first trigger with a BR update (position > batch)
  int64_t U_br;
  int64_t n_sl;        // SL records of the last rollout
  int64_t sl_total0;   // SL inserts before the last rollout
};

struct PrepArgs {
  Memories M;
  LearnBufs LB;
  EngineDev* st;
  AgentPlan A[2];
  int64_t c, rl_cap;
  int B, E;
  uint32_t k0, k1, tag;
  float lr_ar;
};

// ---------------------------------------------------------------------------
// BR prep: rows of update u of agent a (agent/agent.py:217 sample_batch)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(128) k_br_prep(PrepArgs P) {
  __shared__ int64_t cand[MAX_BATCH];
  __shared__ uint32_t key[MAX_BATCH];
  const int a = blockIdx.y;
  const int64_t u = blockIdx.x;
  const AgentPlan& pl = P.A[a];
  if (u >= pl.U_br) return;
  const int b = threadIdx.x;
  const int dbg = a * 2 + 1;
  const int64_t m = pl.m_br0 + u;
  const int64_t pm = m * P.c;
  const int64_t win = pm < P.rl_cap ? pm : P.rl_cap;
  sample_distinct(cand, P.B, pm - win, win, TAG_SAMPLE | (uint32_t)dbg, m, P.k0, P.k1);
  const int64_t slot = (int64_t)a * P.LB.umax + u;
  if (b < P.B) {
    const int64_t row = (int64_t)a * P.M.log_cap + cand[b] % P.M.log_cap;
    const uint4 q = *reinterpret_cast<const uint4*>(&P.M.rl[row]);   // s, s2, meta, a0
    BrRow rr;
    rr.s = q.x;
    rr.s2 = q.y;
    rr.meta = q.z;
    P.LB.br_rows[slot * P.B + b] = rr;
  }
  const bool last = u == pl.U_br - 1;
  for (int e = 0; e < P.E; ++e) {
    int rank;
    draw_perm(key, P.B, e, TAG_PERM | (uint32_t)dbg, m, P.k0, P.k1, rank);
    if (b < P.B) {
      P.LB.br_perm[(slot * P.E + e) * P.B + rank] = (uint8_t)b;
      if (last) P.M.dbg_perms[(dbg * P.E + e) * P.B + rank] = b;
    }
  }
  if (last && b < P.B) P.M.dbg_rows[dbg * P.B + b] = cand[b];
}

// ---------------------------------------------------------------------------
// reservoir slots + per-slot insert lists (utils/ReservoirBuffer.py:18-28)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ar_slots(PrepArgs P) {
  const int a = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const AgentPlan& pl = P.A[a];
  if (q >= pl.n_sl) return;
  const int64_t cap = P.M.sl_cap;
  const int64_t tot = pl.sl_total0 + q;          // adds before this one
  int64_t slot;
  if (tot < cap) {
    slot = tot;                                  // append while count < buffer_size
  } else {
    const u32x4 r = nfsp::philox4x32({TAG_RES | (uint32_t)a, (uint32_t)tot, (uint32_t)(tot >> 32), 0u},
                                     P.k0, P.k1);
    const uint64_t r64 = ((uint64_t)r.x << 32) | r.y;
    const int64_t j = 1 + (int64_t)(r64 % (uint64_t)cap);        // randrange(1, N + 1)
    slot = j < cap ? j : -1;                                     // replace iff j < N
  }
  const int64_t qi = (int64_t)a * P.M.pend_cap + q;
  P.LB.res_slot[qi] = (int32_t)slot;
  if (slot >= 0) {
    const unsigned long long mine = ((unsigned long long)P.tag << 32) | (unsigned long long)q;
    const unsigned long long old = atomicExch(&P.LB.res_head[(int64_t)a * cap + slot], mine);
    P.LB.res_next[qi] = (uint32_t)(old >> 32) == P.tag ? (int32_t)(old & 0xFFFFFFFFull) : -1;
  }
}

// 8 bf16 0/1 values of the layer-1 K slots 8g..8g+7 (bits 4g..4g+3, 16+4g..16+4g+3 of x)
__device__ inline uint4 bits8u(uint32_t x, int g) {
  const uint32_t n0 = (x >> (4 * g)) & 0xFu, n1 = (x >> (16 + 4 * g)) & 0xFu;
  return make_uint4((n0 & 1u) * 0x3F80u + ((n0 >> 1) & 1u) * 0x3F800000u,
                    ((n0 >> 2) & 1u) * 0x3F80u + ((n0 >> 3) & 1u) * 0x3F800000u,
                    (n1 & 1u) * 0x3F80u + ((n1 >> 1) & 1u) * 0x3F800000u,
                    ((n1 >> 2) & 1u) * 0x3F80u + ((n1 >> 3) & 1u) * 0x3F800000u);
}

// The chain records of one (update, epoch): thread b holds fit position b's observation
// mask x (for b < B), targets and the lr; minibatch b >> 5 gets fa / tg of its sample
// b & 31, and ba from the bit transpose of its 32 masks by wave ballot.  Every valid
// sample also carries the bias input (CHAIN_BIAS_BIT).  Whole block (a multiple of 64
// threads) calls.
__device__ inline void emit_recs(StepRec* __restrict__ recs, uint32_t x, float t0, float t1, float t2,
                                 float lr, int B) {
  const int b = threadIdx.x;
  if (b < B) {
    x |= CHAIN_BIAS_BIT;
    StepRec& R = recs[b >> 5];
    const int k = b & 31;
#pragma unroll
    for (int g = 0; g < 4; ++g) R.fa[g][k] = bits8u(x, g);
    R.tg[k] = make_float4(t0, t1, t2, lr);
  }
  const int lane = b & 63;
  unsigned long long mine = 0;
#pragma unroll
  for (int i = 0; i <= CHAIN_BIAS_IN; ++i) {
    const unsigned long long m = __ballot((x >> i) & 1u);
    if (lane == i) mine = m;
  }
  const int mb = (b >> 6) * 2;          // this wave's two minibatches
  if (lane < 32) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (32 * (mb + h) >= B) continue;
      const uint32_t xt = (uint32_t)(mine >> (32 * h));
#pragma unroll
      for (int g = 0; g < 4; ++g) recs[mb + h].ba[g][lane] = bits8u(xt, g);
    }
  }
}

// latest insert of this rollout into `slot` with index < limit (-1: none)
__device__ inline int64_t latest_insert(const LearnBufs& LB, const Memories& M, int a, int64_t slot,
                                        int64_t limit, uint32_t tag) {
  const unsigned long long h = LB.res_head[(int64_t)a * M.sl_cap + slot];
  if ((uint32_t)(h >> 32) != tag) return -1;
  int64_t best = -1;
  int32_t q = (int32_t)(h & 0xFFFFFFFFull);
  while (q >= 0) {
    if (q < limit && q > best) best = q;
    q = LB.res_next[(int64_t)a * M.pend_cap + q];
  }
  return best;
}

// ---------------------------------------------------------------------------
// AR prep (agent/agent.py:259-261): M_SL as it was at the trigger
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(128) k_ar_prep(PrepArgs P) {
  __shared__ int64_t cand[MAX_BATCH];
  __shared__ uint32_t key[MAX_BATCH];
  __shared__ uint32_t rx[MAX_BATCH];
  __shared__ float ra[MAX_BATCH][3];
  __shared__ uint32_t px[MAX_BATCH];
  __shared__ float pt[MAX_BATCH][3];
  __shared__ int64_t s_nb;
  const int a = blockIdx.y;
  const int64_t u = blockIdx.x;
  const AgentPlan& pl = P.A[a];
  if (u >= pl.U) return;
  const int b = threadIdx.x;
  const int dbg = a * 2 + 0;
  const int64_t m = pl.m_first + u;
  const int64_t pm = m * P.c;
  const int64_t slot_u = (int64_t)a * P.LB.umax + u;
  if (b == 0) {          // SL inserts made before the trigger: pend_pos is nondecreasing
    const int64_t* pos = P.M.pend_pos + (int64_t)a * P.M.pend_cap;
    int64_t lo = 0, hi = pl.n_sl;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (pos[mid] <= pm) lo = mid + 1; else hi = mid;
    }
    s_nb = lo;
  }
  __syncthreads();
  const int64_t nb = s_nb;
  const int64_t tot = pl.sl_total0 + nb;
  const int64_t count = tot < P.M.sl_cap ? tot : P.M.sl_cap;
  if (count <= P.B) {                         // size() > minibatch_size fails
    if (b == 0) P.LB.ar_active[slot_u] = 0;
    return;
  }
  if (b == 0) {
    P.LB.ar_active[slot_u] = 1;
    atomicAdd((unsigned long long*)&P.st->ar_updates[a], 1ull);
  }
  sample_distinct(cand, P.B, 0, count, TAG_SAMPLE | (uint32_t)dbg, m, P.k0, P.k1);
  if (b < P.B) {
    const int64_t j = cand[b];
    const int64_t q = latest_insert(P.LB, P.M, a, j, nb, P.tag);
    if (q >= 0) {
      const int64_t qi = (int64_t)a * P.M.pend_cap + q;
      rx[b] = P.M.pend_x[qi];
      ra[b][0] = P.M.pend_a[qi * 3 + 0];
      ra[b][1] = P.M.pend_a[qi * 3 + 1];
      ra[b][2] = P.M.pend_a[qi * 3 + 2];
    } else {
      const SlRec r = P.M.sl[(int64_t)a * P.M.sl_cap + j];
      rx[b] = r.x;
      ra[b][0] = r.a0;
      ra[b][1] = r.a1;
      ra[b][2] = r.a2;
    }
  }
  const bool last = u == pl.U - 1;
  for (int e = 0; e < P.E; ++e) {
    int rank;
    draw_perm(key, P.B, e, TAG_PERM | (uint32_t)dbg, m, P.k0, P.k1, rank);
    if (b < P.B) {        // fit position rank <- sampled row b
      px[rank] = rx[b];
      pt[rank][0] = ra[b][0]; pt[rank][1] = ra[b][1]; pt[rank][2] = ra[b][2];
      if (last) P.M.dbg_perms[(dbg * P.E + e) * P.B + rank] = b;
    }
    __syncthreads();
    const bool in = b < P.B;
    // targets / batch: the AR chain's cross-entropy gradient takes them pre-scaled (exact)
    const float sc = 1.0f / (float)CHAIN_MB;
    emit_recs(P.LB.ar_rec + (slot_u * P.E + e) * (P.B / CHAIN_MB), in ? px[b] : 0u, in ? pt[b][0] * sc : 0.f,
              in ? pt[b][1] * sc : 0.f, in ? pt[b][2] * sc : 0.f, P.lr_ar, P.B);
    __syncthreads();
  }
  if (last && b < P.B) P.M.dbg_rows[dbg * P.B + b] = cand[b];
}

__global__ void __launch_bounds__(256) k_res_apply(PrepArgs P) {
  const int a = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P.A[a].n_sl) return;
  const int64_t qi = (int64_t)a * P.M.pend_cap + q;
  const int64_t slot = P.LB.res_slot[qi];
  if (slot < 0) return;
  if (latest_insert(P.LB, P.M, a, slot, P.A[a].n_sl, P.tag) != q) return;   // a later add wins
  SlRec r;
  r.x = P.M.pend_x[qi];
  r.a0 = P.M.pend_a[qi * 3 + 0];
  r.a1 = P.M.pend_a[qi * 3 + 1];
  r.a2 = P.M.pend_a[qi * 3 + 2];
  P.M.sl[(int64_t)a * P.M.sl_cap + slot] = r;
}

// ---------------------------------------------------------------------------
// DQN targets of one BR segment (agent/agent.py:219-241), one update per workgroup
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_br_targets(LearnBufs LB, const float* __restrict__ tw, int a,
                                                    int64_t u0, int B, int E, double gamma,
                                                    unsigned quirks, int64_t it0, double lr0) {
  // threads 0..127: Q_target(s) of row b (waves 0-1); threads 128..255: Q_target(s2) of
  // row b - 128 (waves 2-3) -- the two forwards of a row run side by side
  __shared__ __attribute__((aligned(16))) float sw[NET_LDS];
  __shared__ float q[MAX_BATCH][3];
  __shared__ float val[MAX_BATCH];
  __shared__ uint32_t sb[MAX_BATCH];
  __shared__ uint8_t am[MAX_BATCH];
  __shared__ double part[2];
  __shared__ int lastw[2][3];
  const int tid = threadIdx.x;
  const int b = tid & (MAX_BATCH - 1);
  const bool s2half = tid >= MAX_BATCH;
  const int64_t u = u0 + blockIdx.x;
  const int64_t slot = (int64_t)a * LB.umax + u;
  BrRow rr{};
  if (b < B) rr = LB.br_rows[slot * B + b];
  stage_net_lds(sw, tw, tid, blockDim.x);
  __syncthreads();
  if (b < B) {
    float y[3];
    if (!s2half) {
      fwd_lds(sw, rr.s, NFSP_ACT_RELU, y);
      q[b][0] = y[0]; q[b][1] = y[1]; q[b][2] = y[2];
      am[b] = (uint8_t)(rr.meta & 0xFFu);
      sb[b] = rr.s;
    } else {
      fwd_lds(sw, rr.s2, NFSP_ACT_RELU, y);
      const float qmax = fmaxf(fmaxf(y[0], y[1]), y[2]);
      const float r = (float)(int8_t)((rr.meta >> 16) & 0xFFu) * 0.5f;
      const bool terminal = !(quirks & NFSP_QUIRK_TERMINAL_BOOTSTRAP) && ((rr.meta >> 8) & 1u);
      val[b] = (float)(terminal ? (double)r : (double)r + gamma * (double)qmax);
    }
  }
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6;
  if (!s2half) {
    // exploitability proxy (agent/agent.py:235-238): mean of the row maxima, before the
    // row-0 overwrite; and for the quirk, the last row k with argmax a_k == action
    double m = b < B ? (double)fmaxf(fmaxf(q[b][0], q[b][1]), q[b][2]) : 0.0;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m += __shfl_xor(m, off);
    if (lane == 0) part[wv] = m;
#pragma unroll
    for (int act = 0; act < 3; ++act) {
      const unsigned long long bal = __ballot(b < B && am[b] == act);
      if (lane == 0) lastw[wv][act] = bal ? 64 * wv + 63 - __builtin_clzll(bal) : -1;
    }
  }
  __syncthreads();
  if (tid == 0) LB.br_expl[slot] = (part[0] + part[1]) / B;
  if (quirks & NFSP_QUIRK_ROW0_TARGET) {
    if (tid < 3) {       // target[0][argmax a_k] = v_k for k = 0..B-1: the last k wins
      const int last = lastw[1][tid] >= 0 ? lastw[1][tid] : lastw[0][tid];
      if (last >= 0) q[0][tid] = val[last];
    }
  } else if (!s2half && b < B) {
    q[b][am[b]] = val[b];
  }
  __syncthreads();
  // lr of this update: lr0 / (1 + 0.003 sqrt(iteration)) with iteration = it0 + 2 u
  // (agent/agent.py:249, iteration += 2 per BR update), in the reference's double arithmetic
  const float lr = (float)(lr0 / (1.0 + 0.003 * sqrt((double)(it0 + 2 * u))));
  for (int e = 0; e < E; ++e) {
    uint32_t x = 0;
    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
    if (!s2half && b < B) {
      const int k = LB.br_perm[(slot * E + e) * B + b];
      x = sb[k];
      t0 = q[k][0]; t1 = q[k][1]; t2 = q[k][2];
    }
    emit_recs(LB.br_rec + (slot * E + e) * (B / CHAIN_MB), x, t0, t1, t2, lr, B);
  }
}

// ---------------------------------------------------------------------------
// SGD chains: one workgroup (4 waves) per (agent, net) runs that net's updates back to
// back with the whole net in registers (k_chain3).  Reference: agent/agent.py:241-264
// (model.fit(batch_size=32, epochs=2) of the BR Q-net and the AR policy net).
// ---------------------------------------------------------------------------
struct ChainArgs {
  float* w[2];                    // weights of (agent, net)
  float* sync_to[2];              // BR: target net to copy into at the end (or null)
  const StepRec* rec;             // [2][umax][E][B / 32] step records (prep kernels)
  const uint8_t* active;          // AR: per-update flag, 0..0 1..1 in u (null for BR)
  int64_t umax;
  int64_t u0[2], u1[2];           // update range per agent
  int agents[2];                  // blockIdx -> agent
  int B, E;
  unsigned long long* stamps;     // diagnostic build only (NFSP_CHAIN_STAMPS): phase cycles
  float* loss_out;                // optional: [2][umax][E] Keras epoch losses (the values the
                                  // reference's TensorBoard callbacks log, agent/agent.py:84-88)
};

// In-kernel phase stamps (cdna_hip_programming.md §7): a separate diagnostic build only.
#ifdef NFSP_CHAIN_STAMPS
#define CHAIN_STAMP(k)                                                                   \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    unsigned long long _t;                                                              \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");          \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    st_acc[k] += _t - st_last;                                                          \
    st_last = _t;                                                                       \
  } while (0)
#else
#define CHAIN_STAMP(k) do { } while (0)
#endif

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ inline float dpp_f(float x, int ctrl) {
  switch (ctrl) {   // the control word must be an immediate
    case 0x128: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
    case 0xB1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
    case 0x4E: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));
  }
}

__device__ inline float dpp_any(float x, int ctrl) {
  switch (ctrl) {
    case 0x121: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xF, 0xF, false));
    case 0x122: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xF, 0xF, false));
    case 0x124: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));
    default: return dpp_f(x, ctrl);
  }
}

// x + partner(lane ^ 32) in every lane
__device__ inline float sum_x32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// x + partner(lane ^ 16) in every lane
__device__ inline float sum_x16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ---------------------------------------------------------------------------
// k_chain3: the SGD chain on bf16 matrix cores with exact-f32 operands.
//
// An f32 value v is split exactly into three bf16 terms v = hi + mid + lo (8 + 8 + 8
// significand bits, round-to-nearest at each cut), and a Leduc observation is 0/1, so
// X.W = X.lo + X.mid + X.hi with every product exact and f32 accumulation: the 16 chained
// v_mfma_f32_16x16x4_f32 of a layer-1 product become 3 v_mfma_f32_16x16x32_bf16 per tile
// (K = 32 covers all 30 inputs).  Per wave (hidden slice 16w..16w+15, lane (g, c) =
// (l >> 4, l & 15)):
//   * layer-1 K slot 8g + j <-> input pi(g, j) = 4g + j (j < 4) or 16 + 4g + j - 4, so the
//     dW1 accumulator lands in the registers that hold W1 (wr[j] = W1[pi(g, j)][16w + c]).
//     Input 30 is the constant 1 (CHAIN_BIAS_BIT).  Its row holds b1, so the layer-1
//     products include the bias, and dW1's row 30 is gb1;
//   * forward twice from the same registers: Z1 sample-major (D row = sample, for the
//     backward and dW1) and Z1^T hidden-major (D row = hidden: layer 2 is then 4 lane-local
//     FMAs per output plus two permlane swaps instead of a 16-lane reduction);
//   * dW1 = X^T dZ1 with K = samples (K slot 8g + j <-> sample 16 (j >> 2) + 4g + (j & 3));
//   * every bit operand comes ready-made from the step record (StepRec: the prep kernels
//     expand the masks and their bit transpose).  Records pass through a 4-slot LDS ring:
//     each wave loads a quarter of record t + 2 during step t, and step t + 1's barrier
//     publishes it;
//   * one barrier per step (the 4 waves' layer-2 partials); all other exchange is
//     wave-private (LDS dm / w2t) or cross-lane (DPP, permlane).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifdef NFSP_CHAIN_STAMPS
// diagnostic build: [AR blk 0, AR blk 1, BR, -][wave][phase 0-5, -, -, kernel cycles, steps]
__device__ unsigned long long g_chain_stamps[4][4][10];
#endif

// Stores are unconditional: lanes whose copy is redundant (the odd lane rows of po / dm, the
// rows g > 0 of w2t, the lanes past a record quarter) write to sink rows nobody reads, so
// the loop has no exec-mask branches.
struct Chain3Smem {
  float po[2][4][64][4];     // per-wave partial layer-2 outputs by sample (rows 32..63: sink),
                             // double-buffered by step parity
  float dm[4][3][64];        // wave-private: dL/dz2 of the 32 samples, by output (32..63: sink)
  float4 w2t[4][64];         // wave-private: W2[h][0..2] of the slice for Z1^T (lane l writes
                             // row l; rows 0..15 are read)
  StepRec ring[4];           // step records t .. t + 2 (slot t & 3), a quarter per wave
  uint4 rec_sink[64];
};
constexpr int REC_CHUNKS = (int)(sizeof(StepRec) / 16);    // 288 x 16 B
constexpr int REC_QUARTER = REC_CHUNKS / 4;                 // 72 per wave
static_assert(REC_CHUNKS % 4 == 0 && REC_QUARTER > 64 && REC_QUARTER <= 128, "record chunking");
// Reserve (nearly) all of a CU's LDS for a chain workgroup: a chain then has its CU to
// itself -- no prep / target kernel's waves share its SIMDs.
constexpr int CHAIN_LDS = 150 * 1024;
static_assert(sizeof(Chain3Smem) <= CHAIN_LDS, "chain LDS");

// exact three-term bf16 split of 8 f32 values, a pair at a time: one packed conversion
// per pair and level (v_cvt_pk_bf16_f32, round to nearest even), the two f32 values of the
// packed pair by shift / mask, and the two residuals.  v = hi + mid + lo exactly.
// (inline asm: as plain conversions the compiler re-derives the low half by a second
// single-value conversion instead of shifting the packed word)
__device__ inline uint32_t cvt_pk_bf16(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ inline void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma clang fp contract(off)
  uint32_t h[4], m[4], o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = v[2 * k], b = v[2 * k + 1];
    h[k] = cvt_pk_bf16(a, b);
    const float ra = a - __uint_as_float(h[k] << 16), rb = b - __uint_as_float(h[k] & 0xFFFF0000u);
    m[k] = cvt_pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(m[k] << 16), sb = rb - __uint_as_float(m[k] & 0xFFFF0000u);
    o[k] = cvt_pk_bf16(sa, sb);
  }
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  mid = __builtin_bit_cast(bf16x8, make_uint4(m[0], m[1], m[2], m[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
}

__device__ inline floatx4 mfma3(bf16x8 a, bf16x8 bhi, bf16x8 bmid, bf16x8 blo) {
  floatx4 z = {};
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, blo, z, 0, 0, 0);
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bmid, z, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bhi, z, 0, 0, 0);
}
__device__ inline floatx4 mfma3t(bf16x8 ahi, bf16x8 amid, bf16x8 alo, bf16x8 b) {
  floatx4 z = {};
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, b, z, 0, 0, 0);
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(amid, b, z, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, b, z, 0, 0, 0);
}

template <int RELU, int LOSS>
__global__ void __launch_bounds__(256) k_chain3(ChainArgs C) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Chain3Smem& sm = *reinterpret_cast<Chain3Smem*>(smem_raw);
  const int a = C.agents[blockIdx.x];
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = tid & 63;
  const int g = l >> 4, c = l & 15;
  const int hid = 16 * w + c;
  const int sl = 16 * (g >> 1) + c;            // this lane's loss sample
  float* gw = C.w[blockIdx.x];
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
  const int64_t slot0 = (int64_t)a * C.umax;
  const int64_t u1 = C.u1[blockIdx.x];
  int64_t u0 = C.u0[blockIdx.x];
  if (C.active) {          // AR: skip the inactive prefix (M_SL <= batch; monotone in u)
    while (u0 < u1) {
      const int64_t q = u0 + l;
      const unsigned long long m = __ballot(q < u1 && C.active[slot0 + q]);
      if (m) { u0 += __builtin_ctzll(m); break; }
      u0 += 64;
    }
    if (u0 > u1) u0 = u1;
  }
  const int T1 = (int)(u1 * spu);
  int t = (int)(u0 * spu);
  const uint4* recb = reinterpret_cast<const uint4*>(C.rec + slot0 * spu);
  // this wave's quarter of record p (clamped), into two registers / back into ring slot p & 3;
  // the lanes past the quarter load a duplicate chunk and store it to the sink
  const bool in_q = l < REC_QUARTER - 64;
  const int lb = in_q ? 64 + l : REC_QUARTER - 1;
  auto issue = [&](int p, uint4& va, uint4& vb) {
    const uint4* src = recb + (size_t)(p < T1 ? p : T1 - 1) * REC_CHUNKS + REC_QUARTER * w;
    va = src[l];
    vb = src[lb];
  };
  auto stash = [&](int p, const uint4& va, const uint4& vb) {
    uint4* dst = reinterpret_cast<uint4*>(&sm.ring[p & 3]) + REC_QUARTER * w;
    dst[l] = va;
    *(in_q ? dst + 64 + l : &sm.rec_sink[l]) = vb;
  };
  auto publish = [&]() {   // this wave's W2 rows for its own Z1^T layer 2
    sm.w2t[w][l] = make_float4(W2_0, W2_1, W2_2, 0.f);
  };
  const int prow = 32 * (g & 1) + sl;          // po / dm row: the sample, or the sink
#ifdef NFSP_CHAIN_STAMPS
  unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_last = 0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
  const unsigned long long st_t0 = st_last;
#endif
  // Records reach the lanes through an LDS ring: at step t each wave loads its quarter of
  // record t + 2 and stores it at the end of step t; barrier(t + 1) publishes it.  Every
  // load is consumed inside its own step (nothing loop-carried in registers), and the 4
  // waves share one copy of each record.
  float loss_acc = 0.f;                        // wave 0 lane 0: running epoch loss
  auto step = [&]() {
    uint4 va, vb;
    issue(t + 2, va, vb);
    const StepRec& R = sm.ring[t & 3];
    const bf16x8 fa0 = __builtin_bit_cast(bf16x8, R.fa[g][c]);
    const bf16x8 fa1 = __builtin_bit_cast(bf16x8, R.fa[g][16 + c]);
    const bf16x8 ba0 = __builtin_bit_cast(bf16x8, R.ba[g][c]);
    const bf16x8 ba1 = __builtin_bit_cast(bf16x8, R.ba[g][16 + c]);
    // ---- layer 1, both orientations
    bf16x8 whi, wmid, wlo;
    split3(wr, whi, wmid, wlo);
    float W2h[4][3];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float4 q = sm.w2t[w][4 * g + r];
      W2h[r][0] = q.x; W2h[r][1] = q.y; W2h[r][2] = q.z;
    }
    // Z1^T first (layer 2 waits on it); Z1 (needed only by the backward) is issued after
    // layer 2, so its matrix-core time overlaps the barrier wait
    const floatx4 zh0 = mfma3t(whi, wmid, wlo, fa0);     // Z1^T: hidden 16w+4g+r, sample c
    const floatx4 zh1 = mfma3t(whi, wmid, wlo, fa1);     //                      sample 16+c
    __builtin_amdgcn_sched_barrier(0);
    CHAIN_STAMP(0);
    // ---- layer 2 partial over the slice, from Z1^T
    float p0[3], p1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { p0[k] = 0.f; p1[k] = 0.f; }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float h0 = fmaxf(zh0[r], 0.f);        // b1 is W1's row 30 (CHAIN_BIAS_IN)
      const float h1 = fmaxf(zh1[r], 0.f);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        p0[k] = p0[k] + h0 * W2h[r][k];
        p1[k] = p1[k] + h1 * W2h[r][k];
      }
    }
    float q[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {   // rows g, g ^ 2 (tile halves), then g ^ 1
      const auto rr = __builtin_amdgcn_permlane32_swap(__float_as_uint(p0[k]), __float_as_uint(p1[k]),
                                                       false, false);
      q[k] = sum_x16(__uint_as_float(rr[0]) + __uint_as_float(rr[1]));
    }
    const int buf = t & 1;
    *reinterpret_cast<float4*>(&sm.po[buf][w][prow][0]) = make_float4(q[0], q[1], q[2], 0.f);
    __builtin_amdgcn_sched_barrier(0);
    const floatx4 zs0 = mfma3(fa0, whi, wmid, wlo);      // Z1: sample 4g+r, hidden 16w+c
    const floatx4 zs1 = mfma3(fa1, whi, wmid, wlo);      //     sample 16+4g+r
    const float4 tg = R.tg[sl];                          // read before the barrier pins it early
    __builtin_amdgcn_sched_barrier(0);                   // ... and the Z1 MFMAs issue before it
    CHAIN_STAMP(1);
    __syncthreads();
    CHAIN_STAMP(2);
    // ---- output + loss of sample sl (every wave redundantly, identical results)
    float d0, d1, d2, lr_step;
    float o_keep[3], tt_keep[3], p_keep[3];     // for the optional loss log
    {
      const float4 a0 = *reinterpret_cast<const float4*>(&sm.po[buf][0][sl][0]);
      const float4 a1 = *reinterpret_cast<const float4*>(&sm.po[buf][1][sl][0]);
      const float4 a2 = *reinterpret_cast<const float4*>(&sm.po[buf][2][sl][0]);
      const float4 a3 = *reinterpret_cast<const float4*>(&sm.po[buf][3][sl][0]);
      const float o0 = (((a0.x + a1.x) + a2.x) + a3.x) + b2_0;
      const float o1 = (((a0.y + a1.y) + a2.y) + a3.y) + b2_1;
      const float o2 = (((a0.z + a1.z) + a2.z) + a3.z) + b2_2;
      lr_step = tg.w;
      const float tt[3] = {tg.x, tg.y, tg.z};
      o_keep[0] = o0; o_keep[1] = o1; o_keep[2] = o2;
      tt_keep[0] = tg.x; tt_keep[1] = tg.y; tt_keep[2] = tg.z;
      if (RELU) {          // Huber on ReLU outputs, mean over 3 x batch
        const float oz[3] = {o0, o1, o2};
        float dd[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float ee = tt[k] - fmaxf(oz[k], 0.f);
          // |e| > 1 ? sign(e) : e  ==  clamp(e, -1, 1)
          const float gg = __builtin_amdgcn_fmed3f(ee, -1.f, 1.f);
          dd[k] = oz[k] > 0.f ? gg * -inv3m : 0.f;
        }
        d0 = dd[0]; d1 = dd[1]; d2 = dd[2];
      } else {
        // Keras categorical cross-entropy on the softmax (normalise p = y / S, clip p to
        // [1e-7, 1 - 1e-7], loss -sum t log p; mean over the batch).  Its gradient w.r.t.
        // the logits in closed form, with M = the unclipped outputs (the clip's gradient
        // is 0 elsewhere) and T_M = sum_{k in M} t_k:
        //   d_k = (y_k T_M / S - [k in M] t_k) / batch
        // (the chain rule through normalise and softmax; the cancelling terms removed --
        // oracle/nn_oracle.py evaluates the unsimplified chain)
        const float mx = fmaxf(fmaxf(o0, o1), o2);
        const float e0 = __expf(o0 - mx), e1 = __expf(o1 - mx), e2 = __expf(o2 - mx);
        const float rs = __builtin_amdgcn_rcpf((e0 + e1) + e2);
        const float y0 = e0 * rs, y1 = e1 * rs, y2 = e2 * rs;
        const float rS = __builtin_amdgcn_rcpf((y0 + y1) + y2);
        const float eps = 1e-7f, hi = 1.0f - 1e-7f;
        const float q0 = y0 * rS, q1 = y1 * rS, q2 = y2 * rS;
        p_keep[0] = q0; p_keep[1] = q1; p_keep[2] = q2;
        // q in [eps, 1 - eps]  <=>  clamp(q, eps, 1 - eps) == q
        const float m0 = __builtin_amdgcn_fmed3f(q0, eps, hi) == q0 ? tt[0] : 0.f;
        const float m1 = __builtin_amdgcn_fmed3f(q1, eps, hi) == q1 ? tt[1] : 0.f;
        const float m2 = __builtin_amdgcn_fmed3f(q2, eps, hi) == q2 ? tt[2] : 0.f;
        // AR records carry t / batch (k_ar_prep; a power-of-two scale, exact), so the 1 / batch
        // of both terms is already in m_k
        const float k = ((m0 + m1) + m2) * rS;
        d0 = y0 * k - m0;
        d1 = y1 * k - m1;
        d2 = y2 * k - m2;
      }
    }
    if (LOSS) {            // fit loss of this minibatch (before its update), Keras' epoch mean
      float Ls;
      if (RELU) {          // huber_loss with py2's 1 / 2 == 0: |e| > 1 ? |e| : e^2 / 2, mean over 3
        float acc = 0.f;
        for (int k = 0; k < 3; ++k) {
          const float e = tt_keep[k] - fmaxf(o_keep[k], 0.f);
          acc += fabsf(e) > 1.0f ? fabsf(e) : 0.5f * e * e;
        }
        Ls = acc * (1.0f / 3.0f);
      } else {             // categorical cross-entropy: -sum t log(clip(y / S))
        float acc = 0.f;
        for (int k = 0; k < 3; ++k)      // (tt_keep = t / batch)
          acc -= (tt_keep[k] * (float)CHAIN_MB) * __logf(fminf(fmaxf(p_keep[k], 1e-7f), 1.0f - 1e-7f));
        Ls = acc;
      }
      float x = (g & 1) == 0 ? Ls : 0.f;     // the 32 distinct samples: rows 0 and 2
      x = x + dpp_any(x, 0x128);
      x = x + dpp_any(x, 0x124);
      x = x + dpp_any(x, 0x122);
      x = x + dpp_any(x, 0x121);
      x = sum_x32(sum_x16(x));
      if (w == 0 && l == 0) {
        const int in_u = t % spu;
        loss_acc += x * invm;
        if (in_u % nmb == nmb - 1) {
          const int64_t uu = t / spu, ee = in_u / nmb;
          C.loss_out[(slot0 + uu) * C.E + ee] = loss_acc / (float)nmb;
          loss_acc = 0.f;
        }
      }
    }
    sm.dm[w][0][prow] = d0;
    sm.dm[w][1][prow] = d1;
    sm.dm[w][2][prow] = d2;
    float gb2[3] = {d0, d1, d2};     // sum over the 32 samples: the row's 16, then rows g ^ 2
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float x = gb2[k];
      x = x + dpp_any(x, 0x128);
      x = x + dpp_any(x, 0x124);
      x = x + dpp_any(x, 0x122);
      x = x + dpp_any(x, 0x121);
      gb2[k] = sum_x32(x);
    }
    CHAIN_STAMP(3);
    // ---- backward in the sample-major layout: samples 16 mt + 4g + r, hidden 16w + c
    float4 dA[3], dB[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      dA[k] = *reinterpret_cast<const float4*>(&sm.dm[w][k][4 * g]);
      dB[k] = *reinterpret_cast<const float4*>(&sm.dm[w][k][16 + 4 * g]);
    }
    float dz[8];
    float g2_0 = 0.f, g2_1 = 0.f, g2_2 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = j & 3;
      const float z = j < 4 ? zs0[r] : zs1[r];
      const float4 e0 = j < 4 ? dA[0] : dB[0], e1 = j < 4 ? dA[1] : dB[1], e2 = j < 4 ? dA[2] : dB[2];
      const float x0 = r == 0 ? e0.x : r == 1 ? e0.y : r == 2 ? e0.z : e0.w;
      const float x1 = r == 0 ? e1.x : r == 1 ? e1.y : r == 2 ? e1.z : e1.w;
      const float x2 = r == 0 ? e2.x : r == 1 ? e2.y : r == 2 ? e2.z : e2.w;
      const float h = fmaxf(z, 0.f);
      g2_0 += h * x0;
      g2_1 += h * x1;
      g2_2 += h * x2;
      const float dh = (x0 * W2_0 + x1 * W2_1) + x2 * W2_2;
      dz[j] = z > 0.f ? dh : 0.f;
    }
    bf16x8 dhi, dmid, dlo;
    split3(dz, dhi, dmid, dlo);
    // dW1[16 it + 4g + r][16w + c] = sum over the 32 samples in dz's K order (row 30: gb1)
    const floatx4 gA = mfma3(ba0, dhi, dmid, dlo);
    const floatx4 gB = mfma3(ba1, dhi, dmid, dlo);
    g2_0 = sum_x16(sum_x32(g2_0));
    g2_1 = sum_x16(sum_x32(g2_1));
    g2_2 = sum_x16(sum_x32(g2_2));
    CHAIN_STAMP(4);
    const float lr = lr_step;
    W2_0 = W2_0 - lr * g2_0;
    W2_1 = W2_1 - lr * g2_1;
    W2_2 = W2_2 - lr * g2_2;
    b2_0 = b2_0 - lr * gb2[0];
    b2_1 = b2_1 - lr * gb2[1];
    b2_2 = b2_2 - lr * gb2[2];
    publish();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      wr[r] = wr[r] - lr * gA[r];
      wr[4 + r] = wr[4 + r] - lr * gB[r];
    }
    stash(t + 2, va, vb);
    CHAIN_STAMP(5);
  };
  if (t < T1) {
    {
      uint4 va, vb;
      issue(t, va, vb);
      stash(t, va, vb);
      issue(t + 1, va, vb);
      stash(t + 1, va, vb);
    }
    publish();
    __syncthreads();
    // drain the prologue's loads: the loop header then merges no pending load into the
    // registers the loop reuses (else every step waits on its fresh record load)
    __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15)
    for (; t < T1; ++t) step();
  }
#ifdef NFSP_CHAIN_STAMPS
  if (l == 0) {
    unsigned long long t_end;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_end)::"memory");
    st_acc[8] = t_end - st_t0;
    st_acc[9] = (unsigned long long)(T1 - (int)(u0 * spu));
    if (C.stamps) {
      for (int k = 0; k < 10; ++k) C.stamps[(blockIdx.x * 4 + w) * 10 + k] = st_acc[k];
    } else {       // engine build: accumulate per (net, block, wave) for nfsp_debug_chain_stamps
      for (int k = 0; k < 10; ++k) atomicAdd(&g_chain_stamps[RELU * 2 + blockIdx.x][w][k], st_acc[k]);
    }
  }
#endif
  float* dsts[2] = {gw, C.sync_to[blockIdx.x]};
  for (int k = 0; k < 2; ++k) {
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
    if (w == 0 && l == 0) {
      dst[nn::OB2 + 0] = b2_0;
      dst[nn::OB2 + 1] = b2_1;
      dst[nn::OB2 + 2] = b2_2;
    }
  }
}

// schedule state after the learner (host-computed values + device-side counters)
struct FinalArgs {
  EngineDev* st;
  const double* br_expl;
  int64_t umax;
  int64_t n_rl[2], n_sl[2], U_br[2];
  int64_t iteration[2], tcount[2], syncs[2];
  double eps[2], temp[2];
  float lr[2];
  int64_t sl_cap;
};

__global__ void k_finalize(FinalArgs F) {
  if (threadIdx.x != 0) return;
  for (int a = 0; a < 2; ++a) {
    EngineDev* st = F.st;
    st->rl_total[a] += F.n_rl[a];
    st->sl_total[a] += F.n_sl[a];
    st->sl_count[a] = st->sl_total[a] < F.sl_cap ? st->sl_total[a] : F.sl_cap;
    if (F.U_br[a] > 0) {
      st->expl[a] = F.br_expl[(int64_t)a * F.umax + F.U_br[a] - 1];
      st->br_updates[a] += F.U_br[a];
      st->iteration[a] = F.iteration[a];
      st->target_count[a] = F.tcount[a];
      st->target_syncs[a] = F.syncs[a];
      st->epsilon[a] = F.eps[a];
      st->temp[a] = F.temp[a];
      st->lr_br[a] = F.lr[a];
    }
  }
}

}  // namespace

#ifdef NFSP_CHAIN_STAMPS
// diagnostic build only: the accumulated chain phase cycles ([4][4][10] u64), then reset
extern "C" int nfsp_debug_chain_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_stamps), sizeof(g_chain_stamps)) != hipSuccess) return -1;
  static const unsigned long long zero[4][4][10] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_chain_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int nfsp_engine_update(nfsp_engine* e) {
  NFSP_REQUIRE(e, "null argument");
  if (!e->pending_update) return NFSP_OK;
  e->pending_update = false;
  hipStream_t s = e->ctx->stream;
  const nfsp_engine_cfg& cfg = e->cfg;
  // the trigger plan needs the rollout's insert counts: one small readback
  EngineDev h;
  NFSP_HIP(hipMemcpyAsync(&h, e->st, sizeof(h), hipMemcpyDeviceToHost, s));
  NFSP_HIP(hipStreamSynchronize(s));
  KTimer kt(e, KT_LEARNER);
  e->learn_tag++;
  PrepArgs P{};
  P.M = e->M;
  P.LB = e->LB;
  P.st = e->st;
  P.c = cfg.inserts_per_update;
  P.rl_cap = cfg.rl_capacity;
  P.B = cfg.batch;
  P.E = cfg.epochs;
  P.k0 = (uint32_t)cfg.seed;
  P.k1 = (uint32_t)(cfg.seed >> 32);
  P.tag = e->learn_tag;
  P.lr_ar = cfg.lr_ar;
  int64_t maxU = 0, maxUbr = 0, maxSL = 0;
  for (int a = 0; a < 2; ++a) {
    AgentPlan& pl = P.A[a];
    pl.P0 = h.rl_total[a];
    const int64_t n = h.last_rl[a];
    pl.m_first = pl.P0 / P.c + 1;
    const int64_t m_last = (pl.P0 + n) / P.c;
    pl.U = m_last >= pl.m_first ? m_last - pl.m_first + 1 : 0;
    // BR update iff min(p_m, cap) > batch  <=>  m * c > batch
    pl.m_br0 = pl.m_first > cfg.batch / P.c + 1 ? pl.m_first : cfg.batch / P.c + 1;
    pl.U_br = m_last >= pl.m_br0 ? m_last - pl.m_br0 + 1 : 0;
    pl.n_sl = h.last_sl[a];
    pl.sl_total0 = h.sl_total[a];
    NFSP_REQUIRE(pl.U <= e->LB.umax, "update plan exceeds the learner buffers");
    maxU = pl.U > maxU ? pl.U : maxU;
    maxUbr = pl.U_br > maxUbr ? pl.U_br : maxUbr;
    maxSL = pl.n_sl > maxSL ? pl.n_sl : maxSL;
  }
  // ---- parallel prep on the ctx stream
  {
  KTimer kprep(e, KT_PREP);
  if (maxUbr > 0) {
    k_br_prep<<<dim3((unsigned)maxUbr, 2), 128, 0, s>>>(P);
    NFSP_LAUNCHED("k_br_prep");
  }
  if (maxSL > 0) {
    k_ar_slots<<<dim3(nfsp_blocks(maxSL, 256), 2), 256, 0, s>>>(P);
    NFSP_LAUNCHED("k_ar_slots");
  }
  if (maxU > 0) {
    k_ar_prep<<<dim3((unsigned)maxU, 2), 128, 0, s>>>(P);
    NFSP_LAUNCHED("k_ar_prep");
  }
  if (maxSL > 0) {
    k_res_apply<<<dim3(nfsp_blocks(maxSL, 256), 2), 256, 0, s>>>(P);
    NFSP_LAUNCHED("k_res_apply");
  }
  }
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)k_chain3<0, 0>, (const void*)k_chain3<1, 0>, (const void*)k_chain3<0, 1>,
                          (const void*)k_chain3<1, 1>})
      NFSP_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN_LDS));
    attr = true;
  }
  for (int a = 0; a < 2; ++a) {
    e->last_U[a] = P.A[a].U;
    e->last_Ubr[a] = P.A[a].U_br;
    if (e->log_loss) {       // NaN = no fit recorded (inactive AR update)
      NFSP_HIP(hipMemsetAsync(e->LB.ar_loss + a * e->LB.umax * cfg.epochs, 0xFF,
                              sizeof(float) * P.A[a].U * cfg.epochs, s));
      NFSP_HIP(hipMemsetAsync(e->LB.br_loss + a * e->LB.umax * cfg.epochs, 0xFF,
                              sizeof(float) * P.A[a].U_br * cfg.epochs, s));
    }
  }
  hipEvent_t fork = take_event(e);
  NFSP_HIP(hipEventRecord(fork, s));
  // ---- AR chains (both agents, one launch) on their own stream
  if (maxU > 0) {
    NFSP_HIP(hipStreamWaitEvent(e->s_ar, fork, 0));
    ChainArgs C{};
    C.rec = e->LB.ar_rec;
    C.loss_out = e->log_loss ? e->LB.ar_loss : nullptr;
    C.active = e->LB.ar_active;
    C.umax = e->LB.umax;
    C.B = cfg.batch;
    C.E = cfg.epochs;
    for (int a = 0; a < 2; ++a) {
      C.agents[a] = a;
      C.w[a] = e->w + (a * 3 + 0) * nn::NP;
      C.sync_to[a] = nullptr;
      C.u0[a] = 0;
      C.u1[a] = P.A[a].U;
    }
    KTimer kc(e, KT_CHAIN_AR, e->s_ar);
    if (C.loss_out) k_chain3<0, 1><<<2, 256, CHAIN_LDS, e->s_ar>>>(C);
    else k_chain3<0, 0><<<2, 256, CHAIN_LDS, e->s_ar>>>(C);
    NFSP_LAUNCHED("k_chain(AR)");
  }
  // diagnostic (NFSP_LEARNER_SERIAL=1): BR work waits for the AR chains, to time them alone
  static const bool serial_ar = getenv("NFSP_LEARNER_SERIAL") && atoi(getenv("NFSP_LEARNER_SERIAL"));
  hipEvent_t ar_done = fork;
  if (serial_ar) {
    ar_done = take_event(e);
    NFSP_HIP(hipEventRecord(ar_done, e->s_ar));
  }
  // ---- BR: per agent, segments between target syncs, each = targets + chain
  FinalArgs F{};
  F.st = e->st;
  F.br_expl = e->LB.br_expl;
  F.umax = e->LB.umax;
  F.sl_cap = cfg.sl_capacity;
  for (int a = 0; a < 2; ++a) {
    const AgentPlan& pl = P.A[a];
    F.n_rl[a] = h.last_rl[a];
    F.n_sl[a] = pl.n_sl;
    F.U_br[a] = pl.U_br;
    hipStream_t sa = e->s_br[a];
    NFSP_HIP(hipStreamWaitEvent(sa, serial_ar ? ar_done : fork, 0));
    int64_t it = h.iteration[a], tc = h.target_count[a], syncs = h.target_syncs[a];
    double eps = h.epsilon[a];
    const int64_t it0 = it;
    float* wbr = e->w + (a * 3 + 1) * nn::NP;
    float* wtg = e->w + (a * 3 + 2) * nn::NP;
    int64_t u = 0;
    while (u < pl.U_br) {
      // segment [u, v): ends after the first update whose target_count % every == 0
      int64_t v = u;
      bool sync = false;
      while (v < pl.U_br) {
        const bool s_here = (tc + (v - 0)) % cfg.target_every == 0;
        ++v;
        if (s_here) { sync = true; break; }
      }
      {
        KTimer kt2(e, KT_TARGETS, sa);
        k_br_targets<<<(unsigned)(v - u), 256, 0, sa>>>(e->LB, wtg, a, u, cfg.batch, cfg.epochs,
                                                         cfg.gamma, cfg.quirks, it0, cfg.lr_br);
      }
      NFSP_LAUNCHED("k_br_targets");
      ChainArgs C{};
      C.rec = e->LB.br_rec;
      C.loss_out = e->log_loss ? e->LB.br_loss : nullptr;
      C.active = nullptr;
      C.umax = e->LB.umax;
      C.B = cfg.batch;
      C.E = cfg.epochs;
      C.agents[0] = a;
      C.w[0] = wbr;
      C.sync_to[0] = sync ? wtg : nullptr;
      C.u0[0] = u;
      C.u1[0] = v;
      {
        KTimer kc(e, KT_CHAIN_BR, sa);
        if (C.loss_out) k_chain3<1, 1><<<1, 256, CHAIN_LDS, sa>>>(C);
        else k_chain3<1, 0><<<1, 256, CHAIN_LDS, sa>>>(C);
      }
      NFSP_LAUNCHED("k_chain(BR)");
      u = v;
    }
    // schedules (agent/agent.py:245-253, 266-273) in the reference's double arithmetic
    for (int64_t k = 0; k < pl.U_br; ++k) {
      if (tc % cfg.target_every == 0) syncs++;
      tc++;
      it += 2;
      eps = eps / (double)it;
    }
    F.iteration[a] = it;
    F.tcount[a] = tc;
    F.syncs[a] = syncs;
    F.eps[a] = eps;
    F.temp[a] = 1.0 / (1.0 + 0.02 * sqrt((double)it));
    F.lr[a] = (float)(cfg.lr_br / (1.0 + 0.003 * sqrt((double)it)));
  }
  // ---- join and publish the schedules
  for (hipStream_t st : {e->s_ar, e->s_br[0], e->s_br[1]}) {
    hipEvent_t j = take_event(e);
    NFSP_HIP(hipEventRecord(j, st));
    NFSP_HIP(hipStreamWaitEvent(s, j, 0));
    e->pool.push_back(j);      // reusable once the wait is enqueued
  }
  e->pool.push_back(fork);
  if (ar_done != fork) e->pool.push_back(ar_done);
  k_finalize<<<1, 64, 0, s>>>(F);
  NFSP_LAUNCHED("k_finalize");
  return NFSP_OK;
}
