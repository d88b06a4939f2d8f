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
#include <string.h>

#include "engine_internal.h"
#include "chain3.h"

using nfsp::u32x4;
namespace nn = nfsp::nn;
using namespace nfsp::eng;
using namespace nfsp::chain;

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
  uint32_t quirks;
};

// ---------------------------------------------------------------------------
// BR prep: rows of update u of agent a (agent/agent.py:217 sample_batch)
// ---------------------------------------------------------------------------
template <int TABLE>   // TABLE: engine groups, blockIdx.z = replica of `tab`
__global__ void __launch_bounds__(128) k_br_prep(PrepArgs P0, const PrepArgs* __restrict__ tab) {
  const PrepArgs& P = TABLE ? tab[blockIdx.z] : P0;
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
template <int TABLE>   // TABLE: engine groups, blockIdx.z = replica of `tab`
__global__ void __launch_bounds__(256) k_ar_slots(PrepArgs P0, const PrepArgs* __restrict__ tab) {
  const PrepArgs& P = TABLE ? tab[blockIdx.z] : P0;
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
    const int64_t j = (P.quirks & NFSP_EXT_RESERVOIR)
                          ? (int64_t)(r64 % (uint64_t)(tot + 1))  // Algorithm R: U{0..tot}
                          : 1 + (int64_t)(r64 % (uint64_t)cap);   // randrange(1, N + 1)
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

// The chain records of one (update, epoch): the thread of fit position b < B holds its
// observation mask x, targets and the lr; minibatch b >> 5 gets the swizzled fa chunks and
// tg of its sample b & 31 (the chain reads the transposed operand from fa itself).  Every
// valid sample also carries the bias input (CHAIN_BIAS_BIT).
__device__ inline void emit_recs(StepRec* __restrict__ recs, uint32_t x, float t0, float t1, float t2,
                                 float lr, int B, int b) {
  if (b < B) {
    x |= CHAIN_BIAS_BIT;
    StepRec& R = recs[b >> 5];
    const int k = b & 31;
#pragma unroll
    for (int g = 0; g < 4; ++g) R.fa[g][fa_slot(g, k)] = bits8u(x, g);
    R.tg[k] = make_float4(t0, t1, t2, lr);
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
template <int TABLE>   // TABLE: engine groups, blockIdx.z = replica of `tab`
__global__ void __launch_bounds__(128) k_ar_prep(PrepArgs P0, const PrepArgs* __restrict__ tab) {
  const PrepArgs& P = TABLE ? tab[blockIdx.z] : P0;
  __shared__ int64_t cand[MAX_BATCH];
  __shared__ uint32_t key[MAX_BATCH];
  __shared__ uint32_t rx[MAX_BATCH];
  __shared__ float ra[MAX_BATCH][3];
  __shared__ uint32_t px[MAX_BATCH];
  __shared__ float pt[MAX_BATCH][3];
  const int a = blockIdx.y;
  const int64_t u = blockIdx.x;
  const AgentPlan& pl = P.A[a];
  if (u >= pl.U) return;
  const int b = threadIdx.x;
  const int dbg = a * 2 + 0;
  const int64_t m = pl.m_first + u;
  const int64_t pm = m * P.c;
  const int64_t slot_u = (int64_t)a * P.LB.umax + u;
  // SL inserts made before the trigger (pend_pos is nondecreasing): a 128-ary search, a few
  // rounds of one probe per thread instead of one thread's ~20 dependent loads.  lo / hi
  // are block-uniform: every thread takes the same rounds.
  const int64_t* pos = P.M.pend_pos + (int64_t)a * P.M.pend_cap;
  const int nt = blockDim.x;
  int64_t lo = 0, hi = pl.n_sl;
  while (hi - lo > nt) {
    const int64_t span = hi - lo;       // probe t at lo + span (t + 1) / (nt + 1): increasing
    const int k = __syncthreads_count(pos[lo + span * (b + 1) / (nt + 1)] <= pm);
    const int64_t below = lo + span * k / (nt + 1);          // probe k - 1 (k >= 1)
    const int64_t above = lo + span * (k + 1) / (nt + 1);    // probe k (k < nt)
    lo = k > 0 ? below + 1 : lo;
    hi = k < nt ? above : hi;
  }
  const int64_t nb = lo + __syncthreads_count(lo + b < hi && pos[lo + b] <= pm);
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
              in ? pt[b][1] * sc : 0.f, in ? pt[b][2] * sc : 0.f, P.lr_ar, P.B, b);
    __syncthreads();
  }
  if (last && b < P.B) P.M.dbg_rows[dbg * P.B + b] = cand[b];
}

template <int TABLE>   // TABLE: engine groups, blockIdx.z = replica of `tab`
__global__ void __launch_bounds__(256) k_res_apply(PrepArgs P0, const PrepArgs* __restrict__ tab) {
  const PrepArgs& P = TABLE ? tab[blockIdx.z] : P0;
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
// One (engine, agent) segment: the agent's learner buffers (update u of the learner call at
// index u), the target net, and the segment's update range [u0, u0 + n).
struct TargetJob {
  const BrRow* rows;   // [umax][B]
  const uint8_t* perm; // [umax][E][B]
  double* expl;        // [umax]
  StepRec* rec;        // [umax][E][B / 32]
  const float* tw;     // target net
  int64_t u0, n;
  int64_t it0;         // the agent's iteration count before the learner call
};

// blockIdx.x = update within the segment; blockIdx.y = job (of `jobs`, else `one`)
__global__ void __launch_bounds__(256) k_br_targets(const TargetJob* __restrict__ jobs, TargetJob one,
                                                    int B, int E, double gamma, unsigned quirks,
                                                    double lr0) {
  const TargetJob J = jobs ? jobs[blockIdx.y] : one;
  const int64_t bx = blockIdx.x;
#include "br_targets_body.inc"
}

// one update's targets by the calling workgroup (k_br_persist's helpers): the same body
__device__ __forceinline__ void br_targets_item(const TargetJob J, int64_t bx, int B, int E, double gamma,
                                                unsigned quirks, double lr0) {
#include "br_targets_body.inc"
}

// ---------------------------------------------------------------------------
// k_br_persist: an engine group's whole BR learner call in one launch (nfsp_group_sched.br_persist;
// round 5, re-landed in round 6 -- DESIGN.md Appendix A.1b).  Workgroups 0 .. njobs - 1 are
// chains, one per (replica, agent) with BR work: each runs its target-sync segments in order,
// in pieces of `chunk` updates, each piece as soon as its targets are written.  The others are
// helpers: they take work items -- (segment, update) -- in queue order and write that update's
// targets and step records (k_br_targets' body).  The host queues the first segments' items; a
// chain queues its next segment's items once the segment's last piece has synced the target
// net they read.  No round waits for another job's segment and no targets launch sits between
// chains.  The same SGD steps as the rounds, bit for bit (a piece resumes from the weights in
// memory).
// Hand-offs, agent scope (per-XCD L2s): the writer's stores, __threadfence in every writing
// thread, the workgroup barrier, then one release atomic; the reader polls relaxed in one
// thread, then one acquire fence and the workgroup barrier.  Every wait is bounded (spin x
// s_sleep 8): on expiry *err is set and the workgroup leaves, so a lost hand-off ends the
// kernel; the host reports it (group_check_err).
// Loop shape: each loop has ONE thread-0 region per iteration, at its top, and the iteration
// ends on a barrier.  The round-5 form also had a thread-0 region at the bottom (the helper's
// "item done" atomic); the compiler merged the two across the back edge into a loop of their
// own, which left the barrier-bearing body as an inner loop that lanes 1-63 of wave 0 and waves
// 1-3 iterated on the stale work word while lane 0 waited for them to leave it: the hang of
// profiles/r05_group_br_persist (found in round 6 in the ISA, profiles/r06/persist_rootcause).
// The words that end the loops (a bail, the next item) are read through readfirstlane, so the
// loops' exits are scalar branches, and a job's fields are made scalar (brp_uniform).
// ---------------------------------------------------------------------------
struct BrPersistArgs {
  ChainArgs C;                  // B, E (the chains' jobs come from seg_job)
  const ChainJob* seg_job;      // [nseg] chain job of each segment (u0, u1: the segment; sync_to)
  const TargetJob* seg_tgt;     // [nseg] its targets job
  const int32_t* seg_chunk0;    // [nseg] its first chunk counter
  const int32_t* job_seg0;      // [njobs + 1] chain workgroup j's segments: [job_seg0[j], job_seg0[j + 1])
  uint32_t* slots;              // [nitems] work items (segment << 16 | update in it); BRP_EMPTY until queued
  uint32_t* ctr;                // [0] helpers' claims, [1] queue reservations
  uint32_t* chunk_done;         // finished items per chunk
  int32_t* err;                 // pinned host: [0] a wait expired, [1] chain bails, [2] helper bails
  int njobs, nitems, chunk;
  int spin;                     // bound of every wait (s_sleep 8 rounds)
  double gamma, lr0;
  unsigned quirks;
};
constexpr uint32_t BRP_EMPTY = 0xFFFFFFFFu, BRP_DONE = 0xFFFFFFFEu;
constexpr int BRP_SPIN = 1 << 18;           // x s_sleep 8 (~56 ms): far past any legitimate wait
constexpr int BRP_CHUNK = 16;               // updates per chain piece (readiness is checked per piece)
constexpr int BRP_HELPERS = 48;             // helper workgroups (c4_emul_r8, timeline tool, with
                                            // the scalar jobs: 96 / 144 / 192 helpers 193.1 /
                                            // 189.5 / 188.1 ms, the AR chains slowing 155 -> 166;
                                            // the rounds 179.6)
constexpr int BRP_STATIC_LDS = 16 * 1024;   // bound on the kernel's static LDS (the targets buffers)

#ifdef NFSP_BRP_STAMPS
// diagnostic build only (tools/build_lib_variant.py brpst -DNFSP_BRP_STAMPS=1, tools/brp_stamps.py):
// per chain [wait cycles, chain cycles, SGD steps, pieces], per helper [wait, work, items, 0]
__device__ unsigned long long g_brp_stamps[2][64][4];
#define BRP_T() __builtin_amdgcn_s_memtime()
#endif

// A job read from the tables arrives in VGPRs (vector loads: the kernel writes global memory,
// so no scalar loads); readfirstlane makes its fields scalar again, as k_chain3's kernel-argument
// jobs are -- otherwise every record load's buffer descriptor becomes a readfirstlane loop
__device__ __forceinline__ int64_t brp_u64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <class T>
__device__ __forceinline__ T* brp_ptr(T* p) { return reinterpret_cast<T*>(brp_u64(reinterpret_cast<int64_t>(p))); }
__device__ __forceinline__ ChainJob brp_uniform(ChainJob J) {
  J.w = brp_ptr(J.w);
  J.sync_to = brp_ptr(J.sync_to);
  J.snap_to = brp_ptr(J.snap_to);
  J.rec = brp_ptr(J.rec);
  J.active = brp_ptr(J.active);
  J.loss_out = brp_ptr(J.loss_out);
  J.u0 = brp_u64(J.u0);
  J.u1 = brp_u64(J.u1);
  return J;
}

__device__ __forceinline__ void brp_bail(int32_t* err, int k) {
  __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_fetch_add(err + k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(256) k_br_persist(BrPersistArgs P) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  __shared__ uint32_t s_word;
#ifdef NFSP_BRP_STAMPS
  unsigned long long st_wait = 0, st_chain = 0, st_steps = 0, st_pieces = 0, st_t1 = 0;
#endif
  if ((int)blockIdx.x < P.njobs) {                         // ---- a chain
    const int j = blockIdx.x;
    for (int s = P.job_seg0[j]; s < P.job_seg0[j + 1]; ++s) {
      const ChainJob JS = brp_uniform(P.seg_job[s]);
      for (int64_t a = JS.u0, c = 0; a < JS.u1; a += P.chunk, ++c) {
        const int64_t b = a + P.chunk < JS.u1 ? a + P.chunk : JS.u1;
        if (threadIdx.x == 0) {                            // the iteration's one thread-0 region
#ifdef NFSP_BRP_STAMPS
          const unsigned long long t0 = BRP_T();
          if (st_t1) st_chain += t0 - st_t1;
#endif
          const uint32_t* done = &P.chunk_done[P.seg_chunk0[s] + c];
          int it = 0;
          while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)(b - a) &&
                 ++it < P.spin)
            __builtin_amdgcn_s_sleep(8);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          s_word = it >= P.spin;
          if (s_word) brp_bail(P.err, 1);
#ifdef NFSP_BRP_STAMPS
          st_t1 = BRP_T();
          st_wait += st_t1 - t0;
          st_steps += (b - a) * P.C.E * (P.C.B / CHAIN_MB);
          ++st_pieces;
#endif
        }
        __syncthreads();
        // readfirstlane: the compiler then knows the value is uniform -- a scalar branch, a loop
        // with uniform exits (with a vector value the loop's exits are divergent, values carried
        // in it are taken as divergent and every record load's buffer descriptor became a
        // readfirstlane loop: 1,280 instructions per 4 steps against k_chain3's 1,217)
        if (__builtin_amdgcn_readfirstlane(s_word)) return; // workgroup-uniform
        ChainJob JP = JS;
        JP.u0 = a;
        JP.u1 = b;
        if (b < JS.u1) JP.sync_to = nullptr;               // the segment's last piece syncs
        chain3_run<1, 0, 1>(P.C, JP, smem_raw);
        __threadfence();        // the piece's weights (and synced target net) out, for the next
        __syncthreads();        // piece's loads by other waves and for the helpers
      }
      if (s + 1 < P.job_seg0[j + 1]) {                     // queue the next segment's items
        const uint32_t m = (uint32_t)P.seg_tgt[s + 1].n;
        if (threadIdx.x == 0) s_word = __hip_atomic_fetch_add(&P.ctr[1], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t base = __builtin_amdgcn_readfirstlane(s_word);
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x)
          __hip_atomic_store(&P.slots[base + i], ((uint32_t)(s + 1) << 16) | i, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();        // s_word is rewritten by the next wait
      }
    }
#ifdef NFSP_BRP_STAMPS
    if (threadIdx.x == 0) {
      if (st_t1) st_chain += BRP_T() - st_t1;
      unsigned long long* d = g_brp_stamps[0][j & 63];
      atomicAdd(d + 0, st_wait); atomicAdd(d + 1, st_chain); atomicAdd(d + 2, st_steps); atomicAdd(d + 3, st_pieces);
    }
#endif
    return;
  }
  uint32_t* prev_done = nullptr;                           // thread 0: the last item's chunk counter
  for (;;) {                                                // ---- a helper
    if (threadIdx.x == 0) {                                // the iteration's one thread-0 region:
#ifdef NFSP_BRP_STAMPS
      const unsigned long long t0 = BRP_T();
      if (st_t1) st_chain += t0 - st_t1;                   // (helpers: work cycles)
#endif
      if (prev_done)                                       // publish the last item, take the next
        __hip_atomic_fetch_add(prev_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t p = __hip_atomic_fetch_add(&P.ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t v = BRP_DONE;
      if (p < (uint32_t)P.nitems) {
        int it = 0;
        while ((v = __hip_atomic_load(&P.slots[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == BRP_EMPTY &&
               ++it < P.spin)
          __builtin_amdgcn_s_sleep(8);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (v == BRP_EMPTY) {
          brp_bail(P.err, 2);
          v = BRP_DONE;
        }
      }
      s_word = v;
#ifdef NFSP_BRP_STAMPS
      st_t1 = BRP_T();
      st_wait += st_t1 - t0;
      if (v != BRP_DONE) ++st_steps;
      if (v == BRP_DONE) {
        unsigned long long* d = g_brp_stamps[1][(blockIdx.x - P.njobs) & 63];
        atomicAdd(d + 0, st_wait); atomicAdd(d + 1, st_chain); atomicAdd(d + 2, st_steps);
      }
#endif
    }
    __syncthreads();
    const uint32_t v = __builtin_amdgcn_readfirstlane(s_word);
    __syncthreads();
    if (v == BRP_DONE) return;                             // workgroup-uniform (scalar)
    const int s = (int)(v >> 16);
    const int64_t i = (int64_t)(v & 0xFFFFu);
    br_targets_item(P.seg_tgt[s], i, P.C.B, P.C.E, P.gamma, P.quirks, P.lr0);
    __threadfence();
    __syncthreads();
    prev_done = &P.chunk_done[P.seg_chunk0[s] + i / P.chunk];
  }
}

// launch with a CU per workgroup: dynamic LDS up to what the CU has left beside the kernel's
// static LDS (the helpers' targets buffers), as the one-engine chains reserve theirs
int launch_br_persist(const BrPersistArgs& P, int helpers, hipStream_t s) {
  static std::atomic<uint64_t> mask{0};
  static std::atomic<int> dyn{0};
  int dev = 0;
  NFSP_HIP(hipGetDevice(&dev));
  const uint64_t bit = 1ull << (dev & 63);
  if (!(mask.load(std::memory_order_acquire) & bit)) {
    hipFuncAttributes fa{};
    NFSP_HIP(hipFuncGetAttributes(&fa, (const void*)k_br_persist));
    if ((int)fa.sharedSizeBytes > BRP_STATIC_LDS) return nfsp::fail(NFSP_EINVAL, "k_br_persist: static LDS");
    const int d = CHAIN_LDS - BRP_STATIC_LDS;
    if (d < (int)sizeof(Chain3Smem)) return nfsp::fail(NFSP_EINVAL, "k_br_persist: LDS");
    NFSP_HIP(hipFuncSetAttribute((const void*)k_br_persist, hipFuncAttributeMaxDynamicSharedMemorySize, d));
    dyn.store(d, std::memory_order_release);
    mask.fetch_or(bit, std::memory_order_acq_rel);
  }
  k_br_persist<<<P.njobs + helpers, 256, dyn.load(std::memory_order_acquire), s>>>(P);
  NFSP_LAUNCHED("k_br_persist");
  return NFSP_OK;
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

// mode bits: 1 = the insert counters (both agents; they must be current before the next
// rollout's commit), 2 << a = agent a's learner results and schedules (after its BR chain)
template <int TABLE>   // TABLE: engine groups, block = replica of `tab`
__global__ void k_finalize(FinalArgs F0, const FinalArgs* __restrict__ tab, int mode) {
  const FinalArgs& F = TABLE ? tab[blockIdx.x] : F0;
  if (threadIdx.x != 0) return;
  for (int a = 0; a < 2; ++a) {
    EngineDev* st = F.st;
    if (mode & 1) {
      st->rl_total[a] += F.n_rl[a];
      st->sl_total[a] += F.n_sl[a];
      st->sl_count[a] = st->sl_total[a] < F.sl_cap ? st->sl_total[a] : F.sl_cap;
    }
    if ((mode & (2 << a)) && F.U_br[a] > 0) {
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

// engine groups: the exchanged nets of all replicas <- W0 + (sum_r (W_r - W0)) * scale, and W0 <-
// that (nfsp_engine_set_exchange's arithmetic over shards, on device, in replica order).
// wtab [3 nets: AR, BR, target][R][2 agents]; nets / bcast: masks over the 3 (bcast: the first
// exchange of a net copies replica 0's everywhere)
__global__ void __launch_bounds__(256) k_group_xchg(float* const* __restrict__ wtab, float* __restrict__ w0 /*[3][2][NP]*/,
                                                    int R, unsigned nets, unsigned bcast, float scale) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * 2 * nn::NP) return;
  const int n = i / (2 * nn::NP), k = i - n * 2 * nn::NP;
  const int a = k / nn::NP, q = k - a * nn::NP;
  const bool b = (bcast >> n) & 1u;
  if (!b && !((nets >> n) & 1u)) return;
  float* const* war = wtab + (size_t)n * R * 2;
  float nw;
  if (b) {
    nw = war[a][q];
  } else {
    const float base = w0[i];
    float s = 0.f;
    // the sum stays in replica order; the unroll lets 16 replicas' loads go out together
    // (one at a time, R = 256 took 0.2 ms of latency per step)
#pragma unroll 16
    for (int r = 0; r < R; ++r) s = s + (war[2 * r + a][q] - base);
    nw = base + s * scale;
  }
  w0[i] = nw;
  for (int r = 0; r < R; ++r) war[2 * r + a][q] = nw;
}

}  // namespace

#ifdef NFSP_CHAIN_STAMPS
// diagnostic build only: the accumulated chain phase cycles ([8][4][10] u64), then reset
extern "C" int nfsp_debug_chain_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_stamps), sizeof(g_chain_stamps)) != hipSuccess) return -1;
  static const unsigned long long zero[8][4][10] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_chain_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

namespace {

// ---------------------------------------------------------------------------
// host side: one learner call = plan (from the rollout's insert counts) + prep launches +
// chain launches + finalize.  nfsp_engine_update runs them for one engine, the group for
// R engines with their chains in shared launches.
// ---------------------------------------------------------------------------
struct Segment {
  int64_t u, v;        // BR updates [u, v) of the learner call
  bool sync;           // ends with a target sync
};

struct LearnPlan {
  PrepArgs P;
  int64_t maxU = 0, maxUbr = 0, maxSL = 0;
  std::vector<Segment> seg[2];
  int64_t it0[2];
  FinalArgs F;
  nfsp_engine::Sched hs;     // the schedules after this call (commit_plan publishes them)
};

// The learner call's plan from the rollout's insert counts and the host's schedule mirror.
// Leaves the engine untouched: commit_plan(e, L) adopts it once every plan of the call (a
// group's replicas) has succeeded, so a failed plan changes no replica's schedules.
int plan_update(const nfsp_engine* e, const EngineDev& h, LearnPlan& L) {
  const nfsp_engine_cfg& cfg = e->cfg;
  PrepArgs& P = L.P;
  P = PrepArgs{};
  P.M = e->M;
  P.LB = e->LB;
  P.st = e->st;
  P.c = cfg.inserts_per_update;
  P.rl_cap = cfg.rl_capacity;
  P.B = cfg.batch;
  P.E = cfg.epochs;
  P.k0 = (uint32_t)cfg.seed;
  P.k1 = (uint32_t)(cfg.seed >> 32);
  P.tag = e->learn_tag + 1;
  P.lr_ar = cfg.lr_ar;
  P.quirks = cfg.quirks;
  L.maxU = L.maxUbr = L.maxSL = 0;
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
    L.maxU = pl.U > L.maxU ? pl.U : L.maxU;
    L.maxUbr = pl.U_br > L.maxUbr ? pl.U_br : L.maxUbr;
    L.maxSL = pl.n_sl > L.maxSL ? pl.n_sl : L.maxSL;
  }
  FinalArgs& F = L.F;
  F = FinalArgs{};
  F.st = e->st;
  F.br_expl = e->LB.br_expl;
  F.umax = e->LB.umax;
  F.sl_cap = cfg.sl_capacity;
  for (int a = 0; a < 2; ++a) {
    const AgentPlan& pl = P.A[a];
    F.n_rl[a] = h.last_rl[a];
    F.n_sl[a] = pl.n_sl;
    F.U_br[a] = pl.U_br;
    // the schedules from the host's mirror (the device copy in EngineDev, written by
    // k_finalize, may still be in flight with cfg.slice_lag 2)
    int64_t it = e->hs.iteration[a], tc = e->hs.target_count[a], syncs = e->hs.target_syncs[a];
    double eps = e->hs.epsilon[a];
    L.it0[a] = it;
    // BR segments between target syncs: [u, v) ends after the first update whose
    // target_count % every == 0 (agent/agent.py:266-273)
    L.seg[a].clear();
    for (int64_t u = 0; u < pl.U_br;) {
      int64_t v = u;
      bool sync = false;
      while (v < pl.U_br) {
        const bool s_here = (tc + v) % cfg.target_every == 0;
        ++v;
        if (s_here) { sync = true; break; }
      }
      L.seg[a].push_back({u, v, sync});
      u = v;
    }
    // schedules (agent/agent.py:245-253, 266-273) in the reference's double arithmetic
    for (int64_t k = 0; k < pl.U_br; ++k) {
      if (tc % cfg.target_every == 0) syncs++;
      tc++;
      it += 2;
      eps = (cfg.quirks & NFSP_EXT_EPS_CONST) ? cfg.epsilon : eps / (double)it;
    }
    if (e->update_limit > 0) {         // test hook: only a prefix of the updates runs
      std::vector<Segment> kept;
      for (const Segment& sg : L.seg[a]) {
        if (sg.u >= e->update_limit) break;
        kept.push_back(sg.v <= e->update_limit ? sg : Segment{sg.u, e->update_limit, false});
      }
      L.seg[a] = kept;
    }
    F.iteration[a] = it;
    F.tcount[a] = tc;
    F.syncs[a] = syncs;
    F.eps[a] = eps;
    L.hs.iteration[a] = it;
    L.hs.target_count[a] = tc;
    L.hs.target_syncs[a] = syncs;
    L.hs.epsilon[a] = eps;
    F.temp[a] = 1.0 / (1.0 + 0.02 * sqrt((double)it));
    F.lr[a] = (float)(cfg.lr_br / (1.0 + 0.003 * sqrt((double)it)));
  }
  return NFSP_OK;
}

void commit_plan(nfsp_engine* e, const LearnPlan& L) {
  e->learn_tag = L.P.tag;
  e->hs = L.hs;
  for (int a = 0; a < 2; ++a) {
    e->last_U[a] = L.P.A[a].U;
    e->last_Ubr[a] = L.P.A[a].U_br;
  }
  e->pending_update = false;
}

int launch_br_prep(nfsp_engine* e, const LearnPlan& L, hipStream_t s) {
  if (L.maxUbr > 0) {
    k_br_prep<0><<<dim3((unsigned)L.maxUbr, 2), 128, 0, s>>>(L.P, nullptr);
    NFSP_LAUNCHED("k_br_prep");
  }
  if (e->log_loss)                     // NaN = no fit recorded
    for (int a = 0; a < 2; ++a)
      NFSP_HIP(hipMemsetAsync(e->LB.br_loss + a * e->LB.umax * e->cfg.epochs, 0xFF,
                              sizeof(float) * L.P.A[a].U_br * e->cfg.epochs, s));
  return NFSP_OK;
}

int launch_ar_prep(nfsp_engine* e, const LearnPlan& L, hipStream_t s) {
  if (L.maxSL > 0) {
    k_ar_slots<0><<<dim3(nfsp_blocks(L.maxSL, 256), 2), 256, 0, s>>>(L.P, nullptr);
    NFSP_LAUNCHED("k_ar_slots");
  }
  if (L.maxU > 0) {
    k_ar_prep<0><<<dim3((unsigned)L.maxU, 2), 128, 0, s>>>(L.P, nullptr);
    NFSP_LAUNCHED("k_ar_prep");
  }
  if (e->log_loss)                     // NaN = no fit recorded (inactive AR update)
    for (int a = 0; a < 2; ++a)
      NFSP_HIP(hipMemsetAsync(e->LB.ar_loss + a * e->LB.umax * e->cfg.epochs, 0xFF,
                              sizeof(float) * L.P.A[a].U * e->cfg.epochs, s));
  return NFSP_OK;
}

int launch_res_apply(const LearnPlan& L, hipStream_t s) {
  if (L.maxSL > 0) {
    k_res_apply<0><<<dim3(nfsp_blocks(L.maxSL, 256), 2), 256, 0, s>>>(L.P, nullptr);
    NFSP_LAUNCHED("k_res_apply");
  }
  return NFSP_OK;
}

int64_t recs_per_update(const nfsp_engine* e) { return (int64_t)e->cfg.epochs * (e->cfg.batch / CHAIN_MB); }

// the AR chain of agent a over the whole learner call
ChainJob ar_job(const nfsp_engine* e, const LearnPlan& L, int a) {
  const int64_t um = e->LB.umax;
  ChainJob j{};
  j.w = e->w + (a * 3 + 0) * nn::NP;
  j.sync_to = nullptr;
  j.snap_to = nullptr;
  j.rec = e->LB.ar_rec + a * um * recs_per_update(e);
  j.active = e->LB.ar_active + a * um;
  j.loss_out = e->log_loss ? e->LB.ar_loss + a * um * e->cfg.epochs : nullptr;
  j.u0 = 0;
  j.u1 = L.P.A[a].U;
  if (e->update_limit > 0 && j.u1 > e->update_limit) j.u1 = e->update_limit;   // test hook
  return j;
}

// BR segment g of agent a: its targets and its chain
TargetJob br_target_job(const nfsp_engine* e, const LearnPlan& L, int a, const Segment& sg) {
  const int64_t um = e->LB.umax, B = e->cfg.batch, E = e->cfg.epochs;
  TargetJob t{};
  t.rows = e->LB.br_rows + a * um * B;
  t.perm = e->LB.br_perm + a * um * E * B;
  t.expl = e->LB.br_expl + a * um;
  t.rec = e->LB.br_rec + a * um * recs_per_update(e);
  t.tw = e->w + (a * 3 + 2) * nn::NP;
  t.u0 = sg.u;
  t.n = sg.v - sg.u;
  t.it0 = L.it0[a];
  return t;
}

ChainJob br_chain_job(const nfsp_engine* e, int a, const Segment& sg) {
  const int64_t um = e->LB.umax;
  ChainJob j{};
  j.w = e->w + (a * 3 + 1) * nn::NP;
  j.sync_to = sg.sync ? e->w + (a * 3 + 2) * nn::NP : nullptr;
  j.snap_to = nullptr;
  j.rec = e->LB.br_rec + a * um * recs_per_update(e);
  j.active = nullptr;
  j.loss_out = e->log_loss ? e->LB.br_loss + a * um * e->cfg.epochs : nullptr;
  j.u0 = sg.u;
  j.u1 = sg.v;
  return j;
}

int launch_br_chain(const ChainArgs& C, int blocks, unsigned quirks, bool loss_log, hipStream_t s) {
  if (quirks & NFSP_EXT_LINEAR_Q)
    return launch_chain_br_linear(C, blocks, loss_log, (quirks & NFSP_EXT_MSE_Q) != 0, s);
  static std::atomic<uint64_t> attr{0};
  return launch_chain<1>(C, blocks, loss_log, s, attr);
}

}  // namespace

// The exchange a pipelined learner call left pending (nfsp_engine_set_exchange), enqueued on
// the AR stream behind that call's AR chain, then the AR snapshot it feeds and its event.
static int flush_exchange(nfsp_engine* e) {
  if (!e->xchg_pending) return NFSP_OK;
  e->xchg_pending = false;
  int rc;
  {
    KTimer kx(e, KT_XCHG, e->s_ar);
    if ((rc = exchange_enqueue(e, e->s_ar)) != NFSP_OK) return rc;
  }
  if (e->xchg_pend_snap) {
    float* snap = e->snap + (size_t)e->xchg_pend_par * 6 * nn::NP;
    for (int a = 0; a < 2; ++a)
      NFSP_HIP(hipMemcpyAsync(snap + (a * 3 + 0) * nn::NP, e->w + (a * 3 + 0) * nn::NP,
                              sizeof(float) * nn::NP, hipMemcpyDeviceToDevice, e->s_ar));
    NFSP_HIP(hipEventRecord(e->snap_ev[e->xchg_pend_par][0], e->s_ar));
  }
  return NFSP_OK;
}

// One learner call for the pending rollout.  par: the learner-buffer set (slice parity; 0
// unless cfg.slice_lag 2).  pipelined: leave the chains running (no join into the ctx
// stream; each BR stream publishes its agent's results itself), and when snap_after, copy
// the nets into snapshot `par` after the chains and record snap_ev[par] for the rollout two
// slices on (step_pipelined).
static int update_impl(nfsp_engine* e, bool pipelined, int par, bool snap_after) {
  if (!e->pending_update) return NFSP_OK;
  hipStream_t s = e->ctx->stream;
  const nfsp_engine_cfg& cfg = e->cfg;
  // the trigger plan needs the rollout's insert counts: one small readback
  EngineDev h;
  NFSP_HIP(hipMemcpyAsync(&h, e->st, sizeof(h), hipMemcpyDeviceToHost, s));
  NFSP_HIP(hipStreamSynchronize(s));
  KTimer kt(e, KT_LEARNER);
  e->LB = e->LBs[par];
  LearnPlan L;
  int rc = plan_update(e, h, L);
  if (rc != NFSP_OK) return rc;
  commit_plan(e, L);
  // the cross-shard exchange after this call's AR chain (nfsp_engine_set_exchange)
  const bool xchg = e->xchg_every > 0 && (++e->xchg_calls) % e->xchg_every == 0;
  if (pipelined && snap_after)         // the rollout two slices on acts with this epsilon
    for (int a = 0; a < 2; ++a) e->snap_eps[par][a] = e->hs.epsilon[a];
  // ---- parallel prep on the ctx stream, in the order the chains need it: the BR rows
  // first (agent 0's BR segments are the learner's critical path), the BR streams fork;
  // then the AR records, the AR stream forks; the final reservoir last (only the next
  // rollout reads it, and it must follow k_ar_prep, which reads the reservoir as it was)
  hipEvent_t fork_br = take_event(e), fork = take_event(e);
  {
    KTimer kprep(e, KT_PREP);
    if ((rc = launch_br_prep(e, L, s)) != NFSP_OK) return rc;
    NFSP_HIP(hipEventRecord(fork_br, s));
    if ((rc = launch_ar_prep(e, L, s)) != NFSP_OK) return rc;
    NFSP_HIP(hipEventRecord(fork, s));
    if ((rc = launch_res_apply(L, s)) != NFSP_OK) return rc;
  }
  if (pipelined) {                     // the counters, before the next rollout's commit
    k_finalize<0><<<1, 64, 0, s>>>(L.F, nullptr, 1);
    NFSP_LAUNCHED("k_finalize");
  }
  float* snap = e->snap + (size_t)par * 6 * nn::NP;
  // diagnostic (cfg.sched NFSP_SCHED_LEARNER_SERIAL): BR work waits for the AR chains, to time
  // them alone
  const bool serial_ar = (e->cfg.sched & NFSP_SCHED_LEARNER_SERIAL) != 0;
  hipEvent_t ar_done = fork;
  // ---- AR chains (both agents, one launch) on their own stream.  With the exchange on and
  // the slices pipelined, this call's exchange (and the AR snapshot it feeds) is enqueued by
  // the NEXT call, after its prep and BR chains and right before its AR chain (or at the
  // step's end): an exchange may hold the host until the AR stream reaches it (RCCL's world-1
  // path synchronises the stream), and this way the host has enqueued everything the other
  // streams need before it can wait -- the AR stream's next chain needs the exchange anyway.
  auto ar_part = [&]() -> int {
    int r;
    if (pipelined && (r = flush_exchange(e)) != NFSP_OK) return r;
    NFSP_HIP(hipStreamWaitEvent(e->s_ar, fork, 0));
    if (L.maxU > 0) {
      ChainArgs C{};
      C.B = cfg.batch;
      C.E = cfg.epochs;
      for (int a = 0; a < 2; ++a) {
        C.job[a] = ar_job(e, L, a);
        if (snap_after && !xchg) C.job[a].snap_to = snap + (a * 3 + 0) * nn::NP;   // written by the chain
      }
      KTimer kc(e, KT_CHAIN_AR, e->s_ar);
      if ((r = launch_chain_ar(C, 2, e->log_loss, e->s_ar)) != NFSP_OK) return r;
    }
    if (xchg) {
      e->xchg_pending = true;
      e->xchg_pend_par = par;
      e->xchg_pend_snap = snap_after;
      if (!pipelined && (r = flush_exchange(e)) != NFSP_OK) return r;
    } else if (snap_after) {
      if (L.maxU == 0)                 // no AR chain this call: copy the nets as they are
        for (int a = 0; a < 2; ++a)
          NFSP_HIP(hipMemcpyAsync(snap + (a * 3 + 0) * nn::NP, e->w + (a * 3 + 0) * nn::NP,
                                  sizeof(float) * nn::NP, hipMemcpyDeviceToDevice, e->s_ar));
      NFSP_HIP(hipEventRecord(e->snap_ev[par][0], e->s_ar));
    }
    if (serial_ar) {
      ar_done = take_event(e);
      NFSP_HIP(hipEventRecord(ar_done, e->s_ar));
    }
    return NFSP_OK;
  };
  // ---- BR: per agent on its own stream, segments between target syncs = targets + chain
  auto br_part = [&]() -> int {
    int r;
    for (int a = 0; a < 2; ++a) {
      hipStream_t sa = e->s_br[a];
      NFSP_HIP(hipStreamWaitEvent(sa, serial_ar ? ar_done : fork_br, 0));
      KTimer kspan(e, KT_BR_STREAM0 + a, sa);     // this agent's BR stream, end to end
      for (size_t gi = 0; gi < L.seg[a].size(); ++gi) {
        const Segment& sg = L.seg[a][gi];
        {
          KTimer kt2(e, KT_TARGETS, sa);
          k_br_targets<<<(unsigned)(sg.v - sg.u), 256, 0, sa>>>(nullptr, br_target_job(e, L, a, sg),
                                                                  cfg.batch, cfg.epochs, cfg.gamma,
                                                                  cfg.quirks, cfg.lr_br);
        }
        NFSP_LAUNCHED("k_br_targets");
        ChainArgs C{};
        C.B = cfg.batch;
        C.E = cfg.epochs;
        C.job[0] = br_chain_job(e, a, sg);
        if (snap_after && gi + 1 == L.seg[a].size())            // the last segment writes the snapshot
          C.job[0].snap_to = snap + (a * 3 + 1) * nn::NP;
        KTimer kc(e, KT_CHAIN_BR, sa);
        if ((r = launch_br_chain(C, 1, cfg.quirks, e->log_loss, sa)) != NFSP_OK) return r;
      }
      if (pipelined) {                   // this agent's learner results, after its chain
        k_finalize<0><<<1, 64, 0, sa>>>(L.F, nullptr, 2 << a);
        NFSP_LAUNCHED("k_finalize");
      }
      if (snap_after) {
        if (L.seg[a].empty())             // no BR chain this call: copy the net as it is
          NFSP_HIP(hipMemcpyAsync(snap + (a * 3 + 1) * nn::NP, e->w + (a * 3 + 1) * nn::NP,
                                  sizeof(float) * nn::NP, hipMemcpyDeviceToDevice, sa));
        NFSP_HIP(hipEventRecord(e->snap_ev[par][1 + a], sa));
      }
    }
    return NFSP_OK;
  };
  // with the exchange on, the BR chains first (they never wait for an exchange), then the AR
  // chain and the exchange (pipelined: the previous call's exchange, then this call's AR chain;
  // else this call's, whose host transport synchronises the AR stream -- the BR streams are
  // busy by then instead of waiting for the host)
  const bool br_first = e->xchg_every > 0 && !serial_ar;
  if (br_first) {
    if ((rc = br_part()) != NFSP_OK) return rc;
    if ((rc = ar_part()) != NFSP_OK) return rc;
  } else {
    if ((rc = ar_part()) != NFSP_OK) return rc;
    if ((rc = br_part()) != NFSP_OK) return rc;
  }
  e->pool.push_back(fork);
  e->pool.push_back(fork_br);
  if (ar_done != fork) e->pool.push_back(ar_done);
  if (pipelined) return NFSP_OK;
  // ---- join and publish the schedules
  for (hipStream_t st : {e->s_ar, e->s_br[0], e->s_br[1]}) {
    hipEvent_t j = take_event(e);
    NFSP_HIP(hipEventRecord(j, st));
    NFSP_HIP(hipStreamWaitEvent(s, j, 0));
    e->pool.push_back(j);      // reusable once the wait is enqueued
  }
  k_finalize<0><<<1, 64, 0, s>>>(L.F, nullptr, 7);
  NFSP_LAUNCHED("k_finalize");
  return NFSP_OK;
}

// the side streams' work so far, joined into the ctx stream
static int join_streams(nfsp_engine* e) {
  for (hipStream_t st : {e->s_ar, e->s_br[0], e->s_br[1]}) {
    hipEvent_t j = take_event(e);
    NFSP_HIP(hipEventRecord(j, st));
    NFSP_HIP(hipStreamWaitEvent(e->ctx->stream, j, 0));
    e->pool.push_back(j);
  }
  return NFSP_OK;
}

extern "C" int nfsp_engine_update(nfsp_engine* e) {
  NFSP_REQUIRE(e, "null argument");
  NFSP_REQUIRE(e->s_ar, "a replica of an engine group is stepped by nfsp_group_step");
  return update_impl(e, false, 0, false);
}

namespace nfsp {
namespace eng {
// nfsp_engine_step with cfg.slice_lag 2.  Slice j's rollout acts with snapshot j & 1: the
// nets as of the step's start for j < 2, else as the chains of slice j - 2 left them (copied
// on each chain stream right after its chain, so slice j - 1's chains may already run).  The
// ctx stream waits only for those copies, never for the running chains: rollout, readback,
// plan and prep of slice j overlap slice j - 1's chains, which the chain streams follow
// without a gap.  The step ends with every stream joined (stats, weights and the next step
// see all of it).
int step_pipelined(nfsp_engine* e) {
  hipStream_t s = e->ctx->stream;
  const int K = e->slices;
  for (int p = 0; p < 2; ++p) {
    NFSP_HIP(hipMemcpyAsync(e->snap + (size_t)p * 6 * nn::NP, e->w, sizeof(float) * 6 * nn::NP,
                            hipMemcpyDeviceToDevice, s));
    for (int a = 0; a < 2; ++a) e->snap_eps[p][a] = e->hs.epsilon[a];
  }
  int rc;
  for (int j = 0; j < K; ++j) {
    const int par = j & 1;
    if (j >= 2)
      for (hipEvent_t ev : e->snap_ev[par]) NFSP_HIP(hipStreamWaitEvent(s, ev, 0));
    if ((rc = rollout_launch_with(e, e->snap + (size_t)par * 6 * nn::NP, e->snap_eps[par])) != NFSP_OK)
      return rc;
    if ((rc = update_impl(e, true, par, j + 2 < K)) != NFSP_OK) return rc;
  }
  if ((rc = flush_exchange(e)) != NFSP_OK) return rc;    // the last slice's
  return join_streams(e);
}
}  // namespace eng
}  // namespace nfsp

// ---------------------------------------------------------------------------
// Engine groups (nfsp_group_*): R replicas stepped together, their chains in shared launches
// ---------------------------------------------------------------------------
constexpr int GROUP_BR_STREAMS = 4;   // at most; nfsp_group_sched.br_streams (group_update)

struct nfsp_group {
  nfsp_ctx* ctx = nullptr;
  int R = 0;
  unsigned flags = 0;
  std::vector<nfsp_engine*> eng;
  hipStream_t s_ar = nullptr, s_br = nullptr;
  // further BR streams: a sliced group's BR jobs run in up to GROUP_BR_STREAMS partitions,
  // each its own rounds on its own stream (partition 0 on s_br); created on first use, so a
  // group with one partition holds no extra stream (and no extra hardware queue)
  hipStream_t s_brp[GROUP_BR_STREAMS - 1] = {};
  void* d_roll = nullptr;        // the replicas' rollout arguments (static device table)
  // per learner call: job / prep / final tables, host (pinned) staging -> device, one copy;
  // two sets by slice parity (a pipelined step's slice j + 1 fills its set while slice j's
  // chains still read theirs)
  char* h_tab[2] = {nullptr, nullptr};
  char* d_tab[2] = {nullptr, nullptr};
  size_t tab_cap[2] = {0, 0};
  hipEvent_t snap_ev[2][2] = {};  // pipelined step: [parity][AR, BR stream] snapshot copies done
  // the replicas' EngineDev, gathered on device and read back in one copy
  EngineDev** d_stp = nullptr;   // [R] -> each replica's state
  EngineDev* d_st = nullptr;     // [R]
  EngineDev* h_st = nullptr;     // [R] pinned
  float** d_war = nullptr;       // [3 nets][R][2] weight pointers (k_group_xchg)
  float* w0 = nullptr;           // [3][2][NP] the exchanged nets after the last exchange
  unsigned w0_valid = 0;         // nets (NFSP_XCHG_*) broadcast from replica 0 already
  unsigned xchg_nets = 0;        // nfsp_group_set_exchange
  int xchg_every = 0;
  float xchg_scale = 1.f;
  int64_t calls = 0;             // learner calls (slices) so far
  int64_t rounds = 0;            // BR rounds of the last learner call (stats)
  nfsp_group_sched sched{};      // nfsp_group_set_sched (from nfsp_group_default_sched)
  int32_t* h_err = nullptr;      // k_br_persist's bail flags (pinned host, mapped): group_check_err
  int chain_lds = 0;             // LDS per chain workgroup: 4R chains on the device's CUs
  bool trace_on = false;         // nfsp_group_set_trace: per call [R][2][AR, BR] update counts
  std::vector<int32_t> trace;
};

namespace {
__global__ void k_gather_st(EngineDev* const* __restrict__ src, EngineDev* __restrict__ dst, int R) {
  constexpr int W = (int)(sizeof(EngineDev) / 8);
  static_assert(sizeof(EngineDev) % 8 == 0, "EngineDev words");
  for (int i = threadIdx.x; i < R * W; i += blockDim.x) {
    const int r = i / W, k = i - r * W;
    reinterpret_cast<uint64_t*>(dst + r)[k] = reinterpret_cast<const uint64_t*>(src[r])[k];
  }
}
}  // namespace

extern "C" int nfsp_group_destroy(nfsp_group* g) {
  if (!g) return NFSP_OK;
  if (g->ctx) (void)hipStreamSynchronize(g->ctx->stream);
  for (hipStream_t st : {g->s_ar, g->s_br})
    if (st) (void)hipStreamSynchronize(st);
  for (hipStream_t st : g->s_brp)
    if (st) (void)hipStreamSynchronize(st);
  for (nfsp_engine* e : g->eng) nfsp_engine_destroy(e);
  for (int p = 0; p < 2; ++p) {
    if (g->h_tab[p]) (void)hipHostFree(g->h_tab[p]);
    if (g->d_tab[p]) (void)hipFree(g->d_tab[p]);
    for (hipEvent_t ev : g->snap_ev[p])
      if (ev) (void)hipEventDestroy(ev);
  }
  if (g->h_st) (void)hipHostFree(g->h_st);
  if (g->h_err) (void)hipHostFree(g->h_err);
  for (void* p : {(void*)g->d_war, (void*)g->w0, g->d_roll, (void*)g->d_stp, (void*)g->d_st})
    if (p) (void)hipFree(p);
  for (hipStream_t st : {g->s_ar, g->s_br})
    if (st) (void)hipStreamDestroy(st);
  for (hipStream_t st : g->s_brp)
    if (st) (void)hipStreamDestroy(st);
  delete g;
  return NFSP_OK;
}

extern "C" int nfsp_group_create(nfsp_ctx* ctx, const nfsp_engine_cfg* cfg, int replicas, unsigned flags,
                                 nfsp_group** out) {
  NFSP_REQUIRE(ctx && cfg && out, "null argument");
  NFSP_REQUIRE(replicas >= 1 && replicas <= NFSP_GROUP_MAX_REPLICAS, "replicas must be in [1, 256]");
  NFSP_REQUIRE((flags & ~NFSP_GROUP_AVG_AR) == 0, "unknown group flags");
  NFSP_REQUIRE(cfg->slices >= 1, "slices must be >= 1");
  *out = nullptr;
  // up to 4R chain workgroups run at once (2R AR + a BR round's 2R): past one per CU they
  // share CUs, each with an equal share of the LDS
  int dev = 0, cus = 0;
  NFSP_HIP(hipGetDevice(&dev));
  NFSP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  nfsp_group* g = new nfsp_group();
  g->ctx = ctx;
  g->R = replicas;
  g->flags = flags;
  if (flags & NFSP_GROUP_AVG_AR) {     // the per-step AR exchange
    g->xchg_nets = NFSP_XCHG_AR;
    g->xchg_every = cfg->slices;
    g->xchg_scale = 1.0f / (float)replicas;
  }
  g->chain_lds = chain_lds_shared((4 * replicas + cus - 1) / (cus > 0 ? cus : 1));
  nfsp_group_default_sched(&g->sched);
  for (int r = 0; r < replicas; ++r) {
    nfsp_engine_cfg c = *cfg;
    c.seed = cfg->seed + (uint64_t)r;
    nfsp_engine* e = nullptr;
    const int rc = nfsp::eng::engine_create(ctx, &c, false, &e);
    if (rc != NFSP_OK) {
      nfsp_group_destroy(g);
      return rc;
    }
    g->eng.push_back(e);
  }
  for (hipStream_t* st : {&g->s_ar, &g->s_br}) {
    const hipError_t sr = hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    if (sr != hipSuccess) {
      nfsp_group_destroy(g);
      return nfsp::hip_fail(sr, "nfsp_group_create: hipStreamCreate");
    }
  }
  for (auto& pe : g->snap_ev)
    for (hipEvent_t& ev : pe) {
      const hipError_t er = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      if (er != hipSuccess) {
        nfsp_group_destroy(g);
        return nfsp::hip_fail(er, "nfsp_group_create: hipEventCreate");
      }
    }
  int rc = nfsp::eng::group_rollout_table(g->eng.data(), replicas, &g->d_roll);
  if (rc != NFSP_OK) {
    nfsp_group_destroy(g);
    return rc;
  }
  std::vector<float*> war(3 * 2 * replicas);
  std::vector<EngineDev*> stp(replicas);
  for (int r = 0; r < replicas; ++r) {
    for (int n = 0; n < 3; ++n)
      for (int a = 0; a < 2; ++a) war[((size_t)n * replicas + r) * 2 + a] = g->eng[r]->w + (a * 3 + n) * nn::NP;
    stp[r] = g->eng[r]->st;
  }
  hipError_t r = hipMalloc((void**)&g->d_war, sizeof(float*) * war.size());
  if (r == hipSuccess) r = hipMalloc((void**)&g->w0, sizeof(float) * 3 * 2 * nn::NP);
  if (r == hipSuccess) r = hipMemcpy(g->d_war, war.data(), sizeof(float*) * war.size(), hipMemcpyHostToDevice);
  if (r == hipSuccess) r = hipMalloc((void**)&g->d_stp, sizeof(EngineDev*) * replicas);
  if (r == hipSuccess) r = hipMalloc((void**)&g->d_st, sizeof(EngineDev) * replicas);
  if (r == hipSuccess) r = hipHostMalloc((void**)&g->h_st, sizeof(EngineDev) * replicas, hipHostMallocDefault);
  if (r == hipSuccess) r = hipHostMalloc((void**)&g->h_err, sizeof(int32_t) * 4, hipHostMallocMapped | hipHostMallocCoherent);
  if (r == hipSuccess) memset(g->h_err, 0, sizeof(int32_t) * 4);
  if (r == hipSuccess) r = hipMemcpy(g->d_stp, stp.data(), sizeof(EngineDev*) * replicas, hipMemcpyHostToDevice);
  if (r != hipSuccess) {
    nfsp_group_destroy(g);
    return nfsp::hip_fail(r, "nfsp_group_create");
  }
  *out = g;
  return NFSP_OK;
}

extern "C" int nfsp_group_engine(nfsp_group* g, int r, nfsp_engine** out) {
  NFSP_REQUIRE(g && out && r >= 0 && r < g->R, "bad argument");
  *out = g->eng[r];
  return NFSP_OK;
}

// the group's exchange (k_group_xchg) on stream `s`
static int group_xchg_launch(nfsp_group* g, hipStream_t s) {
  const unsigned nets = g->xchg_nets ? g->xchg_nets : NFSP_XCHG_AR;
  // nets not broadcast yet take replica 0's (a BR net with its target net)
  unsigned bc = nets & ~g->w0_valid;
  if (bc & NFSP_XCHG_BR) bc |= 4u;
  const float scale = g->xchg_nets ? g->xchg_scale : 1.0f / (float)g->R;
  k_group_xchg<<<nfsp_blocks(3 * 2 * nn::NP, 256), 256, 0, s>>>(g->d_war, g->w0, g->R, nets, bc, scale);
  NFSP_LAUNCHED("k_group_xchg");
  g->w0_valid |= nets;
  return NFSP_OK;
}

extern "C" int nfsp_group_average_ar(nfsp_group* g) {
  NFSP_REQUIRE(g, "null argument");
  return group_xchg_launch(g, g->ctx->stream);
}

extern "C" int nfsp_group_set_exchange(nfsp_group* g, unsigned nets, int every, float scale) {
  NFSP_REQUIRE(g, "null argument");
  NFSP_REQUIRE((nets & ~(NFSP_XCHG_AR | NFSP_XCHG_BR)) == 0, "nets: NFSP_XCHG_AR | NFSP_XCHG_BR");
  NFSP_REQUIRE(every >= 0 && (every == 0 || nets), "every >= 0 (and nets when on)");
  // a net this call turns on starts like the rank path's (AvgPolicyExchange broadcasts rank 0's
  // nets, then nfsp_engine_set_exchange takes them as W0): its next exchange copies replica 0's
  // net everywhere instead of applying deltas against a W0 from before the exchange was off
  const unsigned on = every ? nets : 0;
  g->w0_valid &= ~(on & ~g->xchg_nets);
  g->xchg_nets = on;
  g->xchg_every = every;
  g->xchg_scale = scale;
  g->calls = 0;
  return NFSP_OK;
}

// bump-allocate n items of T in the host / device table pair (8-byte aligned offsets)
struct TabCursor {
  size_t off = 0;
  template <class T>
  size_t take(size_t n) {
    const size_t o = (off + 15) & ~(size_t)15;
    off = o + sizeof(T) * n;
    return o;
  }
};

// One learner call of every replica for their pending rollouts.  par: the learner-buffer and
// table set (slice parity; 0 unless pipelined).  pipelined (nfsp_group_step at slice_lag 2):
// nothing joins the ctx stream -- the counters are published on it after the prep, the BR
// results on the BR stream after the last round; the exchange (when due) follows the AR chains
// on the AR stream; with snap_after each learner stream then copies its nets into snapshot
// `par` and records snap_ev[par] for the rollout two slices on.
// k_br_persist's bounded waits: a hand-off that never came ended that kernel with a bail flag
// set (pinned host memory).  Checked once the kernel has completed: after a learner call's
// readback sync (the ctx stream has then waited for every earlier slice's BR stream) and by
// nfsp_group_check (which synchronises first).
static int group_check_err(nfsp_group* g) {
  volatile int32_t* h = g->h_err;
  if (!h || !h[0]) return NFSP_OK;
  const int cb = h[1], hb = h[2];
  h[0] = h[1] = h[2] = 0;
  return nfsp::fail(NFSP_EHIP, "k_br_persist: a bounded wait expired (work-queue hand-off): chain bails " +
                                   std::to_string(cb) + ", helper bails " + std::to_string(hb));
}

static int group_update(nfsp_group* g, bool pipelined = false, int par = 0, bool snap_after = false) {
  hipStream_t s = g->ctx->stream;
  const int R = g->R;
  nfsp_engine* e0 = g->eng[0];
  const nfsp_engine_cfg& cfg = e0->cfg;
  for (int r = 0; r < R; ++r) NFSP_REQUIRE(g->eng[r]->pending_update, "group replica without a rollout");
  // the trigger plans need every replica's insert counts: one gather, one readback
  k_gather_st<<<1, 256, 0, s>>>(g->d_stp, g->d_st, R);
  NFSP_LAUNCHED("k_gather_st");
  NFSP_HIP(hipMemcpyAsync(g->h_st, g->d_st, sizeof(EngineDev) * R, hipMemcpyDeviceToHost, s));
  NFSP_HIP(hipStreamSynchronize(s));
  int rc;
  if ((rc = group_check_err(g)) != NFSP_OK) return rc;
  KTimer kt(e0, KT_LEARNER);
  std::vector<LearnPlan> L(R);
  int64_t maxU = 0, maxUbr = 0, maxSL = 0;
  const bool loss_log = e0->log_loss;
  for (int r = 0; r < R; ++r) {
    nfsp_engine* e = g->eng[r];
    NFSP_REQUIRE(e->log_loss == loss_log, "the loss log must be on in all replicas of a group or none");
    e->LB = e->LBs[par];
    if ((rc = plan_update(e, g->h_st[r], L[r])) != NFSP_OK) return rc;
    maxU = L[r].maxU > maxU ? L[r].maxU : maxU;
    maxUbr = L[r].maxUbr > maxUbr ? L[r].maxUbr : maxUbr;
    maxSL = L[r].maxSL > maxSL ? L[r].maxSL : maxSL;
  }
  // every plan succeeded: the rollouts are consumed and the schedules advance (a failed
  // plan leaves every replica as it was -- pending, schedules untouched -- so they stay in step)
  for (int r = 0; r < R; ++r) commit_plan(g->eng[r], L[r]);
  if (g->trace_on)
    for (int r = 0; r < R; ++r)
      for (int a = 0; a < 2; ++a) {
        g->trace.push_back((int32_t)L[r].P.A[a].U);
        g->trace.push_back((int32_t)L[r].P.A[a].U_br);
      }
  // ---- tables: prep / final args per replica; the AR chains (2R workgroups, one launch);
  // per BR round k the targets and the chain of every (replica, agent) with a k-th segment
  std::vector<ChainJob> ar_jobs;
  for (int r = 0; r < R; ++r)
    for (int a = 0; a < 2; ++a)
      if (L[r].P.A[a].U > 0) ar_jobs.push_back(ar_job(g->eng[r], L[r], a));
  // BR rounds: round k = one k_br_targets launch (the targets of the segments that start in
  // it, whole segments) + one chain launch (every (replica, agent) with BR work left: the next
  // piece of its current segment, at most `cap` updates; a target sync ends the last piece of
  // its segment).  cap 0: one round per segment index, every job's k-th segment in round k.
  // A round lasts as long as its longest piece, so with whole segments the round structure
  // waits for the longest segment of every round: a sliced group's BR stream ran 1.9 ms per
  // slice against 1.2 ms for its busiest job (tools/group_timeline.py).  Pieces of a segment
  // resume from the weights in memory: the same SGD steps, bit for bit.
  const int64_t cap = g->sched.br_cap >= 0 ? g->sched.br_cap : (e0->slices > 1 ? 40 : 0);
  const bool pace_br = g->sched.br_pace != 0;
  // Partitions: replicas [pr0[p], pr0[p + 1]) are partition p, whose BR jobs run their own
  // rounds on their own stream, followed (pipelined) by the partition's BR results and BR
  // snapshot on that stream.  A round then waits only for the longest piece among its
  // partition's jobs, and one partition's targets overlap the others' chains.  Partitions
  // 1.. go on into the next slice without waiting for the others; partition 0 runs on s_br,
  // which joins every partition at the end of the call (below), so its next-slice rounds wait
  // for the slowest partition: the overlap is asymmetric.  Each job's pieces and targets are
  // the same as with one partition, so are its SGD steps.  Sliced groups only (their rounds
  // are short: the targets between them were ~10% of c4_emul_r8's BR stream); groups whose
  // chains share CUs keep one stream.
  const bool shared_cus = g->chain_lds < CHAIN_LDS;
  // The persistent BR kernel (sched.br_persist) instead of the rounds: one launch, one stream,
  // the reference's BR net (k_chain3<1>), no loss log, its 2R chains and BRP_HELPERS helpers a
  // CU each beside the 2R AR chains (R <= 32, no CU sharing)
  const bool persist = g->sched.br_persist && !loss_log && !(cfg.quirks & NFSP_EXT_LINEAR_Q) && R <= 32 &&
                       !shared_cus;
  int nbs = g->sched.br_streams > 0 ? g->sched.br_streams : (e0->slices > 1 ? 2 : 1);
  nbs = nbs > GROUP_BR_STREAMS ? GROUP_BR_STREAMS : nbs;
  nbs = nbs > R ? R : nbs;
  if (shared_cus || persist) nbs = 1;
  struct BrCursor {
    int r, a;
    size_t s;        // current segment
    int64_t pos;     // next update of it
  };
  struct BrRound {
    int p;                   // partition (stream)
    size_t b0, b1, t0, t1;   // its chain jobs / target jobs in br_jobs / tg_jobs
    int64_t rn;              // the longest segment starting in it (targets grid)
  };
  std::vector<ChainJob> br_jobs;
  std::vector<TargetJob> tg_jobs;
  std::vector<BrRound> rounds_v;
  int pr0[GROUP_BR_STREAMS + 1];
  for (int p = 0; p <= nbs; ++p) pr0[p] = p * R / nbs;
  int64_t max_rounds = 0;
  for (int p = 0; p < (persist ? 0 : nbs); ++p) {
    std::vector<BrCursor> bc;
    for (int r = pr0[p]; r < pr0[p + 1]; ++r)
      for (int a = 0; a < 2; ++a)
        if (!L[r].seg[a].empty()) bc.push_back({r, a, 0, L[r].seg[a][0].u});
    // Paced pieces (capped groups): the partition's busiest job (most BR updates in this call)
    // splits each of its segments into equal pieces of at most `cap`, and in every round the
    // other jobs take at most the busiest job's piece of that round, so no round outlasts the
    // busiest job's own piece and its last piece of a segment is not a short one.  (Plain caps:
    // a 150-update segment ran as 40 + 40 + 40 + 30, and every job's round took 40.)
    std::vector<int64_t> pace;                 // the busiest job's piece per round
    if (cap > 0 && pace_br) {
      int64_t most = -1;
      const std::vector<Segment>* bs = nullptr;
      for (const BrCursor& c : bc) {
        int64_t n = 0;
        for (const Segment& sg : L[c.r].seg[c.a]) n += sg.v - sg.u;
        if (n > most) most = n, bs = &L[c.r].seg[c.a];
      }
      if (bs)
        for (const Segment& sg : *bs) {
          const int64_t len = sg.v - sg.u, np = (len + cap - 1) / cap;
          for (int64_t k = 0; k < np; ++k) pace.push_back(len / np + (k < len % np ? 1 : 0));
        }
    }
    int64_t nr = 0;
    for (;;) {
      const size_t b0 = br_jobs.size(), t0 = tg_jobs.size();
      int64_t rn = 0;
      const int64_t pk = (size_t)nr < pace.size() ? pace[(size_t)nr] : cap;
      for (BrCursor& c : bc) {
        const std::vector<Segment>& segs = L[c.r].seg[c.a];
        if (c.s >= segs.size()) continue;
        const Segment& sg = segs[c.s];
        if (c.pos == sg.u) {
          tg_jobs.push_back(br_target_job(g->eng[c.r], L[c.r], c.a, sg));
          rn = sg.v - sg.u > rn ? sg.v - sg.u : rn;
        }
        const int64_t end = pk > 0 && c.pos + pk < sg.v ? c.pos + pk : sg.v;
        br_jobs.push_back(br_chain_job(g->eng[c.r], c.a, Segment{c.pos, end, sg.sync && end == sg.v}));
        c.pos = end;
        if (end == sg.v && ++c.s < segs.size()) c.pos = segs[c.s].u;
      }
      if (br_jobs.size() == b0) break;
      rounds_v.push_back({p, b0, br_jobs.size(), t0, tg_jobs.size(), rn});
      ++nr;
    }
    max_rounds = nr > max_rounds ? nr : max_rounds;
  }
  // k_br_persist's tables: each segment's chain and targets jobs, its chunk counters, and the
  // work queue holding the first segments' items, chunk by chunk across the jobs
  std::vector<ChainJob> p_job;
  std::vector<TargetJob> p_tgt;
  std::vector<int32_t> p_chunk0, p_jseg0;
  std::vector<uint32_t> p_slots;
  int32_t p_nchunks = 0;
  uint32_t p_npre = 0;
  if (persist) {
    for (int r = 0; r < R; ++r)
      for (int a = 0; a < 2; ++a) {
        if (L[r].seg[a].empty()) continue;
        p_jseg0.push_back((int32_t)p_job.size());
        for (const Segment& sg : L[r].seg[a]) {
          NFSP_REQUIRE(sg.v - sg.u < 65536, "a BR segment of >= 65536 updates");
          p_job.push_back(br_chain_job(g->eng[r], a, sg));
          p_tgt.push_back(br_target_job(g->eng[r], L[r], a, sg));
          p_chunk0.push_back(p_nchunks);
          p_nchunks += (int32_t)((sg.v - sg.u + BRP_CHUNK - 1) / BRP_CHUNK);
        }
      }
    NFSP_REQUIRE(p_job.size() < 65536, "too many BR segments in one learner call");
    const int njobs = (int)p_jseg0.size();
    p_jseg0.push_back((int32_t)p_job.size());
    int64_t nitems = 0, maxn = 0;
    for (const TargetJob& t : p_tgt) nitems += t.n;
    for (int j = 0; j < njobs; ++j) maxn = p_tgt[p_jseg0[j]].n > maxn ? p_tgt[p_jseg0[j]].n : maxn;
    p_slots.assign((size_t)nitems, BRP_EMPTY);
    for (int64_t c0 = 0; c0 < maxn; c0 += BRP_CHUNK)
      for (int j = 0; j < njobs; ++j) {
        const int sgi = p_jseg0[j];
        const int64_t n = p_tgt[sgi].n, c1 = c0 + BRP_CHUNK < n ? c0 + BRP_CHUNK : n;
        for (int64_t i = c0; i < c1; ++i) p_slots[p_npre++] = ((uint32_t)sgi << 16) | (uint32_t)i;
      }
    max_rounds = njobs > 0 ? 1 : 0;
  }
  g->rounds = max_rounds;
  TabCursor cur;
  const size_t o_prep = cur.take<PrepArgs>(R), o_fin = cur.take<FinalArgs>(R);
  const size_t o_ar = cur.take<ChainJob>(ar_jobs.size()), o_br = cur.take<ChainJob>(br_jobs.size());
  const size_t o_tg = cur.take<TargetJob>(tg_jobs.size());
  const size_t o_pj = cur.take<ChainJob>(p_job.size()), o_pt = cur.take<TargetJob>(p_tgt.size());
  const size_t o_pc = cur.take<int32_t>(p_chunk0.size()), o_ps = cur.take<int32_t>(p_jseg0.size());
  const size_t o_pq = cur.take<uint32_t>(p_slots.size()), o_pn = cur.take<uint32_t>(2);
  const size_t o_pd = cur.take<uint32_t>((size_t)p_nchunks);
  const size_t need = cur.off;
  // Every earlier use of set `par` has completed: serially, the call starts with the readback's
  // sync; pipelined, the ctx stream waited for slice j - 2's snapshot events (after its chains)
  // before this slice's rollout.  A grown set is freed and reallocated: the device free
  // synchronises the device.
  char*& h_tab = g->h_tab[par];
  char*& d_tab = g->d_tab[par];
  if (need > g->tab_cap[par]) {
    if (h_tab) NFSP_HIP(hipHostFree(h_tab));
    if (d_tab) NFSP_HIP(hipFree(d_tab));
    h_tab = nullptr;
    d_tab = nullptr;
    g->tab_cap[par] = 0;
    const size_t cap = need * 2;
    NFSP_HIP(hipHostMalloc((void**)&h_tab, cap, hipHostMallocDefault));
    NFSP_HIP(hipMalloc((void**)&d_tab, cap));
    g->tab_cap[par] = cap;
  }
  for (int r = 0; r < R; ++r) {
    memcpy(h_tab + o_prep + sizeof(PrepArgs) * r, &L[r].P, sizeof(PrepArgs));
    memcpy(h_tab + o_fin + sizeof(FinalArgs) * r, &L[r].F, sizeof(FinalArgs));
  }
  memcpy(h_tab + o_ar, ar_jobs.data(), sizeof(ChainJob) * ar_jobs.size());
  memcpy(h_tab + o_br, br_jobs.data(), sizeof(ChainJob) * br_jobs.size());
  memcpy(h_tab + o_tg, tg_jobs.data(), sizeof(TargetJob) * tg_jobs.size());
  if (persist) {
    memcpy(h_tab + o_pj, p_job.data(), sizeof(ChainJob) * p_job.size());
    memcpy(h_tab + o_pt, p_tgt.data(), sizeof(TargetJob) * p_tgt.size());
    memcpy(h_tab + o_pc, p_chunk0.data(), sizeof(int32_t) * p_chunk0.size());
    memcpy(h_tab + o_ps, p_jseg0.data(), sizeof(int32_t) * p_jseg0.size());
    memcpy(h_tab + o_pq, p_slots.data(), sizeof(uint32_t) * p_slots.size());
    const uint32_t ctr[2] = {0u, p_npre};
    memcpy(h_tab + o_pn, ctr, sizeof(ctr));
    memset(h_tab + o_pd, 0, sizeof(uint32_t) * (size_t)p_nchunks);
  }
  const PrepArgs* d_prep = reinterpret_cast<const PrepArgs*>(d_tab + o_prep);
  const FinalArgs* d_fin = reinterpret_cast<const FinalArgs*>(d_tab + o_fin);
  const ChainJob* d_ar = reinterpret_cast<const ChainJob*>(d_tab + o_ar);
  const ChainJob* d_br = reinterpret_cast<const ChainJob*>(d_tab + o_br);
  const TargetJob* d_tg = reinterpret_cast<const TargetJob*>(d_tab + o_tg);
  hipEvent_t fork_br = take_event(e0), fork = take_event(e0);
  {
    KTimer kprep(e0, KT_PREP);
    NFSP_HIP(hipMemcpyAsync(d_tab, h_tab, need, hipMemcpyHostToDevice, s));
    // the same prep kernels as one engine's, every replica in one launch (blockIdx.z)
    if (maxUbr > 0) {
      k_br_prep<1><<<dim3((unsigned)maxUbr, 2, R), 128, 0, s>>>(PrepArgs{}, d_prep);
      NFSP_LAUNCHED("k_br_prep");
    }
    if (loss_log)
      for (int r = 0; r < R; ++r)
        for (int a = 0; a < 2; ++a)
          NFSP_HIP(hipMemsetAsync(g->eng[r]->LB.br_loss + a * g->eng[r]->LB.umax * cfg.epochs, 0xFF,
                                  sizeof(float) * L[r].P.A[a].U_br * cfg.epochs, s));
    NFSP_HIP(hipEventRecord(fork_br, s));
    if (maxSL > 0) {
      k_ar_slots<1><<<dim3(nfsp_blocks(maxSL, 256), 2, R), 256, 0, s>>>(PrepArgs{}, d_prep);
      NFSP_LAUNCHED("k_ar_slots");
    }
    if (maxU > 0) {
      k_ar_prep<1><<<dim3((unsigned)maxU, 2, R), 128, 0, s>>>(PrepArgs{}, d_prep);
      NFSP_LAUNCHED("k_ar_prep");
    }
    if (loss_log)
      for (int r = 0; r < R; ++r)
        for (int a = 0; a < 2; ++a)
          NFSP_HIP(hipMemsetAsync(g->eng[r]->LB.ar_loss + a * g->eng[r]->LB.umax * cfg.epochs, 0xFF,
                                  sizeof(float) * L[r].P.A[a].U * cfg.epochs, s));
    NFSP_HIP(hipEventRecord(fork, s));
    if (maxSL > 0) {
      k_res_apply<1><<<dim3(nfsp_blocks(maxSL, 256), 2, R), 256, 0, s>>>(PrepArgs{}, d_prep);
      NFSP_LAUNCHED("k_res_apply");
    }
  }
  if (pipelined) {                     // the counters, before the next rollout's commit
    k_finalize<1><<<R, 64, 0, s>>>(FinalArgs{}, d_fin, 1);
    NFSP_LAUNCHED("k_finalize");
  }
  // When chains share CUs (R > 64), the first round's BR targets run before the AR chains
  // start: alone they take the chip's issue slots instead of competing with 2R resident AR
  // chains, and the BR stream is the longer one at that size.  (No data dependency.)
  auto launch_ar = [&](hipEvent_t after) -> int {
    NFSP_HIP(hipStreamWaitEvent(g->s_ar, fork, 0));
    if (after) NFSP_HIP(hipStreamWaitEvent(g->s_ar, after, 0));
    ChainArgs C{};
    C.jobs = d_ar;
    C.B = cfg.batch;
    C.E = cfg.epochs;
    C.lds = g->chain_lds;
    KTimer kc(e0, KT_CHAIN_AR, g->s_ar);
    return launch_chain_ar(C, (int)ar_jobs.size(), loss_log, g->s_ar);
  };
  bool ar_launched = ar_jobs.empty();
  if (!shared_cus && !ar_launched) {
    if ((rc = launch_ar(nullptr)) != NFSP_OK) return rc;
    ar_launched = true;
  }
  for (int p = 1; p < nbs; ++p)
    if (!g->s_brp[p - 1]) NFSP_HIP(hipStreamCreateWithFlags(&g->s_brp[p - 1], hipStreamNonBlocking));
  static_assert(GROUP_BR_STREAMS == 4, "sp below");
  hipStream_t sp[GROUP_BR_STREAMS] = {g->s_br, g->s_brp[0], g->s_brp[1], g->s_brp[2]};
  for (int p = 0; p < nbs; ++p) NFSP_HIP(hipStreamWaitEvent(sp[p], fork_br, 0));
  KTimer kspan(e0, KT_BR_STREAM0, g->s_br);     // the group's BR streams, end to end (joined on s_br)
  if (persist && p_jseg0.size() > 1) {
    BrPersistArgs P{};
    P.C.B = cfg.batch;
    P.C.E = cfg.epochs;
    P.seg_job = reinterpret_cast<const ChainJob*>(d_tab + o_pj);
    P.seg_tgt = reinterpret_cast<const TargetJob*>(d_tab + o_pt);
    P.seg_chunk0 = reinterpret_cast<const int32_t*>(d_tab + o_pc);
    P.job_seg0 = reinterpret_cast<const int32_t*>(d_tab + o_ps);
    P.slots = reinterpret_cast<uint32_t*>(d_tab + o_pq);
    P.ctr = reinterpret_cast<uint32_t*>(d_tab + o_pn);
    P.chunk_done = reinterpret_cast<uint32_t*>(d_tab + o_pd);
    NFSP_HIP(hipHostGetDevicePointer((void**)&P.err, g->h_err, 0));
    P.njobs = (int)p_jseg0.size() - 1;
    P.nitems = (int)p_slots.size();
    P.chunk = BRP_CHUNK;
    P.spin = g->sched.br_persist > 1 ? g->sched.br_persist : BRP_SPIN;
    P.gamma = cfg.gamma;
    P.lr0 = cfg.lr_br;
    P.quirks = cfg.quirks;
    KTimer kc(e0, KT_CHAIN_BR, g->s_br);
    if ((rc = launch_br_persist(P, BRP_HELPERS, g->s_br)) != NFSP_OK) return rc;
  }
  for (const BrRound& rd : rounds_v) {
    hipStream_t st = sp[rd.p];
    const int nj = (int)(rd.b1 - rd.b0);
    const int nt = (int)(rd.t1 - rd.t0);
    if (nt > 0) {
      {
        KTimer kt2(e0, KT_TARGETS, st);
        k_br_targets<<<dim3((unsigned)rd.rn, (unsigned)nt), 256, 0, st>>>(
            d_tg + rd.t0, TargetJob{}, cfg.batch, cfg.epochs, cfg.gamma, cfg.quirks, cfg.lr_br);
      }
      NFSP_LAUNCHED("k_br_targets");
    }
    if (!ar_launched) {                      // (one partition: shared_cus)
      hipEvent_t t0 = take_event(e0);
      NFSP_HIP(hipEventRecord(t0, st));
      if ((rc = launch_ar(t0)) != NFSP_OK) return rc;
      e0->pool.push_back(t0);
      ar_launched = true;
    }
    ChainArgs C{};
    C.jobs = d_br + rd.b0;
    C.B = cfg.batch;
    C.E = cfg.epochs;
    C.lds = g->chain_lds;
    KTimer kc(e0, KT_CHAIN_BR, st);
    if ((rc = launch_br_chain(C, nj, cfg.quirks, loss_log, st)) != NFSP_OK) return rc;
  }
  if (!ar_launched && (rc = launch_ar(nullptr)) != NFSP_OK) return rc;
  // each partition's stream: (pipelined) its replicas' BR results, then (snap_after) their BR /
  // target nets and epsilons into snapshot `par`; then the partitions are joined on s_br
  for (int p = 0; p < nbs; ++p) {
    const int r0 = pr0[p], rn = pr0[p + 1] - pr0[p];
    if (pipelined && rn > 0) {
      k_finalize<1><<<rn, 64, 0, sp[p]>>>(FinalArgs{}, d_fin + r0, 6);
      NFSP_LAUNCHED("k_finalize");
      if (snap_after &&
          (rc = nfsp::eng::group_snap_part_launch(g->eng.data() + r0, rn, g->d_roll, par, 1, sp[p], r0)) != NFSP_OK)
        return rc;
    }
    if (p > 0) {
      hipEvent_t j = take_event(e0);
      NFSP_HIP(hipEventRecord(j, sp[p]));
      NFSP_HIP(hipStreamWaitEvent(g->s_br, j, 0));
      e0->pool.push_back(j);
    }
  }
  if (pipelined) {
    if (snap_after) NFSP_HIP(hipEventRecord(g->snap_ev[par][1], g->s_br));
    // AR stream: the exchange when due (after this call's AR chains; AR nets only, so no other
    // stream touches what it writes), then the AR nets into snapshot `par`
    NFSP_HIP(hipStreamWaitEvent(g->s_ar, fork, 0));
    if (g->xchg_every > 0 && (++g->calls) % g->xchg_every == 0 && (rc = group_xchg_launch(g, g->s_ar)) != NFSP_OK)
      return rc;
    if (snap_after) {
      if ((rc = nfsp::eng::group_snap_part_launch(g->eng.data(), R, g->d_roll, par, 0, g->s_ar)) != NFSP_OK) return rc;
      NFSP_HIP(hipEventRecord(g->snap_ev[par][0], g->s_ar));
    }
    e0->pool.push_back(fork);
    e0->pool.push_back(fork_br);
    return NFSP_OK;
  }
  for (hipStream_t st : {g->s_ar, g->s_br}) {
    hipEvent_t j = take_event(e0);
    NFSP_HIP(hipEventRecord(j, st));
    NFSP_HIP(hipStreamWaitEvent(s, j, 0));
    e0->pool.push_back(j);
  }
  e0->pool.push_back(fork);
  e0->pool.push_back(fork_br);
  k_finalize<1><<<R, 64, 0, s>>>(FinalArgs{}, d_fin, 7);
  NFSP_LAUNCHED("k_finalize");
  return NFSP_OK;
}

extern "C" int nfsp_engine_snapshot(nfsp_engine* e, int parity, float** dev_w, double* eps) {
  NFSP_REQUIRE(e && dev_w && eps && (parity == 0 || parity == 1), "bad argument");
  NFSP_REQUIRE(e->snap, "the engine has no snapshots (cfg.slice_lag 1)");
  *dev_w = e->snap + (size_t)parity * 6 * nn::NP;
  if (e->snap_eps_dev) {               // a group replica: its snapshots' epsilons are on device
    NFSP_HIP(hipMemcpyAsync(eps, e->snap_eps_dev + 2 * parity, 2 * sizeof(double), hipMemcpyDeviceToHost,
                            e->ctx->stream));
    NFSP_HIP(hipStreamSynchronize(e->ctx->stream));
    return NFSP_OK;
  }
  eps[0] = e->snap_eps[parity][0];
  eps[1] = e->snap_eps[parity][1];
  return NFSP_OK;
}

extern "C" int nfsp_engine_set_update_limit(nfsp_engine* e, int64_t max_updates) {
  NFSP_REQUIRE(e && max_updates >= 0, "bad argument");
  e->update_limit = max_updates;
  return NFSP_OK;
}

extern "C" int nfsp_group_set_timing(nfsp_group* g, int on) {
  NFSP_REQUIRE(g, "null argument");
  for (nfsp_engine* e : g->eng) e->timing = on != 0;
  return NFSP_OK;
}

// the replicas' rollout / prep marks and the group's shared launches (kept on replica 0)
extern "C" int nfsp_group_get_timings(nfsp_group* g, double* ms, int64_t* launches) {
  NFSP_REQUIRE(g && ms && launches, "null argument");
  for (int k = 0; k < KT_N; ++k) { ms[k] = 0.0; launches[k] = 0; }
  for (nfsp_engine* e : g->eng) {
    double m[KT_N];
    int64_t n[KT_N];
    const int rc = nfsp_engine_get_timings(e, m, n);
    if (rc != NFSP_OK) return rc;
    for (int k = 0; k < KT_N; ++k) { ms[k] += m[k]; launches[k] += n[k]; }
  }
  return NFSP_OK;
}

// Every slice: rollout, then its learner, then (when due) the exchange.  With slice_lag 2 the
// slices run one after another, but slice j acts with snapshot j & 1: the nets and epsilon as
// slice j - 2's learner (and exchange) left them, the step's start for j < 2 -- a pipelined
// engine's arithmetic (step_pipelined).
extern "C" int nfsp_group_step(nfsp_group* g) {
  NFSP_REQUIRE(g, "null argument");
  int rc;
  if (g->xchg_nets & ~g->w0_valid)      // common nets before the first exchange
    if ((rc = nfsp_group_average_ar(g)) != NFSP_OK) return rc;
  const int K = g->eng[0]->slices;
  const bool lag2 = g->eng[0]->slice_lag == 2 && K > 1;
  // Pipelined (as step_pipelined): slice j's rollout waits only for the snapshot copies of
  // slice j - 2, so the rollout, readback, plan and prep of slice j + 1 overlap slice j's
  // chains.  The same arithmetic as the serial loop below.  Not with a BR exchange (it would
  // need both learner streams joined after every exchange) or sched.serial.
  if (lag2 && !(g->xchg_nets & NFSP_XCHG_BR) && !g->sched.serial) {
    hipStream_t s = g->ctx->stream;
    if ((rc = nfsp::eng::group_snap_launch(g->eng.data(), g->R, g->d_roll, -1)) != NFSP_OK) return rc;
    for (int j = 0; j < K; ++j) {
      const int par = j & 1;
      if (j >= 2)
        for (hipEvent_t ev : g->snap_ev[par]) NFSP_HIP(hipStreamWaitEvent(s, ev, 0));
      if ((rc = nfsp::eng::group_rollout_launch(g->eng.data(), g->R, g->d_roll, par)) != NFSP_OK) return rc;
      if ((rc = group_update(g, true, par, j + 2 < K)) != NFSP_OK) return rc;
    }
    for (hipStream_t st : {g->s_ar, g->s_br}) {    // the step ends with every stream joined
      hipEvent_t jv = take_event(g->eng[0]);
      NFSP_HIP(hipEventRecord(jv, st));
      NFSP_HIP(hipStreamWaitEvent(s, jv, 0));
      g->eng[0]->pool.push_back(jv);
    }
    return NFSP_OK;
  }
  if (lag2 && (rc = nfsp::eng::group_snap_launch(g->eng.data(), g->R, g->d_roll, -1)) != NFSP_OK) return rc;
  for (int j = 0; j < K; ++j) {
    if ((rc = nfsp::eng::group_rollout_launch(g->eng.data(), g->R, g->d_roll, lag2 ? (j & 1) : -1)) != NFSP_OK)
      return rc;
    if ((rc = group_update(g)) != NFSP_OK) return rc;
    if (g->xchg_every > 0 && (++g->calls) % g->xchg_every == 0 && (rc = nfsp_group_average_ar(g)) != NFSP_OK)
      return rc;
    if (lag2 && j + 2 < K && (rc = nfsp::eng::group_snap_launch(g->eng.data(), g->R, g->d_roll, j & 1)) != NFSP_OK)
      return rc;
  }
  return NFSP_OK;
}

namespace {
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
}  // namespace

extern "C" int nfsp_group_default_sched(nfsp_group_sched* out) {
  NFSP_REQUIRE(out, "null argument");
  out->br_cap = env_int("NFSP_GROUP_BR_CAP", -1);
  out->br_pace = env_int("NFSP_GROUP_BR_PACE", 1) != 0;
  out->br_streams = env_int("NFSP_GROUP_BR_STREAMS", -1);
  out->serial = env_int("NFSP_GROUP_SERIAL", 0) != 0;
  out->br_persist = env_int("NFSP_GROUP_BR_PERSIST", 0);
  return NFSP_OK;
}

extern "C" int nfsp_group_set_sched(nfsp_group* g, const nfsp_group_sched* sc) {
  NFSP_REQUIRE(g && sc, "null argument");
  NFSP_REQUIRE(sc->br_cap >= -1, "br_cap must be >= -1");
  NFSP_REQUIRE(sc->br_streams == -1 || (sc->br_streams >= 1 && sc->br_streams <= GROUP_BR_STREAMS),
               "br_streams must be -1 or in [1, 4]");
  NFSP_REQUIRE(sc->br_persist >= 0, "br_persist must be >= 0");
  g->sched = *sc;
  g->sched.br_pace = sc->br_pace != 0;
  g->sched.serial = sc->serial != 0;
  return NFSP_OK;
}

extern "C" int nfsp_group_get_sched(nfsp_group* g, nfsp_group_sched* out) {
  NFSP_REQUIRE(g && out, "null argument");
  *out = g->sched;
  return NFSP_OK;
}

#ifdef NFSP_BRP_STAMPS
extern "C" int nfsp_debug_brp_stamps(unsigned long long* out, int reset) {
  NFSP_HIP(hipDeviceSynchronize());
  NFSP_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_brp_stamps), sizeof(g_brp_stamps)));
  if (reset) {
    static unsigned long long zero[2][64][4] = {};
    NFSP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_brp_stamps), zero, sizeof(zero)));
  }
  return NFSP_OK;
}
#endif

extern "C" int nfsp_group_check(nfsp_group* g) {
  NFSP_REQUIRE(g, "null argument");
  NFSP_HIP(hipStreamSynchronize(g->ctx->stream));
  for (hipStream_t st : {g->s_ar, g->s_br})
    if (st) NFSP_HIP(hipStreamSynchronize(st));
  for (hipStream_t st : g->s_brp)
    if (st) NFSP_HIP(hipStreamSynchronize(st));
  return group_check_err(g);
}

extern "C" int nfsp_group_rounds(nfsp_group* g, int64_t* out) {
  NFSP_REQUIRE(g && out, "null argument");
  *out = g->rounds;
  return NFSP_OK;
}

extern "C" int nfsp_group_set_trace(nfsp_group* g, int on) {
  NFSP_REQUIRE(g, "null argument");
  g->trace_on = on != 0;
  g->trace.clear();
  return NFSP_OK;
}

extern "C" int nfsp_group_trace(nfsp_group* g, int32_t* out, int64_t cap, int64_t* n) {
  NFSP_REQUIRE(g && n && cap >= 0 && (out || cap == 0), "bad argument");
  const int64_t m = (int64_t)g->trace.size();
  for (int64_t i = 0; i < m && i < cap; ++i) out[i] = g->trace[i];
  *n = m;
  return NFSP_OK;
}
