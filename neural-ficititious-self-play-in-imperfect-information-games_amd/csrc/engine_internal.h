// Internals shared by engine.hip (rollout, insert, lifecycle) and learner.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <utility>
#include <vector>

#include "nfsp_internal.h"
#include "nn_device.h"

namespace nfsp {
namespace eng {

constexpr int MAXREC = 6;          // records of one kind per lane per hand (<= 6 decisions)
// A net in LDS for fwd_lds (one observation per lane): W1 rows padded to W1S = 66 floats,
// so the per-lane row gathers read 2 hidden units at a time (ds_read_b64, 8-byte aligned)
// and rows i, i' of two lanes hit the bank pairs 2i + j, 2i' + j (mod 64): distinct for
// i, i' < 32.  Per hidden unit j one float4 {b1[j], W2[j][0..2]} (one broadcast
// ds_read_b128).  ZROW, the row of +0.0 that unused gather slots point at, sits on the bank
// pair of row 31 (62 mod 64), which no observation bit uses.  NET_LDS is a multiple of 64
// floats, so every net of the rollout's 4 keeps this bank map.
constexpr int W1S = 66;
constexpr int LHB = 1984;                              // OBS * W1S = 1,980, rounded up to 16 B
constexpr int LB2 = LHB + 4 * nn::H;                   // b2[3]
constexpr int ZROW = 2302;                             // 35 x 64 + 62
constexpr int NET_LDS = 2368;                          // 37 x 64 floats
static_assert(OBS * W1S <= LHB && LHB % 4 == 0 && LB2 + NA <= ZROW, "fwd_lds layout");
static_assert(ZROW % 64 == 62 && ZROW % 2 == 0 && ZROW + nn::H <= NET_LDS && NET_LDS % 64 == 0,
              "fwd_lds zero row / net stride");
// packed weight index (W1[30][H] | b1[H] | W2[H][3] | b2[3]) -> fwd_lds' LDS index
__host__ __device__ inline int net_lds_index(int q) {
  if (q < nn::OB1) return (q / nn::H) * W1S + (q % nn::H);
  if (q < nn::OW2) return LHB + 4 * (q - nn::OB1);
  if (q < nn::OB2) return LHB + 4 * ((q - nn::OW2) / NA) + 1 + (q - nn::OW2) % NA;
  return LB2 + (q - nn::OB2);
}
constexpr int MAX_BATCH = 128;     // learner minibatch (config MiniBatchSize)
constexpr int CHAIN_MB = 32;       // fit minibatch of the SGD chains (Keras batch_size)

// Philox counter word x: the rollout uses the lane id (< 2^24); learner streams use these
constexpr uint32_t TAG_SAMPLE = 0x81000000u, TAG_PERM = 0x82000000u, TAG_RES = 0x83000000u;

// Device-resident engine state (one per engine), read and written by the kernels.
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

// On-device record formats.  The reference tuple (utils/replay_buffer.py:
// 30-41, 53-57: s[30], a[3], r, s2[30], t in fp32 / bool, 257 B) is stored bit-packed: the
// observations are 0/1 so 30 bits each, r is a multiple of 0.5 in [-13, 13] so an int8 in
// half units, t a bit; a is kept whole (3 fp32: the stored action vector, net output or
// uniform draw).  nfsp_engine_memories expands them into the reference's fp32 layout.
struct __attribute__((aligned(16))) RlRec {     // one M_RL record, 32 B
  uint32_t s, s2;      // observation bits before / after
  uint32_t meta;       // argmax(a) | t << 8 | (r in half units, int8) << 16  (= BrRow.meta)
  float a0, a1, a2;    // the stored action vector
  uint32_t pad[2];
};
struct __attribute__((aligned(16))) SlRec {     // one M_SL record, 16 B (utils/ReservoirBuffer.py)
  uint32_t x;          // observation bits
  float a0, a1, a2;    // the behaviour vector (raw Q values or the uniform draw)
};

struct Memories {
  // M_RL: circular logs, agent-major [2][log_cap]
  RlRec* rl;
  int64_t log_cap;
  // M_SL: reservoirs [2][sl_cap]
  SlRec* sl;
  int64_t sl_cap;
  // fp32 export views in the reference layout, allocated on first nfsp_engine_memories
  float *ex_rl_s, *ex_rl_a, *ex_rl_r, *ex_rl_s2, *ex_sl_s, *ex_sl_a;
  uint8_t* ex_rl_t;
  // pending SL records of the last rollout [2][pend_cap], insert order
  uint32_t* pend_x;
  float* pend_a;
  int64_t* pend_pos;
  int64_t pend_cap;
  // learner debug: last update's rows / perms per (agent, role)
  int64_t* dbg_rows;    // [4][batch]
  int32_t* dbg_perms;   // [4][epochs][batch]
};

// Everything one SGD step of a learner chain (learner.hip k_chain3) reads, built by the
// prep kernels so the chain's lanes load their matrix-core operands directly:
//   fa[g][s]  8 bf16 0/1 values: bits 4g..4g+3 and 16+4g..16+4g+3 of sample s's observation
//             (the layer-1 K slots 8g..8g+7 of lane row g), stored at fa[g][fa_slot(g, s)]
//   tg[s]     sample s's three fit targets (AR: divided by the batch, exact) and the step's lr
// 2,560 B per step.  The dW1 = X^T dZ1 operand (the bit-transposed minibatch) is not stored:
// the chain reads it from the fa image in LDS with ds_read_b64_tr_b16 (chain3.h).  The chunks
// of odd rows are XOR-swizzled (fa_slot), so the 16-byte row reads of the image are
// conflict-free and the transposed reads 2-way (the minimum for 8-byte reads of one half of
// each chunk).  AR: 1.21x the reference-layout bytes of its 32 sampled M_SL tuples (32 x
// 132 B per epoch of two); BR: 0.62x (32 x 257 B).
// Input 30 (CHAIN_BIAS_BIT) is the constant 1 of every sample: the chain keeps b1 as W1's
// row 30, so the layer-1 products include the bias and dW1's row 30 is gb1.
constexpr uint32_t CHAIN_BIAS_BIT = 1u << 30;
constexpr int CHAIN_BIAS_IN = 30;
__host__ __device__ constexpr int fa_slot(int g, int s) { return s ^ (12 * (g & 1)); }
struct __attribute__((aligned(16))) StepRec {
  uint4 fa[4][32];
  float4 tg[32];
};

// A sampled M_RL row before its TD target exists.
struct BrRow {
  uint32_t s, s2;
  uint32_t meta;       // argmax(a) | t << 8 | (r half units & 0xFF) << 16
};

struct LearnBufs {
  int64_t umax;        // triggers per agent per rollout, upper bound
  BrRow* br_rows;      // [2][umax][batch]
  uint8_t* br_perm;    // [2][umax][epochs][batch]
  double* br_expl;     // [2][umax]
  StepRec* br_rec;     // [2][umax][epochs][batch / 32]: one record per SGD step
  StepRec* ar_rec;     // [2][umax][epochs][batch / 32]
  float* br_loss;      // [2][umax][epochs] Keras epoch losses when the loss log is on (NaN:
  float* ar_loss;      //   no fit), the values agent/agent.py:243,264's TensorBoard logs
  uint8_t* ar_active;  // [2][umax]
  unsigned long long* res_head;   // [2][sl_cap]  (tag << 32 | q)
  int32_t* res_next;   // [2][pend_cap]
  int32_t* res_slot;   // [2][pend_cap]
};

// per-kernel timing slots (nfsp_engine_get_timings)
enum {
  KT_ROLLOUT = 0, KT_SCAN = 1, KT_COMMIT = 2, KT_LEARNER = 3,   // LEARNER = whole update call
  KT_PREP = 4, KT_TARGETS = 5, KT_CHAIN_BR = 6, KT_CHAIN_AR = 7,
  KT_BR_STREAM0 = 8, KT_BR_STREAM1 = 9,   // span of agent a's BR stream (first targets .. last chain)
  KT_XCHG = 10,                           // the cross-shard AR exchange (delta, all-reduce, apply)
  KT_N = 11
};

// Stage packed weights (W1[30][64] | b1 | W2 | b2) into the padded LDS layout of fwd_lds.
__device__ inline void stage_net_lds(float* sw, const float* __restrict__ w, int tid, int nt) {
  for (int q = tid; q < nn::NP; q += nt) sw[net_lds_index(q)] = w[q];
  for (int j = tid; j < nn::H; j += nt) sw[ZROW + j] = 0.f;
}

// Forward of one 0/1 observation (bits) through a net staged by stage_net_lds.  Same
// operation order as oracle/nn_oracle.py (bit-exact for the ReLU and linear heads).
// The BR / target head: ReLU (the reference) or linear (NFSP_EXT_LINEAR_Q).
__host__ __device__ inline int br_act(unsigned quirks) {
  return (quirks & NFSP_EXT_LINEAR_Q) ? NFSP_ACT_LINEAR : NFSP_ACT_RELU;
}
template <int NR>   // gather rows per hidden unit: 9 covers any Leduc observation
__device__ inline void fwd_lds_n(const float* __restrict__ sw, uint32_t x, int act, float y[3]) {
#pragma clang fp contract(off)
  // the set bits' W1 rows in ascending order; the unused slots point at the zero row, so
  // every hidden unit adds 9 terms without a branch.  Exact: acc starts at +0 and only
  // gains finite values, so it is never -0, and a trailing + 0.0 leaves it unchanged.
  int rows[NR];
  uint32_t b = x;
#pragma unroll
  for (int u = 0; u < NR; ++u) {
    rows[u] = b ? __builtin_ctz(b) * W1S : ZROW;
    b &= b - 1;
  }
  float o0 = 0.f, o1 = 0.f, o2 = 0.f;
  // two hidden units per iteration (one 8-byte gather per set bit), unrolled so the LDS
  // reads of several units go out together; every sum keeps its order (bits ascending per
  // unit, units ascending into o), so the result is unchanged
#pragma unroll 4
  for (int j = 0; j < nn::H; j += 2) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const float2 v = *reinterpret_cast<const float2*>(sw + rows[u] + j);
      a0 = a0 + v.x;
      a1 = a1 + v.y;
    }
    if (NR == 9 && b) {   // > 9 set bits: impossible for Leduc observations, kept exact anyway
      uint32_t rest = b;
      while (rest) {
        const int i = __builtin_ctz(rest);
        rest &= rest - 1;
        a0 = a0 + sw[i * W1S + j];
        a1 = a1 + sw[i * W1S + j + 1];
      }
    }
    const float4 p0 = *reinterpret_cast<const float4*>(sw + LHB + 4 * j);
    const float4 p1 = *reinterpret_cast<const float4*>(sw + LHB + 4 * j + 4);
    float h = a0 + p0.x;
    h = h > 0.f ? h : 0.f;
    o0 = o0 + h * p0.y;
    o1 = o1 + h * p0.z;
    o2 = o2 + h * p0.w;
    h = a1 + p1.x;
    h = h > 0.f ? h : 0.f;
    o0 = o0 + h * p1.y;
    o1 = o1 + h * p1.z;
    o2 = o2 + h * p1.w;
  }
  o0 = o0 + sw[LB2 + 0];
  o1 = o1 + sw[LB2 + 1];
  o2 = o2 + sw[LB2 + 2];
  if (act == NFSP_ACT_RELU) {
    y[0] = o0 > 0.f ? o0 : 0.f;
    y[1] = o1 > 0.f ? o1 : 0.f;
    y[2] = o2 > 0.f ? o2 : 0.f;
  } else if (act == NFSP_ACT_LINEAR) {
    y[0] = o0; y[1] = o1; y[2] = o2;
  } else {
    const float m = fmaxf(fmaxf(o0, o1), o2);
    const float e0 = expf(o0 - m), e1 = expf(o1 - m), e2 = expf(o2 - m);
    const float s = (e0 + e1) + e2;
    y[0] = e0 / s; y[1] = e1 / s; y[2] = e2 / s;
  }
}


// The wave picks the 5-, 7- or 9-row body by the most set bits any active lane has (a
// ballot or two): rows a lane does not have read the zero row, so every body gives the
// same sums.
__device__ inline void fwd_lds(const float* __restrict__ sw, uint32_t x, int act, float y[3]) {
  const int pc = __popc(x);
  if (__ballot(pc > 7)) fwd_lds_n<9>(sw, x, act, y);
  else if (__ballot(pc > 5)) fwd_lds_n<7>(sw, x, act, y);
  else fwd_lds_n<5>(sw, x, act, y);
}

}  // namespace eng
}  // namespace nfsp

struct nfsp_engine {
  nfsp_ctx* ctx = nullptr;
  nfsp_engine_cfg cfg{};
  int N = 0;                   // lanes per rollout (n_lanes / slices)
  int slices = 1;              // cfg.slices
  int nblk = 0;
  uint64_t rollouts = 0;
  uint32_t learn_tag = 0;
  bool pending_update = false;
  float* w = nullptr;
  nfsp::eng::EngineDev* st = nullptr;
  nfsp::eng::Staging S{};
  nfsp::eng::Memories M{};
  nfsp::eng::LearnBufs LB{};        // the learner call's buffers: LBs[parity of the slice]
  nfsp::eng::LearnBufs LBs[2]{};     // [1] only with cfg.slice_lag 2 (double-buffered slices)
  int slice_lag = 1;                 // cfg.slice_lag
  // cfg.slice_lag 2: the acting nets of the next rollouts, [parity][2 agents][3 nets][NP]
  // (target slots unused), and the epsilon each parity's rollout acts with
  float* snap = nullptr;
  double snap_eps[2][2] = {};
  hipEvent_t snap_ev[2][3] = {};     // [parity][AR stream, BR stream 0, BR stream 1]
  double* snap_eps_dev = nullptr;    // a group replica's (slice_lag 2): [parity][agent], on device
  // the cross-shard AR exchange (nfsp_engine_set_exchange; exchange.hip)
  int xchg_every = 0;                // learner calls between exchanges (0: off)
  int64_t xchg_calls = 0, xchg_done = 0;
  float xchg_scale = 1.f;
  float* xchg_w0 = nullptr;          // [2][NP] the AR nets after the last exchange
  float* xchg_buf = nullptr;         // [2][NP] D, then the sum over shards
  void* xchg_comm = nullptr;         // RCCL communicator, or
  nfsp_exchange_fn xchg_fn = nullptr;  // the host transport
  void* xchg_user = nullptr;
  bool xchg_pending = false;         // a pipelined call's exchange, enqueued by the next call
  int xchg_pend_par = 0;             //   (or the step's end), with the AR snapshot it feeds
  bool xchg_pend_snap = false;
  // host mirror of the schedules (agent/agent.py:245-253, 266-273): plan_update computes them
  // in the reference's double arithmetic; k_finalize publishes them to EngineDev for the stats
  struct Sched {
    int64_t iteration[2], target_count[2], target_syncs[2];
    double epsilon[2];
  } hs{};
  hipStream_t s_br[2] = {nullptr, nullptr};
  hipStream_t s_ar = nullptr;
  std::vector<void*> allocs;
  // optional per-kernel timing: (kernel id, start, stop) event triples on the ctx stream
  bool timing = false;
  bool log_loss = false;
  int64_t last_U[2] = {0, 0}, last_Ubr[2] = {0, 0};   // the last learner call's update counts
  int64_t update_limit = 0;    // test hook (nfsp_engine_set_update_limit): chains stop after this many
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> marks;
};

namespace nfsp {
namespace eng {

hipEvent_t take_event(nfsp_engine* e);
int engine_create(nfsp_ctx* ctx, const nfsp_engine_cfg* cfg, bool own_streams, nfsp_engine** out);
int rollout_launch(nfsp_engine* e);   // nfsp_rollout's launches
// the same with the acting nets / epsilon given (cfg.slice_lag 2: a snapshot)
int rollout_launch_with(nfsp_engine* e, const float* w, const double eps[2]);
// nfsp_engine_step with cfg.slice_lag 2 (learner.hip): the slices pipelined
int step_pipelined(nfsp_engine* e);
// engine groups: the replicas' rollout arguments as a device table (static), and every
// replica's rollout through it in one launch per kernel
int group_rollout_table(nfsp_engine* const* eng, int R, void** d_tab);
// par: the snapshot parity the slice acts with (slice_lag 2), -1: the replicas' own nets
int group_rollout_launch(nfsp_engine* const* eng, int R, const void* d_tab, int par);
// slice_lag 2: every replica's nets and epsilon -> snapshot par (-1: both parities)
int group_snap_launch(nfsp_engine* const* eng, int R, const void* d_tab, int par);
// one learner stream's part of it (0: AR nets; 1: BR / target nets and epsilons) on stream s
// replicas r0 .. r0 + R - 1 of the group's rollout table (eng: from replica r0)
int group_snap_part_launch(nfsp_engine* const* eng, int R, const void* d_tab, int par, int part, hipStream_t s,
                           int r0 = 0);
// the cross-shard exchange of the AR nets, enqueued on `s` (the AR chain stream)
int exchange_enqueue(nfsp_engine* e, hipStream_t s);

// RAII bracket: records start/stop events around launches on `stream` when timing is on
struct KTimer {
  nfsp_engine* e;
  int id;
  hipStream_t st;
  hipEvent_t a = nullptr;
  KTimer(nfsp_engine* e_, int id_, hipStream_t s_ = nullptr) : e(e_), id(id_), st(s_ ? s_ : e_->ctx->stream) {
    if (e->timing) {
      a = take_event(e);
      (void)hipEventRecord(a, st);
    }
  }
  ~KTimer() {
    if (e->timing) {
      hipEvent_t b = take_event(e);
      (void)hipEventRecord(b, st);
      e->marks.push_back({id, {a, b}});
    }
  }
};

// `batch` distinct uniform draws from [lo, lo + win) into cand[] (LDS), one per thread
// b < batch: Philox(stream, m, (attempt << 8) | b) % win, duplicates redrawn.  Whole
// workgroup must call.
__device__ inline void sample_distinct(int64_t* cand, int batch, int64_t lo, int64_t win,
                                       uint32_t stream, int64_t m, uint32_t k0, uint32_t k1) {
  const int b = threadIdx.x;
  uint32_t attempt = 0;
  bool redraw = b < batch;
  for (;;) {
    if (redraw) {
      const u32x4 u = philox4x32({stream, (uint32_t)m, (uint32_t)(m >> 32), (attempt << 8) | (uint32_t)b},
                                 k0, k1);
      const uint64_t r64 = ((uint64_t)u.x << 32) | u.y;
      cand[b] = lo + (int64_t)(r64 % (uint64_t)win);
      attempt++;
    }
    __syncthreads();
    bool dup = false;
    if (b < batch)
      for (int k = 0; k < b; ++k) dup |= cand[k] == cand[b];
    redraw = dup;
    if (!__syncthreads_or(dup)) break;
  }
}

// Keras fit's per-epoch shuffle: perm[e][rank] = b where rank = order of a unique random
// key (Philox(stream, m, (e << 8) | b) with b in the low byte).  Whole workgroup calls;
// `key` is LDS scratch of `batch` words.
__device__ inline void draw_perm(uint32_t* key, int batch, int e, uint32_t stream, int64_t m,
                                 uint32_t k0, uint32_t k1, int& rank_out) {
  const int b = threadIdx.x;
  if (b < batch) {
    const u32x4 u = philox4x32({stream, (uint32_t)m, (uint32_t)(m >> 32), ((uint32_t)e << 8) | (uint32_t)b},
                               k0, k1);
    key[b] = (u.x & ~0xFFu) | (uint32_t)b;
  }
  __syncthreads();
  rank_out = 0;
  if (b < batch)
    for (int k = 0; k < batch; ++k) rank_out += key[k] < key[b];
  __syncthreads();
}

}  // namespace eng
}  // namespace nfsp
