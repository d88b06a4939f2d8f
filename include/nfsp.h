/*
 * nfsp.h -- C ABI of libnfsp, the MI355X (gfx950) NFSP-on-Leduc self-play engine.
 *
 * The reference (dantodor/Neural-Ficititious-Self-Play-in-Imperfect-Information-Games)
 * has no FFI: its boundary is the duck-typed Python object API that main.train calls
 * (SURVEY.md §8b).  Every entry point below replaces one of those Python methods, in
 * batched form (n envs / n records per call); the file:line it replaces is cited.
 * The Python host side (the package's leduc.py / agent.py / buffers.py) binds these
 * with ctypes exactly as INTEGRATION.md shows.
 *
 * Conventions
 *   - Every function returns an int status: NFSP_OK (0) or a negative NFSP_E* code;
 *     nfsp_last_error() returns a thread-local message for the last failure.
 *     Game-level misuse is NOT an error, mirroring the reference, which never raises:
 *     illegal raises are remapped (leduc/newenv.py:141-145) and a step after the hand
 *     ended only updates env.s[p] and counts a warning (leduc/newenv.py:346-348).
 *   - Pointers named dev_* are device (HBM) pointers, e.g. torch.Tensor.data_ptr() of a
 *     cuda tensor; everything else is host memory.  Outputs are caller-owned; the ctx
 *     owns env state and its workspaces.
 *   - All work is enqueued on the ctx's stream (default: the null stream; see
 *     nfsp_set_stream) and is asynchronous unless the function says otherwise.
 *   - A ctx is not thread-safe (the reference is single-threaded with one env shared
 *     by both agents, agent/agent.py:28).
 *   - Layouts: observations are float32 [n,30] (24 history bits + 2x3 card bits, values
 *     0/1, leduc/newenv.py:53,118), action vectors float32 [n,3], rewards float32.
 *     Network weights are float32, packed W1[30][H] | b1[H] | W2[H][3] | b2[3]
 *     (= Keras get_weights() order, flattened), H = hidden width (config HiddenLayer).
 */
#ifndef NFSP_H
#define NFSP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NFSP_OK 0
#define NFSP_EINVAL (-1)   /* bad argument (null pointer, size, unsupported width) */
#define NFSP_EHIP (-2)     /* a HIP runtime call failed (message has the HIP error) */
#define NFSP_ENOMEM (-3)

#define NFSP_GAME_LEDUC 0
/* Kuhn swap-in (BASELINE config C5): the same 30-bit observation layout (history bits of
 * round 0, card one-hot at bit 24 + rank), 3 distinct ranks (0 best), antes 1 / 1, one
 * betting round with at most one bet (further raises remap to call), showdown by rank. */
#define NFSP_GAME_KUHN 1

/* MLP output activation / loss (agent/agent.py:103,106,112,115) */
#define NFSP_ACT_RELU 0        /* BR / target-BR head, Huber loss */
#define NFSP_ACT_SOFTMAX 1     /* AR head, categorical cross-entropy */
#define NFSP_ACT_LINEAR 2      /* BR head under NFSP_EXT_LINEAR_Q (engine only) */

/* Reference quirks, reproduced by default (SURVEY.md §7 hard part (b)). */
#define NFSP_QUIRK_TERMINAL_BOOTSTRAP 1u  /* `t_batch[k] is True` never holds: terminal
                                             transitions bootstrap (agent/agent.py:227) */
#define NFSP_QUIRK_ROW0_TARGET 2u         /* TD targets overwrite row 0 only
                                             (agent/agent.py:240-241) */
#define NFSP_QUIRK_ALIAS_RL 4u            /* stored (s, a) of an RL tuple are views of
                                             env.s[p] / env.last_action[p]: every tuple of a
                                             hand ends up with p's LAST pre-action s and a
                                             (utils/replay_buffer.py:30-41 + newenv.py:119) */
#define NFSP_QUIRKS_REFERENCE 7u
/* Textbook-NFSP extensions of the batched engine (Heinrich & Silver 2016), in the same
 * cfg.quirks word.  NOT the reference's algorithm -- NFSP_QUIRKS_REFERENCE leaves them off.
 * They let the same engine run NFSP proper, e.g. for C5's exploitability -> 0 check
 * (DESIGN.md §9); quirks = NFSP_TEXTBOOK is that algorithm with every reference quirk off. */
#define NFSP_EXT_SL_ONEHOT 8u     /* M_SL stores one-hot(argmax) of the BR action, not its raw
                                     vector (the reference: agent/agent.py:147-151) */
#define NFSP_EXT_RESERVOIR 16u    /* M_SL is a true reservoir (Algorithm R): the k-th insert
                                     (k >= N, 0-based) takes slot j = U{0..k} iff j < N (the
                                     reference: utils/ReservoirBuffer.py:22-28) */
#define NFSP_EXT_LINEAR_Q 32u     /* BR / target nets with a linear Q head (the reference's is
                                     ReLU, agent/agent.py:103); Huber on the linear outputs */
#define NFSP_EXT_EPS_CONST 64u    /* eps stays at cfg.epsilon (the reference: eps / iteration
                                     after each BR update, agent/agent.py:253, which ends
                                     exploration within a few updates) */
#define NFSP_EXT_SAMPLE_AR 128u   /* an agent acting with its average policy samples the action
                                     from the AR softmax (Philox counter (lane, hand, 2^31 + k)
                                     for its k-th AR decision) and passes the one-hot vector:
                                     the reference passes the softmax itself, which the env
                                     executes as its argmax (agent/agent.py:143, newenv.py:135) */
#define NFSP_EXT_MSE_Q 256u       /* with NFSP_EXT_LINEAR_Q: the BR / target nets are fitted with
                                     mean squared error, not the reference's Huber loss
                                     (agent/agent.py:91-99).  Huber's clipped gradient makes Q a
                                     robust location estimate (between median and mean), so with
                                     bimodal returns (a +-2 showdown) Q(s, a) sits up to ~1 chip from
                                     the expected return and the greedy "best response" is not one
                                     (tests/studies/kuhn_diag.py).  Requires LINEAR_Q. */
#define NFSP_TEXTBOOK (NFSP_EXT_SL_ONEHOT | NFSP_EXT_RESERVOIR | NFSP_EXT_LINEAR_Q | \
                       NFSP_EXT_EPS_CONST | NFSP_EXT_SAMPLE_AR)
/* NFSP_TEXTBOOK with the expected-return (MSE) Q loss: NFSP as Heinrich & Silver train it */
#define NFSP_TEXTBOOK_MSE (NFSP_TEXTBOOK | NFSP_EXT_MSE_Q)
/* ... with epsilon decaying as the reference's (eps / iteration) instead of NFSP_EXT_EPS_CONST.
 * With SL_ONEHOT, a constant 0.06 stores argmax(rand(3)) -- a uniform action -- for 6 % of the
 * BR decisions, which mixes uniform play into the average policy: Kuhn's exploitability then
 * stops at 0.06-0.09 chips whatever the learning rates; decaying, it reaches 0.01-0.02
 * (profiles/r06/kuhn_*.jsonl). */
#define NFSP_TEXTBOOK_MSE_DECAY (NFSP_TEXTBOOK_MSE & ~NFSP_EXT_EPS_CONST)

typedef struct nfsp_ctx nfsp_ctx;

/* Record columns of an M_RL (utils/replay_buffer.py:30-41) or M_SL
 * (utils/ReservoirBuffer.py:18-28) memory; all device pointers, rows contiguous.
 * M_SL uses s and a only (r, s2, t = NULL). */
typedef struct nfsp_records {
  float* s;     /* [cap, 30] */
  float* a;     /* [cap, 3]  */
  float* r;     /* [cap]     */
  float* s2;    /* [cap, 30] */
  uint8_t* t;   /* [cap]     */
  int64_t cap;
} nfsp_records;

/* ---------------------------------------------------------------- lifecycle */
const char* nfsp_last_error(void);
int nfsp_version(void);
int nfsp_device_count(int* out);

/* Creates a ctx holding n_envs Leduc hands on HIP device `device`.
 * Replaces leduc/newenv.py:14-57 (Env.__init__), batched. */
int nfsp_create(nfsp_ctx** out, int n_envs, uint64_t seed, int game, int device);
int nfsp_destroy(nfsp_ctx* ctx);
/* hip_stream: a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream), 0 = null stream */
int nfsp_set_stream(nfsp_ctx* ctx, void* hip_stream);
int nfsp_synchronize(nfsp_ctx* ctx);
int nfsp_num_envs(const nfsp_ctx* ctx);

/* ---------------------------------------------------------------- env (batched newenv API) */
/* Stores deals (P0, P1, public rank; rank 0 = Ace is best) for the NEXT nfsp_env_reset.
 * Test/host injection of the deck (the reference shuffles the global `random`,
 * leduc/deck.py:42-50; the Python drop-in shuffles there and injects the result).
 * This is how the deal modes of SURVEY §8(b) reach the device.  PHILOX is
 * nfsp_env_reset's own draw.  PY3_MT and PY2_MT are CPython 3 / 2.7 shuffles of the
 * host's MT19937 stream (nfsp_amd.pyrandom.set_python_semantics(3 | 2)), drawn on the host
 * and injected here. */
int nfsp_env_set_deal(nfsp_ctx* ctx, const uint8_t* dev_ranks /* [n,3] */);
/* Deal modes (SURVEY §8(b) deal_mode) of nfsp_env_reset.  The reference reshuffles a fresh
 * 6-card deck with the global `random` at every Env.reset (leduc/deck.py:42-44) and pops
 * P0, P1 and the public card from its end.
 *   PHILOX  (default): the device draw keyed by (ctx seed, env, reset index);
 *   PY3_MT / PY2_MT:   that shuffle on the host, under CPython 3's / 2.7's random seeded
 *                      with random.seed(seed).  Every reset deals env 0, 1, ..., n-1 from
 *                      the one stream, and the deck is its only consumer.  The drop-in
 *                      Python Env shares the process's global random with the rest of
 *                      main.train instead (nfsp_amd.pyrandom).  Leduc only.
 * A pending nfsp_env_set_deal still takes precedence for the next reset. */
#define NFSP_DEAL_PHILOX 0
#define NFSP_DEAL_PY3_MT 1
#define NFSP_DEAL_PY2_MT 2
int nfsp_env_set_deal_mode(nfsp_ctx* ctx, int mode, uint64_t seed);
/* Host only (no device work): the first n deals (P0, P1, public rank) of deal mode PY3_MT or
 * PY2_MT from random.seed(seed), as nfsp_env_reset would draw them for n consecutive resets
 * of a 1-env ctx. */
int nfsp_deal_mt(int mode, uint64_t seed, int64_t n, uint8_t* out /* [n,3] */);
/* Env.reset(dealer) (leduc/newenv.py:76-114) for every env.  Deal = the pending
 * nfsp_env_set_deal if any, else a Philox draw keyed by (seed, env, reset index). */
int nfsp_env_reset(nfsp_ctx* ctx, const uint8_t* dev_dealer /* [n] */);
/* Env.get_state(p) (leduc/newenv.py:116-129).  Player = dev_players[i] if non-null, else p.
 * Any output may be NULL.  s = env.s[p] (obs recorded by p's last step), a =
 * env.last_action[p], r = reward if terminated else 0, s2 = current obs, t = terminated. */
int nfsp_env_get_state(nfsp_ctx* ctx, int p, const uint8_t* dev_players,
                       float* dev_s /*[n,30]*/, float* dev_a /*[n,3]*/, float* dev_r /*[n]*/,
                       float* dev_s2 /*[n,30]*/, uint8_t* dev_t /*[n]*/);
/* Env.step(action, p) (leduc/newenv.py:192-349).  Envs with dev_mask[i] == 0 are left
 * untouched (dev_mask may be NULL = all). */
int nfsp_env_step(nfsp_ctx* ctx, const float* dev_action /*[n,3]*/, int p,
                  const uint8_t* dev_players, const uint8_t* dev_mask);
/* Env.do_action(action, p) (leduc/newenv.py:131-178) alone: argmax, last_action, the
 * illegal-raise remap, then the action recorded (history, pot, actions_done; a fold too).
 * No round change, termination or reward (those are step()'s).  dev_fold[i] = its return
 * value (1 on a fold); dev_fold may be NULL. */
int nfsp_env_do_action(nfsp_ctx* ctx, const float* dev_action /*[n,3]*/, int p,
                       const uint8_t* dev_players, const uint8_t* dev_mask, uint8_t* dev_fold /*[n]*/);
/* Env.game_or_round_has_terminated() (leduc/newenv.py:180-190) on each env's actions_done:
 * 1 = True ([C,C] [R,C] [C,R,C] [R,R,C]), 0 = False (length other than 2 or 3),
 * -1 = None (the reference's fall-through for other length-2 / -3 sequences). */
int nfsp_env_round_status(nfsp_ctx* ctx, int8_t* dev_out /*[n]*/);
/* Env.round_index (leduc/newenv.py:59-61) */
int nfsp_env_round(nfsp_ctx* ctx, uint8_t* dev_round /*[n]*/);
/* Debug/introspection: the 64-byte per-env state (layout nfsp_device.h `Hand`). */
int nfsp_env_export(nfsp_ctx* ctx, void* dev_out /*[n,64] bytes*/);

/* ---------------------------------------------------------------- networks */
/* model.predict(x) (agent/agent.py:126,143,219,230) for B rows; bit-identical to the
 * oracle's fixed summation order for 0/1 inputs. */
int nfsp_mlp_forward(nfsp_ctx* ctx, const float* dev_w, int hidden, int act,
                     const float* dev_x /*[B,30]*/, float* dev_y /*[B,3]*/, int64_t B);
/* model.fit(x, y, epochs, batch_size) with plain SGD (agent/agent.py:243,261): for each
 * epoch, rows dev_perm[e*n .. e*n+n) in slices of batch_size, one SGD step per slice.
 * act selects the loss (RELU -> Huber, SOFTMAX -> categorical cross-entropy).
 * Weights are updated in place.  batch_size <= 64, hidden == 64. */
int nfsp_mlp_fit(nfsp_ctx* ctx, float* dev_w, int hidden, int act,
                 const float* dev_x /*[n,30]*/, const float* dev_t /*[n,3]*/, int n,
                 const int32_t* dev_perm /*[epochs,n]*/, int epochs, int batch_size, float lr);
/* The TD-target construction of update_best_response_network (agent/agent.py:219-241):
 * target = Q_target(s); v_k = r_k + gamma * max Q_target(s2_k) (or r_k if terminal and the
 * TERMINAL_BOOTSTRAP quirk is off); expl = mean_k max target[k] (agent/agent.py:235-238,
 * before the overwrite); then target[row][argmax a_k] = v_k with row = 0 under
 * ROW0_TARGET (sequential, last k wins) else k.  dev_expl: one float64. */
int nfsp_br_targets(nfsp_ctx* ctx, const float* dev_target_w, int hidden,
                    const float* dev_s, const float* dev_a, const float* dev_r,
                    const float* dev_s2, const uint8_t* dev_t, int n, double gamma,
                    unsigned quirks, float* dev_target_out /*[n,3]*/, double* dev_expl);

/* ---------------------------------------------------------------- memories */
/* ReplayBuffer.add / ReservoirBuffer.add (utils/replay_buffer.py:30-41,
 * utils/ReservoirBuffer.py:18-28): copy n records src[i] -> dst[dev_slots[i]].  The slot
 * policy (FIFO head, reservoir j) is the caller's; duplicate slots: last i wins. */
int nfsp_buf_insert(nfsp_ctx* ctx, const nfsp_records* dst, const nfsp_records* src,
                    const int64_t* dev_slots, int64_t n);
/* sample_batch (utils/replay_buffer.py:46-59, utils/ReservoirBuffer.py:33-43): gather
 * dst[i] = src[dev_idx[i]] for i < k (columns that are NULL in dst are skipped). */
int nfsp_buf_sample(nfsp_ctx* ctx, const nfsp_records* src, const int64_t* dev_idx,
                    int64_t k, const nfsp_records* dst);

/* ---------------------------------------------------------------- batched self-play engine
 * The fused hot path (SURVEY.md §8a rows a1-a18 at scale): n_lanes concurrent hands,
 * one hand per lane per nfsp_rollout, both agents' memories and networks on device.
 *
 *   nfsp_rollout       main.train's hand loop (main.py:27-67) x n_lanes in ONE kernel:
 *                      deal (deck.py), eta draws, D/L/D scheduler, Agent.play
 *                      (agent/agent.py:130-156) with the AR / eps-greedy BR forwards,
 *                      env.step; then the RL/SL records are committed in canonical
 *                      order (lane, then play order) to the agents' memories.
 *   nfsp_engine_update the learner for the inserts of the last rollout: update_strategy
 *                      once per `inserts_per_update` RL inserts of an agent (the
 *                      reference's game_step % 128 trigger), each one =
 *                      update_avg_response_network + update_best_response_network with
 *                      the reference schedules; M_SL inserts are applied in stream order
 *                      between the AR updates they precede.
 * Randomness: Philox4x32-10 keyed by cfg.seed; counters (lane, hand, draw) for the
 * rollout and (agent, update, row) for the learner -- results do not depend on
 * scheduling.  Deviation from the sequential reference (declared): all hands of one
 * rollout act with the weights and epsilon at its start (policy lag <= one rollout);
 * repeated triggers while game_step stays on a multiple of 128 are not replayed. */
typedef struct nfsp_engine nfsp_engine;

typedef struct nfsp_engine_cfg {
  int32_t n_lanes;             /* hands in flight */
  int32_t hidden;              /* [Agent] HiddenLayer, must be 64 */
  int64_t rl_capacity;         /* M_RL size (reference: [Utils] Buffersize 40000) */
  int64_t sl_capacity;         /* M_SL size (reference: 40000); < 2^31 */
  int32_t batch;               /* [Agent] MiniBatchSize 128 */
  int32_t inserts_per_update;  /* 128: game_step % 128 (agent/agent.py:153) */
  int32_t target_every;        /* [Agent] TargetModelUpdateRate 150 */
  int32_t epochs;              /* fit epochs, 2 (agent/agent.py:243,261) */
  int32_t fit_batch;           /* Keras default batch_size 32 */
  uint32_t quirks;             /* NFSP_QUIRKS_REFERENCE */
  float eta, lr_br, lr_ar;     /* 0.1, 0.05, 0.1 */
  double gamma, epsilon;       /* 0.95, 0.06 */
  uint64_t seed;
  /* Lane slices (1 = off).  The n_lanes envs are advanced in `slices` equal slices of
   * n_lanes / slices lanes: nfsp_rollout plays one hand on every lane of the next slice, and
   * nfsp_engine_step = `slices` x (nfsp_rollout + nfsp_engine_update), i.e. one hand per lane
   * of all n_lanes, with the learner consuming each slice's inserts before the next slice
   * acts.  That bounds the declared policy lag by one slice instead of all n_lanes hands
   * (the reference has none: main.py:27-67 learns inside the hand loop,
   * agent/agent.py:153-154).  Philox counters and the dealer use the global lane id
   * (slice * n_lanes / slices + lane) and the lane's hand count (rollouts / slices), so a
   * lane's hand does not depend on the slicing.  Staging and learner buffers are sized for
   * one slice.  n_lanes must be a multiple of slices. */
  int32_t slices;
  /* Slice lag inside nfsp_engine_step (slices > 1): 1 = the learner of slice k completes
   * before slice k + 1 acts; 2 = pipelined: slice k + 1's rollout (and the host's plan and the
   * prep kernels of its learner) run while slice k's SGD chains do, so slice k + 1 acts with
   * the nets and epsilon as of the end of slice k - 1's learner (the first two slices of a step:
   * as of the step's start).  The policy lag is then two slices; the chains' streams never
   * wait for a rollout.  Each step starts from the nets as they are (nfsp_engine_weights
   * writes between steps are seen) and ends with every stream joined.  nfsp_rollout /
   * nfsp_engine_update called by themselves always run with lag 1.  Engine groups run their
   * slices one after another, and with slice_lag 2 each replica's slice j acts with the nets
   * and epsilon its learner left after slice j - 2 (snapshots on device): the same arithmetic
   * as a pipelined engine, not its overlap. */
  int32_t slice_lag;
  /* Scheduling flags (NFSP_SCHED_*; they change only the order of launches, never a result).
   * nfsp_engine_default_cfg takes them from the environment (NFSP_LEARNER_SERIAL=1), read at
   * that call; 0 = the production schedule. */
  uint32_t sched;
} nfsp_engine_cfg;
/* diagnostic: an engine's BR work waits for its AR chains, to time each alone */
#define NFSP_SCHED_LEARNER_SERIAL 1u

typedef struct nfsp_engine_stats {
  int64_t hands, rollouts;
  int64_t rl_total[2], sl_total[2];     /* inserts ever, per agent */
  int64_t rl_size[2], sl_size[2];       /* memory sizes (ReplayBuffer/ReservoirBuffer.size);
                                         * sl_size counts the reservoir rows as stored: a
                                         * rollout's SL inserts (in sl_total) are applied to
                                         * them by nfsp_engine_update */
  int64_t last_rl[2], last_sl[2];       /* inserts of the last rollout */
  int64_t br_updates[2], ar_updates[2];
  int64_t iteration[2], target_syncs[2];
  int64_t actions[2][3];                /* Agent.actions counters (agent/agent.py:155) */
  double reward[2];                     /* Agent.reward */
  double epsilon[2], temp[2], lr_br[2];
  double exploitability[2];             /* last BR update's proxy (agent/agent.py:235-238) */
} nfsp_engine_stats;

int nfsp_engine_default_cfg(nfsp_engine_cfg* out);
int nfsp_engine_create(nfsp_ctx* ctx, const nfsp_engine_cfg* cfg, nfsp_engine** out);
int nfsp_engine_destroy(nfsp_engine* e);
/* Device pointer to the packed weights of agent (0|1), net (0 = AR avg_strategy_model,
 * 1 = BR best_response_model, 2 = target_br_model); read or write them in place. */
int nfsp_engine_weights(nfsp_engine* e, int agent, int net, float** dev_w);
int nfsp_rollout(nfsp_engine* e);
/* Test hook: nfsp_rollout acting with the given nets (device [2 agents][3 nets][NP], the
 * target slots unused) and epsilons instead of the engine's -- what a pipelined slice does
 * with its snapshot (cfg.slice_lag 2); lets a test drive a lag-1 engine through the same
 * schedule and compare. */
int nfsp_rollout_with(nfsp_engine* e, const float* dev_w, const double* eps /*[2]*/);
int nfsp_engine_update(nfsp_engine* e);
int nfsp_engine_step(nfsp_engine* e);          /* nfsp_rollout + nfsp_engine_update */
/* After a non-OK return from nfsp_rollout / nfsp_engine_update / nfsp_engine_step the
 * engine's state is unspecified: part of the step's work may have run.  Destroy the
 * engine (nfsp_engine_destroy waits for all of its streams). */
int nfsp_engine_get_stats(nfsp_engine* e, nfsp_engine_stats* out);   /* synchronises */
/* Agent's memories in the reference's fp32 tuple layout (utils/replay_buffer.py:53-57),
 * expanded on the ctx stream at the call from the packed device records (M_RL: 32 B
 * {s bits, s2 bits, argmax|t|r, a[3]}, M_SL: 16 B {bits, a[3]}; the export buffers are
 * allocated on first use).  M_RL is a circular log of rl_log_cap rows whose record k
 * (k-th insert ever) sits at row k % rl_log_cap; the logical M_RL is the last
 * min(rl_total, rl_capacity) records.  sl: the reservoir (rows [0, sl_size)).
 * pending_sl (live views): the last rollout's M_SL records not yet applied by
 * nfsp_engine_update, in insert order, with rl_pos = the agent's RL insert count when each
 * was made. */
int nfsp_engine_memories(nfsp_engine* e, int agent, nfsp_records* rl, int64_t* rl_log_cap,
                         nfsp_records* sl, uint32_t** dev_pending_sl_obs,
                         float** dev_pending_sl_a, int64_t** dev_pending_sl_rl_pos);
/* Per-kernel timing with HIP events recorded around each launch on the stream it runs on:
 * ms / launches [11] = {k_rollout, k_scan1+k_scan2, k_commit, learner (whole
 * nfsp_engine_update), learner prep (k_br_prep..k_res_apply), k_br_targets,
 * k_chain3<BR>, k_chain3<AR>, BR stream of agent 0, BR stream of agent 1, the AR exchange
 * (nfsp_engine_set_exchange: delta, all-reduce, apply on the AR stream)}, accumulated since
 * the previous nfsp_engine_get_timings (which synchronises and resets them).  A "BR stream"
 * entry is the span of one learner call's BR work of that agent on its stream, from its
 * first k_br_targets to its last chain, gaps included (engine groups: their one BR stream in
 * slot 8) -- with k_chain3<AR> (one launch per call, both agents), the per-stream critical
 * path of the learner. */
int nfsp_engine_set_timing(nfsp_engine* e, int on);
/* Loss log (observability; the reference's TensorBoard callbacks on fit, agent/agent.py:
 * 84-88,243,264): when on, the SGD chains also record each update's Keras epoch losses
 * (BR: the py2 huber_loss of agent/agent.py:91-99, where 1 / 2 == 0; AR: categorical
 * cross-entropy), each minibatch's loss taken before its step.  nfsp_engine_losses gives, per
 * agent a and net n (0 = AR, 1 = BR), out[(2a + n) * 2 + 0] = the mean epoch loss over the last
 * nfsp_engine_update's updates and [.. + 1] = its last update's final-epoch loss (NaN: none). */
int nfsp_engine_set_loss_log(nfsp_engine* e, int on);
int nfsp_engine_losses(nfsp_engine* e, double* out /*[2][2][2]*/);
#define NFSP_TIMING_SLOTS 11
int nfsp_engine_get_timings(nfsp_engine* e, double* ms /*[NFSP_TIMING_SLOTS]*/,
                            int64_t* launches /*[NFSP_TIMING_SLOTS]*/);
/* Debug view of the last learner run: per agent and role (0 = AR, 1 = BR) the sampled
 * rows [batch] (int64) and fit permutations [epochs][batch] (int32) of its LAST update. */
int nfsp_engine_last_update(nfsp_engine* e, int agent, int role, int64_t** dev_rows,
                            int32_t** dev_perms);
/* Debug view of the last rollout's per-lane record counts [n_lanes / slices] (uint32, device;
 * local lane i of the slice that rollout played is global lane slice * n_lanes / slices + i):
 * rl0 | rl1 << 4 | sl0 << 8 | sl1 << 12 (RL / SL inserts of agents 0 and 1 by that lane's
 * hand).  Their exclusive prefix over lanes is each lane's first record in the canonical
 * insert order (lane, then play order) -- how a test finds one lane's records in M_RL. */
int nfsp_engine_lane_counts(nfsp_engine* e, uint32_t** dev_counts);

/* Debug view (cfg.slice_lag 2): the acting nets [2 agents][3 nets][NP] (target slots unused)
 * and epsilons of snapshot `parity` -- after a pipelined nfsp_engine_step of K slices, snapshot
 * (K - 1) & 1 holds what the step's last slice acted with. */
int nfsp_engine_snapshot(nfsp_engine* e, int parity, float** dev_w, double* eps /*[2]*/);

/* ---- cross-shard exchange of the average-policy nets (BASELINE C4) ----
 * The reference learns inside its hand loop (main.py:27-67; update_strategy every 128 RL
 * inserts, agent/agent.py:153-154, whose AR fit is agent/agent.py:255-264).  Sharded over N
 * GPUs, each shard's learner trains its own copy of both agents' AR nets; the exchange keeps
 * the copies one net: at the end of every `every`-th learner call (one call per lane slice:
 * every = 1 exchanges after every slice, every = cfg.slices once per step), right behind the
 * call's AR chain on the chain's own stream,
 *     D = W_AR - W0   (both agents, 2 x NP f32),   S = sum over shards of D,
 *     W_AR = W0 + S * scale,   W0 = W_AR
 * (scale 1 / N: the mean of the shards' gradient steps, i.e. data-parallel SGD of one net
 * over every shard's minibatches, exchanged per slice).  Before the AR snapshot of a
 * pipelined slice (cfg.slice_lag 2), so the rollout two slices on acts with the exchanged
 * nets.  Arithmetic: fp contract off, S summed from +0 -- with 2 shards bit-identical to an
 * engine group's on-device exchange (NFSP_GROUP_AVG_AR, nfsp_group_set_exchange).
 * Transports (exactly one):
 *   rccl_comm  an RCCL communicator (nfsp_rccl_comm_create): ncclAllReduce(SUM) of D in place
 *              on the AR chain stream -- stream-ordered, no host round trip;
 *   fn         a host callback, for transports that are not stream-ordered (gloo rehearsals
 *              and CPU-side tests): the engine synchronises the AR stream, calls
 *              fn(user, dev_D, 2 * NP), which must leave S in dev_D (device memory, complete
 *              on return) and return 0; anything else fails the step.
 * Every shard must make the same number of learner calls (the same slices per step).
 * nfsp_engine_set_exchange takes W0 = the AR nets as they are now (call it after the shards'
 * AR nets were made equal, e.g. broadcast from rank 0); every = 0 turns the exchange off. */
typedef int (*nfsp_exchange_fn)(void* user, float* dev_sum, int64_t n);
int nfsp_engine_set_exchange(nfsp_engine* e, int every, float scale, void* rccl_comm,
                             nfsp_exchange_fn fn, void* user);
/* exchanges made so far */
int nfsp_engine_exchanges(nfsp_engine* e, int64_t* out);
/* RCCL (librccl.so.1, loaded on first use): ncclGetUniqueId into out[128] (rank 0), and a
 * communicator of `world` ranks on HIP device `device` from that id (every rank, collectively:
 * ncclCommInitRank blocks until all ranks joined).  nfsp_rccl_ready loads RCCL and selects
 * `device` without joining anything: every rank calls it and the ranks agree (an all-reduce
 * MIN of the results) BEFORE any of them calls nfsp_rccl_comm_create, so a rank that cannot
 * use RCCL never leaves the others blocked in ncclCommInitRank. */
int nfsp_rccl_ready(int device);
int nfsp_rccl_unique_id(uint8_t* out /*[128]*/);
int nfsp_rccl_comm_create(const uint8_t* id /*[128]*/, int world, int rank, int device, void** comm);
int nfsp_rccl_comm_destroy(void* comm);

/* Test hook: from the next nfsp_engine_update on, each agent's AR and BR chains run only the
 * first max_updates updates of the learner call (0 = all).  Everything else still follows
 * the full plan: the prep kernels, the reservoir, and the counters and schedules in the
 * stats.  A test compares the weights with an oracle replay of the same update prefix.  The
 * engine is not meant to train on after that. */
int nfsp_engine_set_update_limit(nfsp_engine* e, int64_t max_updates);

/* ---- engine groups: several learners on one GPU ----
 * A group holds R replicas of the engine.  Each replica is an independent
 * main.train (main.py:21-75) over cfg.n_lanes lanes: its own hands, its own M_RL / M_SL, and
 * its own nets.  Replica r uses cfg.seed + r, and is bit-identical to a standalone engine
 * created with that seed and stepped as often.  nfsp_group_step does rollout + update for
 * every replica.  The SGD chains of all replicas run in shared launches: one AR launch of 2R
 * workgroups; the BR chains in rounds of one targets launch and one chain launch.  Unsliced,
 * round k holds every (replica, agent)'s k-th target-sync segment; sliced (cfg.slices > 1),
 * the replicas are split into 2 halves with their own rounds on their own streams, and a
 * round's pieces are at most 40 updates, paced by the half's busiest job (nfsp_group_sched;
 * DESIGN.md 4.5).  A piece
 * resumes from the weights in memory, so the SGD steps are a standalone engine's.  A chain
 * workgroup occupies one CU, so one learner pair's 4 CUs become 4R.  This is BASELINE C4's
 * shard model inside one GPU.
 * With NFSP_GROUP_AVG_AR, replica 0's AR nets are first copied to every replica.  After every
 * step, each AR net becomes W0 + sum_r (W_r - W0) / R, with W0 = the nets after the
 * previous exchange.  This is shards.AvgPolicyAllReduce's per-step exchange, done on device.
 * A replica's handle (nfsp_group_engine) serves weights, stats, memories, the loss log and
 * timing; nfsp_engine_update / nfsp_engine_step on it are refused. */
typedef struct nfsp_group nfsp_group;
#define NFSP_GROUP_MAX_REPLICAS 256
#define NFSP_GROUP_AVG_AR 1u
int nfsp_group_create(nfsp_ctx* ctx, const nfsp_engine_cfg* cfg, int replicas, unsigned flags,
                      nfsp_group** out);
int nfsp_group_destroy(nfsp_group* g);
int nfsp_group_engine(nfsp_group* g, int replica, nfsp_engine** out);
int nfsp_group_step(nfsp_group* g);
/* The exchange by itself (nfsp_group_step does it when NFSP_GROUP_AVG_AR is set or
 * nfsp_group_set_exchange configured one).  Its first call copies replica 0's exchanged nets
 * everywhere. */
int nfsp_group_average_ar(nfsp_group* g);
/* The group's exchange, as nfsp_engine_set_exchange's over shards: at the end of every
 * `every`-th learner call (slice) of the group, each net in `nets` (NFSP_XCHG_AR: both agents'
 * AR nets; NFSP_XCHG_BR: their BR nets) becomes W0 + (sum_r (W_r - W0)) * scale, summed in
 * replica order from +0, and W0 <- that.  every = 0: off.  NFSP_GROUP_AVG_AR at creation is
 * nets = AR, every = cfg.slices (once per step, after its last slice), scale = 1 / R.  The first
 * exchange of a net (or nfsp_group_average_ar) copies replica 0's net (with BR also its target
 * net) to every replica instead -- also the first after a call that turns the net on again. */
#define NFSP_XCHG_AR 1u
#define NFSP_XCHG_BR 2u
int nfsp_group_set_exchange(nfsp_group* g, unsigned nets, int every, float scale);
/* How a group schedules its BR rounds and slices.  None of these changes an SGD
 * step: a BR piece resumes from the weights in memory, and every partition's jobs run the same
 * pieces and targets (tests/test_gpu_group.py varies them within one process).
 *   br_cap      most updates per BR piece; -1: 40 for sliced groups, whole segments (0) else
 *   br_pace     1: a partition's busiest job splits each segment into equal pieces and the
 *               others follow its piece per round; 0: plain caps
 *   br_streams  BR partitions, each its own rounds on its own stream (1..4); -1: 2 for sliced
 *               groups, else 1 (always 1 when chains share CUs)
 *   serial      1: the slices of a pipelined group run one after another (no overlap)
 *   br_persist  0: BR rounds.  >= 1: a learner call's BR work in ONE launch of the persistent
 *               kernel k_br_persist -- a chain workgroup per (replica, agent) and 48 helper
 *               workgroups writing the targets from a device work queue (groups of <= 32
 *               replicas, the reference's BR net, no loss log; others keep the rounds).  Values
 *               > 1 bound every device wait at that many s_sleep 8 rounds (default 2^18); an
 *               expired wait ends the kernel and the error surfaces at the next learner call or
 *               nfsp_group_check.  br_cap / br_pace / br_streams do not apply to it.
 * nfsp_group_default_sched reads the environment's NFSP_GROUP_BR_CAP / _BR_PACE / _BR_STREAMS /
 * NFSP_GROUP_SERIAL / NFSP_GROUP_BR_PERSIST at that call (nfsp_group_create starts from it);
 * nfsp_group_set_sched applies from the next learner call. */
typedef struct nfsp_group_sched {
  int32_t br_cap, br_pace, br_streams, serial, br_persist;
} nfsp_group_sched;
int nfsp_group_default_sched(nfsp_group_sched* out);
int nfsp_group_set_sched(nfsp_group* g, const nfsp_group_sched* sched);
int nfsp_group_get_sched(nfsp_group* g, nfsp_group_sched* out);
int nfsp_group_set_timing(nfsp_group* g, int on);
/* nfsp_engine_get_timings summed over the replicas.  The shared chain and target launches
 * count once each. */
int nfsp_group_get_timings(nfsp_group* g, double* ms /*[NFSP_TIMING_SLOTS]*/,
                           int64_t* launches /*[NFSP_TIMING_SLOTS]*/);
/* BR rounds of the last learner call: the most any BR partition ran.  Sliced groups split the
 * replicas' BR jobs into 2 partitions (nfsp_group_sched.br_streams, 1..4), each with its own
 * rounds on its own stream; the SGD steps are the same as with one. */
int nfsp_group_rounds(nfsp_group* g, int64_t* out);
/* Synchronise the group's streams and report a k_br_persist wait that expired (NFSP_EHIP). */
int nfsp_group_check(nfsp_group* g);
/* Diagnostic trace of the learner calls' plans (tools/c4_slice_spread.py: the lockstep cost of
 * a per-slice exchange across C4 ranks).  on = 1 clears and starts it; every learner call then
 * appends, per replica r and agent a, its AR and BR update counts: [call][r][a][AR, BR].
 * nfsp_group_trace copies min(cap, size) int32 values and reports the size in *n. */
int nfsp_group_set_trace(nfsp_group* g, int on);
int nfsp_group_trace(nfsp_group* g, int32_t* out, int64_t cap, int64_t* n);

/* ---- evaluation ----
 * Exact exploitability of two average-policy nets (packed weights, device pointers; e.g.
 * nfsp_engine_weights(e, a, 0, ..)) in this Leduc variant as main.train plays it
 * (main.py:21-67; the reference's proxy is agent/agent.py:235-238 summed at main.py:73,
 * its MC evaluator main.py:82-120, commented out).  mode 0: each net's softmax as a mixed
 * strategy (NFSP's average strategy; an illegal raise's mass goes to call); mode 1: the
 * argmax the env executes (leduc/newenv.py:135-145).  out[0] / out[1]: best-response value
 * of seat 0 / 1 against the other seat's policy, over both dealers and all deals;
 * out[2] = out[0] + out[1] (exploitability, chips); out[3] = seat 0's on-policy value.
 * The whole evaluation runs on the device (csrc/exploit.hip k_exploit_walk: the policies,
 * reach top-down and best-response values bottom-up over the public tree, in f64); only
 * the 4 results come back.  Synchronises the ctx stream. */
int nfsp_exploitability(nfsp_ctx* ctx, const float* dev_w_ar0, const float* dev_w_ar1, int mode,
                        double* out /*[4]*/);
/* The same for n pairs of nets at once (one workgroup per pair; e.g. every replica of an
 * engine group): dev_w_ar0[k] / dev_w_ar1[k] are host arrays of device pointers, out[4k..4k+3]
 * pair k's results as above. */
int nfsp_exploitability_batch(nfsp_ctx* ctx, const float* const* dev_w_ar0, const float* const* dev_w_ar1,
                              int n, int mode, double* out /*[4n]*/);

#ifdef __cplusplus
}
#endif
#endif /* NFSP_H */
