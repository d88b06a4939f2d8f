// Device-side building blocks shared by every kernel of libnfsp: counter-based RNG,
// the Leduc-variant state machine and the fixed-order MLP forward.
//
// Reference semantics restated here (file:line in /root/reference):
//   leduc/newenv.py:76-114   reset (blinds, fresh per-hand state, deal P0 then P1)
//   leduc/newenv.py:116-129  get_state (s = pre-action obs of p, a = last action of p,
//                            r = reward if terminated else 0, s2 = current obs, t)
//   leduc/newenv.py:131-178  do_action (argmax, raise->call remaps, contributions)
//   leduc/newenv.py:180-190  round-end patterns
//   leduc/newenv.py:192-349  step (pre-action obs, public card, fold/showdown rewards)
//   agent/agent.py:90-116    the 30 -> H -> 3 MLP heads (relu | softmax output)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nfsp {

// ---------------------------------------------------------------------------
// constants
// ---------------------------------------------------------------------------
constexpr int OBS = 30;          // 24 history bits + 2 rounds x 3 ranks
constexpr int NA = 3;            // fold, call, raise
constexpr int CARD_OFF = 24;
constexpr int A_FOLD = 0, A_CALL = 1, A_RAISE = 2;

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11).  Every random draw of the engine is a pure
// function of (seed, counter), so results never depend on scheduling.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

__host__ __device__ inline u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c.x, hi0, lo0);
    mulhilo32(0xCD9E8D57u, c.z, hi1, lo1);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// [0,1) with 24 random bits: exact in fp32 and in fp64.
__host__ __device__ inline float u01(uint32_t u) { return (float)(u >> 8) * 5.9604644775390625e-08f; }
// floor(u * n / 2^32): the engine's randbelow(n).
__host__ __device__ inline uint32_t below(uint32_t u, uint32_t n) {
  return (uint32_t)(((uint64_t)u * (uint64_t)n) >> 32);
}

// Deal from three randbelow draws j5 = below(6), j4 = below(5), j3 = below(4).  These are
// the first three swaps of CPython's shuffle (i = 5, 4, 3) over the ordered deck
// [r0s0, r0s1, r1s0, r1s1, r2s0, r2s1] (leduc/deck.py:35-40); pop() then returns
// positions 5, 4, 3 = P0, P1, public (leduc/newenv.py:109-114, 221).
__host__ __device__ inline void deal_from_draws(uint32_t j5, uint32_t j4, uint32_t j3,
                                                uint8_t& r0, uint8_t& r1, uint8_t& rp) {
  uint8_t d[6] = {0, 1, 2, 3, 4, 5};
  uint8_t t;
  t = d[5]; d[5] = d[j5]; d[j5] = t;
  t = d[4]; d[4] = d[j4]; d[j4] = t;
  t = d[3]; d[3] = d[j3]; d[j3] = t;
  r0 = d[5] >> 1;
  r1 = d[4] >> 1;
  rp = d[3] >> 1;
}

// Kuhn swap-in (BASELINE config C5): a 3-card deck of distinct ranks
// (0 = best); P0's card = below(3) of the deck, P1's = one of the two left.
constexpr int GAME_LEDUC = 0, GAME_KUHN = 1;
__host__ __device__ inline void deal_kuhn(uint32_t j3, uint32_t j2, uint8_t& r0, uint8_t& r1) {
  r0 = (uint8_t)j3;
  r1 = (uint8_t)((j3 + 1 + j2) % 3);
}

// numpy.argmax over 3 floats: the first maximum; a NaN counts as the maximum.
__host__ __device__ inline int argmax3(float a0, float a1, float a2) {
  if (a0 != a0) return 0;
  if (a1 != a1) return 1;
  if (a2 != a2) return 2;
  int v = 0;
  float m = a0;
  if (a1 > m) { v = 1; m = a1; }
  if (a2 > m) { v = 2; }
  return v;
}

// ---------------------------------------------------------------------------
// Leduc-variant hand state (one per env / lane).  64 bytes.
// ---------------------------------------------------------------------------
struct alignas(16) Hand {
  uint32_t hist;        // history[p][round][slot][act] at 12p + 6round + 2slot + act
  uint32_t s[2];        // env.s[p]: observation recorded by p's last step (bits)
  uint32_t warn;        // steps attempted after termination
  float la[2][3];       // env.last_action[p]
  float rew[2];         // env.reward
  uint8_t rank[3];      // P0, P1, public
  uint8_t dealer;
  uint8_t rnd, term, raises0, raises1;
  uint8_t slot, ndone, done0, done1;
  uint8_t done2, c0, c1, game;  // contributions in half units; GAME_LEDUC | GAME_KUHN
};

// Leduc: blinds dealer 0.5 / other 1.0 (leduc/newenv.py:76-114).  Kuhn: antes 1 / 1, one
// betting round, at most one bet, showdown by rank (no public card).
__host__ __device__ inline void hand_reset(Hand& h, int dealer, uint8_t r0, uint8_t r1, uint8_t rp,
                                           int game = GAME_LEDUC) {
  h.hist = 0; h.s[0] = h.s[1] = 0; h.warn = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) { h.la[0][i] = 0.f; h.la[1][i] = 0.f; }
  h.rew[0] = h.rew[1] = 0.f;
  h.rank[0] = r0; h.rank[1] = r1; h.rank[2] = rp;
  h.dealer = (uint8_t)dealer;
  h.rnd = 0; h.term = 0; h.raises0 = 0; h.raises1 = 0;
  h.slot = 0; h.ndone = 0; h.done0 = h.done1 = h.done2 = 0;
  h.game = (uint8_t)game;
  if (game == GAME_KUHN) {
    h.c0 = h.c1 = 2;              // antes 1.0 each
  } else {
    h.c0 = dealer == 0 ? 1 : 2;   // blinds: dealer 0.5, other 1.0
    h.c1 = dealer == 1 ? 1 : 2;
  }
}

// The observation get_state(p) builds (history ++ specific_cards[p]) as 30 bits.
__host__ __device__ inline uint32_t hand_obs(const Hand& h, int p) {
  uint32_t b = h.hist | (1u << (CARD_OFF + h.rank[p]));
  if (h.rnd == 1) b |= (1u << (CARD_OFF + 3 + h.rank[p])) | (1u << (CARD_OFF + 3 + h.rank[2]));
  return b;
}

__host__ __device__ inline uint8_t& hand_contrib(Hand& h, int p) { return p ? h.c1 : h.c0; }
__host__ __device__ inline uint8_t& hand_raises(Hand& h, int p) { return p ? h.raises1 : h.raises0; }

// Whether a raise by p is executed as a raise (else do_action remaps it to a call):
// Leduc leduc/newenv.py:141-145 (p raised this round, or the round so far is [C, R]);
// Kuhn: one bet per hand.
__host__ __device__ inline bool hand_raise_legal(const Hand& h, int p) {
  if (h.game == GAME_KUHN) return h.raises0 + h.raises1 == 0;
  return !((p ? h.raises1 : h.raises0) > 0 || (h.ndone == 2 && h.done0 == A_CALL && h.done1 == A_RAISE));
}

// Env.do_action(action, p) (leduc/newenv.py:131-178): argmax (first max wins), store
// last_action, remap an illegal raise to a call, then record the action.  A fold is recorded
// too (actions_done.append('Fold')) and returns true; termination and round changes are
// step()'s.
__host__ __device__ inline bool hand_do_action(Hand& h, int p, float a0, float a1, float a2) {
  int v = argmax3(a0, a1, a2);
  h.la[p][0] = a0; h.la[p][1] = a1; h.la[p][2] = a2;
  const bool kuhn = h.game == GAME_KUHN;
  if (v == A_RAISE && !hand_raise_legal(h, p)) v = A_CALL;
  if (v != A_FOLD) {
    const bool prev_raise = h.ndone > 0 &&
        (h.ndone == 1 ? h.done0 : (h.ndone == 2 ? h.done1 : h.done2)) == A_RAISE;
    const bool opener = h.rnd == 0 && h.ndone == 0;
    h.hist |= 1u << (12 * p + 6 * h.rnd + 2 * h.slot + (v == A_RAISE ? 1 : 0));
    h.slot++;
    uint8_t& c = hand_contrib(h, p);
    if (v == A_CALL) {
      c += prev_raise ? 2 : 0;
    } else {
      hand_raises(h, p)++;
      c += prev_raise ? 4 : 2;
    }
    if (opener && !kuhn) c += 1;                 // the dealer completes its blind
  }
  if (h.ndone == 0) h.done0 = (uint8_t)v;        // a round holds at most 3 actions
  else if (h.ndone == 1) h.done1 = (uint8_t)v;
  else h.done2 = (uint8_t)v;
  h.ndone++;
  return v == A_FOLD;
}

// Env.game_or_round_has_terminated() (leduc/newenv.py:180-190) on actions_done:
// 1 = True ([C,C] [R,C] [C,R,C] [R,R,C]), 0 = False (length other than 2 or 3),
// -1 = None (a length-2 or -3 sequence that does not end the round).
__host__ __device__ inline int hand_round_status(const Hand& h) {
  if (h.ndone == 2)
    return ((h.done0 == A_CALL || h.done0 == A_RAISE) && h.done1 == A_CALL) ? 1 : -1;
  if (h.ndone == 3)
    return ((h.done0 == A_CALL || h.done0 == A_RAISE) && h.done1 == A_RAISE && h.done2 == A_CALL) ? 1 : -1;
  return 0;
}

// env.step(action, p).  Returns nothing; mirrors every side effect of the reference.
__host__ __device__ inline void hand_step(Hand& h, int p, float a0, float a1, float a2) {
  h.s[p] = hand_obs(h, p);                      // newenv.py:200-202, even after the end
  if (h.term) { h.warn++; return; }             // newenv.py:346-348
  const int o = 1 - p;
  const int raw = argmax3(a0, a1, a2);
  const bool kuhn = h.game == GAME_KUHN;
  if (hand_do_action(h, p, a0, a1, a2)) {
    h.term = 1;
  } else if (hand_round_status(h) == 1) {
    if (h.rnd == 1 || kuhn) {
      h.term = 1;
    } else {
      h.rnd = 1;
      h.raises0 = h.raises1 = 0;
      h.slot = 0;
      h.ndone = 0;
    }
  }
  if (h.term) {
    const float cp = 0.5f * hand_contrib(h, p), co = 0.5f * hand_contrib(h, o);
    float rp_, ro_;
    if (raw == A_FOLD) {
      rp_ = -cp; ro_ = cp;
    } else {
      const int kp = h.rank[p], ko = h.rank[o], kb = h.rank[2];
      if (!kuhn && kp == kb)      { rp_ = co;  ro_ = -cp; }   // pair with the public card
      else if (!kuhn && ko == kb) { rp_ = -co; ro_ = cp; }    // (Kuhn: no public card)
      else if (kp < ko)  { rp_ = co;  ro_ = -cp; }   // lower rank index wins
      else if (kp > ko)  { rp_ = -co; ro_ = cp; }
      else               { rp_ = 0.f; ro_ = 0.f; }   // draw
    }
    h.rew[p] = rp_;
    h.rew[o] = ro_;
  }
}

// ---------------------------------------------------------------------------
// MLP forward, one observation per lane.  Weights are packed
//   W1[30][H] | b1[H] | W2[H][3] | b2[3]
// Order of operations = oracle/nn_oracle.py dense_seq: acc = +0; acc += x_i * W[i] for
// i ascending; then + bias; no FMA contraction (bit-identical to the oracle).  The
// input is 0/1, so layer 1 only adds the rows whose bit is set (x_i * W = +-0 exactly
// otherwise, and adding a signed zero never changes a sum that starts at +0).
// ---------------------------------------------------------------------------
template <int H>
__host__ __device__ inline int mlp_params() { return OBS * H + H + H * NA + NA; }

template <int H, typename WPtr>
__device__ inline void mlp_forward_bits(WPtr w, uint32_t x, int act, float& y0, float& y1, float& y2) {
#pragma clang fp contract(off)
  const int oW2 = OBS * H + H;
  const int ob1 = OBS * H;
  float o0 = 0.f, o1 = 0.f, o2 = 0.f;
  for (int j = 0; j < H; ++j) {
    float acc = 0.f;
    uint32_t bits = x;
    while (bits) {
      const int i = __builtin_ctz(bits);
      bits &= bits - 1;
      acc = acc + w[i * H + j];
    }
    float hj = acc + w[ob1 + j];
    hj = hj > 0.f ? hj : 0.f;
    o0 = o0 + hj * w[oW2 + j * NA + 0];
    o1 = o1 + hj * w[oW2 + j * NA + 1];
    o2 = o2 + hj * w[oW2 + j * NA + 2];
  }
  o0 = o0 + w[oW2 + H * NA + 0];
  o1 = o1 + w[oW2 + H * NA + 1];
  o2 = o2 + w[oW2 + H * NA + 2];
  if (act == 0) {
    y0 = o0 > 0.f ? o0 : 0.f;
    y1 = o1 > 0.f ? o1 : 0.f;
    y2 = o2 > 0.f ? o2 : 0.f;
  } else {
    const float m = fmaxf(fmaxf(o0, o1), o2);
    const float e0 = expf(o0 - m), e1 = expf(o1 - m), e2 = expf(o2 - m);
    const float s = (e0 + e1) + e2;
    y0 = e0 / s; y1 = e1 / s; y2 = e2 / s;
  }
}

}  // namespace nfsp
