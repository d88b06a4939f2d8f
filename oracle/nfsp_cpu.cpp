// TEST INFRASTRUCTURE ONLY -- C++ restatement of the reference's self-play loop (main.train
// with its Env, Agent and memories) for the CPU side of the measurement.
//
// Only tests/ (the parity check against oracle/nfsp_oracle.py) and bench.py's cpu_baseline
// leg load this library (oracle/build/libnfsp_cpu.so, built by oracle/Makefile).  It is never
// part of the product path.
//
// It is the same algorithm as nfsp_oracle.py, hand for hand:
//  * CPython `random` is MT19937 seeded by init_by_array over the seed's 32-bit words:
//    random() takes 53 bits from two draws, _randbelow rejects getrandbits(bit_length(n)),
//    and shuffle / randrange / randint / sample(range(n), k) follow CPython 3.10 (sample:
//    the pool method when n <= 21 + 4^ceil(log4(3k)), else the set method).
//  * numpy's global legacy RandomState is MT19937 seeded by init_genrand.  rand() is res53,
//    uniform is low + range * res53, and shuffle draws with masked rejection
//    (random_interval).
//    Calls into both generators happen in the reference's order:
//     - leduc/deck.py:44 shuffle;
//     - main.py:36-45 the eta draws;
//     - agent/agent.py:125-128 eps and rand(1,1,3);
//     - utils/*Buffer*.py the sample / randrange;
//     - Keras fit's per-epoch np.random.shuffle.
//  * Env: leduc/newenv.py:76-349, including the aliasing of stored RL tuples.  s and a are
//    views of env.s[p] / env.last_action[p] (newenv.py:119,126), so they keep changing
//    until the next reset allocates fresh arrays.  Records made during the current hand
//    read the live env arrays and are frozen at the next reset.
//  * Agent: agent/agent.py:130-273.  This includes:
//     - the np.average(a) != 0 store rule and the game_step % 128 trigger;
//     - the terminal flag that is never True (`is True` on np.bool_);
//     - the row-0 targets;
//     - eps ** 1 / iteration and the lr / temp schedules;
//     - target sync when count % 150 == 0.
//    The quirks can be turned off as in nfsp_oracle (quirks=False).
//  * Networks: nn_oracle.py's Keras restatement.
//     - Forwards sum in dense_seq's order (acc += x_i * W_i, then + b; built with
//       -ffp-contract=off), so the ReLU heads match numpy bit for bit.
//     - The softmax uses expf; numpy's SIMD float32 exp differs by up to 2 ulp.
//     - Gradients sum in row order; numpy uses BLAS.
//    So weights agree with nn_oracle to float32 rounding, not bitwise.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <thread>
#include <unordered_set>
#include <vector>

namespace {

// ---------------------------------------------------------------- MT19937 -----------
struct MT19937 {
  uint32_t mt[624];
  int idx = 625;
  void init_genrand(uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + uint32_t(i);
    idx = 624;
  }
  void init_by_array(const uint32_t* key, int n) {
    init_genrand(19650218u);
    int i = 1, j = 0;
    for (int k = std::max(624, n); k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + uint32_t(j);
      ++i; ++j;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= n) j = 0;
    }
    for (int k = 623; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - uint32_t(i);
      ++i;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
    idx = 624;
  }
  uint32_t u32() {
    if (idx >= 624) {
      for (int k = 0; k < 624; ++k) {
        uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
        mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      idx = 0;
    }
    uint32_t y = mt[idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double res53() {
    uint32_t a = u32() >> 5, b = u32() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
};

// CPython 3.10 Lib/random.py over _randommodule.c
struct PyRandom {
  MT19937 m;
  void seed(uint64_t s) {
    uint32_t key[2] = {uint32_t(s), uint32_t(s >> 32)};
    m.init_by_array(key, key[1] ? 2 : 1);
  }
  double random() { return m.res53(); }
  uint64_t randbelow(uint64_t n) {  // _randbelow_with_getrandbits (n < 2^32 here)
    if (n == 0) return 0;
    int k = 64 - __builtin_clzll(n);
    uint64_t r;
    do r = m.u32() >> (32 - k); while (r >= n);
    return r;
  }
  template <class T> void shuffle(T* x, int n) {
    for (int i = n - 1; i > 0; --i) std::swap(x[i], x[randbelow(uint64_t(i) + 1)]);
  }
  // sample(range(n), k) -> out[k]
  void sample(int64_t n, int k, int64_t* out, std::vector<int64_t>& pool,
              std::unordered_set<int64_t>& sel) {
    int64_t setsize = 21;
    if (k > 5) setsize += int64_t(std::pow(4.0, std::ceil(std::log(double(k * 3)) / std::log(4.0))));
    if (n <= setsize) {
      pool.resize(size_t(n));
      for (int64_t i = 0; i < n; ++i) pool[size_t(i)] = i;
      for (int i = 0; i < k; ++i) {
        int64_t j = int64_t(randbelow(uint64_t(n - i)));
        out[i] = pool[size_t(j)];
        pool[size_t(j)] = pool[size_t(n - i - 1)];
      }
    } else {
      sel.clear();
      for (int i = 0; i < k; ++i) {
        int64_t j = int64_t(randbelow(uint64_t(n)));
        while (sel.count(j)) j = int64_t(randbelow(uint64_t(n)));
        sel.insert(j);
        out[i] = j;
      }
    }
  }
};

// numpy mtrand.RandomState (legacy)
struct NpRandom {
  MT19937 m;
  void seed(uint32_t s) { m.init_genrand(s); }
  double rand() { return m.res53(); }
  uint32_t interval(uint32_t mx) {
    if (mx == 0) return 0;
    uint32_t mask = mx;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (m.u32() & mask)) > mx) {}
    return v;
  }
  void shuffle(int* x, int n) {
    for (int i = n - 1; i > 0; --i) std::swap(x[i], x[interval(uint32_t(i))]);
  }
};

// ---------------------------------------------------------------- networks -----------
constexpr int NIN = 30, NH = 64, NOUT = 3;
constexpr int NPARAM = NIN * NH + NH + NH * NOUT + NOUT;   // 2,179: W1 | b1 | W2 | b2

struct Net {
  float w[NPARAM];
  bool softmax;
  float* W1() { return w; }
  float* b1() { return w + NIN * NH; }
  float* W2() { return w + NIN * NH + NH; }
  float* b2() { return w + NIN * NH + NH + NH * NOUT; }
  const float* W1() const { return w; }
  const float* b1() const { return w + NIN * NH; }
  const float* W2() const { return w + NIN * NH + NH; }
  const float* b2() const { return w + NIN * NH + NH + NH * NOUT; }

  void glorot(NpRandom& r) {   // rng.uniform(-l, l, size).astype(float32), W1 then W2
    auto fill = [&](float* W, int fi, int fo) {
      double lim = std::sqrt(6.0 / double(fi + fo)), lo = -lim, range = lim - lo;
      for (int i = 0; i < fi * fo; ++i) W[i] = float(lo + range * r.rand());
    };
    fill(W1(), NIN, NH);
    std::fill(b1(), b1() + NH, 0.f);
    fill(W2(), NH, NOUT);
    std::fill(b2(), b2() + NOUT, 0.f);
  }

  static float relu(float z) { return (z >= 0.f || std::isnan(z)) ? z : 0.f; }  // np.maximum

  // dense_seq order; x is a 30-bit observation (0/1 inputs: x_i * W = W, 0 * W adds +-0).
  void forward(uint32_t x, float* z1, float* h, float* z2, float* y) const {
    float acc[NH];
    for (int j = 0; j < NH; ++j) acc[j] = 0.f;
    for (int i = 0; i < NIN; ++i)
      if ((x >> i) & 1u) {
        const float* Wi = W1() + i * NH;
        for (int j = 0; j < NH; ++j) acc[j] = acc[j] + Wi[j];
      }
    for (int j = 0; j < NH; ++j) {
      z1[j] = acc[j] + b1()[j];
      h[j] = relu(z1[j]);
    }
    float o[NOUT] = {0.f, 0.f, 0.f};
    for (int j = 0; j < NH; ++j)
      for (int k = 0; k < NOUT; ++k) o[k] = o[k] + h[j] * W2()[j * NOUT + k];
    for (int k = 0; k < NOUT; ++k) z2[k] = o[k] + b2()[k];
    if (!softmax) {
      for (int k = 0; k < NOUT; ++k) y[k] = relu(z2[k]);
    } else {
      float mx = std::max(std::max(z2[0], z2[1]), z2[2]);
      float e[NOUT];
      for (int k = 0; k < NOUT; ++k) e[k] = std::exp(z2[k] - mx);
      float s = (e[0] + e[1]) + e[2];
      for (int k = 0; k < NOUT; ++k) y[k] = e[k] / s;
    }
  }
  void predict(uint32_t x, float* y) const {
    float z1[NH], h[NH], z2[NOUT];
    forward(x, z1, h, z2, y);
  }

  // One SGD step on rows idx[0..m) of (xs, ts): nn_oracle.MLP.grads + sgd_step.
  void sgd_step(const uint32_t* xs, const float (*ts)[NOUT], const int* idx, int m, float lr) {
    static thread_local float Z1[32][NH], H[32][NH], DZ1[32][NH];
    float gW1[NIN * NH], gb1[NH], gW2[NH * NOUT], gb2[NOUT];
    float DZ2[32][NOUT];
    const float fm = float(m);
    for (int r = 0; r < m; ++r) {
      float z2[NOUT], y[NOUT];
      forward(xs[idx[r]], Z1[r], H[r], z2, y);
      const float* t = ts[idx[r]];
      if (!softmax) {                                   // Huber, agent/agent.py:91-99
        for (int k = 0; k < NOUT; ++k) {
          float e = t[k] - y[k];
          float d = std::fabs(e) > 1.f ? (e > 0.f ? 1.f : -1.f) : e;
          d = -d / float(3 * m);
          DZ2[r][k] = d * (z2[k] > 0.f ? 1.f : 0.f);
        }
      } else {                                          // categorical cross-entropy
        const float eps = 1e-7f, one_m = 1.f - eps;
        float S = (y[0] + y[1]) + y[2];
        float dldp[NOUT], dldy[NOUT];
        for (int k = 0; k < NOUT; ++k) {
          float p = y[k] / S;
          float pc = std::min(std::max(p, eps), one_m);
          float mask = (p >= eps && p <= one_m) ? 1.f : 0.f;
          dldp[k] = (-t[k] / pc) * mask / fm;
        }
        float sdy = (dldp[0] * y[0] + dldp[1] * y[1]) + dldp[2] * y[2];
        for (int k = 0; k < NOUT; ++k) dldy[k] = dldp[k] / S - sdy / (S * S);
        float s2 = (dldy[0] * y[0] + dldy[1] * y[1]) + dldy[2] * y[2];
        for (int k = 0; k < NOUT; ++k) DZ2[r][k] = y[k] * (dldy[k] - s2);
      }
    }
    std::fill(gW2, gW2 + NH * NOUT, 0.f);
    std::fill(gb2, gb2 + NOUT, 0.f);
    std::fill(gW1, gW1 + NIN * NH, 0.f);
    std::fill(gb1, gb1 + NH, 0.f);
    for (int r = 0; r < m; ++r) {
      for (int j = 0; j < NH; ++j)
        for (int k = 0; k < NOUT; ++k) gW2[j * NOUT + k] += H[r][j] * DZ2[r][k];
      for (int k = 0; k < NOUT; ++k) gb2[k] += DZ2[r][k];
      for (int j = 0; j < NH; ++j) {
        const float* w2 = W2() + j * NOUT;
        float dh = (DZ2[r][0] * w2[0] + DZ2[r][1] * w2[1]) + DZ2[r][2] * w2[2];
        DZ1[r][j] = dh * (Z1[r][j] > 0.f ? 1.f : 0.f);
        gb1[j] += DZ1[r][j];
      }
      uint32_t x = xs[idx[r]];
      for (int i = 0; i < NIN; ++i)
        if ((x >> i) & 1u) {
          float* g = gW1 + i * NH;
          for (int j = 0; j < NH; ++j) g[j] += DZ1[r][j];
        }
    }
    for (int i = 0; i < NIN * NH; ++i) W1()[i] = W1()[i] - lr * gW1[i];
    for (int j = 0; j < NH; ++j) b1()[j] = b1()[j] - lr * gb1[j];
    for (int i = 0; i < NH * NOUT; ++i) W2()[i] = W2()[i] - lr * gW2[i];
    for (int k = 0; k < NOUT; ++k) b2()[k] = b2()[k] - lr * gb2[k];
  }

  // Keras fit(x, t, epochs=2, batch_size=32, shuffle=True): np.random.shuffle per epoch.
  void fit(const uint32_t* xs, const float (*ts)[NOUT], int n, float lr, NpRandom& np_rng) {
    int idx[128];
    for (int ep = 0; ep < 2; ++ep) {
      for (int i = 0; i < n; ++i) idx[i] = i;
      np_rng.shuffle(idx, n);
      for (int b0 = 0; b0 < n; b0 += 32) sgd_step(xs, ts, idx + b0, std::min(32, n - b0), lr);
    }
  }
};

// numpy's float32 add.reduce (pairwise_sum, PW_BLOCKSIZE 128), then / n: np.average of a
// float32 list (agent/agent.py:235-238).
float np_mean_f32(const float* a, int n) {
  struct P {
    static float sum(const float* a, int n) {
      if (n < 8) {
        float r = 0.f;
        for (int i = 0; i < n; ++i) r += a[i];
        return r;
      }
      if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i = 8;
        for (; i < n - (n % 8); i += 8)
          for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
      }
      int n2 = n / 2;
      n2 -= n2 % 8;
      return sum(a, n2) + sum(a + n2, n - n2);
    }
  };
  return P::sum(a, n) / float(n);
}

int argmax3(const double* a) {
  int i = 0;
  if (a[1] > a[i]) i = 1;
  if (a[2] > a[i]) i = 2;
  return i;
}
int argmax3f(const float* a) {
  int i = 0;
  if (a[1] > a[i]) i = 1;
  if (a[2] > a[i]) i = 2;
  return i;
}

// ---------------------------------------------------------------- env ----------------
enum { FOLD = 0, CALL = 1, RAISE = 2 };

struct Env {
  bool kuhn = false;
  int dealer = 0, round = 0, slot = 0;
  bool terminated = false;
  uint32_t hist = 0;
  int ranks[3] = {0, 0, 0};
  int raises[2] = {0, 0};
  int done[4];
  int ndone = 0;
  int contrib[2] = {0, 0};          // half units
  double reward[2] = {0, 0};
  uint32_t s[2] = {0, 0};           // env.s[p] (bits of the pre-action observation)
  double last_action[2][3] = {};
  int64_t warnings = 0;
  struct Live { struct Replay* buf; int64_t seq; };
  std::vector<Live> live;           // RL records aliasing this hand's s / last_action
  PyRandom* py = nullptr;

  void freeze_live();
  void deal() {                     // leduc/deck.py:29-50 (pop from the end)
    if (kuhn) {
      int c[3] = {0, 1, 2};
      py->shuffle(c, 3);
      ranks[0] = c[2]; ranks[1] = c[1]; ranks[2] = 0;
      return;
    }
    int c[6] = {0, 1, 2, 3, 4, 5};
    py->shuffle(c, 6);
    ranks[0] = c[5] / 2; ranks[1] = c[4] / 2; ranks[2] = c[3] / 2;
  }
  void reset(int d) {               // leduc/newenv.py:76-114
    freeze_live();
    dealer = d;
    if (kuhn) { contrib[0] = contrib[1] = 2; }
    else { contrib[d] = 1; contrib[1 - d] = 2; }
    deal();
    s[0] = s[1] = 0;
    hist = 0; round = 0; terminated = false;
    raises[0] = raises[1] = 0;
    reward[0] = reward[1] = 0;
    slot = 0; ndone = 0;
    std::memset(last_action, 0, sizeof last_action);
  }
  uint32_t obs(int p) const {
    uint32_t b = hist | (1u << (24 + ranks[p]));
    if (round == 1) b |= (1u << (27 + ranks[p])) | (1u << (27 + ranks[2]));
    return b;
  }
  bool round_over() const {
    const int* d = done;
    return (ndone == 2 && d[1] == CALL && (d[0] == CALL || d[0] == RAISE)) ||
           (ndone == 3 && d[2] == CALL && d[1] == RAISE && (d[0] == CALL || d[0] == RAISE));
  }
  bool apply(const double* a, int p) {      // do_action, leduc/newenv.py:131-178
    int v = argmax3(a);
    for (int k = 0; k < 3; ++k) last_action[p][k] = a[k];
    if (v == RAISE && (kuhn ? (raises[0] + raises[1] > 0)
                            : (raises[p] > 0 || (ndone == 2 && done[0] == CALL && done[1] == RAISE))))
      v = CALL;
    if (v == FOLD) { done[ndone++] = FOLD; return true; }
    bool prev_raise = ndone > 0 && done[ndone - 1] == RAISE;
    bool opener = round == 0 && ndone == 0;
    hist |= 1u << (12 * p + 6 * round + 2 * slot + (v == CALL ? 0 : 1));
    ++slot;
    if (v == CALL) contrib[p] += prev_raise ? 2 : 0;
    else { raises[p] += 1; contrib[p] += prev_raise ? 4 : 2; }
    if (opener && !kuhn) contrib[p] += 1;
    done[ndone++] = v;
    return false;
  }
  void step(const double* a, int p) {       // leduc/newenv.py:192-349
    s[p] = obs(p);
    if (terminated) { ++warnings; return; }
    int o = 1 - p;
    terminated = apply(a, p);
    if (!terminated && round_over()) {
      if (round == 1 || kuhn) terminated = true;
      else { round = 1; raises[0] = raises[1] = 0; slot = 0; ndone = 0; }
    }
    if (!terminated) return;
    if (argmax3(a) == FOLD) {
      reward[p] = -contrib[p] / 2.0;
      reward[o] = contrib[p] / 2.0;
      return;
    }
    int rp = ranks[p], ro = ranks[o], pub = ranks[2];
    double win_p = contrib[o] / 2.0, win_o = contrib[p] / 2.0;
    if (rp == pub && !kuhn) { reward[p] = win_p; reward[o] = -win_o; }
    else if (ro == pub && !kuhn) { reward[p] = -win_p; reward[o] = win_o; }
    else if (rp < ro) { reward[p] = win_p; reward[o] = -win_o; }
    else if (rp > ro) { reward[p] = -win_p; reward[o] = win_o; }
    else { reward[0] = reward[1] = 0; }
  }
};

// ---------------------------------------------------------------- memories -----------
struct RlRec {
  uint32_t s, s2;
  double a[3];
  double r;
  bool t;
  int8_t live_p;                    // >= 0: s / a are views of the env's arrays of that player
};

struct Replay {                     // utils/replay_buffer.py:20-59 (FIFO deque)
  std::vector<RlRec> ring;
  int64_t cap = 0, count = 0, total = 0;
  RlRec& at(int64_t seq) { return ring[size_t(seq % cap)]; }
  RlRec& item(int64_t j) { return at(total - count + j); }   // deque index j
  void add(const RlRec& r) {
    if (count < cap) ++count;
    at(total) = r;
    ++total;
  }
};

struct Reservoir {                  // utils/ReservoirBuffer.py:8-43
  std::vector<uint32_t> s;
  std::vector<std::array<double, 3>> a;
  int64_t cap = 0, count = 0;
  void add(uint32_t x, const double* av, PyRandom& py) {
    if (count < cap) {
      s[size_t(count)] = x;
      a[size_t(count)] = {av[0], av[1], av[2]};
      ++count;
      return;
    }
    int64_t j = 1 + int64_t(py.randbelow(uint64_t(cap)));
    if (j < cap) { s[size_t(j)] = x; a[size_t(j)] = {av[0], av[1], av[2]}; }
  }
};

void Env::freeze_live() {
  for (const Live& l : live) {
    Replay& b = *l.buf;
    if (l.seq < b.total - b.count) continue;      // evicted already
    RlRec& r = b.at(l.seq);
    int p = r.live_p;
    r.s = s[p];
    for (int k = 0; k < 3; ++k) r.a[k] = last_action[p][k];
    r.live_p = -1;
  }
  live.clear();
}

}  // namespace

// ---------------------------------------------------------------- C ABI --------------
extern "C" {

typedef struct {
  int64_t rl_capacity, sl_capacity;
  double lr_br, lr_ar, gamma, epsilon, eta;
  int32_t batch, target_every;
  int64_t seed;          // random.seed (every buffer constructor) and np.random.seed
  int64_t init_seed;     // RandomState of the Glorot draws (nfsp_oracle.make_main)
  int32_t quirks;        // 1: the reference as written; 0: nfsp_oracle quirks=False
  int32_t game;          // 0 Leduc, 1 Kuhn
  int32_t workload;      // BASELINE.md's CPU workloads: 0 (c) main.train end to end; 1 (a) env +
                         // scheduler with uniform-random action vectors; 2 (b) Agent.play with
                         // the MLP forwards and memory inserts, no update_strategy
} nfsp_cpu_cfg;

typedef struct {
  int64_t hands;
  int64_t rl_inserts[2], sl_inserts[2], rl_size[2], sl_size[2];
  int64_t iteration[2], br_updates[2], ar_updates[2], game_step[2], played[2];
  double actions[2][3], reward[2], epsilon[2], lr_br[2], temp[2], exploitability[2];
  int64_t warnings;
} nfsp_cpu_stats;

}  // extern "C"

namespace {

struct Agent {
  Net ar, br, tgt;
  Replay rl;
  Reservoir sl;
  double epsilon, temp = 1.0, lr_br0, lr_ar, gamma;
  float cur_lr_br;
  int64_t iteration = 0, target_count = 0, game_step = 0, played = 0;
  int64_t rl_inserts = 0, sl_inserts = 0, br_updates = 0, ar_updates = 0;
  int target_every, batch;
  bool quirks;
  double actions[3] = {0, 0, 0}, reward = 0, exploitability = 0;

  // scratch for updates
  std::vector<int64_t> pick, pool;
  std::unordered_set<int64_t> sel;
  uint32_t xs[128], xs2[128];
  float ts[128][NOUT];
};

struct Game {
  nfsp_cpu_cfg cfg;
  PyRandom py;
  NpRandom np;
  Env env;
  Agent ag[2];
  int64_t hands = 0;

  explicit Game(const nfsp_cpu_cfg& c) : cfg(c) {
    env.kuhn = c.game == 1;
    env.py = &py;
    np.seed(uint32_t(c.seed));                    // main.py: np.random.seed(Seed)
    NpRandom init;
    init.seed(uint32_t(c.init_seed));
    for (Agent& a : ag) {                          // agent/agent.py:23-88 construction order
      a.rl.cap = c.rl_capacity;
      a.rl.ring.resize(size_t(c.rl_capacity));
      a.sl.cap = c.sl_capacity;
      a.sl.s.resize(size_t(c.sl_capacity));
      a.sl.a.resize(size_t(c.sl_capacity));
      a.ar.softmax = true;
      a.br.softmax = a.tgt.softmax = false;
      a.ar.glorot(init);
      a.br.glorot(init);
      a.tgt.glorot(init);
      a.tgt = a.br;                                // target_br_model.set_weights(br)
      a.epsilon = c.epsilon;
      a.lr_br0 = c.lr_br;
      a.cur_lr_br = float(c.lr_br);
      a.lr_ar = c.lr_ar;
      a.gamma = c.gamma;
      a.target_every = c.target_every;
      a.batch = c.batch;
      a.quirks = c.quirks != 0;
      a.pick.resize(size_t(c.batch));
    }
    py.seed(uint64_t(c.seed));                     // random.seed(random_seed) in each buffer
  }

  void update_avg(Agent& a) {                      // agent/agent.py:255-264
    if (a.sl.count <= a.batch) return;
    int n = a.batch;
    py.sample(a.sl.count, n, a.pick.data(), a.pool, a.sel);
    for (int k = 0; k < n; ++k) {
      size_t j = size_t(a.pick[size_t(k)]);
      a.xs[k] = a.sl.s[j];
      for (int q = 0; q < NOUT; ++q) a.ts[k][q] = float(a.sl.a[j][q]);
    }
    a.ar.fit(a.xs, a.ts, n, float(a.lr_ar), np);
    ++a.ar_updates;
  }

  void update_br(Agent& a) {                       // agent/agent.py:209-253
    if (a.rl.count <= a.batch) return;
    ++a.iteration;
    int n = a.batch;
    py.sample(a.rl.count, n, a.pick.data(), a.pool, a.sel);
    double av[128][3], r[128];
    bool t[128];
    for (int k = 0; k < n; ++k) {
      RlRec& rec = a.rl.item(a.pick[size_t(k)]);
      if (rec.live_p >= 0) {
        a.xs[k] = env.s[rec.live_p];
        for (int q = 0; q < 3; ++q) av[k][q] = env.last_action[rec.live_p][q];
      } else {
        a.xs[k] = rec.s;
        for (int q = 0; q < 3; ++q) av[k][q] = rec.a[q];
      }
      a.xs2[k] = rec.s2;
      r[k] = rec.r;
      t[k] = rec.t;
    }
    float qmax[128];
    for (int k = 0; k < n; ++k) {
      a.tgt.predict(a.xs[k], a.ts[k]);
      qmax[k] = std::max(std::max(a.ts[k][0], a.ts[k][1]), a.ts[k][2]);
    }
    a.exploitability = double(np_mean_f32(qmax, n));
    for (int k = 0; k < n; ++k) {
      float y2[NOUT];
      a.tgt.predict(a.xs2[k], y2);
      float qn = std::max(std::max(y2[0], y2[1]), y2[2]);
      bool terminal = a.quirks ? false : t[k];
      // gamma * q_next[k]: a Python float times np.float32 is float32 under numpy 2
      // (NEP 50; nfsp_oracle.Agent.br_targets); r + that is float64.
      double v = terminal ? r[k] : r[k] + double(float(a.gamma) * qn);
      int row = a.quirks ? 0 : k;
      a.ts[row][argmax3(av[k])] = float(v);
    }
    a.br.fit(a.xs, a.ts, n, a.cur_lr_br, np);
    ++a.br_updates;
    ++a.iteration;
    a.temp = 1.0 / (1.0 + 0.02 * std::sqrt(double(a.iteration)));
    if (a.target_count % a.target_every == 0) a.tgt = a.br;    // agent/agent.py:266-270
    ++a.target_count;
    a.cur_lr_br = float(a.lr_br0 / (1.0 + 0.003 * std::sqrt(double(a.iteration))));
    a.epsilon = a.epsilon / double(a.iteration);
  }

  // Agent.play (agent/agent.py:130-156); s2_in: the dealer's first call passes d_s.
  bool play(int pi, bool avg_policy, int index, const uint32_t* s2_in) {
    Agent& a = ag[pi];
    uint32_t s2;
    bool t = false;
    if (!s2_in) {
      const double* la = env.last_action[index];
      double r = env.terminated ? env.reward[index] : 0.0;
      s2 = env.obs(index);
      t = env.terminated;
      a.reward += r;
      if (((la[0] + la[1]) + la[2]) / 3.0 != 0.0) {          // np.average(a) != 0
        RlRec rec{};
        rec.s = env.s[index];
        for (int q = 0; q < 3; ++q) rec.a[q] = la[q];
        rec.r = r;
        rec.s2 = s2;
        rec.t = t;
        rec.live_p = int8_t(index);
        env.live.push_back({&a.rl, a.rl.total});
        a.rl.add(rec);
        ++a.rl_inserts;
        ++a.game_step;
      }
      if (t) return t;
    } else {
      s2 = *s2_in;
    }
    int act;
    if (avg_policy) {
      float y[NOUT];
      a.ar.predict(s2, y);
      double yd[3] = {y[0], y[1], y[2]};
      env.step(yd, index);
      act = argmax3f(y);
    } else {
      double at[3];
      if (py.random() > a.epsilon) {                         // act_best_response
        float y[NOUT];
        a.br.predict(s2, y);
        for (int q = 0; q < 3; ++q) at[q] = y[q];
      } else {
        for (int q = 0; q < 3; ++q) at[q] = np.rand();
      }
      double e[3], es = 0;                                   // boltzmann (stats only)
      for (int q = 0; q < 3; ++q) e[q] = std::exp(at[q] / a.temp);
      es = (e[0] + e[1]) + e[2];
      for (int q = 0; q < 3; ++q) e[q] /= es;
      act = argmax3(e);
      env.step(at, index);
      a.sl.add(s2, at, py);
      ++a.sl_inserts;
    }
    ++a.played;
    if (cfg.workload == 0 && a.game_step % 128 == 0) {     // update_strategy
      update_avg(a);
      update_br(a);
    }
    a.actions[act] += 1;
    return t;
  }

  // workload (a): a player that observes (Env.get_state) and steps the env with np.random.rand
  // vectors -- main.train's scheduler around the env with no agent
  bool play_random(int index, bool first) {
    if (!first) {
      (void)env.obs(index);
      if (env.terminated) return true;
    }
    double at[3];
    for (int q = 0; q < 3; ++q) at[q] = np.rand();
    env.step(at, index);
    return false;
  }

  void play_hand(int dealer) {                     // main.py:24-67
    int lhand = 1 - dealer;
    env.reset(dealer);
    bool pol[2];
    pol[dealer] = py.random() > cfg.eta;            // "a" (average policy)
    pol[lhand] = py.random() > cfg.eta;
    uint32_t d_s = env.obs(dealer);
    bool first = true, d_t = false, l_t = false;
    if (cfg.workload == 1) {
      while (!(d_t && l_t)) {
        int rnd = env.round;
        if (!d_t) { d_t = play_random(dealer, first); first = false; }
        if (!l_t) l_t = play_random(lhand, false);
        if (rnd == env.round && !d_t) d_t = play_random(dealer, false);
      }
      ++hands;
      return;
    }
    while (!(d_t && l_t)) {
      int rnd = env.round;
      if (!d_t) { d_t = play(dealer, pol[dealer], dealer, first ? &d_s : nullptr); first = false; }
      if (!l_t) l_t = play(lhand, pol[lhand], lhand, nullptr);
      if (rnd == env.round && !d_t) d_t = play(dealer, pol[dealer], dealer, nullptr);
    }
    ++hands;
  }

  // main.train (nfsp_oracle.train): one call = one dealer draw + `episodes` hands, with the
  // sampled_actions reset every stats_every hands after the first 150.
  void train(int64_t episodes, int stats_every, double* curve, int64_t* n_curve) {
    int dealer = int(py.randbelow(2));
    int64_t nc = 0;
    for (int64_t i = 0; i < episodes; ++i) {
      dealer = 1 - dealer;
      play_hand(dealer);
      if (stats_every > 0 && i > 150 && i % stats_every == 0) {
        for (Agent& a : ag) { a.actions[0] = a.actions[1] = a.actions[2] = 0; a.played = 0; }
        if (curve) curve[nc] = ag[0].exploitability + ag[1].exploitability;
        ++nc;
      }
    }
    if (n_curve) *n_curve = nc;
  }
};

}  // namespace

extern "C" {

void* nfsp_cpu_create(const nfsp_cpu_cfg* cfg) { return new Game(*cfg); }
void nfsp_cpu_destroy(void* g) { delete static_cast<Game*>(g); }

int nfsp_cpu_train(void* h, int64_t episodes, int32_t stats_every, double* curve, int64_t* n_curve) {
  static_cast<Game*>(h)->train(episodes, stats_every, curve, n_curve);
  return 0;
}

int nfsp_cpu_get_stats(void* h, nfsp_cpu_stats* out) {
  Game& g = *static_cast<Game*>(h);
  std::memset(out, 0, sizeof *out);
  out->hands = g.hands;
  out->warnings = g.env.warnings;
  for (int p = 0; p < 2; ++p) {
    const Agent& a = g.ag[p];
    out->rl_inserts[p] = a.rl_inserts;
    out->sl_inserts[p] = a.sl_inserts;
    out->rl_size[p] = a.rl.count;
    out->sl_size[p] = a.sl.count;
    out->iteration[p] = a.iteration;
    out->br_updates[p] = a.br_updates;
    out->ar_updates[p] = a.ar_updates;
    out->game_step[p] = a.game_step;
    out->played[p] = a.played;
    for (int q = 0; q < 3; ++q) out->actions[p][q] = a.actions[q];
    out->reward[p] = a.reward;
    out->epsilon[p] = a.epsilon;
    out->lr_br[p] = a.cur_lr_br;
    out->temp[p] = a.temp;
    out->exploitability[p] = a.exploitability;
  }
  return 0;
}

// net: 0 = AR (avg_strategy_model), 1 = BR, 2 = target BR; out: 2,179 floats (W1|b1|W2|b2).
int nfsp_cpu_weights(void* h, int32_t agent, int32_t net, float* out) {
  Game& g = *static_cast<Game*>(h);
  if (agent < 0 || agent > 1 || net < 0 || net > 2) return -1;
  const Agent& a = g.ag[agent];
  const Net& n = net == 0 ? a.ar : net == 1 ? a.br : a.tgt;
  std::memcpy(out, n.w, sizeof n.w);
  return 0;
}

// Memories in the reference's order: M_RL as the deque (oldest first; records of the
// current hand read the live env arrays), M_SL as the reservoir list.  Returns the count
// written (at most max_n); null pointers skip a field.
int64_t nfsp_cpu_rl(void* h, int32_t agent, int64_t max_n, uint32_t* s, double* a, double* r,
                    uint32_t* s2, uint8_t* t) {
  Game& g = *static_cast<Game*>(h);
  Agent& ag = g.ag[agent & 1];
  int64_t n = std::min(max_n, ag.rl.count);
  for (int64_t j = 0; j < n; ++j) {
    const RlRec& rec = ag.rl.item(j);
    bool live = rec.live_p >= 0;
    if (s) s[j] = live ? g.env.s[rec.live_p] : rec.s;
    if (a) for (int q = 0; q < 3; ++q) a[3 * j + q] = live ? g.env.last_action[rec.live_p][q] : rec.a[q];
    if (r) r[j] = rec.r;
    if (s2) s2[j] = rec.s2;
    if (t) t[j] = rec.t;
  }
  return n;
}

int64_t nfsp_cpu_sl(void* h, int32_t agent, int64_t max_n, uint32_t* s, double* a) {
  Game& g = *static_cast<Game*>(h);
  Agent& ag = g.ag[agent & 1];
  int64_t n = std::min(max_n, ag.sl.count);
  for (int64_t j = 0; j < n; ++j) {
    if (s) s[j] = ag.sl.s[size_t(j)];
    if (a) for (int q = 0; q < 3; ++q) a[3 * j + q] = ag.sl.a[size_t(j)][q];
  }
  return n;
}

// CPU throughput: `threads` independent replicas of main.train (replica i: seed + i,
// init_seed + i), each playing hands until `seconds` of wall time have passed.  Returns
// the hands played by all replicas; *elapsed = the wall time until the last replica stopped.
int64_t nfsp_cpu_bench(const nfsp_cpu_cfg* cfg, int32_t threads, double seconds, double* elapsed) {
  std::vector<std::thread> pool;
  std::vector<int64_t> done(size_t(std::max(threads, 1)), 0);
  std::atomic<int> ready{0};
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < threads; ++i) {
    pool.emplace_back([&, i] {
      nfsp_cpu_cfg c = *cfg;
      c.seed += i;
      c.init_seed += i;
      auto g = std::make_unique<Game>(c);
      int dealer = int(g->py.randbelow(2));
      ready.fetch_add(1);
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        for (int k = 0; k < 64; ++k) {
          dealer = 1 - dealer;
          g->play_hand(dealer);
        }
      }
      done[size_t(i)] = g->hands;
    });
  }
  for (auto& t : pool) t.join();
  if (elapsed) *elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int64_t tot = 0;
  for (int64_t d : done) tot += d;
  return tot;
}

int nfsp_cpu_cfg_size(void) { return int(sizeof(nfsp_cpu_cfg)); }
int nfsp_cpu_stats_size(void) { return int(sizeof(nfsp_cpu_stats)); }

}  // extern "C"
