// The reference's deck shuffle on the host, for a C caller (nfsp_env_set_deal_mode,
// nfsp_deal_mt; SURVEY §8(b) deal_mode).  The reference shuffles a fresh 6-card deck with the
// global `random` at every Env.reset (leduc/deck.py:42-44, random.shuffle) and pops P0, P1 and
// later the public card from its end (leduc/deck.py:46-50, leduc/newenv.py:98-109,225).
// CPython's random is MT19937:
//   * seed(n): init_by_array over the 32-bit words of |n|, low word first ([0] for 0);
//   * CPython 3: shuffle's j = _randbelow(i + 1) = getrandbits(bit_length(i + 1)), redrawn
//     while >= i + 1; getrandbits(k <= 32) = genrand_uint32() >> (32 - k);
//   * CPython 2.7: j = int(random() * (i + 1)), random() = (a * 2^26 + b) / 2^53 with
//     a = genrand >> 5, b = genrand >> 6.
// This is host code (no device work); the deals reach the device through the ctx's pending
// deal buffer, like nfsp_env_set_deal.
#include <stdint.h>

#include <vector>

#include "nfsp_internal.h"

namespace nfsp {

struct Mt19937 {
  uint32_t mt[624];
  int mti = 625;

  void init_genrand(uint32_t s) {
    mt[0] = s;
    for (mti = 1; mti < 624; ++mti) mt[mti] = 1812433253u * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
  }
  void init_by_array(const uint32_t* key, int len) {
    init_genrand(19650218u);
    int i = 1, j = 0;
    for (int k = 624 > len ? 624 : len; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      ++i;
      ++j;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= len) j = 0;
    }
    for (int k = 623; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      ++i;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
    mti = 624;
  }
  void seed_python(uint64_t n) {     // random.seed(n) for a non-negative int n
    uint32_t key[2] = {(uint32_t)n, (uint32_t)(n >> 32)};
    init_by_array(key, key[1] ? 2 : 1);
  }
  uint32_t genrand() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    if (mti >= 624) {
      int kk = 0;
      for (; kk < 624 - 397; ++kk) {
        const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; ++kk) {
        const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
      mti = 0;
    }
    uint32_t y = mt[mti++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double random() {
    const uint32_t a = genrand() >> 5, b = genrand() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
  uint32_t randbelow3(uint32_t n) {  // CPython 3 _randbelow (n < 2^32)
    int k = 0;
    while ((n >> k) != 0) ++k;       // n.bit_length()
    uint32_t r = genrand() >> (32 - k);
    while (r >= n) r = genrand() >> (32 - k);
    return r;
  }
};

struct DealMt {
  Mt19937 mt;
  int mode = NFSP_DEAL_PHILOX;
  uint8_t* staging = nullptr;       // pinned [n_envs][3]: one reset's deals
  hipEvent_t copied = nullptr;      // the last staging -> device copy
  bool in_flight = false;
};

// one reset's deal: shuffle the ordered deck (card c = rank c >> 1, suit c & 1;
// leduc/deck.py:35-38), P0 = pop(), P1 = pop(), public = the next pop
static void draw_deal(DealMt& d, uint8_t out[3]) {
  int cards[6] = {0, 1, 2, 3, 4, 5};
  for (int i = 5; i >= 1; --i) {
    const uint32_t j = d.mode == NFSP_DEAL_PY2_MT ? (uint32_t)(d.mt.random() * (double)(i + 1))
                                                   : d.mt.randbelow3((uint32_t)(i + 1));
    const int t = cards[i];
    cards[i] = cards[j];
    cards[j] = t;
  }
  out[0] = (uint8_t)(cards[5] >> 1);
  out[1] = (uint8_t)(cards[4] >> 1);
  out[2] = (uint8_t)(cards[3] >> 1);
}

// nfsp_env_reset's host part in an MT deal mode: the ctx's next n deals into pending_deal,
// through a pinned staging buffer.  Only the previous reset's copy out of that buffer is
// waited for (its event), not the whole stream.
int deal_mt_stage(nfsp_ctx* c) {
  DealMt& d = *static_cast<DealMt*>(c->deal_mt);
  const size_t bytes = 3 * (size_t)c->n_envs;
  if (!d.staging) {
    NFSP_HIP(hipHostMalloc((void**)&d.staging, bytes, hipHostMallocDefault));
    NFSP_HIP(hipEventCreateWithFlags(&d.copied, hipEventDisableTiming));
  }
  if (d.in_flight) NFSP_HIP(hipEventSynchronize(d.copied));
  for (int i = 0; i < c->n_envs; ++i) draw_deal(d, d.staging + 3 * (size_t)i);
  NFSP_HIP(hipMemcpyAsync(c->pending_deal, d.staging, bytes, hipMemcpyHostToDevice, c->stream));
  NFSP_HIP(hipEventRecord(d.copied, c->stream));
  d.in_flight = true;
  c->has_pending_deal = true;
  return NFSP_OK;
}

void deal_mt_free(nfsp_ctx* c) {
  DealMt* d = static_cast<DealMt*>(c->deal_mt);
  if (d) {
    if (d->in_flight) (void)hipEventSynchronize(d->copied);
    if (d->copied) (void)hipEventDestroy(d->copied);
    if (d->staging) (void)hipHostFree(d->staging);
  }
  delete d;
  c->deal_mt = nullptr;
}

}  // namespace nfsp

extern "C" int nfsp_env_set_deal_mode(nfsp_ctx* c, int mode, uint64_t seed) {
  NFSP_REQUIRE(c, "null argument");
  NFSP_REQUIRE(mode == NFSP_DEAL_PHILOX || mode == NFSP_DEAL_PY3_MT || mode == NFSP_DEAL_PY2_MT,
               "unknown deal mode");
  NFSP_REQUIRE(mode == NFSP_DEAL_PHILOX || c->game == NFSP_GAME_LEDUC,
               "the MT deal modes reproduce the reference's Leduc deck");
  nfsp::deal_mt_free(c);
  if (mode != NFSP_DEAL_PHILOX) {
    auto* d = new nfsp::DealMt();
    d->mode = mode;
    d->mt.seed_python(seed);
    c->deal_mt = d;
  }
  return NFSP_OK;
}

extern "C" int nfsp_deal_mt(int mode, uint64_t seed, int64_t n, uint8_t* out) {
  NFSP_REQUIRE(out && n >= 0, "bad argument");
  NFSP_REQUIRE(mode == NFSP_DEAL_PY3_MT || mode == NFSP_DEAL_PY2_MT, "mode must be PY3_MT or PY2_MT");
  nfsp::DealMt d;
  d.mode = mode;
  d.mt.seed_python(seed);
  for (int64_t i = 0; i < n; ++i) nfsp::draw_deal(d, out + 3 * i);
  return NFSP_OK;
}
