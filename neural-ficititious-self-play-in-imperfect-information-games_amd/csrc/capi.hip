// libnfsp C ABI: ctx lifecycle, the batched Leduc env (newenv API) and the memory
// insert/sample kernels.  Declarations and reference citations: include/nfsp.h.
#include <stdio.h>

#include "nfsp_internal.h"

using nfsp::Hand;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

namespace nfsp {
void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) { g_err = msg; return code; }
int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return NFSP_EHIP;
}
}  // namespace nfsp

extern "C" const char* nfsp_last_error(void) { return g_err.c_str(); }
extern "C" int nfsp_version(void) { return 1; }

extern "C" int nfsp_device_count(int* out) {
  NFSP_REQUIRE(out, "out is null");
  NFSP_HIP(hipGetDeviceCount(out));
  return NFSP_OK;
}

// ---------------------------------------------------------------------------
// env kernels: one lane per env (state is a 64-B struct, touched once per call)
// ---------------------------------------------------------------------------
__global__ void k_env_reset(Hand* __restrict__ hands, int n, const uint8_t* __restrict__ dealer,
                            const uint8_t* __restrict__ ranks, uint32_t k0, uint32_t k1,
                            uint32_t reset_lo, uint32_t reset_hi, int game) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t r0, r1, rp = 0;
  if (ranks) {
    r0 = ranks[3 * i]; r1 = ranks[3 * i + 1]; rp = ranks[3 * i + 2];
  } else {
    const nfsp::u32x4 u = nfsp::philox4x32({(uint32_t)i, reset_lo, reset_hi, 0xDEA1u}, k0, k1);
    if (game == nfsp::GAME_KUHN)
      nfsp::deal_kuhn(nfsp::below(u.x, 3), nfsp::below(u.y, 2), r0, r1);
    else
      nfsp::deal_from_draws(nfsp::below(u.x, 6), nfsp::below(u.y, 5), nfsp::below(u.z, 4), r0, r1, rp);
  }
  Hand h;
  nfsp::hand_reset(h, dealer[i] & 1, r0, r1, rp, game);
  hands[i] = h;
}

// one lane per (env, feature) so the [n,30] outputs are written coalesced
__global__ void k_env_get_state(const Hand* __restrict__ hands, int n, int p,
                                const uint8_t* __restrict__ players, float* __restrict__ s,
                                float* __restrict__ a, float* __restrict__ r,
                                float* __restrict__ s2, uint8_t* __restrict__ t) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * nfsp::OBS) return;
  const int i = (int)(e / nfsp::OBS);
  const int f = (int)(e - (int64_t)i * nfsp::OBS);
  const Hand& h = hands[i];
  const int q = players ? (players[i] & 1) : p;
  if (s) s[e] = (float)((h.s[q] >> f) & 1u);
  if (s2) s2[e] = (float)((nfsp::hand_obs(h, q) >> f) & 1u);
  if (f < nfsp::NA && a) a[3 * i + f] = h.la[q][f];
  if (f == 0) {
    if (r) r[i] = h.term ? h.rew[q] : 0.f;
    if (t) t[i] = h.term;
  }
}

__global__ void k_env_step(Hand* __restrict__ hands, int n, const float* __restrict__ action, int p,
                           const uint8_t* __restrict__ players, const uint8_t* __restrict__ mask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (mask && !mask[i]) return;
  Hand h = hands[i];
  const int q = players ? (players[i] & 1) : p;
  nfsp::hand_step(h, q, action[3 * i], action[3 * i + 1], action[3 * i + 2]);
  hands[i] = h;
}

__global__ void k_env_do_action(Hand* __restrict__ hands, int n, const float* __restrict__ action, int p,
                                const uint8_t* __restrict__ players, const uint8_t* __restrict__ mask,
                                uint8_t* __restrict__ fold) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (mask && !mask[i]) return;
  Hand h = hands[i];
  const int q = players ? (players[i] & 1) : p;
  const bool f = nfsp::hand_do_action(h, q, action[3 * i], action[3 * i + 1], action[3 * i + 2]);
  hands[i] = h;
  if (fold) fold[i] = f ? 1 : 0;
}

__global__ void k_env_round_status(const Hand* __restrict__ hands, int n, int8_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int8_t)nfsp::hand_round_status(hands[i]);
}

__global__ void k_env_round(const Hand* __restrict__ hands, int n, uint8_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = hands[i].rnd;
}

// ---------------------------------------------------------------------------
// lifecycle
// ---------------------------------------------------------------------------
extern "C" int nfsp_create(nfsp_ctx** out, int n_envs, uint64_t seed, int game, int device) {
  NFSP_REQUIRE(out, "out is null");
  NFSP_REQUIRE(n_envs > 0, "n_envs must be > 0");
  NFSP_REQUIRE(game == NFSP_GAME_LEDUC || game == NFSP_GAME_KUHN, "unsupported game");
  *out = nullptr;
  NFSP_HIP(hipSetDevice(device));
  nfsp_ctx* c = new nfsp_ctx();
  c->n_envs = n_envs;
  c->device = device;
  c->game = game;
  c->seed = seed;
  hipError_t e = hipMalloc(&c->hands, sizeof(Hand) * (size_t)n_envs);
  if (e == hipSuccess) e = hipMalloc(&c->pending_deal, 3 * (size_t)n_envs);
  if (e == hipSuccess) e = hipMalloc(&c->scratch_f64, 64 * sizeof(double));
  if (e == hipSuccess) e = hipMemset(c->hands, 0, sizeof(Hand) * (size_t)n_envs);
  if (e != hipSuccess) {
    nfsp_destroy(c);
    return nfsp::hip_fail(e, "nfsp_create: device allocation");
  }
  *out = c;
  return NFSP_OK;
}

extern "C" int nfsp_destroy(nfsp_ctx* c) {
  if (!c) return NFSP_OK;
  if (c->hands) (void)hipFree(c->hands);
  if (c->pending_deal) (void)hipFree(c->pending_deal);
  nfsp::deal_mt_free(c);
  if (c->scratch_f64) (void)hipFree(c->scratch_f64);
  if (c->scratch_i64) (void)hipFree(c->scratch_i64);
  delete c;
  return NFSP_OK;
}

extern "C" int nfsp_set_stream(nfsp_ctx* c, void* s) {
  NFSP_REQUIRE(c, "ctx is null");
  c->stream = (hipStream_t)s;
  return NFSP_OK;
}

extern "C" int nfsp_synchronize(nfsp_ctx* c) {
  NFSP_REQUIRE(c, "ctx is null");
  NFSP_HIP(hipStreamSynchronize(c->stream));
  return NFSP_OK;
}

extern "C" int nfsp_num_envs(const nfsp_ctx* c) { return c ? c->n_envs : 0; }

// ---------------------------------------------------------------------------
// env API
// ---------------------------------------------------------------------------
extern "C" int nfsp_env_set_deal(nfsp_ctx* c, const uint8_t* ranks) {
  NFSP_REQUIRE(c && ranks, "null argument");
  NFSP_HIP(hipMemcpyAsync(c->pending_deal, ranks, 3 * (size_t)c->n_envs, hipMemcpyDeviceToDevice,
                          c->stream));
  c->has_pending_deal = true;
  return NFSP_OK;
}

extern "C" int nfsp_env_reset(nfsp_ctx* c, const uint8_t* dealer) {
  NFSP_REQUIRE(c && dealer, "null argument");
  if (c->deal_mt && !c->has_pending_deal) {       // nfsp_env_set_deal_mode: CPython's shuffle
    const int rc = nfsp::deal_mt_stage(c);
    if (rc != NFSP_OK) return rc;
  }
  const uint64_t ri = c->resets++;
  k_env_reset<<<nfsp_blocks(c->n_envs, 256), 256, 0, c->stream>>>(
      c->hands, c->n_envs, dealer, c->has_pending_deal ? c->pending_deal : nullptr,
      (uint32_t)c->seed, (uint32_t)(c->seed >> 32), (uint32_t)ri, (uint32_t)(ri >> 32), c->game);
  NFSP_LAUNCHED("k_env_reset");
  c->has_pending_deal = false;
  return NFSP_OK;
}

extern "C" int nfsp_env_get_state(nfsp_ctx* c, int p, const uint8_t* players, float* s, float* a,
                                  float* r, float* s2, uint8_t* t) {
  NFSP_REQUIRE(c, "ctx is null");
  NFSP_REQUIRE(p == 0 || p == 1 || players, "player must be 0 or 1");
  const int64_t total = (int64_t)c->n_envs * nfsp::OBS;
  k_env_get_state<<<nfsp_blocks(total, 256), 256, 0, c->stream>>>(c->hands, c->n_envs, p & 1,
                                                                   players, s, a, r, s2, t);
  NFSP_LAUNCHED("k_env_get_state");
  return NFSP_OK;
}

extern "C" int nfsp_env_step(nfsp_ctx* c, const float* action, int p, const uint8_t* players,
                             const uint8_t* mask) {
  NFSP_REQUIRE(c && action, "null argument");
  NFSP_REQUIRE(p == 0 || p == 1 || players, "player must be 0 or 1");
  k_env_step<<<nfsp_blocks(c->n_envs, 256), 256, 0, c->stream>>>(c->hands, c->n_envs, action,
                                                                  p & 1, players, mask);
  NFSP_LAUNCHED("k_env_step");
  return NFSP_OK;
}

extern "C" int nfsp_env_do_action(nfsp_ctx* c, const float* action, int p, const uint8_t* players,
                                  const uint8_t* mask, uint8_t* fold) {
  NFSP_REQUIRE(c && action, "null argument");
  NFSP_REQUIRE(p == 0 || p == 1 || players, "player must be 0 or 1");
  k_env_do_action<<<nfsp_blocks(c->n_envs, 256), 256, 0, c->stream>>>(c->hands, c->n_envs, action,
                                                                       p & 1, players, mask, fold);
  NFSP_LAUNCHED("k_env_do_action");
  return NFSP_OK;
}

extern "C" int nfsp_env_round_status(nfsp_ctx* c, int8_t* out) {
  NFSP_REQUIRE(c && out, "null argument");
  k_env_round_status<<<nfsp_blocks(c->n_envs, 256), 256, 0, c->stream>>>(c->hands, c->n_envs, out);
  NFSP_LAUNCHED("k_env_round_status");
  return NFSP_OK;
}

extern "C" int nfsp_env_round(nfsp_ctx* c, uint8_t* out) {
  NFSP_REQUIRE(c && out, "null argument");
  k_env_round<<<nfsp_blocks(c->n_envs, 256), 256, 0, c->stream>>>(c->hands, c->n_envs, out);
  NFSP_LAUNCHED("k_env_round");
  return NFSP_OK;
}

extern "C" int nfsp_env_export(nfsp_ctx* c, void* out) {
  NFSP_REQUIRE(c && out, "null argument");
  NFSP_HIP(hipMemcpyAsync(out, c->hands, sizeof(Hand) * (size_t)c->n_envs,
                          hipMemcpyDeviceToDevice, c->stream));
  return NFSP_OK;
}

// ---------------------------------------------------------------------------
// memories: row copies between record tables (one lane per 4-byte word)
// ---------------------------------------------------------------------------
// Row layout of one record seen as 65 words: s[30] a[3] r s2[30] t.  `scatter` selects
// insert (dst row = idx[i]) vs sample (src row = idx[i]).
__global__ void k_rows_copy(nfsp_records dst, nfsp_records src, const int64_t* __restrict__ idx,
                            int64_t n, int scatter) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int W = 65;
  if (e >= n * W) return;
  const int64_t i = e / W;
  const int w = (int)(e - i * W);
  const int64_t j = idx[i];
  const int64_t di = scatter ? j : i;
  const int64_t si = scatter ? i : j;
  if (w < 30) {
    if (dst.s && src.s) dst.s[di * 30 + w] = src.s[si * 30 + w];
  } else if (w < 33) {
    if (dst.a && src.a) dst.a[di * 3 + (w - 30)] = src.a[si * 3 + (w - 30)];
  } else if (w == 33) {
    if (dst.r && src.r) dst.r[di] = src.r[si];
  } else if (w < 64) {
    if (dst.s2 && src.s2) dst.s2[di * 30 + (w - 34)] = src.s2[si * 30 + (w - 34)];
  } else {
    if (dst.t && src.t) dst.t[di] = src.t[si];
  }
}

// Duplicate destination slots in one insert batch: the reference applies adds one at a
// time, so the LAST record aimed at a slot must win.  Mark the earlier ones dead first.
__global__ void k_last_writer(const int64_t* __restrict__ slots, int64_t n, int64_t* __restrict__ live) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = slots[i];
  int64_t out = s;
  for (int64_t k = i + 1; k < n; ++k)
    if (slots[k] == s) { out = -1; break; }
  live[i] = out;
}

__global__ void k_rows_insert_live(nfsp_records dst, nfsp_records src, const int64_t* __restrict__ live,
                                   int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int W = 65;
  if (e >= n * W) return;
  const int64_t i = e / W;
  const int64_t di = live[i];
  if (di < 0) return;
  const int w = (int)(e - i * W);
  if (w < 30) {
    if (dst.s && src.s) dst.s[di * 30 + w] = src.s[i * 30 + w];
  } else if (w < 33) {
    if (dst.a && src.a) dst.a[di * 3 + (w - 30)] = src.a[i * 3 + (w - 30)];
  } else if (w == 33) {
    if (dst.r && src.r) dst.r[di] = src.r[i];
  } else if (w < 64) {
    if (dst.s2 && src.s2) dst.s2[di * 30 + (w - 34)] = src.s2[i * 30 + (w - 34)];
  } else {
    if (dst.t && src.t) dst.t[di] = src.t[i];
  }
}

extern "C" int nfsp_buf_insert(nfsp_ctx* c, const nfsp_records* dst, const nfsp_records* src,
                               const int64_t* slots, int64_t n) {
  NFSP_REQUIRE(c && dst && src && slots, "null argument");
  NFSP_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return NFSP_OK;
  if (n <= 4096) {
    // small batches (the drop-in's per-call adds): resolve duplicates on device, no host sync
    if (c->scratch_i64_cap < n) {
      NFSP_HIP(hipStreamSynchronize(c->stream));
      if (c->scratch_i64) NFSP_HIP(hipFree(c->scratch_i64));
      c->scratch_i64 = nullptr;
      c->scratch_i64_cap = 0;
      NFSP_HIP(hipMalloc(&c->scratch_i64, sizeof(int64_t) * 4096));
      c->scratch_i64_cap = 4096;
    }
    int64_t* live = c->scratch_i64;
    k_last_writer<<<nfsp_blocks(n, 256), 256, 0, c->stream>>>(slots, n, live);
    NFSP_LAUNCHED("k_last_writer");
    k_rows_insert_live<<<nfsp_blocks(n * 65, 256), 256, 0, c->stream>>>(*dst, *src, live, n);
    NFSP_LAUNCHED("k_rows_insert_live");
  } else {
    // large batches: caller guarantees distinct slots (FIFO ring segments)
    k_rows_copy<<<nfsp_blocks(n * 65, 256), 256, 0, c->stream>>>(*dst, *src, slots, n, 1);
    NFSP_LAUNCHED("k_rows_copy(insert)");
  }
  return NFSP_OK;
}

extern "C" int nfsp_buf_sample(nfsp_ctx* c, const nfsp_records* src, const int64_t* idx, int64_t k,
                               const nfsp_records* dst) {
  NFSP_REQUIRE(c && dst && src && idx, "null argument");
  NFSP_REQUIRE(k >= 0, "k < 0");
  if (k == 0) return NFSP_OK;
  k_rows_copy<<<nfsp_blocks(k * 65, 256), 256, 0, c->stream>>>(*dst, *src, idx, k, 0);
  NFSP_LAUNCHED("k_rows_copy(sample)");
  return NFSP_OK;
}
