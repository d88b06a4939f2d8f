// Host-side internals shared by the libnfsp translation units: the ctx object and
// the error plumbing behind nfsp_last_error().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "nfsp.h"
#include "nfsp_device.h"

struct nfsp_ctx {
  int n_envs = 0;
  int device = 0;
  int game = NFSP_GAME_LEDUC;
  uint64_t seed = 0;
  hipStream_t stream = nullptr;
  nfsp::Hand* hands = nullptr;        // [n_envs]
  uint8_t* pending_deal = nullptr;    // [n_envs*3]
  bool has_pending_deal = false;
  uint64_t resets = 0;                // reset index (Philox counter word)
  double* scratch_f64 = nullptr;      // small device scratch
  int64_t* scratch_i64 = nullptr;     // insert de-duplication scratch
  int64_t scratch_i64_cap = 0;
  void* deal_mt = nullptr;            // nfsp_env_set_deal_mode's MT19937 state (deal_mt.hip)
};

namespace nfsp {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);
int deal_mt_stage(nfsp_ctx* c);       // MT deal modes: the next reset's deals -> pending_deal
void deal_mt_free(nfsp_ctx* c);

}  // namespace nfsp

#define NFSP_HIP(expr)                                         \
  do {                                                         \
    hipError_t _e = (expr);                                    \
    if (_e != hipSuccess) return nfsp::hip_fail(_e, #expr);    \
  } while (0)

#define NFSP_LAUNCHED(what)                                    \
  do {                                                         \
    hipError_t _e = hipGetLastError();                         \
    if (_e != hipSuccess) return nfsp::hip_fail(_e, what);     \
  } while (0)

#define NFSP_REQUIRE(cond, msg)                                \
  do {                                                         \
    if (!(cond)) return nfsp::fail(NFSP_EINVAL, msg);          \
  } while (0)

inline unsigned nfsp_blocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }
