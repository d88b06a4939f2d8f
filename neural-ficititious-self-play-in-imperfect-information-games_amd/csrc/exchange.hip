// The cross-shard exchange of the average-policy nets (BASELINE C4; the C ABI
// and its arithmetic: include/nfsp.h nfsp_engine_set_exchange).
//
// Each shard (one engine per GPU) trains its own copy of both agents' AR nets
// (agent/agent.py:255-264 at the reference cadence).  At the end of every `every`-th learner
// call the shards' gradient steps since the last exchange are summed and applied to the common
// base, right behind the call's AR chain on the AR chain stream:
//   k_xchg_delta   D = W_AR - W0
//   transport      S = sum over shards of D: ncclAllReduce on the same stream (RCCL over xGMI,
//                  stream-ordered: no host round trip), or a host callback (gloo rehearsals)
//   k_xchg_apply   W_AR = W0 + S * scale, W0 = W_AR
// 2 x 2,179 f32 = 17.4 KB per exchange; with 16 slices per C3 step and every = 1 that is 16
// collectives per ~165 ms step.  The arithmetic is learner.hip k_group_xchg's (contract off,
// S summed from +0), so 2 shards equal a 2-replica engine group bit for bit.
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>

#include <rccl/rccl.h>

#include "engine_internal.h"

namespace nn = nfsp::nn;
using namespace nfsp::eng;

namespace {

// the AR net of agent a sits at e->w + (3a + 0) NP; the exchange buffers are [2][NP]
__global__ void __launch_bounds__(256) k_xchg_delta(const float* __restrict__ w, const float* __restrict__ w0,
                                                    float* __restrict__ d) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * nn::NP) return;
  const int a = i / nn::NP, q = i - a * nn::NP;
  d[i] = w[(a * 3) * nn::NP + q] - w0[i];
}

__global__ void __launch_bounds__(256) k_xchg_apply(float* __restrict__ w, float* __restrict__ w0,
                                                    const float* __restrict__ s, float scale) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * nn::NP) return;
  const int a = i / nn::NP, q = i - a * nn::NP;
  // 0.f + S: the group kernel's sum starts from +0 (turns a -0 sum of one shard into +0)
  const float nw = w0[i] + (0.f + s[i]) * scale;
  w0[i] = nw;
  w[(a * 3) * nn::NP + q] = nw;
}

__global__ void __launch_bounds__(256) k_xchg_base(const float* __restrict__ w, float* __restrict__ w0) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * nn::NP) return;
  const int a = i / nn::NP, q = i - a * nn::NP;
  w0[i] = w[(a * 3) * nn::NP + q];
}

// RCCL, loaded on first use (a process that never exchanges never loads it)
struct Rccl {
  bool tried = false;
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};
Rccl g_rccl;
std::mutex g_rccl_mu;

int rccl_load() {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!g_rccl.tried) {
    g_rccl.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (h) {
      g_rccl.get_unique_id = reinterpret_cast<decltype(g_rccl.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
      g_rccl.comm_init_rank = reinterpret_cast<decltype(g_rccl.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
      g_rccl.comm_destroy = reinterpret_cast<decltype(g_rccl.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
      g_rccl.all_reduce = reinterpret_cast<decltype(g_rccl.all_reduce)>(dlsym(h, "ncclAllReduce"));
      g_rccl.error_string = reinterpret_cast<decltype(g_rccl.error_string)>(dlsym(h, "ncclGetErrorString"));
      if (g_rccl.get_unique_id && g_rccl.comm_init_rank && g_rccl.comm_destroy && g_rccl.all_reduce &&
          g_rccl.error_string)
        g_rccl.h = h;
    }
  }
  if (!g_rccl.h) return nfsp::fail(NFSP_EINVAL, "RCCL (librccl.so.1) could not be loaded");
  return NFSP_OK;
}

int rccl_fail(ncclResult_t r, const char* what) {
  return nfsp::fail(NFSP_EHIP, std::string(what) + ": " + g_rccl.error_string(r));
}

}  // namespace

namespace nfsp {
namespace eng {
int exchange_enqueue(nfsp_engine* e, hipStream_t s) {
  NFSP_REQUIRE(e->xchg_comm || e->xchg_fn, "the exchange has no transport");
  const unsigned nb = nfsp_blocks(2 * nn::NP, 256);
  k_xchg_delta<<<nb, 256, 0, s>>>(e->w, e->xchg_w0, e->xchg_buf);
  NFSP_LAUNCHED("k_xchg_delta");
  if (e->xchg_comm) {
    const ncclResult_t r = g_rccl.all_reduce(e->xchg_buf, e->xchg_buf, 2 * nn::NP, ncclFloat32, ncclSum,
                                             static_cast<ncclComm_t>(e->xchg_comm), s);
    if (r != ncclSuccess) return rccl_fail(r, "ncclAllReduce (AR exchange)");
  } else {
    NFSP_HIP(hipStreamSynchronize(s));
    const int rc = e->xchg_fn(e->xchg_user, e->xchg_buf, 2 * nn::NP);
    if (rc != 0) return nfsp::fail(NFSP_EINVAL, "the exchange callback failed (rc " + std::to_string(rc) + ")");
  }
  k_xchg_apply<<<nb, 256, 0, s>>>(e->w, e->xchg_w0, e->xchg_buf, e->xchg_scale);
  NFSP_LAUNCHED("k_xchg_apply");
  e->xchg_done++;
  return NFSP_OK;
}
}  // namespace eng
}  // namespace nfsp

extern "C" int nfsp_engine_set_exchange(nfsp_engine* e, int every, float scale, void* rccl_comm,
                                        nfsp_exchange_fn fn, void* user) {
  NFSP_REQUIRE(e, "null argument");
  NFSP_REQUIRE(e->s_ar, "a replica of an engine group exchanges through nfsp_group_set_exchange");
  NFSP_REQUIRE(every >= 0, "every must be >= 0");
  NFSP_REQUIRE(every == 0 || ((rccl_comm != nullptr) != (fn != nullptr)),
               "exactly one transport: an RCCL communicator or a host callback");
  NFSP_REQUIRE(!e->pending_update && !e->xchg_pending,
               "set the exchange between steps (a rollout or an exchange is pending)");
  if (every > 0 && !e->xchg_w0) {
    for (float** p : {&e->xchg_w0, &e->xchg_buf}) {
      NFSP_HIP(hipMalloc((void**)p, sizeof(float) * 2 * nn::NP));
      e->allocs.push_back(*p);
    }
  }
  e->xchg_every = every;
  e->xchg_scale = scale;
  e->xchg_comm = every ? rccl_comm : nullptr;
  e->xchg_fn = every ? fn : nullptr;
  e->xchg_user = user;
  e->xchg_calls = 0;
  if (every > 0) {     // W0 = the AR nets as they are (after every stream of the last step)
    for (hipStream_t st : {e->s_ar, e->s_br[0], e->s_br[1]}) NFSP_HIP(hipStreamSynchronize(st));
    k_xchg_base<<<nfsp_blocks(2 * nn::NP, 256), 256, 0, e->ctx->stream>>>(e->w, e->xchg_w0);
    NFSP_LAUNCHED("k_xchg_base");
    NFSP_HIP(hipStreamSynchronize(e->ctx->stream));
  }
  return NFSP_OK;
}

extern "C" int nfsp_engine_exchanges(nfsp_engine* e, int64_t* out) {
  NFSP_REQUIRE(e && out, "null argument");
  *out = e->xchg_done;
  return NFSP_OK;
}

extern "C" int nfsp_rccl_ready(int device) {
  int rc = rccl_load();
  if (rc != NFSP_OK) return rc;
  int n = 0;
  NFSP_HIP(hipGetDeviceCount(&n));
  NFSP_REQUIRE(device >= 0 && device < n, "no such HIP device");
  NFSP_HIP(hipSetDevice(device));
  return NFSP_OK;
}

extern "C" int nfsp_rccl_unique_id(uint8_t* out) {
  NFSP_REQUIRE(out, "null argument");
  int rc = rccl_load();
  if (rc != NFSP_OK) return rc;
  ncclUniqueId id;
  const ncclResult_t r = g_rccl.get_unique_id(&id);
  if (r != ncclSuccess) return rccl_fail(r, "ncclGetUniqueId");
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return NFSP_OK;
}

extern "C" int nfsp_rccl_comm_create(const uint8_t* id, int world, int rank, int device, void** comm) {
  NFSP_REQUIRE(id && comm && world >= 1 && rank >= 0 && rank < world, "bad argument");
  int rc = rccl_load();
  if (rc != NFSP_OK) return rc;
  NFSP_HIP(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = g_rccl.comm_init_rank(&c, world, u, rank);
  if (r != ncclSuccess) return rccl_fail(r, "ncclCommInitRank");
  *comm = c;
  return NFSP_OK;
}

extern "C" int nfsp_rccl_comm_destroy(void* comm) {
  if (!comm) return NFSP_OK;
  int rc = rccl_load();
  if (rc != NFSP_OK) return rc;
  const ncclResult_t r = g_rccl.comm_destroy(static_cast<ncclComm_t>(comm));
  if (r != ncclSuccess) return rccl_fail(r, "ncclCommDestroy");
  return NFSP_OK;
}
