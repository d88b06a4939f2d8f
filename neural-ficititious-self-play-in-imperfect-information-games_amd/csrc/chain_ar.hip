// The AR chain's instantiation of k_chain3 (chain3.h), in its own translation unit.  The
// BR instantiation is in learner.hip.  The two are compiled with different scheduler flags
// (__graft_entry__.FILE_FLAGS): the AMDGPU register-pressure trackers speed the BR chain
// and slow this one.  Reference: agent/agent.py:255-264 (update_avg_response_network).
#include "chain3.h"

namespace nfsp {
namespace chain {

int launch_chain_ar(const ChainArgs& C, int blocks, bool loss_log, hipStream_t s) {
  static std::atomic<uint64_t> attr{0};
  const int rc = set_chain_lds(attr, (const void*)k_chain3<0, 0>, (const void*)k_chain3<0, 1>);
  if (rc != NFSP_OK) return rc;
  if (loss_log) k_chain3<0, 1><<<blocks, 256, CHAIN_LDS, s>>>(C);
  else k_chain3<0, 0><<<blocks, 256, CHAIN_LDS, s>>>(C);
  NFSP_LAUNCHED("k_chain(AR)");
  return NFSP_OK;
}

}  // namespace chain
}  // namespace nfsp
