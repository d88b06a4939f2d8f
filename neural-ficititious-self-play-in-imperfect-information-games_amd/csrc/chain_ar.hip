// The AR chain's instantiation of k_chain3 (chain3.h), in its own translation unit.  The
// BR instantiation is in learner.hip.  The two are compiled with different scheduler flags
// (__graft_entry__.FILE_FLAGS): the AMDGPU register-pressure trackers speed the BR chain
// and slow this one.  Reference: agent/agent.py:255-264 (update_avg_response_network).
#include "chain3.h"

namespace nfsp {
namespace chain {

int launch_chain_ar(const ChainArgs& C, int blocks, bool loss_log, hipStream_t s) {
  static std::atomic<uint64_t> attr{0};
  return launch_chain<0>(C, blocks, loss_log, s, attr);
}

}  // namespace chain
}  // namespace nfsp
