// The BR chain with a linear Q head (k_chain3<2, *>, chain3.h), used only under the
// textbook-NFSP extension NFSP_EXT_LINEAR_Q.  Its own translation unit, so the reference
// BR chain in learner.hip keeps its code and placement; built with learner.hip's flags
// (__graft_entry__.FILE_FLAGS).
#include "chain3.h"

namespace nfsp {
namespace chain {

int launch_chain_br_linear(const ChainArgs& C, int blocks, bool loss_log, bool mse, hipStream_t s) {
  static std::atomic<uint64_t> attr{0}, attr_mse{0};
  if (mse) return launch_chain<3>(C, blocks, loss_log, s, attr_mse);   // NFSP_EXT_MSE_Q
  return launch_chain<2>(C, blocks, loss_log, s, attr);
}

}  // namespace chain
}  // namespace nfsp
