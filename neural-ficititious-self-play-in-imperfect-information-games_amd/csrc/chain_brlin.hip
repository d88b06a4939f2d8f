// The BR chain with a linear Q head (k_chain3<2, *>, chain3.h), used only under the
// textbook-NFSP extension NFSP_EXT_LINEAR_Q.  Its own translation unit, so the reference
// BR chain in learner.hip keeps its code and placement; built with learner.hip's flags
// (__graft_entry__.FILE_FLAGS).
#include "chain3.h"

namespace nfsp {
namespace chain {

int launch_chain_br_linear(const ChainArgs& C, bool loss_log, hipStream_t s) {
  static std::atomic<uint64_t> attr{0};
  const int rc = set_chain_lds(attr, (const void*)k_chain3<2, 0>, (const void*)k_chain3<2, 1>);
  if (rc != NFSP_OK) return rc;
  if (loss_log) k_chain3<2, 1><<<1, 256, CHAIN_LDS, s>>>(C);
  else k_chain3<2, 0><<<1, 256, CHAIN_LDS, s>>>(C);
  NFSP_LAUNCHED("k_chain(BR, linear)");
  return NFSP_OK;
}

}  // namespace chain
}  // namespace nfsp
