// config.cpp — quorum sizes of the commit-stream producers (SURVEY.md §8(a)
// row a14: the deps of an Atlas / EPaxos commit are the union over a fast
// quorum, so d <= fast quorum size).  Restates fantoch/src/config.rs:294-312.
#include "fantoch_amd.h"

extern "C" int fx_quorum_sizes(uint32_t protocol, uint32_t n, uint32_t f, uint32_t* fast_quorum,
                               uint32_t* write_quorum) {
  if (!fast_quorum || !write_quorum || n == 0) return FX_ERR_INVALID_ARG;
  switch (protocol) {
    case FX_PROTOCOL_ATLAS:  // Config::atlas_quorum_sizes (config.rs:294-301)
      if (f > n / 2) return FX_ERR_INVALID_ARG;
      *fast_quorum = n / 2 + f;
      *write_quorum = f + 1;
      return FX_OK;
    case FX_PROTOCOL_EPAXOS: {  // Config::epaxos_quorum_sizes (config.rs:303-312): f ignored
      const uint32_t fe = n / 2;
      *fast_quorum = fe + (fe + 1) / 2;
      *write_quorum = fe + 1;
      return FX_OK;
    }
    default:
      return FX_ERR_INVALID_ARG;
  }
}
