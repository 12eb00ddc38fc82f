// fx_internal.h — declarations shared between the kernel TU and the host TU.
#pragma once
#include <stdint.h>

namespace fx {
// Decodes the pending vertices of lane `lane` from a saved state block
// (tier layout of graph_exec.hip).  Writes up to cap (dot, waiting_on) pairs;
// returns the count.
uint32_t decode_pending(uint32_t tier, const uint32_t* block, uint32_t lane, uint32_t* dots,
                        uint32_t* waits, uint32_t cap);
}  // namespace fx
