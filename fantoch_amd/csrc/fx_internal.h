// fx_internal.h — declarations shared by the kernel and host translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>
#include <stddef.h>
#include <stdint.h>

namespace fx {

// Arguments of one executor launch (fx_batch_execute).
struct KArgs {
  const uint32_t* dot;
  const uint32_t* hdr;
  const uint32_t* deps;
  const uint32_t* lengths;
  uint32_t S, steps, dmax, n;
  size_t plane;
  uint32_t* order;
  uint32_t* release;
  uint32_t* nexec;
  uint32_t* err;
  const uint32_t* stream_map;
  uint32_t num_lanes;
  uint32_t* state;
  uint32_t step_begin, step_end, flags;
  const uint32_t* init_frontier;
  uint32_t* dbg;  // per-lane diagnostic counters (FX_LANE_DEBUG), normally null
  const uint32_t* lanes_dev;  // device lane count (FX_TIER_SPLIT sub-launches), normally null
  uint32_t drift;             // lane tier: max blocks (4 steps) a lane runs ahead of the slowest, 0 = unbounded
  // partial replication (FX_FLAG_PARTIAL, wide HBM tier): per lane a ring of
  // (step, parent dot) pairs, one per dep missing for the first time
  // (PendingIndex::index found no entry, index.rs:180-198): word 0 = count,
  // then req_cap pairs
  uint32_t* req;
  uint32_t req_cap;
};

// One workgroup per stream, streams read from the plane tiles (fx_index: 16
// bytes per stream and tile row, so 8 consecutive streams share a 128-byte
// line).  Hardware deals workgroups round-robin to the 8 XCDs, whose L2s are
// separate: with the identity mapping the 8 streams of a line run on 8 XCDs
// and each fetches the line.  A launch whose grid is a multiple of 64 maps
// workgroup 64g + 8i + x (XCD x) to stream slot 64g + 8x + i, so a line's
// streams share one L2; xcd_grid pads launches of >= 256 slots to that shape
// (slots >= the lane count exit at once).
__device__ __forceinline__ uint32_t xcd_slot(uint32_t b) {
  return (gridDim.x & 63u) ? b : (b & ~63u) | ((b & 7u) << 3) | ((b >> 3) & 7u);
}
inline uint32_t xcd_grid(uint32_t lanes) { return lanes >= 256u ? (lanes + 63u) & ~63u : lanes; }

// Lane-per-stream executor tiers (graph_exec.hip) and the 16-lanes-per-stream
// group tier (graph_group.hip).
int launch_group(const KArgs& a, hipStream_t stream);
size_t group_state_bytes(uint32_t streams);
uint32_t group_state_words_per_stream();
uint32_t group_decode_pending(const uint32_t* block, uint32_t stream_in_block, uint32_t* dots,
                              uint32_t* waits, uint32_t cap);
constexpr uint32_t GROUP_LANES = 16;        // lanes per stream in the group tier
constexpr uint32_t GROUP_SLOTS = 16;        // pending vertices per stream
constexpr uint32_t GROUP_CACHE = 8;         // cached deps per pending vertex
constexpr uint32_t GROUP_WINDOW_BITS = 32;  // executed-clock window per source

// Wavefront-per-stream tier (graph_wave.hip).
int launch_wave(const KArgs& a, hipStream_t stream);
size_t wave_state_bytes(uint32_t streams);
uint32_t wave_state_words_per_stream();
uint32_t wave_decode_pending(const uint32_t* block, uint32_t stream_in_launch, uint32_t* dots,
                             uint32_t* waits, uint32_t cap);
constexpr uint32_t WAVE_SLOTS = 64;        // pending vertices per stream (one per lane)
constexpr uint32_t WAVE_CACHE = 8;         // cached deps per pending vertex
constexpr uint32_t WAVE_WINDOW_BITS = 32;  // executed-clock window per source
constexpr uint32_t WAVE_MAX_DEPS = 14;     // dep planes read per Add

// Lane-per-stream tier with a register-resident slot table (graph_lane.hip).
int launch_lane(const KArgs& a, hipStream_t stream);
size_t lane_state_bytes(uint32_t streams);
uint32_t lane_state_words_per_stream();
uint32_t lane_decode_pending(const uint32_t* block, uint32_t lane, uint32_t* dots, uint32_t* waits,
                             uint32_t cap);
constexpr uint32_t LANE_SLOTS = 12;         // pending vertices per stream
constexpr uint32_t LANE_MAX_DEPS = 8;       // dep planes (and cached deps per vertex)
constexpr uint32_t LANE_WINDOW_BITS = 32;   // executed-clock window per source
constexpr size_t LANE_MAX_PLANE_BYTES = 0xFFFFFFF0u;  // input planes are read with 32-bit buffer offsets

// FX_TIER_SPLIT (graph_split.hip): per-tile choice between the group and the
// lane tier, both launched concurrently.
int launch_split(const KArgs& a, void* scratch, hipStream_t stream);
size_t split_scratch_bytes(uint32_t streams);
constexpr uint32_t SPLIT_DEFAULT_THRESHOLD = 16;  // mean deps per Add x 8 at or above which
                                                  // a tile runs on the group tier

// Per-kernel profiling of the split tier (fx_profile_last_kernel_ms): HIP
// events recorded on each kernel's own stream around its launch, so the
// dominant kernel's duration is measured where it runs.
bool profile_on();
void split_profile_record(int which, bool end, hipStream_t s);
// the drop-in handle's persistent executor kernel (graph_wave.hip, persist::)
struct PersistArgs {
  uint32_t* ctl;        // host-mapped control words (PERSIST_*)
  const uint32_t* rows; // host-mapped ring of published rows (persist::PRW words each)
  uint32_t* out;        // host-mapped ring of (order word, release step) pairs
  uint32_t* state;      // device: the wave tier's saved state of one stream
  uint32_t row_slots, out_slots;  // powers of two
  uint32_t n, at_commit, init, done0;
  // test hooks (fx_graph_executor_debug_hooks; 0 = off): the k-th flush of
  // this launch publishes no status, so the host's bounded wait must expire;
  // the kernel ignores the stop request and the idle exit until it has been
  // idle this many 100 MHz ticks (bounded: it still exits by itself), so the
  // host's stop request goes unanswered
  uint32_t debug_skip_status;
  uint32_t debug_hold_ticks;
};
constexpr uint32_t PERSIST_ROW_WORDS = 16;  // dot, hdr, 14 deps
constexpr uint32_t PERSIST_CTL_WORDS = 64;
constexpr uint32_t PERSIST_MB_DEPS = 12;    // deps a mailbox row carries (tag, dot, hdr, 12 deps, checksum)
constexpr uint32_t PERSIST_INLINE = 4;      // pairs a flush reports in the control words
// Control words, four 64-byte lines.  Line 0 host -> device: PUB (rows
// published), EXIT.  Line 1: the mailbox (tag, dot, hdr, 12 deps, a checksum of
// the other 15 words: persist_mb_sum).  Line 2
// device -> host: the status as two tagged 64-bit words {DONE, NEXEC | bit 31 on
// an error} and {DONE2, ERR}, the timing words, RUN.  Line 3: up to
// PERSIST_INLINE (order word, release step) pairs as tagged 64-bit words
// {tag, order} {tag, release}.  Every device -> host word is a system-scope
// store and the host checks the tags, so a flush with at most PERSIST_INLINE
// pairs needs no release fence; a larger one goes through the out ring and one
// fence before the status.
enum : uint32_t { PERSIST_PUB = 0, PERSIST_EXIT = 1, PERSIST_MB = 16, PERSIST_DONE = 32, PERSIST_NEXEC = 33,
                  PERSIST_DONE2 = 34, PERSIST_ERR = 35, PERSIST_TCOMP = 36, PERSIST_TFENCE = 37,
                  PERSIST_TPOLLS = 38, PERSIST_TRTT = 39, PERSIST_TCYC = 40, PERSIST_TITER = 41,
                  PERSIST_TSTEP = 42, PERSIST_TMB = 43, PERSIST_RUN = 47,
                  PERSIST_PAIRS = 48 };
constexpr uint32_t PERSIST_ERR_BIT = 0x80000000u;
int persist_launch(const PersistArgs& a, hipStream_t stream);
// The mailbox checksum: XOR over k of fmix32(word k ^ (k + 1) * golden) for
// the tag, dot, hdr and the 12 deps (k = 0..14).  The kernel reads the line with
// 32 independent 4-byte loads, which a host write can interleave with; a line
// whose words come from two different one-Add flushes fails this check (the
// tag is mixed in) and the kernel reads the row from the ring instead.
__host__ __device__ inline uint32_t persist_mb_mix(uint32_t w, uint32_t k) {
  uint32_t h = w ^ ((k + 1u) * 0x9E3779B9u);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
// fx_profile_slot_ms: events around one kernel slot's launch (graph_exec.hip)
void profile_slot_record(uint32_t slot, bool end, hipStream_t s);

// Single-stream gather used by the executor handle: out[k - k0] =
// release[rec(order[k])] for k in [k0, k1), so a flush reads back only the
// release steps of the commands it converts (bytes linear in the executed count).
// the drop-in handle's transfers (graph_exec.hip)
int scatter_rows(const uint32_t* stage, uint32_t nplanes, uint32_t r0, uint32_t rows, uint32_t cap, uint32_t* dot,
                 uint32_t* hdr, uint32_t* deps, hipStream_t stream);
int flush_pack(const uint32_t* order, const uint32_t* release, const uint32_t* nexec, const uint32_t* err,
               uint32_t cap, uint32_t k0, uint32_t* out, hipStream_t stream);
int gather_release(const uint32_t* order, const uint32_t* release, uint32_t steps, uint32_t k0,
                   uint32_t k1, uint32_t* out, hipStream_t stream);

// Decodes the pending vertices of lane `lane` from a saved state block
// (tier layout of graph_exec.hip).  Writes up to cap (dot, waiting_on) pairs;
// returns the count.
uint32_t decode_pending(uint32_t tier, const uint32_t* block, uint32_t lane, uint32_t* dots,
                        uint32_t* waits, uint32_t cap);

// Device scratch that persists across calls: slot `slot` grown to at least
// `bytes` (never shrunk; hipMalloc of multi-GB buffers per call costs more
// than the kernels of a configs[4] step).  NULL on allocation failure.
// Callers hold scratch_mutex() while they use their slots.
void* scratch(uint32_t slot, size_t bytes);
std::recursive_mutex& scratch_mutex();
enum : uint32_t {
  SCRATCH_TIERED_STATE = 0,
  SCRATCH_TIERED_MAP = 1,
  SCRATCH_TIERED_MAP2 = 2,
  SCRATCH_TIERED_CNT = 3,
  SCRATCH_CUT_FIRST = 4,
  SCRATCH_SLOTS = 40
};

// The wide tiers (graph_wide.hip): tables in LDS (whole streams) or HBM (also resumable).
int launch_wide(const KArgs& a, bool hbm, hipStream_t stream);
size_t wide_state_bytes(uint32_t tier, uint32_t n, uint32_t lanes);
bool wide_lds_fits(uint32_t n, uint32_t dmax);  // the LDS wide tier's tables fit a workgroup
// pending (dot, waiting_on) pairs of a saved HBM wide-tier table block (one
// stream); with partial replication one pair per (vertex, parent) registration
uint32_t wide_decode_pending(const uint32_t* block, uint32_t n, uint32_t* dots, uint32_t* waits, uint32_t cap,
                             bool partial = false);
size_t wide_partial_state_bytes(uint32_t n, uint32_t lanes);  // FX_FLAG_PARTIAL tables

// fx_batch_run_tiered over all streams (only == NULL) or the listed ones.
int run_tiered(const fx_stream_batch* in, const fx_order_batch* out, uint32_t flags, void* hip_stream,
               const std::vector<uint32_t>* only, uint32_t* tier_counts);
}  // namespace fx
