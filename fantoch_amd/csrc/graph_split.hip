// graph_split.hip — FX_TIER_SPLIT: each 64-stream tile runs on the executor
// layout that suits its dependency density, both layouts concurrently.
//
// The per-stream work of GraphExecutor::handle (fantoch_ps/src/executor/graph/
// mod.rs:213-642) grows with the number of deps per Add: at low conflict rates
// an Add has ~1 dep (its own client's previous command), almost never waits,
// and one lane per stream (k_graph_lane, tier 5: independent lane progress, 64
// streams per wavefront) is fastest; at high conflict rates every Add depends
// on every process's latest command, the Tarjan / check_pending slow path
// dominates, and the lockstep maximum over 64 lanes makes tier 5 lose to the
// 16-lanes-per-stream group layout (k_graph_group, tier 0).  Both tiers produce
// the oracle's output bit for bit, so the choice is purely a schedule:
//   1. k_split_score: one wavefront per tile reads the header plane of the
//      first SPLIT_SAMPLE_STEPS steps and quantises the tile's mean deps per
//      Add to a bucket (deps x 8, 0..63);
//   2. k_split_plan: one workgroup lists the tiles by descending bucket
//      (heaviest first, so the longest chains start first) into a heavy map
//      (bucket >= threshold, group tier) and a light map (lane tier), 64
//      entries per tile (padding lanes of a ragged last tile get a sentinel
//      stream index >= S and stay idle), and writes both lane counts;
//   3. the lane kernel (light map) goes on an auxiliary HIP stream and the
//      group kernel (heavy map) on the caller's stream, forked and joined with
//      events; both grids cover every tile and read their lane count from
//      device memory, so nothing returns to the host in between.
// Map entries of a tile stay contiguous and in order, so a wavefront's loads
// are the same 1 KiB tile loads as an unmapped launch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace split {

constexpr uint32_t NB = 64;                  // score buckets (mean deps x 8)
constexpr uint32_t SAMPLE_BLOCKS = 64;       // 4-step blocks sampled per tile
constexpr uint32_t PLAN_THREADS = 1024;
constexpr uint32_t SENTINEL = 0xFFFFFFFFu;

__global__ __launch_bounds__(64) void k_split_score(const uint32_t* __restrict__ hdr,
                                                    const uint32_t* __restrict__ lengths, uint32_t S,
                                                    uint32_t steps, uint32_t* __restrict__ score) {
  const uint32_t t = blockIdx.x, l = threadIdx.x;
  const uint32_t s = t * 64 + l;
  const uint32_t steps4 = (steps + 3) >> 2;
  const uint32_t nb = min(steps4, SAMPLE_BLOCKS);
  uint32_t len = s < S ? (lengths ? min(lengths[s], steps) : steps) : 0u;
  len = min(len, nb * 4);
  uint32_t nd = 0;
  const uint32_t* p = hdr + (size_t)t * steps4 * 256 + l * 4;
  for (uint32_t b = 0; b < nb; ++b) {
    const uint4 h = *reinterpret_cast<const uint4*>(p + (size_t)b * 256);
    const uint32_t i = b * 4;
    nd += (i + 0 < len ? (h.x >> 24) & 31u : 0u) + (i + 1 < len ? (h.y >> 24) & 31u : 0u) +
          (i + 2 < len ? (h.z >> 24) & 31u : 0u) + (i + 3 < len ? (h.w >> 24) & 31u : 0u);
  }
  uint32_t cnt = len;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    nd += (uint32_t)__shfl_xor((int)nd, (int)o, 64);
    cnt += (uint32_t)__shfl_xor((int)cnt, (int)o, 64);
  }
  if (l == 0) score[t] = min((nd * 8u) / max(cnt, 1u), NB - 1);
}

// One workgroup: stable counting sort of the tiles by descending bucket.
__global__ __launch_bounds__(PLAN_THREADS) void k_split_plan(const uint32_t* __restrict__ score,
                                                             uint32_t tiles, uint32_t S, uint32_t thr,
                                                             uint32_t* __restrict__ heavy,
                                                             uint32_t* __restrict__ light,
                                                             uint32_t* __restrict__ counts) {
  __shared__ uint32_t wsum[PLAN_THREADS / 64];
  const uint32_t tid = threadIdx.x, w = tid >> 6, l = tid & 63u;
  uint32_t nh = 0, nl = 0;  // tiles placed so far (block-uniform)
  for (int b = NB - 1; b >= 0; --b) {
    const bool hv = (uint32_t)b >= thr;
    uint32_t* map = hv ? heavy : light;
    for (uint32_t c0 = 0; c0 < tiles; c0 += PLAN_THREADS) {
      const uint32_t t = c0 + tid;
      const bool f = t < tiles && score[t] == (uint32_t)b;
      const uint64_t m = __ballot(f);
      const uint32_t below = __popcll(m & ((1ull << l) - 1ull));
      if (l == 0) wsum[w] = __popcll(m);
      __syncthreads();
      uint32_t off = 0, tot = 0;
      for (uint32_t q = 0; q < PLAN_THREADS / 64; ++q) {
        off += q < w ? wsum[q] : 0u;
        tot += wsum[q];
      }
      if (f) {
        const uint32_t pos = (hv ? nh : nl) + off + below;
        uint32_t* e = map + (size_t)pos * 64;
        for (uint32_t i = 0; i < 64; ++i) {
          const uint32_t s = t * 64 + i;
          e[i] = s < S ? s : SENTINEL;
        }
      }
      if (hv) nh += tot; else nl += tot;
      __syncthreads();
    }
  }
  if (tid == 0) {
    counts[0] = nh * 64;
    counts[1] = nl * 64;
  }
}

static hipStream_t g_aux = nullptr;
static hipEvent_t g_fork = nullptr, g_join = nullptr;

static uint32_t threshold() {
  static int thr = -1;
  if (thr < 0) {
    const char* e = getenv("FX_SPLIT_THRESHOLD");  // tuning knob: bucket = mean deps x 8
    thr = e ? atoi(e) : (int)SPLIT_DEFAULT_THRESHOLD;
    if (thr < 0) thr = 0;
  }
  return (uint32_t)thr;
}

}  // namespace split

size_t split_scratch_bytes(uint32_t streams) {
  const size_t tiles = (streams + 63) / 64;
  return (tiles + 2 * tiles * 64 + 4) * 4;
}

int launch_split(const KArgs& a0, void* scratch, hipStream_t hs) {
  using namespace split;
  const uint32_t S = a0.S;
  const uint32_t tiles = (S + 63) / 64;
  if (tiles == 0) return FX_OK;
  if (a0.dmax > GROUP_LANES) return FX_ERR_INVALID_ARG;
  uint32_t* score = (uint32_t*)scratch;
  uint32_t* heavy = score + tiles;
  uint32_t* light = heavy + (size_t)tiles * 64;
  uint32_t* counts = light + (size_t)tiles * 64;
  // the lane tier holds n <= 8 sources and <= LANE_MAX_DEPS deps and reads
  // planes of < 4 GiB: otherwise every tile is heavy
  const bool lane_ok = a0.n <= 8 && a0.dmax <= LANE_MAX_DEPS && a0.plane * 4 <= LANE_MAX_PLANE_BYTES;
  const uint32_t thr = lane_ok ? threshold() : 0u;
  if (!g_aux) {
    if (hipStreamCreateWithFlags(&g_aux, hipStreamNonBlocking) != hipSuccess) return FX_ERR_HIP;
    if (hipEventCreateWithFlags(&g_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g_join, hipEventDisableTiming) != hipSuccess)
      return FX_ERR_HIP;
  }
  hipLaunchKernelGGL(k_split_score, dim3(tiles), dim3(64), 0, hs, a0.hdr, a0.lengths, S, a0.steps, score);
  hipLaunchKernelGGL(k_split_plan, dim3(1), dim3(PLAN_THREADS), 0, hs, score, tiles, S, thr, heavy, light,
                     counts);
  if (hipGetLastError() != hipSuccess) return FX_ERR_HIP;
  KArgs h = a0, lt = a0;
  h.stream_map = heavy;
  h.num_lanes = tiles * 64;
  h.lanes_dev = counts + 0;
  lt.stream_map = light;
  lt.num_lanes = tiles * 64;
  lt.lanes_dev = counts + 1;
  int st = FX_OK;
  if (thr < NB) {
    if (hipEventRecord(g_fork, hs) != hipSuccess || hipStreamWaitEvent(g_aux, g_fork, 0) != hipSuccess)
      return FX_ERR_HIP;
    if (thr > 0) {
      split_profile_record(2, false, g_aux);
      st = launch_lane(lt, g_aux);
      split_profile_record(2, true, g_aux);
    }
    split_profile_record(1, false, hs);
    const int st2 = launch_group(h, hs);
    split_profile_record(1, true, hs);
    if (hipEventRecord(g_join, g_aux) != hipSuccess || hipStreamWaitEvent(hs, g_join, 0) != hipSuccess)
      return FX_ERR_HIP;
    if (st2) return st2;
  } else {
    st = launch_lane(lt, hs);
  }
  return st;
}

}  // namespace fx
