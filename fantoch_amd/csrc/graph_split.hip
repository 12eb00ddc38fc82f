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
//   2. k_plan_*: a grid-wide stable counting sort lists the tiles by
//      descending bucket (heaviest first, so the longest chains start first)
//      into a heavy map
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

// Stable counting sort of the tiles by descending bucket (heavy map: buckets
// >= thr, light map: the rest), in four grid-wide passes:
//   k_plan_count  per block of PB tiles, a histogram of its buckets;
//   k_plan_scan   one workgroup: each (bucket, block)'s first position in its
//                 map (buckets descending, blocks ascending) and both counts;
//   k_plan_place  each tile's position = its (bucket, block) offset + its rank
//                 among the block's tiles of that bucket; inv[pos] = tile;
//   k_plan_fill   one thread per map entry: stream = inv[entry / 64] * 64 + i.
// The order is the one-workgroup sort's (bucket descending, tile ascending).
constexpr uint32_t PB = 256;  // tiles per block of the plan passes

__global__ __launch_bounds__(PB) void k_plan_count(const uint32_t* __restrict__ score, uint32_t tiles,
                                                   uint32_t nblk, uint32_t* __restrict__ bh) {
  __shared__ uint32_t h[NB];
  const uint32_t tid = threadIdx.x, blk = blockIdx.x;
  if (tid < NB) h[tid] = 0;
  __syncthreads();
  const uint32_t t = blk * PB + tid;
  if (t < tiles) atomicAdd(&h[score[t]], 1u);
  __syncthreads();
  if (tid < NB) bh[tid * nblk + blk] = h[tid];
}

__global__ __launch_bounds__(1024) void k_plan_scan(uint32_t* __restrict__ bh, uint32_t nblk, uint32_t thr,
                                                    uint32_t* __restrict__ counts) {
  // bh[b * nblk + k] -> exclusive offset in map(b) in the order (b desc, k asc)
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry[2];
  const uint32_t tid = threadIdx.x, l = tid & 63u, w = tid >> 6;
  if (tid < 2) carry[tid] = 0;
  __syncthreads();
  for (int b = NB - 1; b >= 0; --b) {
    const uint32_t side = (uint32_t)b >= thr ? 0u : 1u;
    for (uint32_t k0 = 0; k0 < nblk; k0 += 1024) {
      const uint32_t k = k0 + tid;
      const uint32_t v = k < nblk ? bh[(uint32_t)b * nblk + k] : 0u;
      uint32_t x = v;  // inclusive scan within the wavefront
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (l >= o) x += y;
      }
      if (l == 63) wsum[w] = x;
      __syncthreads();
      uint32_t before = 0, tot = 0;
      for (uint32_t q = 0; q < 16; ++q) {
        before += q < w ? wsum[q] : 0u;
        tot += wsum[q];
      }
      const uint32_t c = carry[side];
      if (k < nblk) bh[(uint32_t)b * nblk + k] = c + before + x - v;
      __syncthreads();
      if (tid == 0) carry[side] = c + tot;
      __syncthreads();
    }
  }
  if (tid == 0) {
    counts[0] = carry[0] * 64;
    counts[1] = carry[1] * 64;
  }
}

__global__ __launch_bounds__(PB) void k_plan_place(const uint32_t* __restrict__ score, uint32_t tiles,
                                                   uint32_t nblk, uint32_t thr, const uint32_t* __restrict__ bh,
                                                   uint32_t* __restrict__ inv_heavy,
                                                   uint32_t* __restrict__ inv_light) {
  __shared__ uint32_t sc[PB];
  const uint32_t tid = threadIdx.x, blk = blockIdx.x;
  const uint32_t t = blk * PB + tid;
  sc[tid] = t < tiles ? score[t] : 0xFFFFFFFFu;
  __syncthreads();
  if (t >= tiles) return;
  const uint32_t b = sc[tid];
  uint32_t r = 0;
  for (uint32_t q = 0; q < tid; ++q) r += sc[q] == b ? 1u : 0u;
  const uint32_t pos = bh[b * nblk + blk] + r;
  (b >= thr ? inv_heavy : inv_light)[pos] = t;
}

__global__ __launch_bounds__(256) void k_plan_fill(const uint32_t* __restrict__ inv, const uint32_t* __restrict__ counts,
                                                   uint32_t which, uint32_t entries, uint32_t S,
                                                   uint32_t* __restrict__ map) {
  const uint32_t e = blockIdx.x * 256 + threadIdx.x;
  if (e >= entries || e >= counts[which]) return;
  const uint32_t s = inv[e >> 6] * 64 + (e & 63u);
  map[e] = s < S ? s : SENTINEL;
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
  using namespace split;
  const size_t tiles = (streams + 63) / 64, nblk = (tiles + PB - 1) / PB;
  // score, heavy / light maps, counts, per-(bucket, block) offsets, inverse maps
  return (tiles + 2 * tiles * 64 + 4 + NB * nblk + 2 * tiles) * 4;
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
  const uint32_t nblk = (tiles + PB - 1) / PB;
  uint32_t* bh = counts + 4;
  uint32_t* inv_heavy = bh + (size_t)NB * nblk;
  uint32_t* inv_light = inv_heavy + tiles;
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
  hipLaunchKernelGGL(k_plan_count, dim3(nblk), dim3(PB), 0, hs, score, tiles, nblk, bh);
  hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, hs, bh, nblk, thr, counts);
  hipLaunchKernelGGL(k_plan_place, dim3(nblk), dim3(PB), 0, hs, score, tiles, nblk, thr, bh, inv_heavy, inv_light);
  const uint32_t entries = tiles * 64;
  hipLaunchKernelGGL(k_plan_fill, dim3((entries + 255) / 256), dim3(256), 0, hs, inv_heavy, counts, 0u, entries, S,
                     heavy);
  hipLaunchKernelGGL(k_plan_fill, dim3((entries + 255) / 256), dim3(256), 0, hs, inv_light, counts, 1u, entries, S,
                     light);
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
