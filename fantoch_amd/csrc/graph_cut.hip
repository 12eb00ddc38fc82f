// graph_cut.hip — one huge commit stream as many independent ones
// (BASELINE configs[4]: a single instance whose executors each see 10^6 Adds).
//
// The reference's DependencyGraph (fantoch_ps/src/executor/graph/mod.rs:
// 213-642) is a sequential state machine: every handle_add sees the pending
// vertices, the pending index and the executed clock the previous Adds left.
// A stream still splits exactly at its *quiescent cuts*: step t is a cut when
// every dep of every Add at steps <= t was itself added at a step <= t (the
// prefix is dependency-closed).  Then every Add of the prefix has executed by
// the end of step t (a vertex runs as soon as its dependency closure is
// committed), so the state after step t is: no pending vertex, an empty
// pending index, and an executed clock holding exactly the prefix's dots.
// The segment after the cut therefore runs the same from an empty graph,
// provided that
//   * its deps on prefix dots are dropped (they are executed: find_scc skips
//     them, tarjan.rs:128-145),
//   * its dots are renumbered per source by rank inside the segment, which
//     keeps every comparison the executor makes (deps ascending C1, SCC members
//     ascending, waiters ascending C2 — all within one source's order or by
//     source first) and keeps the segment's executed clock compact.
// Every segment then is an ordinary stream of a batch (fx_batch_run_tiered),
// and its outputs map back by the segment's first step a: order rows and
// arrival indices shift by a (segment k's commands are the stream's rows
// [a, a + len), since each segment executes completely), release steps shift
// by a.
//
// Exactness does not rest on the argument above: a stream whose segments do
// not all execute completely, whose last step is not a cut (a dep that never
// arrives), with a segment longer than MAX_SEG, or with anything unusual (a
// double index, an index-only record, a dot out of range) is run whole by the
// ordinary tiered driver instead.  The oracle check found no violation of the
// closure argument in 288 k cuts of synthetic streams with 60 % cycles.
//
// Work per Add is O(d + segment length) and every phase is a flat kernel over
// (stream, step): position table scatter, dependency reach, a two-level
// prefix max (cut flags), a two-level prefix count (segment ids), segment
// build, the batched executor, scatter back.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace cut {

constexpr uint32_t INF = 0xFFFFFFFFu;
constexpr uint32_t MAX_SEG = 4096;  // longer segments: the stream runs whole
constexpr uint32_t CHUNK = 1024;    // steps per scan block (256 threads x 4)
constexpr uint32_t BT = 256;

struct In {
  const uint32_t* dot;
  const uint32_t* hdr;
  const uint32_t* deps;
  const uint32_t* lengths;
  uint32_t S, steps, dmax, n;
  size_t pw;  // plane words
};

__device__ __forceinline__ uint32_t len_of(const In& in, uint32_t s) {
  return in.lengths ? min(in.lengths[s], in.steps) : in.steps;
}

// Work item t -> (stream s, step i) of the flat kernels that read the input
// planes.  With one tile column of streams (S <= 64; configs[4]: 5) the items
// run in plane order: the S streams' 16-byte pieces of a 4-step tile row are
// adjacent words, so a wave reads whole lines once.  Stream-major items (each
// wave walking one stream's steps) read 16 bytes of each line per stream, and
// each line came from HBM once per stream.  i may be >= steps (steps are
// rounded up to 4).
__device__ __forceinline__ uint64_t n_items(const In& in) {
  return in.S <= FX_TILE_STREAMS ? (uint64_t)in.S * ((in.steps + 3u) & ~3u) : (uint64_t)in.S * in.steps;
}
__device__ __forceinline__ void item(const In& in, uint64_t t, uint32_t& s, uint32_t& i) {
  if (in.S <= FX_TILE_STREAMS) {
    const uint32_t w = 4u * in.S;
    s = (uint32_t)(t % w) >> 2;
    i = (uint32_t)(t / w) * 4u + (uint32_t)(t & 3u);
  } else {
    s = (uint32_t)(t / in.steps);
    i = (uint32_t)(t % in.steps);
  }
}

// position-table slot of dot d in stream s, or INF when out of the table
__device__ __forceinline__ uint64_t pos_slot(const In& in, const uint64_t* base, const uint32_t* maxseq,
                                             uint32_t s, uint32_t d) {
  const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
  const uint32_t ms = maxseq[s];
  if (src < 1 || src > in.n || sq > ms) return ~0ull;
  return base[s] + (uint64_t)(src - 1) * (ms + 1) + sq;
}

// Per-stream max over a grid-stride loop: each wave keeps a running (stream,
// max) pair and issues one atomicMax per stream it leaves (a handful per wave)
// instead of one per iteration: with a few long streams, per-iteration
// atomics on a few addresses serialised at L2 and dominated the cut analysis.
struct WaveMax {
  uint32_t s = 0xFFFFFFFFu, m = 0;  // wave-uniform
  __device__ __forceinline__ void add(uint32_t* out, uint32_t sl, uint32_t v) {
    uint64_t todo = __ballot(true);
    while (todo) {
      const uint32_t lead = __builtin_ctzll(todo);
      const uint32_t s0 = (uint32_t)__shfl((int)sl, (int)lead);
      const bool mine = sl == s0;
      uint32_t mm = mine ? v : 0u;
      for (uint32_t off = 32; off; off >>= 1) mm = max(mm, (uint32_t)__shfl_xor((int)mm, off));
      if (s0 == s) {
        m = max(m, mm);
      } else {
        flush(out);
        s = s0;
        m = mm;
      }
      todo &= ~__ballot(mine);
    }
  }
  __device__ __forceinline__ void flush(uint32_t* out) const {
    if (s != 0xFFFFFFFFu && (threadIdx.x & 63u) == 0) atomicMax(&out[s], m);
  }
  // the block's waves usually end on the same stream: combine them in LDS
  // first, so a block issues one atomic per distinct stream, not one per wave
  __device__ __forceinline__ void flush_block(uint32_t* out) const {
    __shared__ uint32_t bs[BT / 64], bm[BT / 64];
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) {
      bs[w] = s;
      bm[w] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (uint32_t i = 0; i < BT / 64; ++i) {
        if (bs[i] == 0xFFFFFFFFu) continue;
        uint32_t mx = bm[i];
        bool first = true;
        for (uint32_t j = 0; j < i; ++j) first = first && bs[j] != bs[i];
        if (!first) continue;
        for (uint32_t j = i + 1; j < BT / 64; ++j)
          if (bs[j] == bs[i]) mx = max(mx, bm[j]);
        atomicMax(&out[bs[i]], mx);
      }
    }
  }
};

// With few streams (configs[4]: 5), per-stream maxima from thousands of
// blocks would all hit the same few addresses: the atomics serialise at L2.
// Then the block's waves combine in LDS and the block writes its S partial
// maxima (part[block][S]), reduced per stream by k_part_max.
constexpr uint32_t SMALL_S = 64;

// out[s] = max(out[s], max over blocks b of part[b][s]); one block per stream
__global__ void k_part_max(const uint32_t* part, uint32_t blocks, uint32_t S, uint32_t* out) {
  const uint32_t s = blockIdx.x;
  uint32_t m = 0;
  for (uint32_t b = threadIdx.x; b < blocks; b += blockDim.x) m = max(m, part[(size_t)b * S + s]);
  for (uint32_t off = 32; off; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
  __shared__ uint32_t sh[BT / 64];
  if ((threadIdx.x & 63u) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t i = 1; i < blockDim.x / 64; ++i) m = max(m, sh[i]);
    out[s] = max(out[s], max(m, sh[0]));
  }
}

__global__ void k_maxseq(In in, uint32_t* maxseq, uint32_t* bad, uint32_t* part) {
  const uint64_t total = n_items(in);
  WaveMax acc;
  __shared__ uint32_t lm[SMALL_S];
  const bool small = part != nullptr;
  if (small) {
    if (threadIdx.x < SMALL_S) lm[threadIdx.x] = 0;
    __syncthreads();
  }
  uint32_t* out = small ? lm : maxseq;
  // wave-uniform trip count (the reduction needs every lane active)
  for (uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x; b0 < total; b0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t t = b0 + threadIdx.x;
    uint32_t s, i;
    item(in, min(t, total - 1), s, i);
    const bool valid = t < total && i < len_of(in, s);
    uint32_t sq = 0;
    if (valid) {
      const size_t at = fx_index(i, s, in.steps);
      const uint32_t d = in.dot[at];
      const uint32_t src = FX_DOT_SRC(d);
      if (src < 1 || src > in.n) bad[s] = 1;  // (the record kind: k_reach, which reads hdr anyway)
      sq = FX_DOT_SEQ(d);
    }
    acc.add(out, s, sq);
  }
  if (small) {
    acc.flush(lm);
    __syncthreads();
    if (threadIdx.x < in.S) part[(size_t)blockIdx.x * in.S + threadIdx.x] = lm[threadIdx.x];
  } else {
    acc.flush_block(maxseq);
  }
}

__global__ void k_pos(In in, const uint64_t* base, const uint32_t* maxseq, uint32_t* pos, uint32_t* bad) {
  const uint64_t total = n_items(in);
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t s, i;
    item(in, t, s, i);
    if (i >= len_of(in, s)) continue;
    const uint64_t slot = pos_slot(in, base, maxseq, s, in.dot[fx_index(i, s, in.steps)]);
    if (slot == ~0ull) {
      bad[s] = 1;
      continue;
    }
    if (atomicExch(&pos[slot], i) != INF) bad[s] = 1;  // double index: run whole, report there
  }
}

// reach(i) = max(i, position of every dep); INF for a dep never added
__global__ void k_reach(In in, const uint64_t* base, const uint32_t* maxseq, const uint32_t* pos, uint32_t* reach,
                        uint32_t* bad) {
  const uint64_t total = n_items(in);
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t s, i;
    item(in, t, s, i);
    if (i >= len_of(in, s)) continue;
    const size_t at = fx_index(i, s, in.steps);
    const uint32_t h = in.hdr[at];
    if (FX_HDR_KIND(h) != FX_KIND_ADD) bad[s] = 1;  // an index-only or executed record: the stream runs whole
    const uint32_t nd = FX_HDR_ND(h);
    uint32_t r = i;
    for (uint32_t j = 0; j < nd && j < in.dmax; ++j) {
      const uint64_t slot = pos_slot(in, base, maxseq, s, in.deps[j * in.pw + at]);
      r = max(r, slot == ~0ull ? INF : pos[slot]);
    }
    reach[(size_t)s * in.steps + i] = r;
  }
}

// block-wide exclusive scan (256 threads) with op = max or +
template <bool SUM>
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* sh) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, off);
    if (lane >= off) x = SUM ? x + y : max(x, y);
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t p = 0;
  for (uint32_t k = 0; k < w; ++k) p = SUM ? p + sh[k] : max(p, sh[k]);
  uint32_t e = (uint32_t)__shfl_up((int)x, 1);
  if (lane == 0) e = 0;
  __syncthreads();
  return SUM ? p + e : max(p, e);
}

// per (chunk, stream): max of reach over the chunk
__global__ void k_chunk_max(In in, const uint32_t* reach, uint32_t nch, uint32_t* cagg) {
  const uint32_t c = blockIdx.x % nch, s = blockIdx.x / nch;
  const uint32_t L = len_of(in, s);
  __shared__ uint32_t sh[4];
  uint32_t m = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t i = c * CHUNK + threadIdx.x * 4 + k;
    if (i < L) m = max(m, reach[(size_t)s * in.steps + i]);
  }
  // block max
  for (uint32_t off = 32; off; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
  if ((threadIdx.x & 63u) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) cagg[(size_t)s * nch + c] = max(max(sh[0], sh[1]), max(sh[2], sh[3]));
}

// per stream: chunk aggregates -> exclusive prefix (max or sum)
template <bool SUM>
__global__ void k_chunk_excl(uint32_t S, uint32_t nch, uint32_t* cagg, uint32_t* total) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  uint32_t run = 0;
  for (uint32_t c = 0; c < nch; ++c) {
    const uint32_t v = cagg[(size_t)s * nch + c];
    cagg[(size_t)s * nch + c] = run;
    run = SUM ? run + v : max(run, v);
  }
  if (total) total[s] = run;
}

// the same for long streams (configs[4]: 5 streams of ~4,900 chunks, where a
// thread per stream walked its chunks one dependent load at a time, 0.11 ms
// per scan): one block per stream scans CHUNK aggregates per round, carrying
// the running value between rounds
template <bool SUM>
__global__ void k_chunk_excl_blk(uint32_t nch, uint32_t* cagg, uint32_t* total) {
  const uint32_t s = blockIdx.x;
  __shared__ uint32_t sh[4];
  __shared__ uint32_t carry_sh;
  uint32_t* a = cagg + (size_t)s * nch;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nch; b0 += CHUNK) {
    uint32_t v[4], loc = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t i = b0 + threadIdx.x * 4 + k;
      v[k] = i < nch ? a[i] : 0u;
      loc = SUM ? loc + v[k] : max(loc, v[k]);
    }
    const uint32_t ex = block_excl<SUM>(loc, sh);
    uint32_t run = SUM ? carry + ex : max(carry, ex);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t i = b0 + threadIdx.x * 4 + k;
      if (i < nch) a[i] = run;
      run = SUM ? run + v[k] : max(run, v[k]);
    }
    if (threadIdx.x == BT - 1) carry_sh = run;  // the last thread's inclusive value
    __syncthreads();
    carry = carry_sh;
    __syncthreads();
  }
  if (total && threadIdx.x == 0) total[s] = carry;
}

// exclusive chunk scan per stream: a block per stream when streams are long
template <bool SUM>
static void chunk_excl(uint32_t S, uint32_t nch, uint32_t* cagg, uint32_t* total, hipStream_t hs) {
  if (nch > 64) hipLaunchKernelGGL(k_chunk_excl_blk<SUM>, dim3(S), dim3(BT), 0, hs, nch, cagg, total);
  else hipLaunchKernelGGL(k_chunk_excl<SUM>, dim3((S + 255) / 256), dim3(256), 0, hs, S, nch, cagg, total);
}

// cut flags: prefix max of reach <= i; per-chunk cut counts
__global__ void k_flags(In in, const uint32_t* reach, uint32_t nch, const uint32_t* cmax_excl, uint8_t* flag,
                        uint32_t* ccnt, uint32_t* lastok) {
  const uint32_t c = blockIdx.x % nch, s = blockIdx.x / nch;
  const uint32_t L = len_of(in, s);
  __shared__ uint32_t sh[4];
  uint32_t v[4], m = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t i = c * CHUNK + threadIdx.x * 4 + k;
    v[k] = i < L ? reach[(size_t)s * in.steps + i] : 0u;
    m = max(m, v[k]);
  }
  uint32_t run = max(block_excl<false>(m, sh), cmax_excl[(size_t)s * nch + c]);
  uint32_t cnt = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t i = c * CHUNK + threadIdx.x * 4 + k;
    run = max(run, v[k]);
    const bool f = i < L && run <= i;
    if (i < in.steps) flag[(size_t)s * in.steps + i] = f ? 1 : 0;
    cnt += f ? 1u : 0u;
    if (i + 1 == L) lastok[s] = f ? 1u : 0u;
  }
  for (uint32_t off = 32; off; off >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, off);
  if ((threadIdx.x & 63u) == 0) sh[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) ccnt[(size_t)s * nch + c] = sh[0] + sh[1] + sh[2] + sh[3];
}

// segment ids: segment of step i = cuts strictly before i; a cut ends its segment
__global__ void k_segs(In in, const uint8_t* flag, uint32_t nch, const uint32_t* ccnt_excl, const uint64_t* segbase,
                       uint32_t* seg_of, uint32_t* seg_end, uint32_t* seg_stream) {
  const uint32_t c = blockIdx.x % nch, s = blockIdx.x / nch;
  const uint32_t L = len_of(in, s);
  __shared__ uint32_t sh[4];
  uint32_t f[4], cnt = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t i = c * CHUNK + threadIdx.x * 4 + k;
    f[k] = i < L ? flag[(size_t)s * in.steps + i] : 0u;
    cnt += f[k];
  }
  uint32_t run = block_excl<true>(cnt, sh) + ccnt_excl[(size_t)s * nch + c];
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t i = c * CHUNK + threadIdx.x * 4 + k;
    if (i >= L) break;
    const uint64_t id = segbase[s] + run;
    seg_of[(size_t)s * in.steps + i] = (uint32_t)id;
    if (f[k]) {
      seg_end[id] = i;
      seg_stream[id] = s;
    }
    run += f[k];
  }
}

// segment starts and lengths; longest segment per stream
__global__ void k_seglen(uint64_t nseg, const uint64_t* segbase, const uint32_t* seg_end, const uint32_t* seg_stream,
                         uint32_t* seg_start, uint32_t* smax, uint32_t S, uint32_t* part) {
  WaveMax acc;
  __shared__ uint32_t lm[SMALL_S];
  const bool small = part != nullptr;
  if (small) {
    if (threadIdx.x < SMALL_S) lm[threadIdx.x] = 0;
    __syncthreads();
  }
  uint32_t* out = small ? lm : smax;
  for (uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x; b0 < nseg; b0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = b0 + threadIdx.x;
    const bool valid = k < nseg;
    const uint32_t s = seg_stream[valid ? k : nseg - 1];
    uint32_t len = 0;
    if (valid) {
      const uint32_t a = (k == segbase[s]) ? 0u : seg_end[k - 1] + 1u;
      seg_start[k] = a;
      len = seg_end[k] - a + 1u;
    }
    acc.add(out, s, len);
  }
  if (small) {
    acc.flush(lm);
    __syncthreads();
    if (threadIdx.x < S) part[(size_t)blockIdx.x * S + threadIdx.x] = lm[threadIdx.x];
  } else {
    acc.flush_block(smax);
  }
}

// Segments one Add long (an Add whose deps all lie in the executed prefix;
// at 2 % conflicts nine in ten segments) need no executor: the Add is a
// singleton SCC found by the search handle_add starts from it
// (graph/mod.rs:244-250, tarjan.rs:96-316), so it executes at its own step,
// after the whole prefix: order row a = a | SCC start, release[a] = a.
// k_build writes those directly, and only the longer segments form the batch,
// ordered by length class, longest first: the batch executor runs one segment
// per lane, so a wave lasts as long as its longest segment, and neighbours of
// like length keep its lanes busy (S5: lengths 2 to 110; the lane tier 4.8 ->
// 2.6 ms).  It scatters k_build's writes into the batch planes (0.75 -> 1.14
// ms); ordering only inside chunks of 1,024 segments kept them local but lost
// more in the executor (S5 5.58 against 4.26 ms per step, same box).  Class of
// a length L >= 2: ceil(log2 L), 1..12, 13 beyond MAX_SEG (those streams run
// whole; their segments keep an empty batch slot).  Deterministic: within a
// class the segments keep their id order (per-chunk class counts, an
// exclusive scan of each class over the chunks, ranks by ballots inside a
// chunk).
constexpr uint32_t NCLS = 16;
__device__ __forceinline__ uint32_t seg_class(uint64_t g, uint64_t nseg, const uint32_t* seg_start,
                                              const uint32_t* seg_end) {
  if (g >= nseg) return 0;
  const uint32_t len = seg_end[g] - seg_start[g] + 1u;
  if (len < 2) return 0;
  return len > MAX_SEG ? 13u : 32u - (uint32_t)__builtin_clz(len - 1u);
}

// per chunk of CHUNK segments: the count of each class (ccnt[chunk][class])
// and of the batch's segments in all (cm[chunk])
__global__ void k_class_count(uint64_t nseg, const uint32_t* seg_start, const uint32_t* seg_end, uint32_t nch,
                              uint32_t* ccnt) {
  __shared__ uint32_t cnt[NCLS];
  if (threadIdx.x < NCLS) cnt[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t c = seg_class((uint64_t)blockIdx.x * CHUNK + k * BT + threadIdx.x, nseg, seg_start, seg_end);
    if (c) atomicAdd(&cnt[c], 1u);
  }
  __syncthreads();
  if (threadIdx.x < NCLS) ccnt[(size_t)threadIdx.x * nch + blockIdx.x] = cnt[threadIdx.x];
}

// batch index of every segment (INF for a single) and its inverse.  cm: the
// exclusive prefix of the chunks' batch counts
__global__ void k_class_fill(uint64_t nseg, const uint32_t* seg_start, const uint32_t* seg_end, uint32_t nch,
                             const uint32_t* ccnt, const uint32_t* ctot, uint32_t* bidx, uint32_t* bseg) {
  __shared__ uint32_t base[NCLS], run[NCLS], cw[BT / 64][NCLS];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  if (threadIdx.x < NCLS) {
    uint32_t b = 0;  // longest class first
    for (uint32_t c = threadIdx.x + 1; c < NCLS; ++c) b += ctot[c];
    base[threadIdx.x] = b + ccnt[(size_t)threadIdx.x * nch + blockIdx.x];
    run[threadIdx.x] = 0;
  }
  for (uint32_t k = 0; k < 4; ++k) {
    const uint64_t g = (uint64_t)blockIdx.x * CHUNK + k * BT + threadIdx.x;
    const uint32_t c = seg_class(g, nseg, seg_start, seg_end);
    if (lane < NCLS) cw[w][lane] = 0;
    __syncthreads();
    uint32_t rank = 0;
    uint64_t todo = __ballot(c != 0);
    while (todo) {
      const uint32_t lead = __builtin_ctzll(todo);
      const uint32_t c0 = (uint32_t)__shfl((int)c, (int)lead);
      const uint64_t same = __ballot(c == c0);
      if (lane == lead) cw[w][c0] = (uint32_t)__popcll(same);
      if (c == c0) rank = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
      todo &= ~same;
    }
    __syncthreads();
    if (g < nseg) {
      if (c) {
        uint32_t b = base[c] + run[c] + rank;
        for (uint32_t v = 0; v < w; ++v) b += cw[v][c];
        bidx[g] = b;
        bseg[b] = (uint32_t)g;
      } else {
        bidx[g] = INF;
      }
    }
    __syncthreads();
    if (threadIdx.x < NCLS) {
      uint32_t t = 0;
      for (uint32_t v = 0; v < BT / 64; ++v) t += cw[v][threadIdx.x];
      run[threadIdx.x] += t;
    }
    __syncthreads();
  }
}

struct Seg {
  uint32_t* dot;
  uint32_t* hdr;
  uint32_t* deps;
  uint32_t* lengths;
  uint32_t steps;  // longest segment
  size_t pw;
};

// rank of the seq of source `src` among the segment's dots of that source
__device__ __forceinline__ uint32_t seg_rank(const In& in, uint32_t s, uint32_t a, uint32_t b, uint32_t src,
                                             uint32_t sq) {
  uint32_t r = 1;
  for (uint32_t t = a; t <= b; ++t) {
    const uint32_t d = in.dot[fx_index(t, s, in.steps)];
    r += (FX_DOT_SRC(d) == src && FX_DOT_SEQ(d) < sq) ? 1u : 0u;
  }
  return r;
}

// Renumbering needs each dot's rank among the segment's dots of its source.
// A segment of at most RANK_INLINE Adds is scanned by k_build itself, once
// per Add and per dep.  For longer ones k_rank writes every Add's own rank
// once (rk, stream-major) and k_build takes a dep's rank at the dep's
// position (a dep outside the prefix lies in the segment: it ends at a cut):
// S5, 3 deps per Add, k_build 1.14 ms -> k_rank 0.11 + k_build 0.29 ms.
// k_rank walks the stream's Adds (each reads its segment bounds to skip the
// short ones); when the longer segments hold few Adds (2 % conflicts: most
// segments are 1-4 Adds) k_rank_slots walks only their batch slots instead
// (a prefix of the batch, which is ordered longest class first).  At S5 the
// slot walk read 1.45x the bytes of the Add walk and took 0.20 against 0.11 ms.
constexpr uint32_t RANK_INLINE = 4;    // class <= 2
constexpr uint32_t RANK_CLASS_MIN = 3;  // classes ranked by k_rank / k_rank_slots

__global__ void k_rank_slots(In in, uint32_t nl, uint32_t seg_steps, const uint32_t* bseg, const uint32_t* seg_stream,
                             const uint32_t* seg_start, const uint32_t* seg_end, const uint32_t* whole, uint32_t* rk) {
  const uint64_t total = fx_plane_words(nl, seg_steps);
  const uint32_t steps4 = (seg_steps + 3u) >> 2;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t row = t >> 8;  // (tile, 4-step block) of the batch planes
    const uint32_t bb = (uint32_t)(row / steps4) * 64u + ((uint32_t)(t & 255u) >> 2);
    const uint32_t j = (uint32_t)(row % steps4) * 4u + (uint32_t)(t & 3u);
    if (bb >= nl) continue;
    const uint32_t k = bseg[bb];
    const uint32_t a = seg_start[k], b = seg_end[k], s = seg_stream[k];
    if (j > b - a || whole[s]) continue;  // (segments over MAX_SEG belong to whole streams)
    const uint32_t d = in.dot[fx_index(a + j, s, in.steps)];
    rk[(size_t)s * in.steps + a + j] = seg_rank(in, s, a, b, FX_DOT_SRC(d), FX_DOT_SEQ(d));
  }
}

__global__ void k_rank(In in, const uint32_t* seg_of, const uint32_t* seg_start, const uint32_t* seg_end,
                       const uint32_t* whole, uint32_t* rk) {
  const uint64_t total = n_items(in);
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t s, i;
    item(in, t, s, i);
    if (i >= len_of(in, s) || whole[s]) continue;
    const uint32_t k = seg_of[(size_t)s * in.steps + i];
    const uint32_t a = seg_start[k], b = seg_end[k];
    if (b - a < RANK_INLINE) continue;  // k_build ranks these itself
    const uint32_t d = in.dot[fx_index(i, s, in.steps)];
    rk[(size_t)s * in.steps + i] = seg_rank(in, s, a, b, FX_DOT_SRC(d), FX_DOT_SEQ(d));
  }
}

__global__ void k_build(In in, const uint64_t* base, const uint32_t* maxseq, const uint32_t* pos,
                        const uint32_t* seg_of, const uint32_t* seg_start, const uint32_t* seg_end,
                        const uint32_t* bidx, const uint32_t* whole, const uint8_t* flag, const uint32_t* rk, Seg sg,
                        uint32_t* order, uint32_t* release) {
  const uint64_t total = n_items(in);
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t s, i;
    item(in, t, s, i);
    if (i >= len_of(in, s) || whole[s]) continue;
    const size_t at = fx_index(i, s, in.steps);
    // a single Add (cuts after i - 1 and after i) executes at its own step; the
    // cut flags (a byte per step, read in order) tell without the segment
    // tables (at 2 % conflicts, 82 % of the Adds)
    const uint8_t* sf = flag + (size_t)s * in.steps;
    if (sf[i] && (i == 0 || sf[i - 1])) {
      order[at] = i | FX_ORDER_SCC_START;
      release[at] = i;
      continue;
    }
    const uint32_t k = seg_of[(size_t)s * in.steps + i];
    const uint32_t a = seg_start[k], b = seg_end[k], j = i - a;
    const uint32_t bk = bidx[k];
    const size_t to = fx_index(j, bk, sg.steps);
    const uint32_t d = in.dot[at];
    const uint32_t* srk = rk + (size_t)s * in.steps;
    const bool inl = b - a < RANK_INLINE;
    sg.dot[to] = FX_PACK_DOT(FX_DOT_SRC(d), inl ? seg_rank(in, s, a, b, FX_DOT_SRC(d), FX_DOT_SEQ(d)) : srk[i]);
    const uint32_t h = in.hdr[at];
    const uint32_t nd = min(FX_HDR_ND(h), in.dmax);
    uint32_t nk = 0;
    for (uint32_t x = 0; x < nd; ++x) {  // ascending stays ascending: per-source ranks, source first
      const uint32_t u = in.deps[x * in.pw + at];
      const uint32_t p = pos[pos_slot(in, base, maxseq, s, u)];
      if (p < a) continue;  // executed in the prefix
      sg.deps[nk * sg.pw + to] =
          FX_PACK_DOT(FX_DOT_SRC(u), inl ? seg_rank(in, s, a, b, FX_DOT_SRC(u), FX_DOT_SEQ(u)) : srk[p]);
      ++nk;
    }
    sg.hdr[to] = FX_MAKE_HDR(FX_HDR_T(h), nk, FX_HDR_KIND(h));
    if (j == 0) sg.lengths[bk] = b - a + 1u;
  }
}

// batch outputs -> the stream's planes; a segment that did not execute
// completely sends its stream to the whole-stream path.  Items in the batch
// planes' own order (t = plane word), so a wave reads 1 KiB of them at once
__global__ void k_scatter(uint32_t nb, uint32_t seg_steps, const uint32_t* bseg, const uint32_t* seg_stream,
                          const uint32_t* seg_start, const uint32_t* blen, const uint32_t* sorder,
                          const uint32_t* srelease, const uint32_t* snexec, const uint32_t* serr, uint32_t steps,
                          uint32_t* order, uint32_t* release, uint32_t* fail) {
  const uint64_t total = fx_plane_words(nb, seg_steps);
  const uint32_t steps4 = (seg_steps + 3u) >> 2;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t row = t >> 8;  // (tile, 4-step block)
    const uint32_t b = (uint32_t)(row / steps4) * 64u + ((uint32_t)(t & 255u) >> 2);
    const uint32_t j = (uint32_t)(row % steps4) * 4u + (uint32_t)(t & 3u);
    if (b >= nb) continue;
    const uint32_t len = blen[b];
    if (j >= len) continue;
    const uint32_t k = bseg[b];
    const uint32_t s = seg_stream[k], a = seg_start[k];
    if (serr[b] != FX_OK || snexec[b] != len) {
      if (j == 0) fail[s] = 1;
      continue;
    }
    const size_t from = t;  // fx_index(j, b, seg_steps)
    const size_t to = fx_index(a + j, s, steps);
    const uint32_t o = sorder[from];
    order[to] = (a + FX_ORDER_REC(o)) | (o & FX_ORDER_SCC_START);
    const uint32_t r = srelease[from];
    release[to] = r == FX_RELEASE_NONE ? FX_RELEASE_NONE : a + r;
  }
}

__global__ void k_finish(In in, const uint32_t* whole, const uint32_t* fail, uint32_t* nexec, uint32_t* err) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= in.S || whole[s] || fail[s]) return;
  nexec[s] = len_of(in, s);
  err[s] = FX_OK;
}

// the driver's device buffers: persistent scratch slots (fx_internal.h)
struct DevBufs {
  hipStream_t hs;
  uint32_t next = SCRATCH_CUT_FIRST;
  template <typename T>
  T* alloc(size_t count, int fill = -1) {
    if (next >= SCRATCH_SLOTS) return nullptr;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 4);
    void* p = scratch(next++, bytes);
    if (p && fill >= 0) (void)hipMemsetAsync(p, fill, bytes, hs);
    return (T*)p;
  }
};

static uint32_t grid_for(uint64_t work) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((work + BT - 1) / BT, 256u * 64u));
}
// per-stream max reductions (WaveMax): fewer, longer-running waves, so each
// flushes one atomic per stream after many iterations (8 blocks per CU)
static uint32_t grid_for_max(uint64_t work) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((work + BT - 1) / BT, 256u * 8u));
}

}  // namespace cut
}  // namespace fx

using namespace fx;
using namespace fx::cut;

extern "C" int fx_batch_run_cut(const fx_stream_batch* in_, const fx_order_batch* out, uint32_t flags,
                                void* hip_stream, fx_cut_stats* stats) {
  if (!in_ || !out) return FX_ERR_INVALID_ARG;
  if (stats) *stats = fx_cut_stats{};
  // execute-at-commit has no graph to cut
  if (flags & FX_FLAG_EXECUTE_AT_COMMIT) return run_tiered(in_, out, flags, hip_stream, nullptr, nullptr);
  if (fx_device_count() <= 0) return FX_ERR_NO_DEVICE;
  if (!in_->dot || !in_->hdr || (in_->dmax && !in_->deps) || !out->order || !out->release || !out->nexec || !out->err)
    return FX_ERR_INVALID_ARG;
  if (in_->n < 1 || in_->n > 8 || in_->steps >= (1u << 26) || in_->dmax > 31) return FX_ERR_INVALID_ARG;
  hipStream_t hs = (hipStream_t)hip_stream;
  In in{in_->dot, in_->hdr, in_->deps, in_->lengths, in_->num_streams, in_->steps, in_->dmax, in_->n,
        fx_plane_words(in_->num_streams, in_->steps)};
  const uint32_t S = in.S;
  if (S == 0 || in.steps == 0) return FX_OK;
  std::lock_guard<std::recursive_mutex> lock(scratch_mutex());
  DevBufs db;
  db.hs = hs;
  const uint64_t work = (uint64_t)S * in.steps;
  // 1. position table
  uint32_t* maxseq = db.alloc<uint32_t>(S, 0);
  uint32_t* bad = db.alloc<uint32_t>(S, 0);
  if (!maxseq || !bad) return FX_ERR_HIP;
  const uint32_t gmax = grid_for_max(work);
  uint32_t* part = S <= SMALL_S ? db.alloc<uint32_t>((size_t)gmax * S) : nullptr;
  if (S <= SMALL_S && !part) return FX_ERR_HIP;
  hipLaunchKernelGGL(k_maxseq, dim3(gmax), dim3(BT), 0, hs, in, maxseq, bad, part);
  if (part) hipLaunchKernelGGL(k_part_max, dim3(S), dim3(BT), 0, hs, part, gmax, S, maxseq);
  std::vector<uint32_t> h_maxseq(S), h_bad(S);
  (void)hipMemcpyAsync(h_maxseq.data(), maxseq, (size_t)S * 4, hipMemcpyDeviceToHost, hs);
  if (hipStreamSynchronize(hs) != hipSuccess) return FX_ERR_HIP;
  std::vector<uint64_t> h_base(S);
  uint64_t ptotal = 0;
  for (uint32_t s = 0; s < S; ++s) {
    h_base[s] = ptotal;
    ptotal += (uint64_t)in.n * ((uint64_t)h_maxseq[s] + 1);
  }
  if (ptotal > (1ull << 32)) return run_tiered(in_, out, flags, hip_stream, nullptr, nullptr);  // sparse seqs
  uint64_t* base = db.alloc<uint64_t>(S);
  uint32_t* pos = db.alloc<uint32_t>(ptotal, 0xFF);
  uint32_t* reach = db.alloc<uint32_t>(work);
  if (!base || !pos || !reach) return FX_ERR_HIP;
  (void)hipMemcpyAsync(base, h_base.data(), (size_t)S * 8, hipMemcpyHostToDevice, hs);
  hipLaunchKernelGGL(k_pos, dim3(grid_for(work)), dim3(BT), 0, hs, in, base, maxseq, pos, bad);
  hipLaunchKernelGGL(k_reach, dim3(grid_for(work)), dim3(BT), 0, hs, in, base, maxseq, pos, reach, bad);
  // 2. cut flags (prefix max of reach) and segment counts
  const uint32_t nch = (in.steps + CHUNK - 1) / CHUNK;
  uint32_t* cagg = db.alloc<uint32_t>((size_t)S * nch);
  uint32_t* ccnt = db.alloc<uint32_t>((size_t)S * nch);
  uint8_t* flag = db.alloc<uint8_t>(work);
  uint32_t* lastok = db.alloc<uint32_t>(S, 0);
  uint32_t* nseg = db.alloc<uint32_t>(S);
  if (!cagg || !ccnt || !flag || !lastok || !nseg) return FX_ERR_HIP;
  hipLaunchKernelGGL(k_chunk_max, dim3(nch * S), dim3(BT), 0, hs, in, reach, nch, cagg);
  chunk_excl<false>(S, nch, cagg, (uint32_t*)nullptr, hs);
  hipLaunchKernelGGL(k_flags, dim3(nch * S), dim3(BT), 0, hs, in, reach, nch, cagg, flag, ccnt, lastok);
  chunk_excl<true>(S, nch, ccnt, nseg, hs);
  std::vector<uint32_t> h_nseg(S), h_lastok(S);
  (void)hipMemcpyAsync(h_nseg.data(), nseg, (size_t)S * 4, hipMemcpyDeviceToHost, hs);
  (void)hipMemcpyAsync(h_lastok.data(), lastok, (size_t)S * 4, hipMemcpyDeviceToHost, hs);
  (void)hipMemcpyAsync(h_bad.data(), bad, (size_t)S * 4, hipMemcpyDeviceToHost, hs);
  if (hipStreamSynchronize(hs) != hipSuccess) return FX_ERR_HIP;
  std::vector<uint64_t> h_segbase(S);
  uint64_t NS = 0;
  for (uint32_t s = 0; s < S; ++s) {
    h_segbase[s] = NS;
    NS += h_nseg[s];
  }
  // 3. segments
  uint64_t* segbase = db.alloc<uint64_t>(S);
  uint32_t* seg_of = db.alloc<uint32_t>(work);
  uint32_t* seg_end = db.alloc<uint32_t>(NS);
  uint32_t* seg_stream = db.alloc<uint32_t>(NS);
  uint32_t* seg_start = db.alloc<uint32_t>(NS);
  uint32_t* smax = db.alloc<uint32_t>(S, 0);
  if (!segbase || !seg_of || !seg_end || !seg_stream || !seg_start || !smax) return FX_ERR_HIP;
  (void)hipMemcpyAsync(segbase, h_segbase.data(), (size_t)S * 8, hipMemcpyHostToDevice, hs);
  hipLaunchKernelGGL(k_segs, dim3(nch * S), dim3(BT), 0, hs, in, flag, nch, ccnt, segbase, seg_of, seg_end, seg_stream);
  if (NS) {
    const uint32_t gs = grid_for_max(NS);
    uint32_t* spart = S <= SMALL_S ? db.alloc<uint32_t>((size_t)gs * S) : nullptr;
    if (S <= SMALL_S && !spart) return FX_ERR_HIP;
    hipLaunchKernelGGL(k_seglen, dim3(gs), dim3(BT), 0, hs, NS, segbase, seg_end, seg_stream, seg_start, smax, S,
                       spart);
    if (spart) hipLaunchKernelGGL(k_part_max, dim3(S), dim3(BT), 0, hs, spart, gs, S, smax);
  }
  // the batch: segments longer than one Add, by chunks and, inside a chunk,
  // longest class first (k_class_fill)
  uint32_t* ctot = db.alloc<uint32_t>(NCLS, 0);
  uint32_t* bidx = nullptr;
  uint32_t* bseg = nullptr;
  if (!ctot) return FX_ERR_HIP;
  if (NS && NS < (1ull << 31)) {
    const uint32_t nchS = (uint32_t)((NS + CHUNK - 1) / CHUNK);
    uint32_t* ccls = db.alloc<uint32_t>((size_t)NCLS * nchS);
    bidx = db.alloc<uint32_t>(NS);
    bseg = db.alloc<uint32_t>(NS);
    if (!ccls || !bidx || !bseg) return FX_ERR_HIP;
    hipLaunchKernelGGL(k_class_count, dim3(nchS), dim3(BT), 0, hs, NS, seg_start, seg_end, nchS, ccls);
    chunk_excl<true>(NCLS, nchS, ccls, ctot, hs);
    hipLaunchKernelGGL(k_class_fill, dim3(nchS), dim3(BT), 0, hs, NS, seg_start, seg_end, nchS, ccls, ctot, bidx,
                       bseg);
  }
  std::vector<uint32_t> h_smax(S), h_ctot(NCLS);
  (void)hipMemcpyAsync(h_smax.data(), smax, (size_t)S * 4, hipMemcpyDeviceToHost, hs);
  (void)hipMemcpyAsync(h_ctot.data(), ctot, NCLS * 4, hipMemcpyDeviceToHost, hs);
  if (hipStreamSynchronize(hs) != hipSuccess) return FX_ERR_HIP;
  uint32_t h_nbatch = 0;
  for (uint32_t c = 1; c < NCLS; ++c) h_nbatch += h_ctot[c];
  std::vector<uint32_t> h_len(S, in.steps);
  if (in_->lengths) {
    (void)hipMemcpyAsync(h_len.data(), in_->lengths, (size_t)S * 4, hipMemcpyDeviceToHost, hs);
    if (hipStreamSynchronize(hs) != hipSuccess) return FX_ERR_HIP;
  }
  std::vector<uint32_t> h_whole(S, 0), whole_list;
  uint32_t seg_steps = 1;
  uint64_t nseg_used = 0;
  for (uint32_t s = 0; s < S; ++s) {
    const bool any = std::min(h_len[s], in.steps) > 0;
    if (h_bad[s] || (any && !h_lastok[s]) || h_smax[s] > MAX_SEG) {
      h_whole[s] = 1;  // no usable cut decomposition: the stream runs whole
      whole_list.push_back(s);
    } else {
      seg_steps = std::max(seg_steps, h_smax[s]);
      nseg_used += h_nseg[s];
    }
  }
  if (NS >= (1ull << 31)) {  // too many segments for one batch: every stream runs whole
    for (uint32_t s = 0; s < S; ++s)
      if (!h_whole[s]) {
        h_whole[s] = 1;
        whole_list.push_back(s);
      }
    nseg_used = 0;
  }
  uint32_t* whole = db.alloc<uint32_t>(S);
  uint32_t* fail = db.alloc<uint32_t>(S, 0);
  if (!whole || !fail) return FX_ERR_HIP;
  (void)hipMemcpyAsync(whole, h_whole.data(), (size_t)S * 4, hipMemcpyHostToDevice, hs);
  if (stats) {
    stats->segments = nseg_used;
    stats->max_segment = seg_steps;
    stats->single_segments = nseg_used ? NS - h_nbatch : 0;
  }
  if (nseg_used) {
    // 4. the segment batch: one stream per segment longer than one Add (the
    // single ones are written by k_build); NB = 0 still runs k_build
    const uint32_t SS = std::max(h_nbatch, 1u);
    Seg sg;
    sg.steps = seg_steps;
    sg.pw = fx_plane_words(SS, seg_steps);
    // rows past a segment's length and dep planes past its ndeps are never read
    sg.dot = db.alloc<uint32_t>(sg.pw);
    sg.hdr = db.alloc<uint32_t>(sg.pw);
    sg.deps = db.alloc<uint32_t>(sg.pw * std::max(in.dmax, 1u));
    sg.lengths = db.alloc<uint32_t>(SS, 0);
    uint32_t* sorder = db.alloc<uint32_t>(sg.pw);
    uint32_t* srelease = db.alloc<uint32_t>(sg.pw);
    uint32_t* snexec = db.alloc<uint32_t>(SS);
    uint32_t* serr = db.alloc<uint32_t>(SS);
    if (!sg.dot || !sg.hdr || !sg.deps || !sg.lengths || !sorder || !srelease || !snexec || !serr) return FX_ERR_HIP;
    uint32_t* rk = db.alloc<uint32_t>(work);
    if (!rk) return FX_ERR_HIP;
    // the longer segments' Adds, bounded by their class (<= 2^c each)
    uint32_t nl = 0;
    uint64_t nl_adds = 0;
    for (uint32_t c = RANK_CLASS_MIN; c < NCLS; ++c) {
      nl += h_ctot[c];
      nl_adds += (uint64_t)h_ctot[c] << std::min(c, 12u);
    }
    if (nl_adds * 8 < work)
      hipLaunchKernelGGL(k_rank_slots, dim3(grid_for(fx_plane_words(std::max(nl, 1u), seg_steps))), dim3(BT), 0, hs,
                         in, nl, seg_steps, bseg, seg_stream, seg_start, seg_end, whole, rk);
    else
      hipLaunchKernelGGL(k_rank, dim3(grid_for(work)), dim3(BT), 0, hs, in, seg_of, seg_start, seg_end, whole, rk);
    hipLaunchKernelGGL(k_build, dim3(grid_for(work)), dim3(BT), 0, hs, in, base, maxseq, pos, seg_of, seg_start,
                       seg_end, bidx, whole, flag, rk, sg, out->order, out->release);
    if (h_nbatch) {
      fx_stream_batch sin{sg.dot, sg.hdr, sg.deps, sg.lengths, SS, seg_steps, in.dmax, in.n};
      fx_order_batch sout{sorder, srelease, snexec, serr};
      // the batch starts at FX_TIER_DEFAULT unless the caller names a first
      // tier.  The group tier first is 4-8 % faster per step (same box: S5 3.97
      // against 4.30 ms, 2 % 1.01 against 1.08, 100 % 6.03 against 6.17) but
      // reads 2.2x the HBM bytes at S5 (its 8 cached deps: 2.74 GB per step
      // against the lane tier's 0.28) and 1.3x at 2 %, so it stays opt-in
      // (FX_FLAG_FIRST_TIER(FX_TIER_GROUP)); the wave tier 5.27 / 8.48 ms and
      // the wide tier 17.1 / 22.2 ms are slower
      const int st = run_tiered(&sin, &sout, flags, hip_stream, nullptr, stats ? stats->tier_counts : nullptr);
      if (st == FX_ERR_HIP || st == FX_ERR_NO_DEVICE || st == FX_ERR_INVALID_ARG) return st;
      // (per-segment failures are handled below: their streams run whole)
      hipLaunchKernelGGL(k_scatter, dim3(grid_for(fx_plane_words(SS, seg_steps))), dim3(BT), 0, hs, SS, seg_steps,
                         bseg, seg_stream, seg_start, sg.lengths, sorder, srelease, snexec, serr, in.steps,
                         out->order, out->release, fail);
    }
  }
  // every stream that neither runs whole nor failed a segment executed all
  // its Adds — including the empty ones, which have no segment at all
  hipLaunchKernelGGL(k_finish, dim3((S + 255) / 256), dim3(256), 0, hs, in, whole, fail, out->nexec, out->err);
  std::vector<uint32_t> h_fail(S);
  (void)hipMemcpyAsync(h_fail.data(), fail, (size_t)S * 4, hipMemcpyDeviceToHost, hs);
  if (hipStreamSynchronize(hs) != hipSuccess) return FX_ERR_HIP;
  uint32_t failed = 0;
  for (uint32_t s = 0; s < S; ++s)
    if (h_fail[s] && !h_whole[s]) {
      whole_list.push_back(s);
      ++failed;
    }
  if (stats) stats->failed_streams = failed;
  std::sort(whole_list.begin(), whole_list.end());
  if (stats) stats->whole_streams = (uint32_t)whole_list.size();
  if (whole_list.empty()) return FX_OK;
  // 5. the rest, whole: the ordinary tiered driver (exact by construction)
  return run_tiered(in_, out, flags, hip_stream, &whole_list, nullptr);
}
