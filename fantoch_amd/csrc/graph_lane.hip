// graph_lane.hip — tier 5 of the batched GraphExecutor: one lane per stream,
// register-resident slot table, lanes progress independently.
//
// Same algorithm as the other tiers (DependencyGraph::handle_add,
// fantoch_ps/src/executor/graph/mod.rs:213-642, canonical orders C1/C2), laid
// out for the measured shape of the work: at the bench workload an Add costs
// on average 1.0-2.9 Tarjan visits, 1-10 dep edges and < 1 waiter retry
// (oracle counters), so the executor is a long sequential chain of SHORT
// micro-ops.  The layout therefore spends nothing on cross-lane traffic and
// keeps every stream of a GPU resident at once:
//
//   * one lane = one stream (one (instance, process) executor,
//     executor.rs:19-29); no shuffles, no ballots inside an executor;
//   * VertexIndex (index.rs:18-51) as 16 slots in VGPRs: dot, PendingIndex
//     registration (index.rs:145-208), arrival record, Tarjan word.  A dot
//     lookup is 16 parallel compares; a field read is a one-hot masked OR;
//   * TarjanSCCFinder (tarjan.rs:25-316) without an explicit stack: ids are
//     handed out in push order, so "the stack above v" is {on-stack slots with
//     id >= id(v)} (an on-stack bit mask), and each slot's Tarjan word keeps its
//     DFS parent and resume index, so the frame stack is the parent chain;
//   * check_pending's LIFO of released dots (mod.rs:556-587) stores, per
//     released dot, the mask of slots registered on it at release time — the
//     set can only shrink before it is popped (registrations are only made on
//     missing dots), so `mask & registered` at pop equals the reference's
//     PendingIndex::remove at pop;
//   * AEClock (threshold 0.9.1) per source: frontier + 32-bit exception window
//     in VGPRs;
//   * LDS holds only the cached deps of pending vertices (16 x DC words) and
//     the worklist: 88 words per lane at DC = 5, so 7 wavefronts fit a CU and
//     the 102,400 streams of the bench (1,600 wavefronts) are all resident;
//   * input: a 2-block register pipeline per lane (block = 4 steps = one
//     16-byte load per plane).  Every 4 iterations the wavefront refills: lanes
//     that have finished their block take the next one and every lane issues
//     the same 2 + DC loads (static count, clamped addresses), so the loads a
//     refill waits for were issued 4 iterations earlier, and a lane never waits
//     for its neighbours to finish a block (the lockstep of tier 3).
//
// A stream that outgrows 16 pending vertices, DC cached deps or a 32-bit clock
// window stops with FX_ERR_CAPACITY and is rerun at tier 1.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace lane {

constexpr uint32_t WV = 64;
constexpr uint32_t P = LANE_SLOTS;  // pending slots
constexpr uint32_t PM = (1u << P) - 1u;
constexpr uint32_t ROOTPAR = 15u;   // parent field of a DFS root
static_assert(LANE_SLOTS <= 15, "slots are nibbles, 15 marks the DFS root");
constexpr uint32_t WLC = P + 2;     // check_pending worklist capacity (u16 masks)
// saved state words per stream (any instantiation)
constexpr uint32_t S_CLK = 4 * P, S_DEP = S_CLK + 16, S_WL = S_DEP + 8 * P, S_SC = S_WL + (WLC + 1) / 2;
constexpr uint32_t WORDS = S_SC + 4;

enum : uint32_t { PH_IDLE = 0, PH_DFS = 1, PH_TRY = 2, PH_CHECK = 3, PH_SAVE = 4 };

// Tarjan word: id 5 | low 5 | visited epoch 8 | DFS parent 4 | parent's resume
// index 4 | Tarjan stack position 4 (the last three only while on the DFS path)
__device__ __forceinline__ uint32_t tw_id(uint32_t t) { return t & 31u; }
__device__ __forceinline__ uint32_t tw_low(uint32_t t) { return (t >> 5) & 31u; }
__device__ __forceinline__ uint32_t tw_ep(uint32_t t) { return (t >> 10) & 0xFFu; }
__device__ __forceinline__ uint32_t tw_par(uint32_t t) { return (t >> 18) & 15u; }
__device__ __forceinline__ uint32_t tw_fdi(uint32_t t) { return (t >> 23) & 15u; }
__device__ __forceinline__ uint32_t tw_mk(uint32_t id, uint32_t low, uint32_t ep, uint32_t par,
                                          uint32_t fdi) {
  return id | (low << 5) | (ep << 10) | (par << 18) | (fdi << 23);
}

// all-ones if bit q of v is set (one v_bfe_i32)
__device__ __forceinline__ uint32_t bitm(uint32_t v, uint32_t q) {
  return (uint32_t)((int32_t)(v << (31u - q)) >> 31);
}
// a[i] for a one-hot oh = 1 << i (arithmetic masks: a select chain is folded
// into a dynamically indexed load, which sends the array to scratch)
template <uint32_t N>
__device__ __forceinline__ uint32_t oget(const uint32_t (&a)[N], uint32_t oh) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t q = 0; q < N; ++q) r |= a[q] & bitm(oh, q);
  return r;
}
template <uint32_t N>
__device__ __forceinline__ void oput(uint32_t (&a)[N], uint32_t oh, uint32_t v) {
#pragma unroll
  for (uint32_t q = 0; q < N; ++q) {
    const uint32_t m = bitm(oh, q);
    a[q] = (v & m) | (a[q] & ~m);
  }
}
__device__ __forceinline__ uint32_t pick4(const uint4& v, uint32_t q) {
  return (v.x & (0u - (uint32_t)(q == 0))) | (v.y & (0u - (uint32_t)(q == 1))) |
         (v.z & (0u - (uint32_t)(q == 2))) | (v.w & (0u - (uint32_t)(q == 3)));
}

// cached dep word: (source - 1) 3 | seq 24 | slot hint + 1 (5 bits)
__device__ __forceinline__ uint32_t cdep_dot(uint32_t w) {
  return ((((w >> 24) & 7u) + 1u) << FX_SEQ_BITS) | (w & FX_SEQ_MASK);
}

template <uint32_t NS, uint32_t DC>
struct Lane {
  // LDS words of a lane (word w at lds[w * 64], so every lane hits its own bank);
  // the clock rows are u64 (frontier | window << 32) at clk[si * 64] so one
  // ds_read_b64 fetches a source's state
  static constexpr uint32_t L_CLK = 0;            // [NS] u64 clock rows (2 words each)
  static constexpr uint32_t L_DEP = 2 * NS;       // [P][DC] cached deps
  static constexpr uint32_t L_TW = L_DEP + P * DC;  // [P] Tarjan words
  static constexpr uint32_t L_REC = L_TW + P;     // [P] arrival index | ncached << 26
  static constexpr uint32_t L_WL = L_REC + P;     // worklist: u16 masks, two per word
  static constexpr uint32_t LW = L_WL + (WLC + 1) / 2;

  uint32_t* lds;
  uint64_t* clk;            // this lane's clock row 0 (row si at clk[si * 64])
  uint32_t sd[P], sw[P];    // slot dot / dot the slot is registered on (matched in parallel)
  uint32_t occ = 0, wmask = 0, tmask = 0;
  uint64_t stk = 0;         // Tarjan stack: slot nibbles, entry j at bits 4j
  uint32_t nts = 0;
  uint32_t k = 0, err = 0, epoch = 1, nwl = 0, cur = 0;
  uint32_t phase = PH_IDLE, root = 0, idc = 0, missing = 0;
  // current DFS frame: vertex, its id / low / stack position / parent / parent's resume index
  uint32_t fv = 0, fid = 0, flow = 0, fpos = 0, fpar = 0, fpdi = 0, fdi = 0, fnc = 0;
  uint32_t in_try = 0, emitted = 0;
  uint32_t smem = 0, sall = 0, sfirst = 0;  // SCC being saved: members left / all / next opens it
  uint32_t stream = 0, n = 0, steps = 0;
  uint32_t* order = nullptr;
  uint4 ob = make_uint4(0, 0, 0, 0);  // order words k & ~3 .. k - 1, not yet stored
  uint32_t* release = nullptr;
  // release words of the block of `cur` (steps cur & ~3 .. +3), stored when the
  // next block starts: a release in the block being read (every fast-path
  // singleton) lands in the buffer, older ones go straight to memory after it
  // was stored.  rlo: the block's first step this launch processed (NONE: no
  // block yet); the words below rlo belong to an earlier launch and are not
  // rewritten.
  uint4 rb = make_uint4(FX_RELEASE_NONE, FX_RELEASE_NONE, FX_RELEASE_NONE, FX_RELEASE_NONE);
  uint32_t rlo = 0xFFFFFFFFu;

  __device__ __forceinline__ uint32_t& w(uint32_t i) { return lds[i * WV]; }
  __device__ __forceinline__ uint32_t& tw(uint32_t sl) { return w(L_TW + sl); }
  __device__ __forceinline__ uint32_t& rec(uint32_t sl) { return w(L_REC + sl); }
  __device__ __forceinline__ size_t at(uint32_t step) const { return fx_index(step, stream, steps); }

  // ------------------------------------------------------------ clock
  // AEClock (threshold 0.9.1) per source: frontier f + exception bits above it
  __device__ __forceinline__ uint64_t& crow(uint32_t si) { return clk[(si < NS ? si : NS - 1) * WV]; }
  // AEClock::contains (tarjan.rs:131-132) given the source's row
  __device__ __forceinline__ bool row_contains(uint64_t row, uint32_t d) const {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    const uint32_t f = (uint32_t)row, wv = (uint32_t)(row >> 32);
    const uint32_t seq = d & FX_SEQ_MASK, off = seq - f - 1u;
    return si < n && (seq <= f || (off < 32u && ((wv >> (off & 31u)) & 1u)));
  }
  __device__ __forceinline__ bool contains(uint32_t d) { return row_contains(crow((d >> FX_SEQ_BITS) - 1u), d); }
  // AEClock::add (tarjan.rs:293)
  __device__ __forceinline__ void clk_add(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) { err = FX_ERR_DOT_RANGE; return; }
    uint64_t& row = crow(si);
    const uint64_t r0 = row;
    uint32_t f = (uint32_t)r0, wv = (uint32_t)(r0 >> 32);
    const uint32_t seq = d & FX_SEQ_MASK;
    if (seq <= f) return;
    const uint32_t off = seq - f - 1u;
    if (off >= 32u) { err = FX_ERR_CAPACITY; return; }
    if (off != 0) {
      wv |= 1u << off;
    } else {
      const uint32_t win = wv >> 1;               // bit j <-> seq f + 2 + j
      const uint32_t ones = __builtin_ctz(~win);  // top bit of win is 0 -> <= 31
      f = f + 1 + ones;
      wv = win >> ones;
    }
    row = (uint64_t)f | ((uint64_t)wv << 32);
  }

  // ------------------------------------------------------ slot table
  __device__ __forceinline__ uint32_t match(const uint32_t (&a)[P], uint32_t d) const {
    uint32_t m = 0;
#pragma unroll
    for (uint32_t q = 0; q < P; ++q) m |= (a[q] == d ? 1u : 0u) << q;
    return m;
  }
  // slot holding dot d (VertexIndex lookup), or -1
  __device__ __forceinline__ int find(uint32_t d) const {
    const uint32_t m = match(sd, d) & occ;
    return m ? (int)__builtin_ctz(m) : -1;
  }
  // slots registered on d (PendingIndex entry of d)
  __device__ __forceinline__ uint32_t waiters(uint32_t d) const { return match(sw, d) & wmask; }
  // slot with the smallest dot in m (canonical C2 / BTreeSet order), m != 0
  __device__ __forceinline__ uint32_t argmin(uint32_t m, uint32_t& dot) const {
    uint32_t bd = 0xFFFFFFFFu, bs = 0;
#pragma unroll
    for (uint32_t q = 0; q < P; ++q) {
      const uint32_t t = bitm(m, q) & (0u - (uint32_t)(sd[q] < bd));
      bd = (sd[q] & t) | (bd & ~t);
      bs = (q & t) | (bs & ~t);
    }
    dot = bd;
    return bs;
  }

  __device__ __forceinline__ void new_epoch() {
    epoch = (epoch + 1) & 0xFFu;
    if (epoch == 0) {
      for (uint32_t q = 0; q < P; ++q) tw(q) &= ~(0xFFu << 10);
      epoch = 1;
    }
  }

  __device__ __forceinline__ void wl_push(uint32_t m) {
    if (nwl >= WLC) { err = FX_ERR_CAPACITY; return; }
    uint32_t& x = w(L_WL + (nwl >> 1));
    x = (nwl & 1u) ? ((x & 0xFFFFu) | (m << 16)) : m;
    ++nwl;
  }
  __device__ __forceinline__ uint32_t wl_pop() {
    --nwl;
    return (w(L_WL + (nwl >> 1)) >> ((nwl & 1u) << 4)) & 0xFFFFu;
  }

  // order[at(k)] = w, stored 16 bytes at a time: the 4 order words of steps
  // 4j..4j+3 of one stream are contiguous in the tile layout, so a lane writes
  // whole 16-byte segments instead of four scattered words
  __device__ __forceinline__ void put_order(uint32_t w) {
    const uint32_t q = k & 3u;
    ob.x = q == 0 ? w : ob.x;
    ob.y = q == 1 ? w : ob.y;
    ob.z = q == 2 ? w : ob.z;
    ob.w = q == 3 ? w : ob.w;
    if (q == 3) *reinterpret_cast<uint4*>(order + at(k - 3)) = ob;
  }
  __device__ __forceinline__ void put_release(uint32_t r, uint32_t v) {
    if (rlo != 0xFFFFFFFFu && (r >> 2) == (cur >> 2) && r >= rlo) {
      const uint32_t q = r & 3u;
      rb.x = q == 0 ? v : rb.x;
      rb.y = q == 1 ? v : rb.y;
      rb.z = q == 2 ? v : rb.z;
      rb.w = q == 3 ? v : rb.w;
    } else {
      release[at(r)] = v;
    }
  }
  // stores the release words of the block of `cur`, steps [rlo, cur]: one
  // 16-byte store for a whole block, else word by word
  __device__ __forceinline__ void flush_release() {
    if (rlo == 0xFFFFFFFFu) return;
    const uint32_t b = cur & ~3u;
    if (rlo == b && cur == b + 3u) {
      *reinterpret_cast<uint4*>(release + at(b)) = rb;
    } else {
      for (uint32_t t = rlo; t <= cur; ++t) {
        const uint32_t q = t & 3u;
        release[at(t)] = q == 0 ? rb.x : q == 1 ? rb.y : q == 2 ? rb.z : rb.w;
      }
    }
    rlo = 0xFFFFFFFFu;
  }
  // stores the buffered words of an incomplete segment (kernel end)
  __device__ __forceinline__ void flush_order() {
    const uint32_t q = k & 3u, b = k - q;
    if (q > 0) order[at(b)] = ob.x;
    if (q > 1) order[at(b + 1)] = ob.y;
    if (q > 2) order[at(b + 2)] = ob.z;
  }

  __device__ __forceinline__ void emit(uint32_t r, uint32_t d, bool start) {
    if (k >= steps) { err = FX_ERR_ORDER_OVERFLOW; return; }
    put_order(r | (start ? FX_ORDER_SCC_START : 0u));
    put_release(r, cur);
    ++k;
    clk_add(d);
  }

  // VertexIndex::index(Vertex::new(dot, cmd, deps, time)) (index.rs:33-37).
  // Only the deps not executed now are kept (executed deps are ignored by
  // every later search, tarjan.rs:128-145, and the clock only grows), ascending.
  __device__ __forceinline__ int insert_vertex(uint32_t i, uint32_t d, const uint32_t (&dv)[DC], uint32_t notex) {
    const uint32_t fre = ~occ & PM;
    if (!fre) { err = FX_ERR_CAPACITY; return -1; }
    const uint32_t sl = __builtin_ctz(fre);
    uint32_t nc = 0;
#pragma unroll
    for (uint32_t j = 0; j < DC; ++j) {
      if ((notex >> j) & 1u) {
        const uint32_t dep = dv[j];
        w(L_DEP + sl * DC + nc) = ((((dep >> FX_SEQ_BITS) - 1u) & 7u) << 24) | (dep & FX_SEQ_MASK);
        ++nc;
      }
    }
    oput(sd, 1u << sl, d);
    rec(sl) = i | (nc << 26);
    tw(sl) = 0;
    occ |= 1u << sl;
    return (int)sl;
  }

  // ------------------------------ find_scc as a micro-op state machine
  __device__ __forceinline__ void dfs_start(uint32_t r, bool intry) {
    root = r;
    in_try = intry;
    emitted = 0;
    missing = 0;
    idc = 1;
    tw(r) = tw_mk(1, 1, tw_ep(tw(r)), ROOTPAR, 0);  // stack position 0
    stk = r;
    nts = 1;
    fv = r;
    fid = 1;
    flow = 1;
    fpos = 0;
    fpar = ROOTPAR;
    fpdi = 0;
    fdi = 0;
    fnc = rec(r) >> 26;
    phase = PH_DFS;
  }

  // finalize (tarjan.rs:60-93) + the caller's handling of the FinderInfo
  // (handle_add mod.rs:240-262, try_pending mod.rs:604-640)
  __device__ __forceinline__ void dfs_finish() {
    // reset ids of the vertices left on the stack; in try_pending a failed
    // search that saved no SCC marks them visited
    const bool mark = in_try && missing != 0 && !emitted;
    for (uint32_t j = 0; j < nts; ++j) {
      uint32_t& t = tw((uint32_t)(stk >> (4 * j)) & 15u);
      t = mark ? (epoch << 10) : (t & (0xFFu << 10));
    }
    nts = 0;
    if (missing) wmask |= 1u << root;  // index_pending(dot, missing) (mod.rs:525-554); sw written by the caller
    if (in_try) {
      if (!missing || emitted) new_epoch();  // visited.clear() (mod.rs:607, 621-623)
      phase = PH_TRY;
    } else {
      phase = PH_CHECK;
    }
  }

  // fv is closed and not an SCC root, or its SCC was saved: return to the
  // parent (low = min(low, child.low), tarjan.rs:211) or end the search
  __device__ __forceinline__ void dfs_return() {
    if (fv == root) {  // root done: Found
      dfs_finish();
      return;
    }
    const uint32_t p = fpar;
    const uint32_t tp = tw(p);
    fdi = fpdi;
    flow = min(tw_low(tp), flow);
    fid = tw_id(tp);
    fpar = tw_par(tp);
    fpdi = tw_fdi(tp);
    fpos = tp >> 27;
    fv = p;
    fnc = rec(p) >> 26;
  }

  // One iteration = one micro-op of this lane's executor.  The 12-wide
  // primitives (clock tests, slot match, registration match, argmin, clock
  // add) run once per iteration with operands chosen by the phase, so a
  // wavefront whose lanes sit in different phases pays each of them once,
  // not once per call site.
  //   IDLE + input  GraphExecutor::handle(Add) -> handle_add (mod.rs:213-275)
  //   DFS           one edge of strong_connect (tarjan.rs:96-316) after
  //                 skipping executed deps (tarjan.rs:128-145), or closing fv
  //   SAVE          save_scc (mod.rs:488-523): one SCC member, ascending dot
  //   TRY           try_pending (mod.rs:589-642): next waiter, ascending (C2)
  //   CHECK         check_pending (mod.rs:556-587): pop one released dot (LIFO)
  __device__ __forceinline__ void iterate(bool start, uint32_t i, uint32_t d, uint32_t h,
                                          const uint32_t (&dv)[DC], uint32_t dmax, bool at_commit) {
    // ---- A: operands
    const uint32_t nd = (h >> 24) & 31u, kind = h >> 29;
    const bool dfs = phase == PH_DFS;
    uint32_t vec[DC], dw[DC];
    uint32_t lo = 0, hi = 0;
    if (start) {
      if (rlo != 0xFFFFFFFFu && (i >> 2) != (cur >> 2)) flush_release();
      if (rlo == 0xFFFFFFFFu) {
        rb = make_uint4(FX_RELEASE_NONE, FX_RELEASE_NONE, FX_RELEASE_NONE, FX_RELEASE_NONE);
        rlo = i;
      }
      cur = i;
      nwl = 0;
      uint32_t e0 = 0, prev = 0;
      if (nd > dmax) e0 = FX_ERR_INVALID_ARG;
      if ((d >> FX_SEQ_BITS) - 1u >= n || (d & FX_SEQ_MASK) == 0) e0 = FX_ERR_DOT_RANGE;
#pragma unroll
      for (uint32_t j = 0; j < DC; ++j) {
        if (j < nd) {
          if (dv[j] <= prev) e0 = FX_ERR_DEPS_UNSORTED;
          if ((dv[j] >> FX_SEQ_BITS) - 1u >= 8u) e0 = FX_ERR_DOT_RANGE;
          prev = dv[j];
        }
      }
      err = e0;
      hi = nd;
    }
#pragma unroll
    for (uint32_t j = 0; j < DC; ++j) {
      dw[j] = dfs ? w(L_DEP + fv * DC + j) : 0u;
      vec[j] = start ? dv[j] : cdep_dot(dw[j]);
    }
    if (dfs) {
      lo = fdi;
      hi = fnc;
    }
    // ---- B: executed-clock tests (AEClock::contains, tarjan.rs:131-132)
    uint64_t rows[DC];
#pragma unroll
    for (uint32_t j = 0; j < DC; ++j) rows[j] = crow((vec[j] >> FX_SEQ_BITS) - 1u);
    uint32_t notex = 0;
#pragma unroll
    for (uint32_t j = 0; j < DC; ++j)
      if (j >= lo && j < hi && !(start && vec[j] == d) && !row_contains(rows[j], vec[j])) notex |= 1u << j;
    // ---- C: one slot lookup (VertexIndex, index.rs:18-51)
    const uint32_t jn = notex ? __builtin_ctz(notex) : 0u;
    uint32_t x1 = d;
#pragma unroll
    for (uint32_t j = 0; j < DC; ++j) x1 = j == jn && dfs ? vec[j] : x1;
    const uint32_t m1 = match(sd, x1) & occ;
    // ---- D: one argmin (waiter order C2 / SCC order)
    const uint32_t am = phase == PH_TRY ? tmask : phase == PH_SAVE ? smem : 0u;
    uint32_t bd = 0;
    const uint32_t bs = argmin(am ? am : 1u, bd);
    // ---- E: one emission (to_execute + executed clock + waiters)
    const bool fast = start && !err && !at_commit && kind != FX_KIND_INDEX_ONLY && !notex && !(occ && m1);
    const bool save = phase == PH_SAVE && am != 0;
    uint32_t wt = 0;
    if (fast || save) {
      const uint32_t r = fast ? i : (rec(bs) & 0x03FFFFFFu);
      const uint32_t ed = fast ? d : bd;
      if (k >= steps) {
        err = FX_ERR_ORDER_OVERFLOW;
      } else {
        put_order(r | (fast || sfirst ? FX_ORDER_SCC_START : 0u));
        put_release(r, cur);
        ++k;
        clk_add(ed);
        wt = waiters(ed);
      }
    }
    uint32_t swv = 0, swoh = 0;  // registration write (PendingIndex::index)
    // ---- F: transitions
    if (start) {
      if (at_commit && !err) {  // execute_at_commit bypass (executor.rs:72-73)
        if (k >= steps) {
          err = FX_ERR_ORDER_OVERFLOW;
        } else {
          put_order(i | FX_ORDER_SCC_START);
          put_release(i, i);
          ++k;
        }
      } else if (!err && occ && m1) {
        err = FX_ERR_DOUBLE_INDEX;  // mod.rs:233-237
      } else if (!err && kind == FX_KIND_INDEX_ONLY) {
        insert_vertex(i, d, dv, notex);
      } else if (fast) {  // a singleton SCC; check_pending([dot]) pops it at once
        if (wt && !err) {
          wmask &= ~wt;
          tmask = wt;
          new_epoch();
          phase = PH_TRY;
        }
      } else if (!err) {
        const int sl = insert_vertex(i, d, dv, notex);
        if (sl >= 0) dfs_start((uint32_t)sl, false);
      }
    } else if (dfs) {
      if (notex) {
        fdi = jn + 1;
        if (!m1) {  // missing: give up (tarjan.rs:148-157, shard_count == 1)
          missing = x1;
          swv = x1;
          swoh = 1u << root;
          dfs_finish();
        } else {
          const uint32_t x = __builtin_ctz(m1);
          const uint32_t tx = tw(x);
          if (tw_id(tx) == 0) {  // not visited: recurse (tarjan.rs:172-214)
            ++idc;
            tw(fv) = tw_mk(fid, flow, tw_ep(tw(fv)), fpar, fpdi) | (fpos << 27);
            tw(x) = tw_mk(idc, idc, tw_ep(tx), fv, fdi) | (nts << 27);
            stk |= (uint64_t)x << (4 * nts);
            fpos = nts;
            ++nts;
            fpar = fv;
            fpdi = fdi;
            fv = x;
            fid = idc;
            flow = idc;
            fdi = 0;
            fnc = rec(x) >> 26;
          } else {  // visited and on the stack (tarjan.rs:215-225)
            flow = min(flow, tw_id(tx));
          }
        }
      } else if (fid == flow) {  // SCC root (tarjan.rs:233-312): its members are stack [fpos, nts)
        uint32_t mem = 0;
        for (uint32_t j = fpos; j < nts; ++j) mem |= 1u << ((uint32_t)(stk >> (4 * j)) & 15u);
        smem = mem;
        sall = mem;
        sfirst = 1;
        phase = PH_SAVE;
      } else {
        dfs_return();
      }
    } else if (save) {
      sfirst = 0;
      if (wt) wl_push(wt);
      smem &= ~(1u << bs);
      if (!smem && !err) {  // the SCC is out: drop it from the index and the stack
        occ &= ~sall;
        wmask &= ~sall;
        tmask &= ~sall;
        nts = fpos;
        stk &= (fpos ? (~0ull >> (64 - 4 * fpos)) : 0ull);
        emitted = 1;
        phase = PH_DFS;
        dfs_return();
      }
    } else if (phase == PH_TRY) {
      if (!tmask) {
        phase = PH_CHECK;
      } else {
        tmask &= ~(1u << bs);
        if (tw_ep(tw(bs)) != epoch) dfs_start(bs, true);  // else visited: skipped, not re-registered
      }
    }
    if (phase == PH_CHECK) {
      if (nwl == 0 || !wmask) {
        nwl = 0;
        phase = PH_IDLE;
      } else {
        const uint32_t t = wl_pop() & wmask;
        if (t) {
          wmask &= ~t;  // PendingIndex::remove(x)
          tmask = t;
          new_epoch();  // try_pending's fresh `visited`
          phase = PH_TRY;
        }
      }
    }
    oput(sw, swoh, swv);
    if (err) phase = PH_IDLE;
  }

  // --------------------------------------------------- state save/restore
  // Saved layout (lane-interleaved, word w of lane l at block[w * 64 + l]) is
  // the same for every instantiation: slots, 8 clock sources, 8 deps per slot.
  __device__ __forceinline__ void load_state(const uint32_t* g) {  // g = block + lane
#pragma unroll
    for (uint32_t q = 0; q < P; ++q) {
      sd[q] = g[(0 * P + q) * WV];
      sw[q] = g[(1 * P + q) * WV];
      rec(q) = g[(2 * P + q) * WV];
      tw(q) = g[(3 * P + q) * WV];
    }
#pragma unroll
    for (uint32_t q = 0; q < NS; ++q)
      clk[q * WV] = (uint64_t)g[(S_CLK + q) * WV] | ((uint64_t)g[(S_CLK + 8 + q) * WV] << 32);
    for (uint32_t sl = 0; sl < P; ++sl)
      for (uint32_t j = 0; j < DC; ++j) w(L_DEP + sl * DC + j) = g[(S_DEP + sl * 8 + j) * WV];
    for (uint32_t q = 0; q < (WLC + 1) / 2; ++q) w(L_WL + q) = g[(S_WL + q) * WV];
    occ = g[S_SC * WV] & 0xFFFFu;
    wmask = g[S_SC * WV] >> 16;
    k = g[(S_SC + 1) * WV];
    err = g[(S_SC + 2) * WV] & 0xFFFFu;
    epoch = g[(S_SC + 2) * WV] >> 16;
  }
  __device__ __forceinline__ void save_state(uint32_t* g) {
#pragma unroll
    for (uint32_t q = 0; q < P; ++q) {
      g[(0 * P + q) * WV] = sd[q];
      g[(1 * P + q) * WV] = sw[q];
      g[(2 * P + q) * WV] = rec(q);
      g[(3 * P + q) * WV] = tw(q);
    }
#pragma unroll
    for (uint32_t q = 0; q < NS; ++q) {
      g[(S_CLK + q) * WV] = (uint32_t)clk[q * WV];
      g[(S_CLK + 8 + q) * WV] = (uint32_t)(clk[q * WV] >> 32);
    }
    for (uint32_t sl = 0; sl < P; ++sl)
      for (uint32_t j = 0; j < DC; ++j) g[(S_DEP + sl * 8 + j) * WV] = w(L_DEP + sl * DC + j);
    for (uint32_t q = 0; q < (WLC + 1) / 2; ++q) g[(S_WL + q) * WV] = w(L_WL + q);
    g[S_SC * WV] = occ | (wmask << 16);
    g[(S_SC + 1) * WV] = k;
    g[(S_SC + 2) * WV] = (err & 0xFFFFu) | (epoch << 16);
  }
};

// Two waves per SIMD where the LDS allows it: the 8-cached-deps builds take
// 35-37 KB of LDS per wavefront, so a CU holds four (one per SIMD) whatever
// the register count, and they declare one (their 256 VGPRs then cost nothing)
template <uint32_t NS, uint32_t DC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DC <= 5 ? 2 : 1)))
void k_graph_lane(KArgs a) {
  using L = Lane<NS, DC>;
  constexpr uint32_t NP = 2 + DC;  // planes per block: dot, hdr, deps
  __shared__ __attribute__((aligned(16))) uint32_t smem[L::LW * WV];
  static_assert(L::LW <= 160, "LDS words per lane");
  const uint32_t lane = threadIdx.x;
  const uint32_t gl = blockIdx.x * WV + lane;
  const uint32_t nl = a.lanes_dev ? min(a.num_lanes, *a.lanes_dev) : a.num_lanes;
  if (blockIdx.x * WV >= nl) return;  // wavefront past a device-side lane count
  // map entries >= S are padding lanes (FX_TIER_SPLIT's ragged last tile)
  const uint32_t s0 = gl < nl ? (a.stream_map ? a.stream_map[gl] : gl) : 0xFFFFFFFFu;
  const bool active = s0 < a.S;
  const uint32_t s = active ? s0 : 0u;
  const uint32_t len = active ? (a.lengths ? min(a.lengths[s], a.steps) : a.steps) : 0u;
  uint32_t* gst = a.state ? a.state + (size_t)blockIdx.x * WORDS * WV + lane : nullptr;

  L e;
  e.lds = smem + lane;
  e.clk = reinterpret_cast<uint64_t*>(smem + L::L_CLK * WV) + lane;
  e.stream = s;
  e.n = a.n;
  e.steps = a.steps;
  e.order = a.order;
  e.release = a.release;
#pragma unroll
  for (uint32_t q = 0; q < P; ++q) e.sd[q] = e.sw[q] = 0;
  if (a.flags & FX_FLAG_INIT) {
#pragma unroll
    for (uint32_t q = 0; q < NS; ++q)
      e.clk[q * WV] = (a.init_frontier && active) ? a.init_frontier[(size_t)s * 8 + q] : 0u;
  } else if (active) {
    e.load_state(gst);
    // a resumed stream part-way through a 16-byte order segment: the previous
    // launch stored its first words (flush_order)
    if (e.k & 3u) e.ob = *reinterpret_cast<const uint4*>(a.order + e.at(e.k & ~3u));
  }
  if (!active) e.err = FX_ERR_INVALID_ARG;  // idle lane (its loads read stream 0)

  const bool at_commit = (a.flags & FX_FLAG_EXECUTE_AT_COMMIT) != 0;
  const uint32_t dmax = a.dmax;
  const uint32_t steps4 = (a.steps + 3) >> 2;
  const size_t soff = (size_t)(s >> 6) * steps4 * 256 + ((s & 63u) << 2);
  const uint32_t lim = min(len, a.step_end);
  const uint32_t b_last = a.step_end ? (a.step_end - 1) >> 2 : 0u;
  const size_t plane = dmax ? a.plane : 0;
  const uint32_t jlast = dmax ? dmax - 1 : 0;
  // Refill loads go through range-checked buffer descriptors (one per plane,
  // built from kernel arguments only, so they stay in SGPRs): a lane that keeps
  // its block passes an out-of-range offset, and the load returns zeros
  // without a memory request.  The instruction count stays static (vmcnt(N),
  // not vmcnt(0)), and only lanes that moved to a new block fetch it.
  const uint32_t pbytes = (uint32_t)min(a.plane * 4, (size_t)0xFFFFFFF0u);
  const uint32_t* depb = dmax ? a.deps : a.dot;
  __amdgpu_buffer_rsrc_t rs[NP];
  rs[0] = __builtin_amdgcn_make_buffer_rsrc((void*)a.dot, 0, (int)pbytes, 0x00020000);
  rs[1] = __builtin_amdgcn_make_buffer_rsrc((void*)a.hdr, 0, (int)pbytes, 0x00020000);
#pragma unroll
  for (uint32_t j = 0; j < DC; ++j)
    rs[2 + j] = __builtin_amdgcn_make_buffer_rsrc((void*)(depb + (size_t)min(j, jlast) * plane), 0,
                                                  (int)pbytes, 0x00020000);
  constexpr uint32_t OOB = 0xFFFFFFF0u;
  const uint32_t sbyte = (uint32_t)(soff * 4);
  auto boff = [&](uint32_t b) -> uint32_t { return sbyte + min(b, b_last) * 1024u; };
  auto ld = [&](uint32_t off, uint32_t p) -> uint4 {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs[p], off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };

  // Pipeline: c = block blk (readable); x = block blk + 1 (dot / hdr, and the
  // dep planes its headers need); y = dot / hdr of block blk + 2.  A lane that
  // moves to the next block issues the dep loads of its new x, skipping the
  // planes no Add of that block uses (the headers came one block earlier, in
  // y), and the dot / hdr loads of its new y, into t; the next refill merges t
  // (tl: t holds this lane's loads).  Sparse streams so read ~3 of the 2 + DC
  // planes.
  uint32_t i = a.step_begin;
  uint32_t blk = i >> 2;
  uint4 c[NP], x[NP], y[2], t[NP];
#pragma unroll
  for (uint32_t p = 0; p < NP; ++p) c[p] = ld(boff(blk), p);
#pragma unroll
  for (uint32_t p = 0; p < NP; ++p) x[p] = ld(boff(blk + 1), p);
#pragma unroll
  for (uint32_t p = 0; p < 2; ++p) y[p] = ld(boff(blk + 2), p);
#pragma unroll
  for (uint32_t p = 0; p < NP; ++p) t[p] = make_uint4(0, 0, 0, 0);
  uint32_t tl = 0;  // all-ones: t holds the loads of the last refill
  // Drift bound: a lane moves to block blk + 1 only while that block is fewer
  // than `drift` blocks past the slowest live lane's, so the lanes of a
  // wavefront read (and write) each 1 KiB tile row within a short window and
  // the row's cache lines are fetched once instead of once per straggler.
  const uint32_t drift = a.drift ? a.drift : 0xFFFFFFFFu;
  auto mset = [](uint4& d, const uint4& v, uint32_t m) {
    d.x = (v.x & m) | (d.x & ~m);
    d.y = (v.y & m) | (d.y & ~m);
    d.z = (v.z & m) | (d.z & ~m);
    d.w = (v.w & m) | (d.w & ~m);
  };

  for (uint32_t it = 0;; ++it) {
    if ((it & 3u) == 0) {
      const bool live = e.phase != PH_IDLE || (i < lim && !e.err);
      if (!__any(live)) break;
      uint32_t lo = (i < lim && !e.err) ? (i >> 2) : 0xFFFFFFFFu;
      if (drift != 0xFFFFFFFFu) {
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) lo = min(lo, (uint32_t)__shfl_xor((int)lo, (int)o));
      }
      // merge the last refill's loads (masks, not selects: a select of two
      // arrays becomes a select of their addresses)
#pragma unroll
      for (uint32_t p = 2; p < NP; ++p) mset(x[p], t[p], tl);
      mset(y[0], t[0], tl);
      mset(y[1], t[1], tl);
      const bool sh = (i >> 2) > blk && (drift == 0xFFFFFFFFu || lo == 0xFFFFFFFFu || blk + 1 < lo + drift);
      blk += sh ? 1u : 0u;
      const uint32_t m = 0u - (uint32_t)sh;
#pragma unroll
      for (uint32_t p = 0; p < NP; ++p) mset(c[p], x[p], m);
      mset(x[0], y[0], m);
      mset(x[1], y[1], m);
      tl = m;
      // deps the new x block's Adds carry (its headers are in x[1] now)
      const uint4 h = x[1];
      const uint32_t nd = max(max(FX_HDR_ND(h.x), FX_HDR_ND(h.y)), max(FX_HDR_ND(h.z), FX_HDR_ND(h.w)));
      const uint32_t offx = sh ? boff(blk + 1) : OOB, offy = sh ? boff(blk + 2) : OOB;
#pragma unroll
      for (uint32_t p = 0; p < 2; ++p) t[p] = ld(offy, p);
#pragma unroll
      for (uint32_t j = 0; j < DC; ++j) t[2 + j] = ld(j < nd ? offx : OOB, 2 + j);
    }
    // a lane consumes at most one step per iteration, so between two refills
    // it never runs past the end of x; it only waits (at most 3 iterations)
    // when a slow step left it part-way through c at the previous refill
    if (a.dbg) {
      const uint32_t ph = e.phase;
      const bool stall = ph == PH_IDLE && i < lim && !e.err && (i >> 2) != blk;
      const bool idle = ph == PH_IDLE && !(i < lim && !e.err);
      a.dbg[gl * 8 + 0] += 1;
      a.dbg[gl * 8 + 1] += stall ? 1u : 0u;
      a.dbg[gl * 8 + 2] += idle ? 1u : 0u;
      a.dbg[gl * 8 + 3] += ph == PH_DFS ? 1u : 0u;
      a.dbg[gl * 8 + 4] += ph == PH_TRY ? 1u : 0u;
      a.dbg[gl * 8 + 5] += ph == PH_CHECK ? 1u : 0u;
      a.dbg[gl * 8 + 6] += ph == PH_SAVE ? 1u : 0u;
    }
    const bool start = e.phase == PH_IDLE && i < lim && !e.err && (i >> 2) == blk;
    const uint32_t q = i & 3u;
    uint32_t dv[DC];
#pragma unroll
    for (uint32_t j = 0; j < DC; ++j) dv[j] = pick4(c[2 + j], q);
    if (start || e.phase != PH_IDLE) e.iterate(start, i, pick4(c[0], q), pick4(c[1], q), dv, dmax, at_commit);
    i += start ? 1u : 0u;
  }

  if (!active) return;
  e.flush_release();
  // vertices still pending have no release step (yet)
  for (uint32_t m = e.occ; m; m &= m - 1)
    a.release[e.at(e.rec(__builtin_ctz(m)) & 0x03FFFFFFu)] = FX_RELEASE_NONE;
  e.flush_order();
  a.nexec[s] = e.k;
  a.err[s] = e.err;
  if (a.flags & FX_FLAG_SAVE_STATE) e.save_state(gst);
}

template <uint32_t NS, uint32_t DC>
static int launch_t(const KArgs& a, hipStream_t stream) {
  const uint32_t blocks = (a.num_lanes + WV - 1) / WV;
  if (blocks == 0) return FX_OK;
  hipLaunchKernelGGL((k_graph_lane<NS, DC>), dim3(blocks), dim3(WV), 0, stream, a);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

static uint32_t decode(const uint32_t* block, uint32_t lane, uint32_t* dots, uint32_t* waits,
                       uint32_t cap) {
  const uint32_t* g = block + lane;
  const uint32_t s0 = g[(size_t)S_SC * WV];
  const uint32_t occ = s0 & 0xFFFFu, wm = s0 >> 16;
  uint32_t c = 0;
  for (uint32_t sl = 0; sl < P; ++sl) {
    if (!((occ >> sl) & 1u)) continue;
    if (c < cap) {
      dots[c] = g[(0 * P + sl) * WV];
      waits[c] = ((wm >> sl) & 1u) ? g[(1 * P + sl) * WV] : 0u;
    }
    ++c;
  }
  return c;
}

// drift bound of k_graph_lane in blocks (FX_LANE_DRIFT overrides; 0 = unbounded)
constexpr uint32_t DEFAULT_DRIFT = 3;

// instantiation for a batch: sources rounded to 5 / 8, deps to 3 / 5 / 8
#define FX_LANE_DISPATCH(F, ...)                                         \
  do {                                                                   \
    if (n <= 5) {                                                        \
      if (dmax <= 3) return F<5, 3>(__VA_ARGS__);                        \
      if (dmax <= 5) return F<5, 5>(__VA_ARGS__);                        \
      return F<5, 8>(__VA_ARGS__);                                       \
    }                                                                    \
    if (dmax <= 3) return F<8, 3>(__VA_ARGS__);                          \
    if (dmax <= 5) return F<8, 5>(__VA_ARGS__);                          \
    return F<8, 8>(__VA_ARGS__);                                         \
  } while (0)

}  // namespace lane

static int launch_lane_d(const KArgs& a0, hipStream_t stream) {
  static const uint32_t drift = [] {
    const char* e = getenv("FX_LANE_DRIFT");
    return e ? (uint32_t)atoi(e) : lane::DEFAULT_DRIFT;
  }();
  KArgs a = a0;
  a.drift = drift;
  const uint32_t n = a.n, dmax = a.dmax;
  FX_LANE_DISPATCH(lane::launch_t, a, stream);
}

int launch_lane(const KArgs& a0, hipStream_t stream) {
  if (a0.dmax > LANE_MAX_DEPS || a0.n > 8) return FX_ERR_INVALID_ARG;
  if (a0.plane * 4 > LANE_MAX_PLANE_BYTES) return FX_ERR_INVALID_ARG;  // 32-bit buffer offsets
  if (!getenv("FX_LANE_DEBUG")) return launch_lane_d(a0, stream);
  // diagnostics: per-lane iteration counters, summarised on stderr
  KArgs a = a0;
  const size_t nw = (size_t)(a.num_lanes + 63) / 64 * 64 * 8;
  if (hipMalloc((void**)&a.dbg, nw * 4) != hipSuccess) return FX_ERR_HIP;
  (void)hipMemsetAsync(a.dbg, 0, nw * 4, stream);
  int st = launch_lane_d(a, stream);
  std::vector<uint32_t> h(nw);
  (void)hipMemcpyAsync(h.data(), a.dbg, nw * 4, hipMemcpyDeviceToHost, stream);
  (void)hipStreamSynchronize(stream);
  (void)hipFree(a.dbg);
  double tot[8] = {0};
  uint32_t mx = 0;
  for (size_t l = 0; l < a.num_lanes; ++l) {
    for (int c = 0; c < 8; ++c) tot[c] += h[l * 8 + c];
    mx = std::max(mx, h[l * 8 + 0]);
  }
  const double steps = (double)a.num_lanes * (a.step_end - a.step_begin);
  fprintf(stderr, "[lane dbg] per Add: iters %.2f stall %.2f idle %.2f dfs %.2f try %.2f check %.2f save %.2f; max iters/lane %u\n",
          tot[0] / steps, tot[1] / steps, tot[2] / steps, tot[3] / steps, tot[4] / steps, tot[5] / steps,
          tot[6] / steps, mx);
  return st;
}

uint32_t lane_state_words_per_stream() { return lane::WORDS; }

size_t lane_state_bytes(uint32_t streams) {
  return (size_t)((streams + 63) / 64) * 64 * lane::WORDS * 4;
}

uint32_t lane_decode_pending(const uint32_t* block, uint32_t lane, uint32_t* dots, uint32_t* waits,
                             uint32_t cap) {
  return lane::decode(block, lane, dots, waits, cap);
}

}  // namespace fx
