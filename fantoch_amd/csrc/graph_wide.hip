// graph_wide.hip — the wide tiers: one wavefront per stream, the dependency
// graph in table form (LDS, or HBM for the largest), for streams whose pending
// set outgrows the register/LDS slot tables of tiers 0-6 (BASELINE configs[3]:
// 64 clients per region at 100 % conflicts, SCCs of hundreds of commands and
// hundreds of pending vertices).
//
// It restates DependencyGraph (fantoch_ps/src/executor/graph/mod.rs:213-642)
// and TarjanSCCFinder (tarjan.rs:60-316) over explicit tables, with the
// canonical orders of every other tier (C1 deps ascending, C2 waiters
// ascending):
//   vertex table  dot, arrival index, waited-on dot, Tarjan id / low, marks
//                 (on-stack bit, visited epoch of try_pending's skip rule)
//   dot index     per source, seq mod Q -> vertex (VertexIndex, index.rs:18-51)
//   executed clock per source: frontier + a ring bitmap of W seqs (AEClock)
//   stacks        Tarjan stack, DFS frames, released-dots worklist (LIFO,
//                 check_pending), sorted waiters (try_pending)
// Control flow is wave-uniform; the lanes work together where the reference
// iterates a set: collecting a released dot's waiters (a ballot per 64
// vertices) and ordering them and every SCC by dot (parallel rank sort).
// Capacity (vertices, index collisions, clock window) is reported as
// FX_ERR_CAPACITY, and fx_batch_run_tiered escalates LDS -> HBM tables.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace wide {

constexpr uint32_t NONE = 0xFFFFFFFFu;
enum : uint32_t { FOUND = 0, MISSING = 1, NOT_PENDING = 2 };

constexpr uint32_t PW = 64;  // partial replication: parents a vertex may wait on at once

struct Lay {  // table layout (u32 words) for capacity P, index Q per source, W-bit clock windows
  uint32_t P, Q, WB, n, D;
  uint32_t vdot, vrec, vnd, vdeps, vwait, vid, vlow, vmark, vfree, tstk, fv, fi, wl, tl, tmp, hidx, front, bits, sc, words;
  // partial replication only (0 words otherwise): per-vertex parent lists
  // (count + PW dots), per-frame missing-dep counts, the collected missing deps
  uint32_t vwn, vwl, fm, ml;
  __host__ __device__ void make(uint32_t P_, uint32_t Q_, uint32_t WB_, uint32_t n_, uint32_t D_,
                                bool partial = false) {
    P = P_;
    Q = Q_;
    WB = WB_;
    n = n_;
    D = D_;
    uint32_t o = 0;
    vdot = o; o += P;
    vrec = o; o += P;
    vnd = o; o += P;      // deps of the vertex (copied from the planes at index time:
    vdeps = o; o += P * D;  // the DFS then never waits on HBM)
    vwait = o; o += P;
    vid = o; o += P;
    vlow = o; o += P;
    vmark = o; o += P;
    vfree = o; o += P;
    tstk = o; o += P;
    fv = o; o += P;
    fi = o; o += P;
    wl = o; o += 2 * P;
    tl = o; o += P;
    tmp = o; o += P;
    hidx = o; o += n * Q;
    front = o; o += 8;
    bits = o; o += n * WB;
    sc = o; o += 4;  // saved scalars of a resumable (HBM) stream: nfree, nexec, epoch
    vwn = o; o += partial ? P : 0;
    vwl = o; o += partial ? P * PW : 0;
    fm = o; o += partial ? P : 0;
    ml = o; o += partial ? P : 0;
    words = o;
  }
};

struct W {
  KArgs a;
  Lay L;
  uint32_t* m;  // table memory (LDS or this stream's HBM block)
  uint32_t lid, s;
  uint32_t err = 0;
  uint32_t nfree = 0, tsp = 0, fsp = 0, nwl = 0, idc = 0, epoch = 1, nexec = 0, step = 0;
  uint32_t t_now = 0;
  bool partial = false;  // FX_FLAG_PARTIAL
  uint32_t nml = 0;      // missing deps collected by a first search (partial)

  __device__ __forceinline__ uint32_t& at(uint32_t base, uint32_t i) { return m[base + i]; }
  __device__ __forceinline__ void put(uint32_t base, uint32_t i, uint32_t v) {
    if (lid == 0) m[base + i] = v;
  }
  __device__ __forceinline__ uint32_t rd(uint32_t base, uint32_t i) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)m[base + i]);
  }
  // record fields of arrival r
  __device__ __forceinline__ size_t ix(uint32_t r) const { return fx_index(r, s, a.steps); }
  __device__ __forceinline__ uint32_t ndeps(uint32_t r) const { return min(FX_HDR_ND(a.hdr[ix(r)]), a.dmax); }
  __device__ __forceinline__ uint32_t dep(uint32_t r, uint32_t j) const { return a.deps[j * a.plane + ix(r)]; }

  // ------------------------------------------------------------ clock
  // frv: the frontiers in lanes (lane s = source s + 1), loaded by find_scc
  // and kept in step by clock_add, so the per-edge check reads no LDS word
  // unless the seq is above the frontier
  uint32_t frv = 0;
  __device__ __forceinline__ bool contains(uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
    if (src < 1 || src > L.n) return false;
    const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)frv, (int)(src - 1));
    if (sq <= f) return true;
    const uint32_t off = sq - f - 1;
    if (off >= L.WB * 32u) return false;
    const uint32_t b = sq & (L.WB * 32u - 1u);
    return (rd(L.bits, (src - 1) * L.WB + (b >> 5)) >> (b & 31u)) & 1u;
  }
  __device__ __forceinline__ void clock_add(uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
    if (src < 1 || src > L.n) { err = FX_ERR_DOT_RANGE; return; }
    uint32_t f = rd(L.front, src - 1);
    if (sq <= f) return;
    if (sq - f - 1 >= L.WB * 32u) { err = FX_ERR_CAPACITY; return; }
    const uint32_t mask = L.WB * 32u - 1u;
    const uint32_t b = sq & mask, wi = (src - 1) * L.WB + (b >> 5);
    put(L.bits, wi, rd(L.bits, wi) | (1u << (b & 31u)));
    // advance the frontier over contiguous seqs, clearing their bits
    for (;;) {
      const uint32_t nb = (f + 1) & mask, nw = (src - 1) * L.WB + (nb >> 5);
      const uint32_t word = rd(L.bits, nw);
      if (!((word >> (nb & 31u)) & 1u)) break;
      put(L.bits, nw, word & ~(1u << (nb & 31u)));
      ++f;
    }
    put(L.front, src - 1, f);
    if (lid == src - 1) frv = f;
  }

  // ------------------------------------------------------- vertex index
  __device__ __forceinline__ uint32_t hslot(uint32_t d) const {
    return (FX_DOT_SRC(d) - 1) * L.Q + (FX_DOT_SEQ(d) & (L.Q - 1u));
  }
  // an index word is (vertex + 1) | seq / Q << 16: it names its dot without
  // a read of the vertex table (the slot gives the source and seq mod Q)
  __device__ __forceinline__ uint32_t htag(uint32_t d) const {
    return (FX_DOT_SEQ(d) >> __builtin_ctz(L.Q)) << 16;
  }
  __device__ __forceinline__ uint32_t find(uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d);
    if (src < 1 || src > L.n) return NONE;
    const uint32_t w = rd(L.hidx, hslot(d));
    return ((w & 0xFFFFu) != 0 && (w & 0xFFFF0000u) == htag(d)) ? (w & 0xFFFFu) - 1u : NONE;
  }

  // ------------------------------------------------------- emission
  // save_scc (mod.rs:488-523): members ascending by dot (SCC = BTreeSet)
  __device__ void save_scc(uint32_t base, uint32_t cnt) {
    // members are tstk[base .. base + cnt): rank-sort their dots in the lanes
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
      const uint32_t i = i0 + lid;
      if (i < cnt) {
        const uint32_t v = at(L.tstk, base + i), d = at(L.vdot, v);
        uint32_t r = 0;
        for (uint32_t k = 0; k < cnt; ++k) r += at(L.vdot, at(L.tstk, base + k)) < d ? 1u : 0u;
        at(L.tmp, r) = v;
      }
    }
    __syncthreads();
    for (uint32_t r = 0; r < cnt; ++r) {
      const uint32_t v = rd(L.tmp, r);
      const uint32_t d = rd(L.vdot, v), rec = rd(L.vrec, v);
      if (nexec >= a.steps) { err = FX_ERR_ORDER_OVERFLOW; return; }
      if (lid == 0) {
        a.order[ix(nexec)] = rec | (r == 0 ? FX_ORDER_SCC_START : 0u);
        a.release[ix(rec)] = step;
      }
      ++nexec;
      // remove from the index, free the slot; push to the released list
      put(L.hidx, hslot(d), 0u);
      put(L.vdot, v, 0u);
      put(L.vwait, v, 0u);
      if (partial) put(L.vwn, v, 0u);
      put(L.vfree, nfree++, v);
      if (nwl >= 2 * L.P) { err = FX_ERR_CAPACITY; return; }
      put(L.wl, nwl++, d);
    }
  }

  // find_scc (mod.rs:409-486) + strong_connect (tarjan.rs:96-316) + finalize
  // (tarjan.rs:60-93).  Released dots are appended to the worklist; on a
  // missing dep, *missing = it and the stack members are marked visited with
  // `mark_epoch` (0 = do not mark).
  // With partial replication, the first search of an Add (collect = true)
  // records every missing dep in ml[0, nml) and keeps going; a vertex whose
  // subtree misses deps is no SCC root (tarjan.rs:148-166, 198-200, 233).
  __device__ uint32_t find_scc(uint32_t root_dot, uint32_t* missing, uint32_t mark_epoch, bool* saved,
                               bool collect = false) {
    *saved = false;
    const uint32_t root = find(root_dot);
    if (root == NONE) return NOT_PENDING;
    idc = 1;
    tsp = 0;
    fsp = 0;
    nml = 0;
    frv = lid < L.n ? at(L.front, lid) : 0u;
    put(L.vid, root, 1);
    put(L.vlow, root, 1);
    put(L.vmark, root, rd(L.vmark, root) | 1u);
    put(L.tstk, tsp++, root);
    put(L.fv, fsp, root);
    if (partial) put(L.fm, fsp, 0);
    ++fsp;
    // the top frame lives in registers: its vertex, next dep, id, low, dot,
    // dep count and dep row (lane j = dep j); a frame's position and low go
    // to the tables only when it recurses, and come back when it resumes
    uint32_t cv = root, ci = 0, cid = 1, clow = 1, cdot = root_dot;
    uint32_t cnd = rd(L.vnd, root);
    uint32_t drow = lid < cnd ? at(L.vdeps, root * L.D + lid) : 0u;
    uint32_t result = FOUND;
    while (fsp && !err) {
      if (ci < cnd) {
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)drow, (int)ci);
        ++ci;
        // the clock-window word and the index word both depend on d alone:
        // read them together (one LDS round trip), then decide
        const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
        const bool inr = src >= 1 && src <= L.n;
        const uint32_t si = inr ? src - 1 : 0u;
        const uint32_t bb = sq & (L.WB * 32u - 1u);
        const uint32_t hw = rd(L.hidx, si * L.Q + (sq & (L.Q - 1u)));
        const uint32_t bw = rd(L.bits, si * L.WB + (bb >> 5));
        const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)frv, (int)si);
        const bool executed = inr && (sq <= f || (sq - f - 1u < L.WB * 32u && ((bw >> (bb & 31u)) & 1u)));
        if (d == cdot || executed) continue;  // self or executed (tarjan.rs:128-145)
        const uint32_t w = (inr && (hw & 0xFFFFu) != 0 && (hw & 0xFFFF0000u) == htag(d)) ? (hw & 0xFFFFu) - 1u : NONE;
        if (w == NONE) {
          if (collect) {  // partial replication, first search (tarjan.rs:158-166)
            bool seen = false;
            for (uint32_t k = 0; k < nml && !seen; ++k) seen = rd(L.ml, k) == d;
            if (!seen) {
              if (nml >= L.P) { err = FX_ERR_CAPACITY; break; }
              put(L.ml, nml++, d);
            }
            put(L.fm, fsp - 1, rd(L.fm, fsp - 1) + 1u);
            continue;
          }
          *missing = d;  // missing (tarjan.rs:148-157)
          result = MISSING;
          break;
        }
        const uint32_t idw = rd(L.vid, w), mkw = rd(L.vmark, w);  // both reads in flight at once
        if (idw == 0) {  // recurse
          put(L.fi, fsp - 1, ci);
          put(L.vlow, cv, clow);
          ++idc;
          put(L.vid, w, idc);
          put(L.vmark, w, mkw | 1u);
          put(L.tstk, tsp++, w);
          put(L.fv, fsp, w);
          if (partial) put(L.fm, fsp, 0);
          ++fsp;
          cv = w;
          ci = 0;
          cid = idc;
          clow = idc;
          cdot = d;
          cnd = rd(L.vnd, w);
          drow = lid < cnd ? at(L.vdeps, w * L.D + lid) : 0u;
        } else if (mkw & 1u) {  // on the stack
          clow = min(clow, idw);
        }
        continue;
      }
      // cv finished
      const uint32_t lowv = clow;
      const uint32_t mcount = partial ? rd(L.fm, fsp - 1) : 0u;
      if (mcount == 0 && cid == lowv) {  // SCC root: pop the members (tarjan.rs:233-312)
        uint32_t base = tsp;
        while (base > 0) {
          --base;
          const uint32_t x = rd(L.tstk, base);
          put(L.vmark, x, rd(L.vmark, x) & ~1u);
          clock_add(rd(L.vdot, x));  // executed_clock.add at pop time (tarjan.rs:293)
          if (x == cv) break;
        }
        const uint32_t cnt = tsp - base;
        save_scc(base, cnt);
        tsp = base;
        *saved = true;
      }
      --fsp;
      if (fsp) {  // resume the parent frame (tarjan.rs:211: low = min(low, dep low))
        const uint32_t p = rd(L.fv, fsp - 1);
        cv = p;
        ci = rd(L.fi, fsp - 1);
        cid = rd(L.vid, p);
        clow = min(rd(L.vlow, p), lowv);
        cdot = rd(L.vdot, p);
        cnd = rd(L.vnd, p);
        drow = lid < cnd ? at(L.vdeps, p * L.D + lid) : 0u;
        if (mcount) put(L.fm, fsp - 1, rd(L.fm, fsp - 1) + mcount);  // tarjan.rs:198-200
      } else if (mcount) {
        result = MISSING;  // NotFound -> MissingDependencies(collected) (mod.rs:478-484)
      }
    }
    // finalize: ids of the vertices left on the stack; failed searches mark them visited
    for (uint32_t k = 0; k < tsp; ++k) {
      const uint32_t x = rd(L.tstk, k);
      put(L.vid, x, 0);
      if (mark_epoch && result == MISSING) put(L.vmark, x, (rd(L.vmark, x) & 1u) | (mark_epoch << 1));
    }
    // ids of finished (popped) vertices are gone with their slots; a finished
    // vertex still present was on the stack, handled above
    tsp = 0;
    return result;
  }

  // index_pending (mod.rs:525-554) -> PendingIndex::index (index.rs:168-202):
  // vertex v waits on parent m.  With partial replication v keeps a list of
  // parents, and a parent no vertex waits on yet (a vacant PendingIndex
  // entry) is reported in the request ring; the host keeps the ones this
  // shard does not replicate (is_mine, index.rs:187-197).
  __device__ void index_pending(uint32_t v, uint32_t m) {
    if (!partial) {
      put(L.vwait, v, m);
      return;
    }
    bool seen = false;
    for (uint32_t v0 = 0; v0 < L.P && !seen; v0 += 64) {
      const uint32_t x = v0 + lid;
      bool hit = false;
      if (at(L.vdot, x) != 0) {
        const uint32_t c = at(L.vwn, x);
        for (uint32_t j = 0; j < c && !hit; ++j) hit = at(L.vwl, x * PW + j) == m;
      }
      seen = __ballot(hit) != 0;
    }
    if (!seen) {
      uint32_t* ring = a.req + (size_t)blockIdx.x * (1 + 2 * (size_t)a.req_cap);
      const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)ring[0]);
      if (k >= a.req_cap) { err = FX_ERR_CAPACITY; return; }
      if (lid == 0) {
        ring[1 + 2 * k] = step;
        ring[2 + 2 * k] = m;
        ring[0] = k + 1;
      }
    } else {
      const uint32_t c = rd(L.vwn, v);
      for (uint32_t j = 0; j < c; ++j)
        if (rd(L.vwl, v * PW + j) == m) return;  // HashSet::insert of a present child
    }
    const uint32_t c = rd(L.vwn, v);
    if (c >= PW) { err = FX_ERR_CAPACITY; return; }
    put(L.vwl, v * PW + c, m);
    put(L.vwn, v, c + 1);
    __syncthreads();
  }

  // check_pending (mod.rs:556-587) + try_pending (589-642)
  __device__ void check_pending() {
    while (nwl && !err) {
      const uint32_t d = rd(L.wl, --nwl);
      // PendingIndex::remove(d): every vertex waiting on d, ascending (C2)
      uint32_t cnt = 0;
      for (uint32_t v0 = 0; v0 < L.P; v0 += 64) {
        const uint32_t v = v0 + lid;
        bool w = false;
        if (partial) {
          if (at(L.vdot, v) != 0) {
            const uint32_t c = at(L.vwn, v);
            for (uint32_t j = 0; j < c; ++j)
              if (at(L.vwl, v * PW + j) == d) {  // swap-remove d from v's parents
                at(L.vwl, v * PW + j) = at(L.vwl, v * PW + c - 1);
                at(L.vwn, v) = c - 1;
                w = true;
                break;
              }
          }
        } else {
          w = at(L.vdot, v) != 0 && at(L.vwait, v) == d;
        }
        const uint64_t b = __ballot(w);
        if (w) {
          at(L.tmp, cnt + __builtin_popcountll(b & ((1ull << lid) - 1ull))) = at(L.vdot, v);
          if (!partial) at(L.vwait, v) = 0;
        }
        cnt += __builtin_popcountll(b);
      }
      __syncthreads();
      if (!cnt) continue;
      // rank sort the waiters' dots into tl
      for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
        const uint32_t i = i0 + lid;
        if (i < cnt) {
          const uint32_t x = at(L.tmp, i);
          uint32_t r = 0;
          for (uint32_t k = 0; k < cnt; ++k) r += at(L.tmp, k) < x ? 1u : 0u;
          at(L.tl, r) = x;
        }
      }
      __syncthreads();
      // try_pending: visited-skip set = vertices marked with this epoch
      ++epoch;
      uint32_t cur = epoch;
      for (uint32_t k = 0; k < cnt && !err; ++k) {
        const uint32_t wd = rd(L.tl, k);
        const uint32_t wv = find(wd);
        if (wv != NONE && (rd(L.vmark, wv) >> 1) == cur) continue;  // visited by a failed search
        uint32_t missing = 0;
        bool saved = false;
        const uint32_t r = find_scc(wd, &missing, cur, &saved);
        if (r == FOUND) {
          cur = ++epoch;  // visited.clear()
        } else if (r == MISSING) {
          const uint32_t v2 = find(wd);
          if (v2 != NONE) index_pending(v2, missing);
          if (saved) cur = ++epoch;
        }
      }
    }
  }

  __device__ void handle_add(uint32_t r) {
    const uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.dot[ix(r)]);
    const uint32_t src = FX_DOT_SRC(d);
    if (src < 1 || src > L.n || FX_DOT_SEQ(d) == 0) { err = FX_ERR_DOT_RANGE; return; }
    const uint32_t kind = FX_HDR_KIND(a.hdr[ix(r)]);
    if (kind == FX_KIND_EXECUTED && partial) {  // RequestReply::Executed (mod.rs:394-402)
      clock_add(d);
      __syncthreads();
      nwl = 0;
      put(L.wl, nwl++, d);
      __syncthreads();
      check_pending();
      return;
    }
    if (kind != FX_KIND_ADD && kind != FX_KIND_INDEX_ONLY) { err = FX_ERR_UNSUPPORTED; return; }
    const uint32_t h = hslot(d);
    const uint32_t old = rd(L.hidx, h);
    if (old != 0) {
      if ((old & 0xFFFF0000u) == htag(d)) { err = FX_ERR_DOUBLE_INDEX; return; }
      err = FX_ERR_CAPACITY;  // two pending dots of a source share an index slot
      return;
    }
    if (!nfree) { err = FX_ERR_CAPACITY; return; }
    const uint32_t v = rd(L.vfree, --nfree);
    put(L.vdot, v, d);
    put(L.vrec, v, r);
    const uint32_t nd = ndeps(r);
    put(L.vnd, v, nd);
    if (lid < nd) m[L.vdeps + v * L.D + lid] = dep(r, lid);
    put(L.vwait, v, 0);
    put(L.vid, v, 0);
    put(L.vmark, v, 0);
    if (partial) put(L.vwn, v, 0);
    put(L.hidx, h, (v + 1) | htag(d));
    __syncthreads();
    if (kind == FX_KIND_INDEX_ONLY) return;  // VertexIndex::index without a search (test hook)
    uint32_t missing = 0;
    bool saved = false;
    nwl = 0;
    const uint32_t res = find_scc(d, &missing, 0, &saved, partial);
    if (res == MISSING) {
      const uint32_t v2 = find(d);
      if (v2 != NONE) {  // index_pending (mod.rs:525-554)
        if (partial) {
          for (uint32_t k = 0; k < nml && !err; ++k) index_pending(v2, rd(L.ml, k));
        } else {
          index_pending(v2, missing);
        }
      }
    } else if (res == NOT_PENDING) {
      err = FX_ERR_CAPACITY;  // "just added dot must be pending" (mod.rs:257-259)
      return;
    }
    __syncthreads();
    check_pending();
  }
};

template <bool HBM>
__global__ __launch_bounds__(64) void k_graph_wide(KArgs a, Lay L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t lane_idx = blockIdx.x;
  if (lane_idx >= a.num_lanes) return;
  W w;
  w.a = a;
  w.L = L;
  w.lid = threadIdx.x;
  w.s = a.stream_map ? a.stream_map[lane_idx] : lane_idx;
  w.partial = HBM && (a.flags & FX_FLAG_PARTIAL);
  w.m = HBM ? a.state + (size_t)lane_idx * L.words : smem;
  const uint32_t len = a.lengths ? min(a.lengths[w.s], a.steps) : a.steps;
  if (a.flags & FX_FLAG_INIT) {
    // init tables (the dep rows are written before they are read)
    for (uint32_t i = w.lid; i < L.words; i += 64)
      if (i < L.vdeps || i >= L.vdeps + L.P * L.D) w.m[i] = 0;
    __syncthreads();
    for (uint32_t i = w.lid; i < L.P; i += 64) w.m[L.vfree + i] = L.P - 1u - i;
    if (a.init_frontier && w.lid < L.n) w.m[L.front + w.lid] = a.init_frontier[(size_t)w.s * 8 + w.lid];
    __syncthreads();
    w.nfree = L.P;
    if (w.partial && w.lid == 0) a.req[(size_t)blockIdx.x * (1 + 2 * (size_t)a.req_cap)] = 0;
  } else {  // resume (HBM tables only): the tables are in place, the scalars saved
    w.nfree = w.rd(L.sc, 0);
    w.nexec = w.rd(L.sc, 1);
    w.epoch = w.rd(L.sc, 2);
  }
  const uint32_t end = min(len, a.step_end);
  for (uint32_t r = a.step_begin; r < end && !w.err; ++r) {
    w.step = r;
    if (a.flags & FX_FLAG_EXECUTE_AT_COMMIT) {  // executor.rs:72-73
      if (w.lid == 0) {
        a.order[w.ix(w.nexec)] = r | FX_ORDER_SCC_START;
        a.release[w.ix(r)] = r;
      }
      ++w.nexec;
      continue;
    }
    w.handle_add(r);
  }
  if (HBM && (a.flags & FX_FLAG_SAVE_STATE)) {
    w.put(L.sc, 0, w.nfree);
    w.put(L.sc, 1, w.nexec);
    w.put(L.sc, 2, w.epoch);
  }
  if (w.lid == 0) {
    a.nexec[w.s] = w.nexec;
    a.err[w.s] = w.err;
  }
}

}  // namespace wide

// LDS tables: 512 vertices, 512 index slots per source, 1024-bit windows
// (32 words); HBM tables: 16384 vertices, 32768 index slots, 32768-bit
// windows, dep rows of
// the widest Add (31) so a saved table stays valid when later Adds are wider
static wide::Lay wide_layout(bool hbm, uint32_t n, uint32_t dmax, bool partial = false) {
  wide::Lay L;
  if (hbm) L.make(16384, 32768, 1024, n, 31, partial);
  else L.make(512, 512, 32, n, std::max(dmax, 1u));
  return L;
}

bool wide_lds_fits(uint32_t n, uint32_t dmax) { return (size_t)wide_layout(false, n, dmax).words * 4 <= 160 * 1024; }

size_t wide_state_bytes(uint32_t tier, uint32_t n, uint32_t lanes) {
  return tier == FX_TIER_WIDE_HBM ? (size_t)wide_layout(true, n, 31).words * 4 * lanes : 0;
}

uint32_t wide_decode_pending(const uint32_t* block, uint32_t n, uint32_t* dots, uint32_t* waits, uint32_t cap,
                             bool partial) {
  const wide::Lay L = wide_layout(true, n, 31, partial);
  uint32_t c = 0;
  for (uint32_t v = 0; v < L.P; ++v) {
    const uint32_t d = block[L.vdot + v];
    if (!d) continue;
    if (partial) {  // one (dot, parent) pair per registration; (dot, 0) if none
      const uint32_t k = block[L.vwn + v];
      for (uint32_t j = 0; j < (k ? k : 1u); ++j) {
        if (c < cap) {
          dots[c] = d;
          waits[c] = k ? block[L.vwl + v * wide::PW + j] : 0u;
        }
        ++c;
      }
      continue;
    }
    if (c < cap) {
      dots[c] = d;
      waits[c] = block[L.vwait + v];
    }
    ++c;
  }
  return c;
}

size_t wide_partial_state_bytes(uint32_t n, uint32_t lanes) {
  return (size_t)wide_layout(true, n, 31, true).words * 4 * lanes;
}

int launch_wide(const KArgs& a, bool hbm, hipStream_t hs) {
  // the LDS tables live for one launch: whole streams only (a rerun tier); the
  // HBM tables persist in `state`, so that tier also resumes (the executor handle)
  if (!hbm && (a.step_begin != 0 || a.step_end != a.steps || !(a.flags & FX_FLAG_INIT) ||
               (a.flags & FX_FLAG_SAVE_STATE)))
    return FX_ERR_INVALID_ARG;
  if (a.num_lanes == 0) return FX_OK;
  const bool partial = (a.flags & FX_FLAG_PARTIAL) != 0;
  if (partial && (!hbm || !a.req || a.stream_map)) return FX_ERR_INVALID_ARG;
  const wide::Lay L = wide_layout(hbm, a.n, a.dmax, partial);
  if (!hbm && (size_t)L.words * 4 > 160 * 1024) return FX_ERR_UNSUPPORTED;
  if (hbm) {
    if (!a.state) return FX_ERR_INVALID_ARG;
    hipLaunchKernelGGL(wide::k_graph_wide<true>, dim3(a.num_lanes), dim3(64), 0, hs, a, L);
  } else {
    static bool configured = false;
    if (!configured) {
      (void)hipFuncSetAttribute((const void*)wide::k_graph_wide<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      configured = true;
    }
    hipLaunchKernelGGL(wide::k_graph_wide<false>, dim3(a.num_lanes), dim3(64), (size_t)L.words * 4, hs, a, L);
  }
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

}  // namespace fx
