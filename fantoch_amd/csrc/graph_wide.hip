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

// The LDS tables are packed (PK) so that five streams share a CU: u16 vertex
// lists (free list, Tarjan stack, waiter lists, index slots), one word per DFS
// frame, a vertex's dep count beside its arrival index, and its Tarjan id,
// on-stack bit and visited epoch in one word.  The HBM tables keep one u32
// per field (16,384 vertices do not fit the packed fields).
constexpr uint32_t PK_REC_BITS = 26;                       // arrival index | ndeps << 26
constexpr uint32_t PK_ID_MASK = 0x3FFu, PK_ONSTACK = 0x400u;  // vmark: id | on-stack | epoch << 11
constexpr uint32_t PK_EPOCH_SHIFT = 11, PK_EPOCH_MAX = (1u << 21) - 4096u;

struct Lay {  // table layout (u32 words) for capacity P, index Q per source, W-bit clock windows
  uint32_t P, Q, WB, n, D, wlcap;
  // per-source strides of the index (entries) and the clock windows (words).
  // Packed (LDS): one word more than a source's part, so the same slot /
  // window word of different sources falls in different LDS banks (the deps of
  // one vertex, looked up lane-parallel, come from different sources with
  // nearby seqs: without the pad they hit one bank, a 5-way conflict)
  uint32_t QS, WBS;
  bool pk;
  uint32_t vdot, vrec, vnd, vdeps, vwait, vid, vlow, vmark, vce, vfree, tstk, fv, fi, wl, tl, tmp, hidx, front, bits, sc, words;
  // partial replication only (0 words otherwise): per-vertex parent lists
  // (count + PW dots), per-frame missing-dep counts, the collected missing deps
  uint32_t vwn, vwl, fm, ml;
  __host__ __device__ void make(uint32_t P_, uint32_t Q_, uint32_t WB_, uint32_t n_, uint32_t D_,
                                bool partial = false, bool packed = false) {
    P = P_;
    Q = Q_;
    WB = WB_;
    n = n_;
    D = D_;
    pk = packed;
    QS = packed ? Q + 2u : Q;
    WBS = packed ? WB + 1u : WB;
    uint32_t o = 0;
    const uint32_t h = packed ? P / 2 : P;  // a u16 list of P entries
    vdot = o; o += P;
    vrec = o; o += P;
    vnd = o; o += packed ? 0 : P;
    vdeps = o; o += P * D;  // deps of the vertex (copied from the planes at index time:
                            // the DFS then never waits on HBM)
    vwait = o; o += P;
    vid = o; o += packed ? 0 : P;
    vlow = o; o += packed ? 0 : P;  // per DFS frame: low of the frame's vertex
    vmark = o; o += P;
    vce = o; o += P;  // search-result cache: executions when the vertex's last search failed
    vfree = o; o += h;
    tstk = o; o += h;
    fv = o; o += P;                 // packed: vertex | next dep << 10 | low << 15
    fi = o; o += packed ? 0 : P;
    wlcap = packed ? P : 2 * P;     // released dots of one handle_add: at most the vertices present
    wl = o; o += wlcap;
    tl = o; o += h;
    tmp = o; o += h;
    hidx = o; o += packed ? n * QS / 2 : n * QS;
    front = o; o += 8;
    bits = o; o += n * WBS;
    sc = o; o += 4;  // saved scalars of a resumable (HBM) stream: nfree, nexec, epoch
    vwn = o; o += partial ? P : 0;
    vwl = o; o += partial ? P * PW : 0;
    fm = o; o += partial ? P : 0;
    ml = o; o += partial ? P : 0;
    words = o;
  }
};

// RS = FD != 0 (the compiled-in layout): the states of a frame's deps are
// looked up for all of its deps at once when the frame is entered (lane j:
// dep j, one round trip), so an edge only reads the dep's vertex
constexpr uint32_t RS_EXEC = 0x80000000u;
// WG: several streams (wavefronts) per workgroup, each on its own tables: a
// wave-level barrier orders a wave's LDS accesses (a workgroup barrier would
// couple streams whose control flow differs)
template <bool PK, uint32_t FD = 0, bool WG = false>
struct W {
#ifdef FX_WIDE_NO_RS
  static constexpr bool RS = false;
#else
  static constexpr bool RS = PK && FD != 0;
#endif
  KArgs a;
  Lay L;
  uint32_t* m;  // table memory (LDS or this stream's HBM block)
  uint32_t lid, s, slot = 0;  // slot: the launch's lane index (partial: this lane's request ring)
  uint32_t err = 0;
  uint32_t nfree = 0, tsp = 0, fsp = 0, nwl = 0, idc = 0, epoch = 1, nexec = 0, step = 0;
  uint32_t t_now = 0;
  bool partial = false;  // FX_FLAG_PARTIAL
  uint32_t nml = 0;      // missing deps collected by a first search (partial)

  __device__ __forceinline__ void sync() {
    if constexpr (WG) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      __syncthreads();
    }
  }
  __device__ __forceinline__ uint32_t& at(uint32_t base, uint32_t i) { return m[base + i]; }
  // a uniform store: every lane writes the same word (LDS: no exec-mask
  // save / restore around it; HBM: lane 0)
  __device__ __forceinline__ void put(uint32_t base, uint32_t i, uint32_t v) {
    if (PK || lid == 0) m[base + i] = v;
  }
  __device__ __forceinline__ uint32_t rd(uint32_t base, uint32_t i) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)m[base + i]);
  }
  // vertex lists: u16 entries when packed
  __device__ __forceinline__ uint32_t lget(uint32_t base, uint32_t i) {
    if constexpr (PK) return ((const uint16_t*)(m + base))[i];
    else return m[base + i];
  }
  __device__ __forceinline__ void lset(uint32_t base, uint32_t i, uint32_t v) {
    if constexpr (PK) ((uint16_t*)(m + base))[i] = (uint16_t)v;
    else m[base + i] = v;
  }
  __device__ __forceinline__ uint32_t lrd(uint32_t base, uint32_t i) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)lget(base, i));
  }
  __device__ __forceinline__ void lput(uint32_t base, uint32_t i, uint32_t v) {
    if (PK || lid == 0) lset(base, i, v);
  }
  // vertex fields
  __device__ __forceinline__ uint32_t rec_of(uint32_t w) { return PK ? w & ((1u << PK_REC_BITS) - 1u) : w; }
  __device__ __forceinline__ uint32_t nd_of(uint32_t v) {
    if constexpr (PK) return rd(L.vrec, v) >> PK_REC_BITS;
    else return rd(L.vnd, v);
  }
  // the Tarjan word of v: id (0 = unvisited) and on-stack bit, plus the
  // visited epoch (packed: one word; HBM: id and mark words)
  __device__ __forceinline__ uint32_t epoch_of(uint32_t mk) { return PK ? mk >> PK_EPOCH_SHIFT : mk >> 1; }
  __device__ __forceinline__ bool onstack_of(uint32_t mk) { return PK ? (mk & PK_ONSTACK) != 0 : (mk & 1u) != 0; }
  __device__ __forceinline__ uint32_t rd_mark(uint32_t v) { return rd(L.vmark, v); }
  __device__ __forceinline__ uint32_t rd_id(uint32_t v, uint32_t mk) {
    if constexpr (PK) return mk & PK_ID_MASK;
    else return rd(L.vid, v);
  }
  // v enters the search with id `id` (on the stack)
  __device__ __forceinline__ void visit(uint32_t v, uint32_t mk, uint32_t id) {
    if constexpr (PK) {
      put(L.vmark, v, (mk & ~PK_ID_MASK) | id | PK_ONSTACK);
    } else {
      put(L.vid, v, id);
      put(L.vmark, v, mk | 1u);
    }
  }
  __device__ __forceinline__ void pop_stack(uint32_t x) {
    if constexpr (PK) put(L.vmark, x, rd(L.vmark, x) & ~PK_ONSTACK);
    else put(L.vmark, x, rd(L.vmark, x) & ~1u);
  }
  // DFS frame f: its vertex, next dep and low (packed: one word)
  __device__ __forceinline__ void frame_save(uint32_t f, uint32_t v, uint32_t i, uint32_t low) {
    if constexpr (PK) {
      put(L.fv, f, v | (i << 10) | (low << 15));
    } else {
      put(L.fv, f, v);
      put(L.fi, f, i);
      put(L.vlow, f, low);
    }
  }
  __device__ __forceinline__ void frame_load(uint32_t f, uint32_t& v, uint32_t& i, uint32_t& low) {
    if constexpr (PK) {
      const uint32_t w = rd(L.fv, f);
      v = w & 0x3FFu;
      i = (w >> 10) & 31u;
      low = w >> 15;
    } else {
      v = rd(L.fv, f);
      i = rd(L.fi, f);
      low = rd(L.vlow, f);
    }
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
  __device__ __forceinline__ void clock_add(uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
    if (src < 1 || src > L.n) { err = FX_ERR_DOT_RANGE; return; }
    uint32_t f = rd(L.front, src - 1);
    if (sq <= f) return;
    if (sq - f - 1 >= L.WB * 32u) { err = FX_ERR_CAPACITY; return; }
    const uint32_t mask = L.WB * 32u - 1u;
    const uint32_t b = sq & mask, wi = (src - 1) * L.WBS + (b >> 5);
    put(L.bits, wi, rd(L.bits, wi) | (1u << (b & 31u)));
    // advance the frontier over contiguous seqs, clearing their bits
    for (;;) {
      const uint32_t nb = (f + 1) & mask, nw = (src - 1) * L.WBS + (nb >> 5);
      const uint32_t word = rd(L.bits, nw);
      if (!((word >> (nb & 31u)) & 1u)) break;
      put(L.bits, nw, word & ~(1u << (nb & 31u)));
      ++f;
    }
    put(L.front, src - 1, f);
    if (lid == src - 1) frv = f;
  }

  // executed_clock.contains(d), frontiers read from the table
  __device__ __forceinline__ bool contains(uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
    if (src < 1 || src > L.n) return false;
    const uint32_t f = rd(L.front, src - 1);
    if (sq <= f) return true;
    if (sq - f - 1 >= L.WB * 32u) return false;
    const uint32_t b = sq & (L.WB * 32u - 1u);
    return (rd(L.bits, (src - 1) * L.WBS + (b >> 5)) >> (b & 31u)) & 1u;
  }

  // ------------------------------------------------------- vertex index
  // HBM: an index word is (vertex + 1) | seq / Q << 16, so it names its dot
  // without a read of the vertex table.  Packed: a u16 (vertex + 1), and the
  // vertex's dot is compared (read in the same round trip as its Tarjan word).
  __device__ __forceinline__ uint32_t hslot(uint32_t d) const {
    return (FX_DOT_SRC(d) - 1) * L.QS + (FX_DOT_SEQ(d) & (L.Q - 1u));
  }
  __device__ __forceinline__ uint32_t htag(uint32_t d) const {
    return (FX_DOT_SEQ(d) >> __builtin_ctz(L.Q)) << 16;
  }
  __device__ __forceinline__ uint32_t hword(uint32_t v, uint32_t d) const { return PK ? v + 1u : (v + 1) | htag(d); }
  // the vertex an index word names for dot d (NONE if none); `vd` = that vertex's dot (packed only)
  __device__ __forceinline__ uint32_t hmatch(uint32_t hw, uint32_t d, uint32_t vd) const {
    if constexpr (PK) return (hw != 0 && vd == d) ? hw - 1u : NONE;
    else return ((hw & 0xFFFFu) != 0 && (hw & 0xFFFF0000u) == htag(d)) ? (hw & 0xFFFFu) - 1u : NONE;
  }
  __device__ __forceinline__ uint32_t find(uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d);
    if (src < 1 || src > L.n) return NONE;
    const uint32_t w = lrd(L.hidx, hslot(d));
    return hmatch(w, d, PK && w ? rd(L.vdot, (w & 0xFFFFu) - 1u) : 0u);
  }

  // ------------------------------------------------------- emission
  // save_scc (mod.rs:488-523): members ascending by dot (SCC = BTreeSet)
  __device__ void save_scc(uint32_t base, uint32_t cnt) {
    // members are tstk[base .. base + cnt): rank-sort their dots in the lanes
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
      const uint32_t i = i0 + lid;
      if (i < cnt) {
        const uint32_t v = lget(L.tstk, base + i), d = at(L.vdot, v);
        uint32_t r = 0;
        for (uint32_t k = 0; k < cnt; ++k) r += at(L.vdot, lget(L.tstk, base + k)) < d ? 1u : 0u;
        lset(L.tmp, r, v);
      }
    }
    sync();
    if (nexec + cnt > a.steps) { err = FX_ERR_ORDER_OVERFLOW; return; }
    if (nwl + cnt > L.wlcap) { err = FX_ERR_CAPACITY; return; }
    // emission, one lane per member (members are distinct vertices): the
    // order rows, release steps, index / slot release and the released-dots
    // worklist in the member order (LIFO pops see the same sequence)
    for (uint32_t r0 = 0; r0 < cnt; r0 += 64) {
      const uint32_t r = r0 + lid;
      if (r < cnt) {
        const uint32_t v = lget(L.tmp, r);
        const uint32_t d = at(L.vdot, v), rec = rec_of(at(L.vrec, v));
        a.order[ix(nexec + r)] = rec | (r == 0 ? FX_ORDER_SCC_START : 0u);
        a.release[ix(rec)] = step;
        lset(L.hidx, hslot(d), 0u);
        at(L.vdot, v) = 0u;
        at(L.vwait, v) = 0u;
        if (partial) at(L.vwn, v) = 0u;
        lset(L.vfree, nfree + r, v);
        at(L.wl, nwl + r) = d;
      }
    }
    sync();
    nexec += cnt;
    nfree += cnt;
    nwl += cnt;
  }

  // lane j < nd: RS_EXEC if dep j is executed now, else its index word
  // (vertex + 1; 0 = missing).  Exact for the whole life of the frame with
  // one check at use: no vertex is added during a search, a missing dep
  // cannot execute, and a pending one can only execute (its slot's dot then
  // no longer matches)
  __device__ __forceinline__ uint32_t row_state(uint32_t row, uint32_t nd) {
    const uint32_t src = FX_DOT_SRC(row), sq = FX_DOT_SEQ(row);
    const bool ok = lid < nd && src >= 1 && src <= L.n;
    const uint32_t si = ok ? src - 1u : 0u;
    const uint32_t bb = sq & (L.WB * 32u - 1u);
    const uint32_t f = ok ? at(L.front, si) : 0u;
    const uint32_t bw = ok ? at(L.bits, si * L.WBS + (bb >> 5)) : 0u;
    const uint32_t hw = ok ? lget(L.hidx, si * L.QS + (sq & (L.Q - 1u))) : 0u;
    const bool ex = ok && (sq <= f || (sq - f - 1u < L.WB * 32u && ((bw >> (bb & 31u)) & 1u)));
    return ex ? RS_EXEC : hw;
  }
  uint32_t fst[FD ? FD : 1];  // RS: lane f = the state of dep j of DFS frame f < 64
  __device__ __forceinline__ void fst_save(uint32_t f, uint32_t st) {
    if constexpr (RS) {
      if (f < 64) {
#pragma unroll
        for (uint32_t j = 0; j < FD; ++j) {
          const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)st, (int)j);
          fst[j] = lid == f ? v : fst[j];
        }
      }
    }
  }
  __device__ __forceinline__ uint32_t fst_load(uint32_t f, uint32_t row, uint32_t nd) {
    if constexpr (RS) {
      if (f < 64) {
        uint32_t st = 0;
#pragma unroll
        for (uint32_t j = 0; j < FD; ++j) {
          const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)fst[j], (int)f);
          st = lid == j ? v : st;
        }
        return st;
      }
      return row_state(row, nd);
    }
    return 0u;
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
    visit(root, rd_mark(root), 1);
    lput(L.tstk, tsp++, root);
    if (partial) put(L.fm, fsp, 0);
    ++fsp;
    // the top frame lives in registers: its vertex, next dep, id, low, dot,
    // dep count and dep row (lane j = dep j); a frame's position and low go
    // to the frame table only when it recurses, and come back when it resumes
    uint32_t cv = root, ci = 0, cid = 1, clow = 1, cdot = root_dot;
    uint32_t cnd = nd_of(root);
    uint32_t drow = lid < cnd ? at(L.vdeps, root * L.D + lid) : 0u;
    uint32_t cst = RS ? row_state(drow, cnd) : 0u;
    uint32_t result = FOUND;
    while (fsp && !err) {
      if (RS && ci < cnd) {
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)drow, (int)ci);
        const uint32_t st = (uint32_t)__builtin_amdgcn_readlane((int)cst, (int)ci);
        ++ci;
        if (d == cdot || (st & RS_EXEC)) continue;  // self or executed (tarjan.rs:128-145)
        if (st == 0) {  // missing (tarjan.rs:148-157)
          *missing = d;
          result = MISSING;
          break;
        }
        const uint32_t hx = st - 1u;
        const uint32_t mkw = rd(L.vmark, hx), vd = rd(L.vdot, hx), wnd = nd_of(hx);
        const uint32_t wrow = lid < L.D ? at(L.vdeps, hx * L.D + lid) : 0u;
        if (vd != d) continue;  // executed since the frame was entered
        const uint32_t idw = mkw & PK_ID_MASK;
        if (idw == 0) {  // recurse
          frame_save(fsp - 1, cv, ci, clow);
          fst_save(fsp - 1, cst);
          ++idc;
          visit(hx, mkw, idc);
          lput(L.tstk, tsp++, hx);
          ++fsp;
          cv = hx;
          ci = 0;
          cid = idc;
          clow = idc;
          cdot = d;
          cnd = wnd;
          drow = lid < cnd ? wrow : 0u;
          cst = row_state(drow, cnd);
        } else if (onstack_of(mkw)) {
          clow = min(clow, idw);
        }
        continue;
      }
      if (ci < cnd) {
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)drow, (int)ci);
        ++ci;
        // the clock-window word and the index word both depend on d alone:
        // read them together (one LDS round trip), then decide
        const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
        const bool inr = src >= 1 && src <= L.n;
        const uint32_t si = inr ? src - 1 : 0u;
        const uint32_t bb = sq & (L.WB * 32u - 1u);
        const uint32_t hw = lrd(L.hidx, si * L.QS + (sq & (L.Q - 1u)));
        const uint32_t bw = rd(L.bits, si * L.WBS + (bb >> 5));
        const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)frv, (int)si);
        const bool executed = inr && (sq <= f || (sq - f - 1u < L.WB * 32u && ((bw >> (bb & 31u)) & 1u)));
        if (d == cdot || executed) continue;  // self or executed (tarjan.rs:128-145)
        // the named vertex's Tarjan word (and, packed, its dot), dep count and
        // dep row in one round trip: a recursion into it then waits on nothing
        const uint32_t hv = inr ? (hw & 0xFFFFu) : 0u;
        const uint32_t hx = hv ? hv - 1u : 0u;
        const uint32_t mkw = rd(L.vmark, hx);
        const uint32_t aux = PK ? rd(L.vdot, hx) : rd(L.vid, hx);  // packed: its dot; HBM: its id
        const uint32_t wnd = nd_of(hx);
        const uint32_t wrow = lid < L.D ? at(L.vdeps, hx * L.D + lid) : 0u;
        const uint32_t w = inr ? hmatch(hw, d, aux) : NONE;
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
        const uint32_t idw = PK ? mkw & PK_ID_MASK : aux;
        if (idw == 0) {  // recurse
          frame_save(fsp - 1, cv, ci, clow);
          ++idc;
          visit(w, mkw, idc);
          lput(L.tstk, tsp++, w);
          if (partial) put(L.fm, fsp, 0);
          ++fsp;
          cv = w;
          ci = 0;
          cid = idc;
          clow = idc;
          cdot = d;
          cnd = wnd;
          drow = lid < cnd ? wrow : 0u;
        } else if (onstack_of(mkw)) {  // on the stack
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
          const uint32_t x = lrd(L.tstk, base);
          pop_stack(x);
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
        uint32_t p, pi, plow;
        frame_load(fsp - 1, p, pi, plow);
        cv = p;
        ci = pi;
        cid = rd_id(p, rd_mark(p));
        clow = min(plow, lowv);
        cdot = rd(L.vdot, p);
        cnd = nd_of(p);
        drow = lid < cnd ? at(L.vdeps, p * L.D + lid) : 0u;
        if (RS) cst = fst_load(fsp - 1, drow, cnd);
        if (mcount) put(L.fm, fsp - 1, rd(L.fm, fsp - 1) + mcount);  // tarjan.rs:198-200
      } else if (mcount) {
        result = MISSING;  // NotFound -> MissingDependencies(collected) (mod.rs:478-484)
      }
    }
    // finalize: ids of the vertices left on the stack; failed searches mark
    // them visited (the members are distinct: one lane each)
    const uint32_t ep = (mark_epoch && result == MISSING) ? mark_epoch : 0u;
    for (uint32_t k0 = 0; k0 < tsp; k0 += 64) {
      const uint32_t k = k0 + lid;
      if (k < tsp) {
        const uint32_t x = lget(L.tstk, k);
        if constexpr (PK) {
          const uint32_t mk = at(L.vmark, x);
          at(L.vmark, x) = ep ? (mk & PK_ONSTACK) | (ep << PK_EPOCH_SHIFT) : mk & ~PK_ID_MASK;
        } else {
          at(L.vid, x) = 0u;
          if (ep) at(L.vmark, x) = (at(L.vmark, x) & 1u) | (ep << 1);
        }
      }
    }
    sync();
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
      uint32_t* ring = a.req + (size_t)slot * (1 + 2 * (size_t)a.req_cap);
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
    sync();
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
          lset(L.tmp, cnt + __builtin_popcountll(b & ((1ull << lid) - 1ull)), v);
          if (!partial) at(L.vwait, v) = 0;
        }
        cnt += __builtin_popcountll(b);
      }
      sync();
      if (!cnt) continue;
      // rank sort the waiters by dot into tl
      for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
        const uint32_t i = i0 + lid;
        if (i < cnt) {
          const uint32_t x = lget(L.tmp, i), xd = at(L.vdot, x);
          uint32_t r = 0;
          for (uint32_t k = 0; k < cnt; ++k) r += at(L.vdot, lget(L.tmp, k)) < xd ? 1u : 0u;
          lset(L.tl, r, x);
        }
      }
      sync();
      // try_pending: visited-skip set = vertices marked with this epoch
      ++epoch;
      uint32_t cur = epoch;
      for (uint32_t k = 0; k < cnt && !err; ++k) {
        const uint32_t wv = lrd(L.tl, k);
        // a waiter executed by an earlier search of this round is not pending
        // (its slot is not reused before the next Add)
        const uint32_t wd = rd(L.vdot, wv);
        if (wd == 0) continue;
        if (epoch_of(rd_mark(wv)) == cur) continue;  // visited by a failed search
        uint32_t missing = 0;
        bool saved = false;
        const uint32_t r = find_scc(wd, &missing, cur, &saved);
        if (r == FOUND) {
          cur = ++epoch;  // visited.clear()
        } else if (r == MISSING) {
          if (rd(L.vdot, wv) == wd) {
            index_pending(wv, missing);
            if (!partial) put(L.vce, wv, saved ? NONE : nexec);
          }
          if (saved) cur = ++epoch;
        }
      }
    }
  }

  // packed marks hold 21 epoch bits: restart the epochs before they run out
  // (between Adds no search is running, so every id is 0 and no vertex is on
  // the stack; one Add advances the epoch by at most 2 P + 1 < 4096)
  __device__ void renew_epochs() {
    if constexpr (PK) {
      if (epoch < PK_EPOCH_MAX) return;
      for (uint32_t i = lid; i < L.P; i += 64) m[L.vmark + i] = 0u;
      sync();
      epoch = 1;
    }
  }

  __device__ void handle_add(uint32_t r) {
    renew_epochs();
    const uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.dot[ix(r)]);
    const uint32_t src = FX_DOT_SRC(d);
    if (src < 1 || src > L.n || FX_DOT_SEQ(d) == 0) { err = FX_ERR_DOT_RANGE; return; }
    const uint32_t kind = FX_HDR_KIND(a.hdr[ix(r)]);
    if (kind == FX_KIND_EXECUTED && partial) {  // RequestReply::Executed (mod.rs:394-402)
      clock_add(d);
      sync();
      nwl = 0;
      put(L.wl, nwl++, d);
      sync();
      check_pending();
      return;
    }
    if (kind != FX_KIND_ADD && kind != FX_KIND_INDEX_ONLY) { err = FX_ERR_UNSUPPORTED; return; }
    const uint32_t h = hslot(d);
    const uint32_t old = lrd(L.hidx, h);
    if (old != 0) {
      const bool same = PK ? rd(L.vdot, old - 1u) == d : (old & 0xFFFF0000u) == htag(d);
      if (same) { err = FX_ERR_DOUBLE_INDEX; return; }
      err = FX_ERR_CAPACITY;  // two pending dots of a source share an index slot
      return;
    }
    if (!nfree) { err = FX_ERR_CAPACITY; return; }
    const uint32_t v = lrd(L.vfree, --nfree);
    put(L.vdot, v, d);
    const uint32_t nd = ndeps(r);
    if constexpr (PK) {
      put(L.vrec, v, r | (nd << PK_REC_BITS));
    } else {
      put(L.vrec, v, r);
      put(L.vnd, v, nd);
      put(L.vid, v, 0);
    }
    const uint32_t drj = lid < nd ? dep(r, lid) : 0u;  // lane j: dep j
    if (lid < nd) m[L.vdeps + v * L.D + lid] = drj;
    put(L.vwait, v, 0);
    put(L.vmark, v, 0);
    put(L.vce, v, NONE);
    if (partial) put(L.vwn, v, 0);
    lput(L.hidx, h, hword(v, d));
    sync();
    if (kind == FX_KIND_INDEX_ONLY) return;  // VertexIndex::index without a search (test hook)
    nwl = 0;
    // Search-result cache (as sim_big.hip x_add_): the first search from v
    // enters its first dep u that is neither v nor executed (deps ascend,
    // C1).  If u is pending and the last search rooted at u stopped at
    // missing dep m with no execution here since (vce = executions then; m is
    // the dot u waits on, vwait), and m is still missing and is not v, this
    // search stops at m too having found no SCC: u's walk meets the same deps
    // in the same states (a vertex pending then is still pending; one missing
    // then would have stopped that walk, so only m can have arrived; v was
    // missing then, so it is reachable only through m).  v just waits on m.
    if (!partial) {
      // the executed check of every dep at once (lane j: dep j)
      const uint32_t sj = FX_DOT_SRC(drj), qj = FX_DOT_SEQ(drj);
      const bool okj = lid < nd && sj >= 1 && sj <= L.n;
      const uint32_t bj = qj & (L.WB * 32u - 1u);
      const uint32_t fj = okj ? at(L.front, sj - 1) : 0u;
      const uint32_t wj = okj ? at(L.bits, (sj - 1) * L.WBS + (bj >> 5)) : 0u;
      const bool exj = okj && (qj <= fj || (qj - fj - 1u < L.WB * 32u && ((wj >> (bj & 31u)) & 1u)));
      const uint64_t cand = __ballot(lid < nd && drj != d && !exj);
      const uint32_t u = cand ? (uint32_t)__builtin_amdgcn_readlane((int)drj, (int)__builtin_ctzll(cand)) : 0u;
      const uint32_t uv = u ? find(u) : NONE;
      if (uv != NONE && rd(L.vce, uv) == nexec) {
        const uint32_t cm = rd(L.vwait, uv);
        const uint32_t cs = FX_DOT_SRC(cm);
        if (cm && cm != d && cs >= 1 && cs <= L.n && find(cm) == NONE && !contains(cm)) {
          index_pending(v, cm);
          put(L.vce, v, nexec);
          sync();
          return;  // no search ran: nothing released
        }
      }
    }
    uint32_t missing = 0;
    bool saved = false;
    const uint32_t res = find_scc(d, &missing, 0, &saved, partial);
    if (res == MISSING) {
      const uint32_t v2 = find(d);
      if (v2 != NONE) {  // index_pending (mod.rs:525-554)
        if (partial) {
          for (uint32_t k = 0; k < nml && !err; ++k) index_pending(v2, rd(L.ml, k));
        } else {
          index_pending(v2, missing);
          put(L.vce, v2, saved ? NONE : nexec);
        }
      }
    } else if (res == NOT_PENDING) {
      err = FX_ERR_CAPACITY;  // "just added dot must be pending" (mod.rs:257-259)
      return;
    }
    sync();
    check_pending();
  }
};

// streams per workgroup of the compiled n = 5 LDS build (1: one stream per
// workgroup; k > 1: k neighbouring streams share a CU and their plane lines)
#ifndef FX_WIDE_WPB
#define FX_WIDE_WPB 1
#endif
// FN / FD != 0: the layout of n = FN sources and FD dep planes compiled in
// (the configs[3] shape, n = 5): table offsets become immediates and the
// layout's fields leave the scalar registers, which the DFS is short of
template <bool HBM, uint32_t FN = 0, uint32_t FD = 0, uint32_t WPB = 1>
__global__ __launch_bounds__(64 * WPB) void k_graph_wide(KArgs a, Lay Lrt) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t wv = WPB > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0u;
  const uint32_t lane_idx = xcd_slot(blockIdx.x) * WPB + wv;
  if (lane_idx >= a.num_lanes) return;  // whole wavefront
  Lay L = Lrt;
  if constexpr (FN != 0) L.make(512, 256, 32, FN, FD, false, true);
  W<!HBM, FD, (WPB > 1)> w;
  w.a = a;
  w.L = L;
  w.lid = threadIdx.x & 63u;
  w.slot = lane_idx;
  w.s = a.stream_map ? a.stream_map[lane_idx] : lane_idx;
  w.partial = HBM && (a.flags & FX_FLAG_PARTIAL);
  w.m = HBM ? a.state + (size_t)lane_idx * L.words : smem + wv * L.words;
  const uint32_t len = a.lengths ? min(a.lengths[w.s], a.steps) : a.steps;
  if (a.flags & FX_FLAG_INIT) {
    // init tables (the dep rows are written before they are read)
    for (uint32_t i = w.lid; i < L.words; i += 64)
      if (i < L.vdeps || i >= L.vdeps + L.P * L.D) w.m[i] = 0;
    w.sync();
    for (uint32_t i = w.lid; i < L.P; i += 64) w.lset(L.vfree, i, L.P - 1u - i);
    if (a.init_frontier && w.lid < L.n) w.m[L.front + w.lid] = a.init_frontier[(size_t)w.s * 8 + w.lid];
    w.sync();
    w.nfree = L.P;
    if (w.partial && w.lid == 0) a.req[(size_t)lane_idx * (1 + 2 * (size_t)a.req_cap)] = 0;
  } else {  // resume (HBM tables only): the tables are in place, the scalars saved
    w.nfree = w.rd(L.sc, 0);
    w.nexec = w.rd(L.sc, 1);
    w.epoch = w.rd(L.sc, 2);
  }
  // packed records hold 26-bit arrival indices: longer streams take the HBM tables
  if (!HBM && a.steps >= (1u << PK_REC_BITS)) w.err = FX_ERR_CAPACITY;
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

// LDS tables (packed): 512 vertices, 256 index slots per source, 1024-bit
// windows (32 words): 31.2 KB at n = 5, five streams per CU; HBM tables: 16384 vertices, 32768 index slots, 32768-bit
// windows, dep rows of
// the widest Add (31) so a saved table stays valid when later Adds are wider
static wide::Lay wide_layout(bool hbm, uint32_t n, uint32_t dmax, bool partial = false) {
  wide::Lay L;
  if (hbm) L.make(16384, 32768, 1024, n, 31, partial);
  else L.make(512, 256, 32, n, std::max(dmax, 1u), false, true);
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
  const uint32_t grid = xcd_grid(a.num_lanes);
  if (hbm) {
    if (!a.state) return FX_ERR_INVALID_ARG;
    hipLaunchKernelGGL(wide::k_graph_wide<true>, dim3(grid), dim3(64), 0, hs, a, L);
  } else {
    static bool configured = false;
    if (!configured) {
      (void)hipFuncSetAttribute((const void*)wide::k_graph_wide<false, 5, 5>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)wide::k_graph_wide<false, 5, 5, FX_WIDE_WPB>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)wide::k_graph_wide<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      configured = true;
    }
    constexpr uint32_t WPB = FX_WIDE_WPB;
    if (a.n == 5 && std::max(a.dmax, 1u) == 5 && WPB > 1 && (size_t)L.words * 4 * WPB <= 160 * 1024)
      hipLaunchKernelGGL((wide::k_graph_wide<false, 5, 5, WPB>), dim3(xcd_grid((a.num_lanes + WPB - 1) / WPB)),
                         dim3(64 * WPB), (size_t)L.words * 4 * WPB, hs, a, L);
    else if (a.n == 5 && std::max(a.dmax, 1u) == 5)
      hipLaunchKernelGGL((wide::k_graph_wide<false, 5, 5>), dim3(grid), dim3(64), (size_t)L.words * 4, hs, a, L);
    else
      hipLaunchKernelGGL(wide::k_graph_wide<false>, dim3(grid), dim3(64), (size_t)L.words * 4, hs, a, L);
  }
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

}  // namespace fx
