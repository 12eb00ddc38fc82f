// pred_exec.hip — Caesar's PredecessorsExecutor on the GPU: one wavefront per
// commit stream, the graph as LDS (or HBM) tables, many streams per launch.
//
// PredecessorsGraph (fantoch_ps/src/executor/pred/mod.rs:28-384,
// index.rs:10-120) needs no SCCs: a committed command waits (phase one) until
// every dep is committed, then (phase two) until every dep with a lower Caesar
// clock (seq, process id; common/pred/clocks/mod.rs:15-30) is executed; an
// execution completes the phase two of its waiters, recursively.  Tables:
//   vertex table  dot, arrival, clock (2 words), missing-deps count, deps
//                 (copied at commit) and, per phase, one bit per dep slot
//                 saying whether it is registered in that phase's PendingIndex
//   dot index     per source, seq mod Q -> vertex
//   clocks        committed and executed AEClocks: frontier + ring bitmap
//   recursion     frames (phase, waiter list, position) over a list stack:
//                 try_phase_one_pending / try_phase_two_pending run depth
//                 first exactly as the reference's recursive calls
// PendingIndex::remove(dep) is a lane-parallel scan of the vertex table
// (each vertex holds a dep at most once); the waiters are visited ascending
// by dot (the reference iterates a HashSet; canonical as C2 for the graph
// executor).  Outputs use the batched executor's planes: order row k =
// arrival index of the k-th executed command (every command its own group),
// release[arrival] = the step that executed it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace pred {

constexpr uint32_t NONE = 0xFFFFFFFFu;

struct Lay {
  uint32_t P, Q, WB, n, D, DW, FD, LL;
  uint32_t vdot, vrec, vclo, vchi, vmiss, vnd, vreg, vdeps, vfree, hidx, cfront, cbits, efront, ebits, frames,
      lists, tmp, words;
  __host__ __device__ void make(uint32_t P_, uint32_t Q_, uint32_t WB_, uint32_t n_, uint32_t D_, uint32_t LL_,
                                uint32_t FD_ = 0) {
    P = P_;
    Q = Q_;
    WB = WB_;
    n = n_;
    D = D_;
    DW = (D + 31) / 32;
    FD = FD_ ? FD_ : P;
    LL = LL_;
    uint32_t o = 0;
    vdot = o; o += P;
    vrec = o; o += P;
    vclo = o; o += P;
    vchi = o; o += P;
    vmiss = o; o += P;
    vnd = o; o += P;
    vreg = o; o += 2 * P * DW;  // phase ph, vertex v: words [(ph * P + v) * DW, +DW)
    vdeps = o; o += P * D;
    vfree = o; o += P;
    hidx = o; o += n * Q;
    cfront = o; o += 8;
    cbits = o; o += n * WB;
    efront = o; o += 8;
    ebits = o; o += n * WB;
    frames = o; o += FD * 4;
    lists = o; o += LL;
    tmp = o; o += P;
    words = o;
  }
};

// the SMALL tier of the compiled n = 5 build (k_pred<false, 5, 5, WPB>): 64
// vertices, FX_PRED_Q index slots per source, FX_PRED_WB-word clock windows,
// FX_PRED_FRAMES recursion frames and FX_PRED_LISTS waiter-list entries
// (5.6 KB: 28 streams per CU at 4 per workgroup)
#ifndef FX_PRED_FRAMES
#define FX_PRED_FRAMES 32
#endif
#ifndef FX_PRED_LISTS
#define FX_PRED_LISTS 96
#endif
#ifndef FX_PRED_Q
#define FX_PRED_Q 32
#endif
#ifndef FX_PRED_WB
#define FX_PRED_WB 8
#endif
__host__ __device__ inline Lay small_fixed_layout(uint32_t n, uint32_t D) {
  Lay L{};
  L.make(64, FX_PRED_Q, FX_PRED_WB, n, D, FX_PRED_LISTS, FX_PRED_FRAMES);
  return L;
}

struct PArgs {
  KArgs k;
  const uint32_t* clo;
  const uint32_t* chi;
  const uint32_t* ndeps;
};

// WG: more than one wavefront (stream) per workgroup; each touches only its
// own tables, so a wave-level barrier orders its LDS accesses (a workgroup
// barrier would couple the streams, whose control flow differs)
template <bool WG = false>
struct Pr {
  PArgs a;
  Lay L;
  uint32_t* m;
  uint32_t lid, s;
  uint32_t err = 0, nfree = 0, fsp = 0, ltop = 0, nexec = 0, step = 0;
  // registrations held by each phase's PendingIndex: a removal from an empty
  // index finds no waiter, so its scan of the vertex table is skipped
  uint32_t nreg0 = 0, nreg1 = 0;

  __device__ __forceinline__ void sync() {
    if constexpr (WG) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      __syncthreads();
    }
  }
  __device__ __forceinline__ void put(uint32_t b, uint32_t i, uint32_t v) {
    if (lid == 0) m[b + i] = v;
  }
  __device__ __forceinline__ uint32_t rd(uint32_t b, uint32_t i) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)m[b + i]);
  }
  __device__ __forceinline__ size_t ix(uint32_t r) const { return fx_index(r, s, a.k.steps); }
  __device__ __forceinline__ uint32_t rw(uint32_t ph, uint32_t v, uint32_t j) const {
    return L.vreg + (ph * L.P + v) * L.DW + (j >> 5);
  }
  __device__ __forceinline__ void reg_clear(uint32_t v) {
    for (uint32_t i = lid; i < 2 * L.DW; i += 64) m[L.vreg + ((i / L.DW) * L.P + v) * L.DW + i % L.DW] = 0;
    sync();
  }

  // AEClock over a frontier word + ring bitmap (committed: c*, executed: e*)
  __device__ __forceinline__ bool contains(uint32_t front, uint32_t bits, uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
    if (src < 1 || src > L.n) return false;
    const uint32_t f = rd(front, src - 1);
    if (sq <= f) return true;
    if (sq - f - 1 >= L.WB * 32u) return false;
    const uint32_t b = sq & (L.WB * 32u - 1u);
    return (rd(bits, (src - 1) * L.WB + (b >> 5)) >> (b & 31u)) & 1u;
  }
  __device__ __forceinline__ void clock_add(uint32_t front, uint32_t bits, uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
    if (src < 1 || src > L.n) { err = FX_ERR_DOT_RANGE; return; }
    uint32_t f = rd(front, src - 1);
    if (sq <= f) return;
    if (sq - f - 1 >= L.WB * 32u) { err = FX_ERR_CAPACITY; return; }
    const uint32_t mask = L.WB * 32u - 1u;
    const uint32_t b = sq & mask, wi = (src - 1) * L.WB + (b >> 5);
    put(bits, wi, rd(bits, wi) | (1u << (b & 31u)));
    for (;;) {
      const uint32_t nb = (f + 1) & mask, nw = (src - 1) * L.WB + (nb >> 5);
      const uint32_t word = rd(bits, nw);
      if (!((word >> (nb & 31u)) & 1u)) break;
      put(bits, nw, word & ~(1u << (nb & 31u)));
      ++f;
    }
    put(front, src - 1, f);
  }

  __device__ __forceinline__ uint32_t hslot(uint32_t d) const {
    return (FX_DOT_SRC(d) - 1) * L.Q + (FX_DOT_SEQ(d) & (L.Q - 1u));
  }
  __device__ __forceinline__ uint32_t find(uint32_t d) {
    const uint32_t src = FX_DOT_SRC(d);
    if (src < 1 || src > L.n) return NONE;
    const uint32_t v = rd(L.hidx, hslot(d));
    return (v != 0 && rd(L.vdot, v - 1) == d) ? v - 1 : NONE;
  }
  __device__ __forceinline__ uint64_t clock_of(uint32_t v) {
    return ((uint64_t)rd(L.vchi, v) << 32) | rd(L.vclo, v);
  }

  // execute (mod.rs:369-383)
  __device__ __forceinline__ void execute(uint32_t d, uint32_t rec) {
    clock_add(L.efront, L.ebits, d);
    if (nexec >= a.k.steps) { err = FX_ERR_ORDER_OVERFLOW; return; }
    if (lid == 0) {
      a.k.order[ix(nexec)] = rec | FX_ORDER_SCC_START;
      a.k.release[ix(rec)] = step;
    }
    ++nexec;
  }

  // PendingIndex::remove(d) (index.rs:117-119) of phase `ph` (0 or 1) as a new
  // frame whose waiter list is ascending by dot
  __device__ void push_removed(uint32_t ph, uint32_t d) {
    if ((ph ? nreg1 : nreg0) == 0) return;  // no waiter anywhere: an empty frame
    if (fsp >= L.FD) { err = FX_ERR_CAPACITY; return; }
    const uint32_t base = ltop;
    uint32_t cnt = 0;
    for (uint32_t v0 = 0; v0 < L.P; v0 += 64) {
      const uint32_t v = v0 + lid;
      uint32_t hit = 0;
      if (v < L.P && m[L.vdot + v] != 0) {
        const uint32_t nd = m[L.vnd + v];
        for (uint32_t w = 0; w < L.DW && !hit; ++w) {
          uint32_t reg = m[rw(ph, v, w * 32)];
          while (reg) {
            const uint32_t j = w * 32 + __builtin_ctz(reg);
            reg &= reg - 1;
            if (j < nd && m[L.vdeps + v * L.D + j] == d) {
              hit = j + 1;
              break;
            }
          }
        }
      }
      const uint64_t b = __ballot(hit != 0);
      if (hit) {
        const uint32_t at = cnt + __builtin_popcountll(b & ((1ull << lid) - 1ull));
        m[L.tmp + at] = m[L.vdot + v];
        m[rw(ph, v, hit - 1)] &= ~(1u << ((hit - 1) & 31u));  // removed from the index
      }
      cnt += __builtin_popcountll(b);
    }
    sync();
    if (ph) nreg1 -= cnt;
    else nreg0 -= cnt;
    if (!cnt) return;  // an empty frame does nothing
    if (base + cnt > L.LL || cnt > L.P) { err = FX_ERR_CAPACITY; return; }
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {  // rank sort into the list stack
      const uint32_t i = i0 + lid;
      if (i < cnt) {
        const uint32_t x = m[L.tmp + i];
        uint32_t r = 0;
        for (uint32_t k = 0; k < cnt; ++k) r += m[L.tmp + k] < x ? 1u : 0u;
        m[L.lists + base + r] = x;
      }
    }
    sync();
    ltop += cnt;
    put(L.frames, fsp * 4 + 0, ph);
    put(L.frames, fsp * 4 + 1, base);
    put(L.frames, fsp * 4 + 2, cnt);
    put(L.frames, fsp * 4 + 3, 0);
    ++fsp;
  }

  // save_to_execute (mod.rs:341-367): remove, execute, then (depth first)
  // try_phase_two_pending.  v = find(d): every caller has just found it
  __device__ void save(uint32_t d, uint32_t v) {
    const uint32_t rec = rd(L.vrec, v);
    put(L.hidx, hslot(d), 0);
    put(L.vdot, v, 0);
    // (v's registrations are all gone: each was removed when its dep
    // committed / executed, which is what brought its missing count to 0)
    put(L.vfree, nfree++, v);
    execute(d, rec);
    push_removed(1, d);
  }

  // per-lane forms of contains / find (each lane asks about its own dot)
  __device__ __forceinline__ bool contains_v(uint32_t front, uint32_t bits, uint32_t d) const {
    const uint32_t src = FX_DOT_SRC(d), sq = FX_DOT_SEQ(d);
    if (src < 1 || src > L.n) return false;
    const uint32_t f = m[front + src - 1];
    if (sq <= f) return true;
    if (sq - f - 1 >= L.WB * 32u) return false;
    const uint32_t b = sq & (L.WB * 32u - 1u);
    return (m[bits + (src - 1) * L.WB + (b >> 5)] >> (b & 31u)) & 1u;
  }
  __device__ __forceinline__ uint32_t find_v(uint32_t d) const {
    const uint32_t src = FX_DOT_SRC(d);
    if (src < 1 || src > L.n) return NONE;
    const uint32_t v = m[L.hidx + hslot(d)];
    return (v != 0 && m[L.vdot + v - 1] == d) ? v - 1 : NONE;
  }
  // a phase's PendingIndex::index(dot, dep) for the deps j0 .. j0 + 63 of v
  // whose lanes are set in b: the phase's words of v are still zero (cleared
  // at commit, each phase registers once), so the ballot is the word pair
  __device__ __forceinline__ void reg_mask(uint32_t ph, uint32_t v, uint32_t j0, uint64_t b) {
    if (lid < 2 && j0 / 32 + lid < L.DW) m[rw(ph, v, j0 + 32 * lid)] = (uint32_t)(b >> (32 * lid));
  }

  // move_to_phase_two (mod.rs:208-275): the deps are checked lane-parallel
  // (nothing they read changes while they are checked); v = find(d)
  __device__ void phase_two(uint32_t d, uint32_t v) {
    const uint64_t cv = clock_of(v);
    const uint32_t nd = rd(L.vnd, v);
    uint32_t miss = 0;
    for (uint32_t j0 = 0; j0 < nd; j0 += 64) {
      const uint32_t j = j0 + lid;
      bool lower = false, gone = false;
      if (j < nd) {
        const uint32_t dep = m[L.vdeps + v * L.D + j];
        if (!contains_v(L.efront, L.ebits, dep)) {
          const uint32_t w = find_v(dep);
          if (w == NONE) gone = true;
          else lower = ((((uint64_t)m[L.vchi + w]) << 32) | m[L.vclo + w]) < cv;
        }
      }
      if (__ballot(gone)) { err = FX_ERR_CAPACITY; return; }  // "non-executed dependency must exist"
      const uint64_t b = __ballot(lower);
      reg_mask(1, v, j0, b);  // phase_two_pending_index.index(dot, dep)
      miss += (uint32_t)__builtin_popcountll(b);
    }
    nreg1 += miss;
    if (miss) put(L.vmiss, v, miss);
    else save(d, v);
  }

  // move_to_phase_one (mod.rs:154-206), lane-parallel over the deps; v =
  // find(d), nd its dep count
  __device__ void phase_one(uint32_t d, uint32_t v, uint32_t nd) {
    uint32_t miss = 0;
    for (uint32_t j0 = 0; j0 < nd; j0 += 64) {
      const uint32_t j = j0 + lid;
      const uint64_t b =
          __ballot(j < nd && !contains_v(L.cfront, L.cbits, m[L.vdeps + v * L.D + min(j, nd - 1)]));
      reg_mask(0, v, j0, b);  // phase_one_pending_index.index(dot, dep)
      miss += (uint32_t)__builtin_popcountll(b);
    }
    nreg0 += miss;
    if (miss) put(L.vmiss, v, miss);
    else phase_two(d, v);
  }

  // the frames: try_phase_one_pending / try_phase_two_pending (mod.rs:295-339)
  __device__ void run() {
    while (fsp && !err) {
      const uint32_t f = fsp - 1;
      const uint32_t ph = rd(L.frames, f * 4), base = rd(L.frames, f * 4 + 1), cnt = rd(L.frames, f * 4 + 2),
                     i = rd(L.frames, f * 4 + 3);
      if (i >= cnt) {
        --fsp;
        ltop = base;
        continue;
      }
      put(L.frames, f * 4 + 3, i + 1);
      const uint32_t p = rd(L.lists, base + i);
      const uint32_t v = find(p);
      if (v == NONE) { err = FX_ERR_CAPACITY; return; }  // "command pending ... must exist"
      const uint32_t mc = rd(L.vmiss, v);
      if (mc == 0) { err = FX_ERR_CAPACITY; return; }
      put(L.vmiss, v, mc - 1);
      if (mc == 1) {
        if (ph == 0) phase_two(p, v);
        else save(p, v);
      }
    }
  }

  // the inputs of the 4-step tile row holding step r0 (fx_index: 16 bytes per
  // plane): lane 4q + k holds step r0 + k of plane q -- 0 dot, 1 ndeps (or
  // hdr), 2 clock lo, 3 clock hi, 4 + j dep j (j < 12) -- so a row is one
  // load, issued one row ahead of its use.  r0 + 3 stays inside the padded
  // plane (steps rounded up to 4).
  __device__ __forceinline__ uint32_t row_load(uint32_t r0) const {
    const uint32_t q = lid >> 2, r = r0 + (lid & 3u);
    const size_t at = fx_index(r, s, a.k.steps);
    if (q == 0) return a.k.dot[at];
    if (q == 1) return a.ndeps ? a.ndeps[at] : a.k.hdr[at];
    if (q == 2) return a.clo[at];
    if (q == 3) return a.chi[at];
    const uint32_t j = q - 4;
    return j < a.k.dmax ? a.k.deps[(size_t)j * a.k.plane + at] : 0u;
  }
  __device__ __forceinline__ uint32_t row_at(uint32_t row, uint32_t q, uint32_t k) const {
    return (uint32_t)__builtin_amdgcn_readlane((int)row, (int)(4u * q + k));
  }

  // add (mod.rs:104-152); `row` = row_load(r & ~3)
  __device__ void add(uint32_t r, uint32_t row) {
    const size_t at = ix(r);
    const uint32_t k = r & 3u;
    const uint32_t d = row_at(row, 0, k);
    const uint32_t src = FX_DOT_SRC(d);
    if (src < 1 || src > L.n || FX_DOT_SEQ(d) == 0) { err = FX_ERR_DOT_RANGE; return; }
    // assert!(self.committed_clock.add(..)) (mod.rs:123): a dot commits once,
    // also after it executed (its index slot is gone by then)
    if (contains(L.cfront, L.cbits, d)) { err = FX_ERR_DOUBLE_INDEX; return; }
    clock_add(L.cfront, L.cbits, d);
    if (a.k.flags & FX_FLAG_EXECUTE_AT_COMMIT) {
      execute(d, r);
      return;
    }
    const uint32_t h = hslot(d), old = rd(L.hidx, h);
    if (old != 0) {
      err = rd(L.vdot, old - 1) == d ? FX_ERR_DOUBLE_INDEX : FX_ERR_CAPACITY;
      return;
    }
    if (!nfree) { err = FX_ERR_CAPACITY; return; }
    const uint32_t v = rd(L.vfree, --nfree);
    const uint32_t ndw = row_at(row, 1, k);
    const uint32_t nd = min(a.ndeps ? ndw : FX_HDR_ND(ndw), a.k.dmax);
    put(L.vdot, v, d);
    put(L.vrec, v, r);
    put(L.vclo, v, row_at(row, 2, k));
    put(L.vchi, v, row_at(row, 3, k));
    put(L.vmiss, v, 0);
    put(L.vnd, v, nd);
    reg_clear(v);
    {  // deps 0..11 from the row (every lane takes part in the permute), the rest from HBM
      const uint32_t src = 16u + 4u * min(lid, 11u) + k;
      const uint32_t dj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)row);
      if (lid < nd) m[L.vdeps + v * L.D + lid] = lid < 12u ? dj : a.k.deps[(size_t)lid * a.k.plane + at];
      for (uint32_t j = lid + 64; j < nd; j += 64) m[L.vdeps + v * L.D + j] = a.k.deps[(size_t)j * a.k.plane + at];
    }
    put(L.hidx, h, v + 1);
    sync();
    push_removed(0, d);  // try_phase_one_pending(dot)
    run();
    if (err) return;
    // move_to_phase_one(dot): v is still d's vertex (it holds no registration
    // yet, so nothing run() does can execute and free it)
    phase_one(d, v, nd);
    run();
  }
};

// FN / FD != 0 (the configs[1] shape, n = 5, dmax = 5): the SMALL tier with
// its layout compiled in -- table offsets become immediates, which frees the
// scalar registers the layout's fields held (the generic build spills about
// 50 SGPRs to VGPR lanes) -- and sized for occupancy: smaller tables
// (small_fixed_layout) and WPB streams per workgroup.  A CU holds at most 16
// workgroups, so one stream per workgroup stopped at 16 streams per CU
// whatever the tables; 4 per workgroup on 5.6 KB tables run 28.  Streams that
// outgrow the smaller tables rerun on the LDS tier as before.
#ifndef FX_PRED_WPB
#define FX_PRED_WPB 4  // streams per workgroup of the compiled n = 5 SMALL build
#endif
template <bool HBM, uint32_t FN = 0, uint32_t FD = 0, uint32_t WPB = 1>
__global__ __launch_bounds__(64 * WPB) void k_pred(PArgs a, Lay Lrt) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t wv = WPB > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0u;
  const uint32_t li = xcd_slot(blockIdx.x) * WPB + wv;
  if (li >= a.k.num_lanes) return;  // whole wavefront
  Lay L = Lrt;
  if constexpr (FN != 0) {
    L = small_fixed_layout(FN, FD);
    a.k.n = FN;
    a.k.dmax = FD;
  }
  Pr<(WPB > 1)> w;
  w.a = a;
  w.L = L;
  w.lid = threadIdx.x & 63u;
  w.s = a.k.stream_map ? a.k.stream_map[li] : li;
  w.m = HBM ? a.k.state + (size_t)li * L.words : smem + wv * L.words;
  for (uint32_t i = w.lid; i < L.words; i += 64) w.m[i] = 0;
  w.sync();
  for (uint32_t i = w.lid; i < L.P; i += 64) w.m[L.vfree + i] = L.P - 1u - i;
  w.sync();
  w.nfree = L.P;
  const uint32_t len = a.k.lengths ? min(a.k.lengths[w.s], a.k.steps) : a.k.steps;
  uint32_t row = len ? w.row_load(0) : 0u, next = len > 4 ? w.row_load(4) : 0u;
  for (uint32_t r = 0; r < len && !w.err; ++r) {
    if (r && !(r & 3u)) {
      row = next;
      if (r + 4 < len) next = w.row_load(r + 4);
    }
    w.step = r;
    w.add(r, row);
  }
  if (w.lid == 0) {
    a.k.nexec[w.s] = w.nexec;
    a.k.err[w.s] = w.err;
  }
}

}  // namespace pred

// SMALL: 64 vertices (128 index slots per source, 1024-bit windows, lists 4
// per vertex).  LDS: the most vertices of 512 / 256 / 128 whose tables fit
// 160 KiB (2 index slots per vertex and source, 2048-bit windows, lists 4 per
// vertex).  words == 0 when a tier does not fit.  HBM: 8192 vertices (16384
// index slots, 32768-bit windows, lists 8 per vertex).
static pred::Lay pred_layout(uint32_t tier, uint32_t n, uint32_t dmax) {
  pred::Lay L;
  const uint32_t D = std::max(dmax, 1u);
  if (tier == FX_PRED_TIER_HBM) {
    L.make(8192, 16384, 1024, n, D, 8 * 8192);
    return L;
  }
  if (tier == FX_PRED_TIER_SMALL) {
    L.make(64, 128, 32, n, D, 4 * 64);
    if ((size_t)L.words * 4 > 160 * 1024) L.words = 0;
    return L;
  }
  for (uint32_t P = 512; P >= 128; P /= 2) {
    L.make(P, 2 * P, 64, n, D, 4 * P);
    if ((size_t)L.words * 4 <= 160 * 1024) return L;
  }
  L.words = 0;
  return L;
}

}  // namespace fx

using namespace fx;

extern "C" size_t fx_pred_state_bytes(uint32_t n, uint32_t dmax, uint32_t lanes) {
  return (size_t)pred_layout(FX_PRED_TIER_HBM, std::max(n, 1u), dmax).words * 4 * lanes;
}

extern "C" int fx_pred_execute(const fx_pred_batch* in, const fx_order_batch* out, const uint32_t* stream_map,
                               uint32_t num_lanes, uint32_t tier, void* state, uint32_t flags,
                               void* hip_stream) {
  if (!in || !out || !in->base.dot || !in->base.hdr || (in->base.dmax && !in->base.deps) || !in->clock_lo ||
      !in->clock_hi || !out->order || !out->release || !out->nexec || !out->err)
    return FX_ERR_INVALID_ARG;
  if (in->base.n < 1 || in->base.n > 8 || in->base.dmax > FX_PRED_MAX_DEPS || in->base.steps >= (1u << 26) ||
      (!in->ndeps && in->base.dmax > 31))
    return FX_ERR_INVALID_ARG;
  if (fx_device_count() <= 0) return FX_ERR_NO_DEVICE;
  if (!stream_map && num_lanes > in->base.num_streams) return FX_ERR_INVALID_ARG;
  if (tier > FX_PRED_TIER_HBM || (tier == FX_PRED_TIER_HBM) != (state != nullptr)) return FX_ERR_INVALID_ARG;
  if (num_lanes == 0) return FX_OK;
  const bool hbm = tier == FX_PRED_TIER_HBM;
  pred::PArgs a{};
  a.k.dot = in->base.dot;
  a.k.hdr = in->base.hdr;
  a.k.deps = in->base.deps;
  a.k.lengths = in->base.lengths;
  a.k.S = in->base.num_streams;
  a.k.steps = in->base.steps;
  a.k.dmax = in->base.dmax;
  a.k.n = in->base.n;
  a.k.plane = fx_plane_words(in->base.num_streams, in->base.steps);
  a.k.order = out->order;
  a.k.release = out->release;
  a.k.nexec = out->nexec;
  a.k.err = out->err;
  a.k.stream_map = stream_map;
  a.k.num_lanes = num_lanes;
  a.k.state = (uint32_t*)state;
  a.k.flags = flags;
  a.clo = in->clock_lo;
  a.chi = in->clock_hi;
  a.ndeps = in->ndeps;
  const pred::Lay L = pred_layout(tier, in->base.n, in->base.dmax);
  hipStream_t hs = (hipStream_t)hip_stream;
  if (!hbm && L.words == 0) return FX_ERR_UNSUPPORTED;
  const uint32_t grid = xcd_grid(num_lanes);
  fx::profile_slot_record(FX_PROFILE_SLOT_PRED + tier, false, hs);
  if (hbm) {
    hipLaunchKernelGGL(pred::k_pred<true>, dim3(grid), dim3(64), 0, hs, a, L);
  } else {
    static bool configured = false;
    if (!configured) {
      (void)hipFuncSetAttribute((const void*)pred::k_pred<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      (void)hipFuncSetAttribute((const void*)pred::k_pred<false, 5, 5, FX_PRED_WPB>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      configured = true;
    }
    if (tier == FX_PRED_TIER_SMALL && in->base.n == 5 && std::max(in->base.dmax, 1u) == 5) {
      const pred::Lay L5 = pred::small_fixed_layout(5, 5);
      constexpr uint32_t W = FX_PRED_WPB;
      hipLaunchKernelGGL((pred::k_pred<false, 5, 5, W>), dim3(xcd_grid((num_lanes + W - 1u) / W)), dim3(64 * W),
                         (size_t)L5.words * 4 * W, hs, a, L5);
    } else
      hipLaunchKernelGGL(pred::k_pred<false>, dim3(grid), dim3(64), (size_t)L.words * 4, hs, a, L);
  }
  if (hipGetLastError() != hipSuccess) return FX_ERR_HIP;
  fx::profile_slot_record(FX_PROFILE_SLOT_PRED + tier, true, hs);
  return FX_OK;
}

// Every stream at SMALL, then the ones that ran out of capacity at LDS, then
// HBM (tiers whose tables do not fit are skipped).  Synchronous.
extern "C" int fx_pred_run(const fx_pred_batch* in, const fx_order_batch* out, uint32_t flags, void* hip_stream,
                           uint32_t* reruns) {
  if (reruns) *reruns = 0;
  if (!in) return FX_ERR_INVALID_ARG;
  const uint32_t S = in->base.num_streams, n = std::max(in->base.n, 1u);
  hipStream_t hs = (hipStream_t)hip_stream;
  std::vector<uint32_t> err(S), todo;
  bool first = true;
  uint32_t rr = 0;
  for (uint32_t tier = FX_PRED_TIER_SMALL; tier <= FX_PRED_TIER_HBM; ++tier) {
    if (pred_layout(tier, n, in->base.dmax).words == 0) continue;
    int st;
    if (first) {
      st = fx_pred_execute(in, out, nullptr, S, tier, nullptr, flags, hip_stream);
    } else {
      if (todo.empty()) break;
      std::lock_guard<std::recursive_mutex> lock(scratch_mutex());
      const uint32_t R = (uint32_t)todo.size();
      uint32_t* dmap = (uint32_t*)scratch(SCRATCH_TIERED_MAP, (size_t)R * 4);
      void* dstate = tier == FX_PRED_TIER_HBM ? scratch(SCRATCH_TIERED_STATE, fx_pred_state_bytes(n, in->base.dmax, R))
                                              : nullptr;
      if (!dmap || (tier == FX_PRED_TIER_HBM && !dstate)) return FX_ERR_HIP;
      if (hipMemcpyAsync(dmap, todo.data(), (size_t)R * 4, hipMemcpyHostToDevice, hs) != hipSuccess) return FX_ERR_HIP;
      st = fx_pred_execute(in, out, dmap, R, tier, dstate, flags, hip_stream);
      rr += R;
      if (!st && (hipMemcpyAsync(err.data(), out->err, (size_t)S * 4, hipMemcpyDeviceToHost, hs) != hipSuccess ||
                  hipStreamSynchronize(hs) != hipSuccess))
        return FX_ERR_HIP;
    }
    if (st) return st;
    if (first) {
      if (hipMemcpyAsync(err.data(), out->err, (size_t)S * 4, hipMemcpyDeviceToHost, hs) != hipSuccess ||
          hipStreamSynchronize(hs) != hipSuccess)
        return FX_ERR_HIP;
      first = false;
    }
    todo.clear();
    for (uint32_t s = 0; s < S; ++s)
      if (err[s] == FX_ERR_CAPACITY) todo.push_back(s);
  }
  if (reruns) *reruns = rr;
  for (uint32_t s = 0; s < S; ++s)
    if (err[s]) return (int)err[s];
  return FX_OK;
}
