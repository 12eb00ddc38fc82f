// graph_exec.hip — batched GraphExecutor for gfx950 (MI355X).
//
// One lane = one commit stream = one (instance, process) executor of the
// reference (fantoch_ps/src/executor/graph/executor.rs:19-29 owns one
// DependencyGraph each).  A 64-thread workgroup is one wavefront running 64
// independent executors; there is no inter-lane communication, so nothing
// here depends on dispatch order or XCD placement.
//
// Per-lane executor state lives in LDS in a lane-interleaved layout: state
// word w of lane l is at LDS dword (w * 64 + l), so whatever slot index each
// lane touches, the bank is (l mod 32) and every ds_read/ds_write_b32 is
// conflict-free.  The state restates the reference's containers as fixed
// tables:
//   executed clock AEClock (threshold 0.9.1; tarjan.rs:131-132,293):
//     per source a u32 frontier + a XW-word bitmap of executed seqs above it
//   VertexIndex (index.rs:18-51):  P pending-vertex slots {dot, rec|nd, wait, tarjan}
//   PendingIndex (index.rs:145-208): slot.wait = the missing dot the vertex is
//     registered on (a vertex is registered on at most one dot at a time)
//   TarjanSCCFinder (tarjan.rs:25-33): explicit DFS frame stack + Tarjan stack
//   check_pending's `dots` (mod.rs:556-587): LIFO worklist
// plus per-lane bitmasks in VGPRs: occupied slots, registered waiters, and the
// try_pending snapshot.  A stream whose pending set or clock window outgrows
// its tier stops with FX_ERR_CAPACITY and is rerun at the next tier.
//
// Records stream through a 3-block register pipeline (a block = 4 steps = one
// 16-byte load per lane per plane, see fx_index in fantoch_amd.h).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "fantoch_amd.h"
#include "fx_internal.h"
#include "fx_synth.h"

namespace fx {

constexpr uint32_t WAVE = 64;
constexpr uint32_t DCAP = 8;  // deps of the incoming Add held in registers

template <uint32_t NSRC_, uint32_t P_, uint32_t XW_, uint32_t C_, bool GLOBAL_>
struct Tier {
  static constexpr uint32_t NSRC = NSRC_;  // sources (processes) supported
  static constexpr uint32_t P = P_;        // pending-vertex slots (<= 64: u64 masks)
  static constexpr uint32_t XW = XW_;      // clock window words per source
  static constexpr uint32_t C = C_;        // cached not-yet-executed deps per vertex
  static constexpr bool GLOBAL = GLOBAL_;  // state in HBM instead of LDS
  static constexpr bool HINT = P <= 15;    // cached deps carry the dep's slot + 1
  static constexpr uint32_t CLKS = 1 + XW;
  static constexpr uint32_t CLK = 0;
  static constexpr uint32_t DOT = CLK + NSRC * CLKS;  // packed dot, per slot
  static constexpr uint32_t REC = DOT + P;            // arrival index | ncached << 26
  static constexpr uint32_t WAIT = REC + P;           // registered-on dot (0 = none)
  static constexpr uint32_t TL = WAIT + P;            // id:12 | low:12 | visited epoch:8
  static constexpr uint32_t DEP = TL + P;             // [C][P] cached deps: dot | hint << 28
  static constexpr uint32_t TS = DEP + C * P;         // Tarjan stack, u8 slots
  static constexpr uint32_t FR = TS + (P + 3) / 4;    // DFS frames, u16 slot | dep idx << 8
  static constexpr uint32_t WL = FR + (P + 1) / 2;    // worklist, P + 1 packed dots
  static constexpr uint32_t REG = WL + P + 1;         // words mirrored in LDS
  static constexpr uint32_t WORDS = REG + 6;          // + saved registers (global only)
  static_assert(P <= 64, "slot masks are u64");
  static_assert(P < 256, "slots are u8");
  static_assert(C < 32, "ncached is 5 bits");
};

// LDS bytes / wave: Tier0 37,376 -> 4 waves / CU; Tier1 123,136 -> 1 wave / CU.
using Tier0 = Tier<8, 12, 1, 5, false>;
using Tier1 = Tier<8, 32, 4, 8, false>;
using Tier2 = Tier<8, 64, 32, 16, true>;  // HBM-resident, 1024-bit clock windows

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
};

__device__ __forceinline__ uint32_t hdr_nd(uint32_t h) { return (h >> 24) & 31u; }

template <class T>
struct Exec {
  uint32_t* st;  // this lane's state: word w at st[w * WAVE]
  uint64_t occ = 0, wmask = 0, tmask = 0;
  uint32_t k = 0, err = 0, epoch = 1, nwl = 0, cur = 0;
  uint32_t stream = 0, n = 0, steps = 0, dmax = 0;
  size_t plane = 0;
  const uint32_t* deps = nullptr;
  uint32_t* order = nullptr;
  uint32_t* release = nullptr;

  __device__ __forceinline__ uint32_t& w(uint32_t i) { return st[i * WAVE]; }
  __device__ __forceinline__ uint8_t& ts(uint32_t i) {
    return reinterpret_cast<uint8_t*>(&w(T::TS + (i >> 2)))[i & 3];
  }
  __device__ __forceinline__ uint16_t& fr(uint32_t i) {
    return reinterpret_cast<uint16_t*>(&w(T::FR + (i >> 1)))[i & 1];
  }
  __device__ __forceinline__ uint32_t& wl(uint32_t i) { return w(T::WL + i); }
  __device__ __forceinline__ size_t at(uint32_t step) const { return fx_index(step, stream, steps); }

  // ---------------------------------------------- executed clock (AEClock)
  // AEClock::contains (tarjan.rs:131-132)
  __device__ __forceinline__ bool clk_contains(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) return false;
    const uint32_t seq = d & FX_SEQ_MASK;
    const uint32_t b = T::CLK + si * T::CLKS;
    const uint32_t f = w(b);
    if (seq <= f) return true;
    const uint32_t off = seq - f - 1u;
    if (off >= 32u * T::XW) return false;
    return (w(b + 1 + (off >> 5)) >> (off & 31u)) & 1u;
  }
  // AEClock::add (tarjan.rs:293): frontier + exception window
  __device__ __forceinline__ void clk_add(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) { err = FX_ERR_DOT_RANGE; return; }
    const uint32_t seq = d & FX_SEQ_MASK;
    const uint32_t b = T::CLK + si * T::CLKS;
    const uint32_t f = w(b);
    if (seq <= f) return;
    const uint32_t off = seq - f - 1u;
    if (off >= 32u * T::XW) { err = FX_ERR_CAPACITY; return; }
    if (off != 0) {
      w(b + 1 + (off >> 5)) |= 1u << (off & 31u);
      return;
    }
    if constexpr (T::XW == 1) {
      const uint32_t win = w(b + 1) >> 1;          // bit j <-> seq f + 2 + j
      const uint32_t ones = __builtin_ctz(~win);   // top bit of win is 0 -> <= 31
      w(b) = f + 1 + ones;
      w(b + 1) = win >> ones;
    } else {
      // t = 1 + trailing ones of the window from bit 1
      uint32_t t = 1;
      while (t < 32u * T::XW) {
        const uint32_t word = w(b + 1 + (t >> 5)) >> (t & 31u);
        const uint32_t avail = 32u - (t & 31u);
        const uint32_t inv = ~word;
        const uint32_t run = inv ? (uint32_t)__builtin_ctz(inv) : 32u;
        const uint32_t r = run < avail ? run : avail;
        t += r;
        if (r < avail) break;
      }
      w(b) = f + t;
      const uint32_t ws = t >> 5, sh = t & 31u;
#pragma unroll
      for (uint32_t q = 0; q < T::XW; ++q) {
        const uint32_t lo = q + ws;
        uint32_t v = lo < T::XW ? (w(b + 1 + lo) >> sh) : 0u;
        if (sh && lo + 1 < T::XW) v |= w(b + 2 + lo) << (32u - sh);
        w(b + 1 + q) = v;
      }
    }
  }

  // ----------------------------------------------- VertexIndex slot table
  __device__ __forceinline__ int pt_find(uint32_t d) {
    for (uint64_t m = occ; m; m &= m - 1) {
      const int sl = __builtin_ctzll(m);
      if (w(T::DOT + sl) == d) return sl;
    }
    return -1;
  }
  __device__ __forceinline__ int pt_insert(uint32_t d, uint32_t rec) {
    constexpr uint64_t full = T::P == 64 ? ~0ull : ((1ull << T::P) - 1ull);
    const uint64_t fre = ~occ & full;
    if (!fre) { err = FX_ERR_CAPACITY; return -1; }
    const int sl = __builtin_ctzll(fre);
    occ |= 1ull << sl;
    w(T::DOT + sl) = d;
    w(T::REC + sl) = rec;
    w(T::WAIT + sl) = 0;
    w(T::TL + sl) = 0;
    return sl;
  }
  // Vertex::deps restricted to the deps not executed at insertion (executed
  // deps are ignored by every later search, tarjan.rs:128-145, and the
  // executed clock only grows), ascending; a dep pending at insertion carries
  // its slot (it can only leave that slot by being executed).
  __device__ __forceinline__ void pt_cache_dep(int sl, uint32_t d, uint32_t dep, uint32_t& nc) {
    if (dep == d || clk_contains(dep)) return;
    if ((dep >> FX_SEQ_BITS) > 15u) { err = FX_ERR_DOT_RANGE; return; }
    if (nc >= T::C) { err = FX_ERR_CAPACITY; return; }
    uint32_t hint = 0;
    if constexpr (T::HINT) hint = (uint32_t)(pt_find(dep) + 1);
    w(T::DEP + nc * T::P + sl) = dep | (hint << 28);
    ++nc;
  }
  __device__ __forceinline__ void pt_free(int sl) {
    const uint64_t keep = ~(1ull << sl);
    occ &= keep;
    wmask &= keep;
    tmask &= keep;
  }

  // try_pending's `visited` set (mod.rs:598): an epoch stamp per slot
  __device__ __forceinline__ void new_epoch() {
    epoch = (epoch + 1) & 0xFFu;
    if (epoch == 0) {
      for (uint64_t m = occ; m; m &= m - 1) w(T::TL + __builtin_ctzll(m)) &= 0x00FFFFFFu;
      epoch = 1;
    }
  }

  // save_scc (mod.rs:488-523) for one member: to_execute + executed clock
  __device__ __forceinline__ void emit(uint32_t rec, uint32_t d, bool start) {
    if (k >= steps) { err = FX_ERR_ORDER_OVERFLOW; return; }
    order[at(k)] = rec | (start ? FX_ORDER_SCC_START : 0u);
    release[at(rec)] = cur;
    ++k;
    clk_add(d);
  }

  // find_scc (mod.rs:409-486) + TarjanSCCFinder::strong_connect
  // (tarjan.rs:96-316) + finalize (tarjan.rs:60-93), iterative.  Returns the
  // missing dep (0 = Found).  `emitted` = an SCC was saved by this search.
  __device__ __forceinline__ uint32_t find_scc(int root, bool in_try, bool& emitted) {
    uint32_t idc = 1, nts = 0, nfr = 0, missing = 0;
    emitted = false;
    w(T::TL + root) = (w(T::TL + root) & 0xFF000000u) | 1u | (1u << 12);
    ts(nts++) = (uint8_t)root;
    fr(nfr++) = (uint16_t)root;
    while (nfr > 0) {
      const uint32_t f = fr(nfr - 1);
      const uint32_t v = f & 0xFFu, di = f >> 8;
      const uint32_t nd = w(T::REC + v) >> 26;
      if (di < nd) {
        fr(nfr - 1) = (uint16_t)(v | ((di + 1) << 8));
        const uint32_t cw = w(T::DEP + di * T::P + v);
        const uint32_t dep = cw & 0x0FFFFFFFu;
        // ignore self or already executed (tarjan.rs:128-145); self was dropped at insertion
        if (clk_contains(dep)) continue;
        int x = -1;
        if constexpr (T::HINT) {
          const uint32_t h = cw >> 28;
          if (h && w(T::DOT + h - 1) == dep) x = (int)h - 1;
        }
        if (x < 0) x = pt_find(dep);
        if (x < 0) {  // missing: give up (tarjan.rs:148-157, shard_count == 1)
          missing = dep;
          break;
        }
        const uint32_t tx = w(T::TL + x);
        if ((tx & 0xFFFu) == 0) {  // not visited: recurse (tarjan.rs:172-214)
          ++idc;
          w(T::TL + x) = (tx & 0xFF000000u) | idc | (idc << 12);
          ts(nts++) = (uint8_t)x;
          fr(nfr++) = (uint16_t)x;
        } else {  // visited and on the stack (tarjan.rs:215-225)
          const uint32_t tv = w(T::TL + v);
          const uint32_t idx = tx & 0xFFFu;
          if (idx < ((tv >> 12) & 0xFFFu)) w(T::TL + v) = (tv & 0xFF000FFFu) | (idx << 12);
        }
      } else {
        --nfr;
        const uint32_t tv = w(T::TL + v);
        const uint32_t lowv = (tv >> 12) & 0xFFFu;
        if ((tv & 0xFFFu) == lowv) {  // SCC root (tarjan.rs:233-312)
          uint32_t pos = nts - 1;
          while (ts(pos) != v) --pos;
          // members ascending by dot (SCC = BTreeSet<Dot>, tarjan.rs:15)
          for (uint32_t a = pos + 1; a < nts; ++a) {
            const uint8_t key = ts(a);
            const uint32_t kd = w(T::DOT + key);
            uint32_t b = a;
            while (b > pos && w(T::DOT + ts(b - 1)) > kd) {
              ts(b) = ts(b - 1);
              --b;
            }
            ts(b) = key;
          }
          for (uint32_t a = pos; a < nts; ++a) {
            const uint32_t sl = ts(a);
            const uint32_t d = w(T::DOT + sl);
            emit(w(T::REC + sl) & 0x03FFFFFFu, d, a == pos);
            if (err) return 0;
            wl(nwl++) = d;
            pt_free((int)sl);
          }
          nts = pos;
          emitted = true;
          if (err) return 0;
        }
        if (nfr > 0) {  // low = min(low, dep.low) after the recursion (tarjan.rs:211)
          const uint32_t p = fr(nfr - 1) & 0xFFu;
          const uint32_t tp = w(T::TL + p);
          if (lowv < ((tp >> 12) & 0xFFFu)) w(T::TL + p) = (tp & 0xFF000FFFu) | (lowv << 12);
        }
      }
    }
    // finalize: reset the ids of the vertices left on the stack; in try_pending
    // a failed search that found no SCC adds them to `visited` (mod.rs:621-629)
    const bool mark = in_try && missing != 0 && !emitted;
    for (uint32_t a = 0; a < nts; ++a) {
      const uint32_t sl = ts(a);
      const uint32_t tv = w(T::TL + sl);
      w(T::TL + sl) = mark ? (epoch << 24) : (tv & 0xFF000000u);
    }
    return missing;
  }

  // try_pending (mod.rs:589-642): the snapshot in tmask, tried ascending (C2)
  __device__ __forceinline__ void try_pending() {
    new_epoch();  // visited = {}
    while (tmask && !err) {
      int best = -1;
      uint32_t bd = 0xFFFFFFFFu;
      for (uint64_t m = tmask; m; m &= m - 1) {
        const int sl = __builtin_ctzll(m);
        const uint32_t dd = w(T::DOT + sl);
        if (dd < bd) { bd = dd; best = sl; }
      }
      tmask &= ~(1ull << best);
      if ((w(T::TL + best) >> 24) == epoch) continue;  // visited: skipped, not re-registered
      bool em;
      const uint32_t miss = find_scc(best, true, em);
      if (err) return;
      if (miss == 0) {
        new_epoch();  // Found: visited.clear()
      } else {
        w(T::WAIT + best) = miss;  // index_pending (mod.rs:525-554)
        wmask |= 1ull << best;
        if (em) new_epoch();
      }
    }
  }

  // check_pending (mod.rs:556-587): LIFO over released dots
  __device__ __forceinline__ void check_pending() {
    while (nwl > 0 && !err) {
      if (!wmask) { nwl = 0; return; }
      const uint32_t x = wl(--nwl);
      uint64_t t = 0;
      for (uint64_t m = wmask; m; m &= m - 1) {
        const int sl = __builtin_ctzll(m);
        if (w(T::WAIT + sl) == x) t |= 1ull << sl;
      }
      if (!t) continue;
      wmask &= ~t;  // PendingIndex::remove(x) (index.rs:205-207)
      for (uint64_t m = t; m; m &= m - 1) w(T::WAIT + __builtin_ctzll(m)) = 0;
      tmask = t;
      try_pending();
    }
  }

  // VertexIndex::index(Vertex::new(dot, cmd, deps, time)) (index.rs:33-37):
  // deps j < DCAP come from the prefetched registers, the rest from HBM.
  __device__ __forceinline__ int insert_vertex(uint32_t i, uint32_t d, uint32_t nd, const uint4* rdeps) {
    const int sl = pt_insert(d, i);
    if (sl < 0) return -1;
    uint32_t nc = 0;
#pragma unroll
    for (uint32_t j = 0; j < DCAP; ++j)
      if (j < nd) pt_cache_dep(sl, d, rdeps[j].x, nc);
    for (uint32_t j = DCAP; j < nd; ++j) pt_cache_dep(sl, d, deps[(size_t)j * plane + at(i)], nc);
    if (err) return -1;
    w(T::REC + sl) = i | (nc << 26);
    return sl;
  }

  // GraphExecutor::handle(Add) (executor.rs:69-80) -> handle_add (mod.rs:213-275)
  __device__ __forceinline__ void handle(uint32_t i, uint32_t d, uint32_t h, const uint4* rdeps,
                                         bool at_commit) {
    cur = i;
    const uint32_t nd = hdr_nd(h), kind = h >> 29;
    if (nd > dmax) { err = FX_ERR_INVALID_ARG; return; }  // deps beyond the dep planes
    if ((d >> FX_SEQ_BITS) - 1u >= n || (d & FX_SEQ_MASK) == 0) { err = FX_ERR_DOT_RANGE; return; }
    if (at_commit) {  // execute_at_commit bypass (executor.rs:72-73)
      order[at(k)] = i | FX_ORDER_SCC_START;
      release[at(i)] = i;
      ++k;
      return;
    }
    if (occ && pt_find(d) >= 0) { err = FX_ERR_DOUBLE_INDEX; return; }  // mod.rs:233-237
    if (kind == FX_KIND_INDEX_ONLY) {
      insert_vertex(i, d, nd, rdeps);
      return;
    }
    // Fast path: every dep is self or executed -> strong_connect visits only
    // the new vertex and saves it as a singleton SCC.
    bool fast = nd <= DCAP;
    uint32_t prev = 0;
#pragma unroll
    for (uint32_t j = 0; j < DCAP; ++j) {
      if (j < nd) {
        const uint32_t dep = rdeps[j].x;
        if (dep <= prev) err = FX_ERR_DEPS_UNSORTED;
        prev = dep;
        if (dep != d && !clk_contains(dep)) fast = false;
      }
    }
    if (err) return;
    nwl = 0;
    if (fast) {
      emit(i, d, true);
      if (!wmask || err) return;
      wl(nwl++) = d;
    } else {
      const int sl = insert_vertex(i, d, nd, rdeps);
      if (sl < 0) return;
      bool em;
      const uint32_t miss = find_scc(sl, false, em);
      if (err) return;
      if (miss) {  // index_pending(dot, missing) (mod.rs:251-256)
        w(T::WAIT + sl) = miss;
        wmask |= 1ull << sl;
      }
    }
    check_pending();
  }
};

template <class T>
__global__ __launch_bounds__(64) void k_graph_exec(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t lane = threadIdx.x;
  const uint32_t gl = blockIdx.x * WAVE + lane;
  const bool active = gl < a.num_lanes;
  const uint32_t s = active ? (a.stream_map ? a.stream_map[gl] : gl) : 0u;
  const uint32_t len = active ? (a.lengths ? min(a.lengths[s], a.steps) : a.steps) : 0u;
  uint32_t* gblock = a.state ? a.state + (size_t)blockIdx.x * T::WORDS * WAVE : nullptr;

  Exec<T> e;
  if constexpr (T::GLOBAL) e.st = gblock + lane;
  else e.st = smem + lane;
  e.stream = s;
  e.n = a.n;
  e.steps = a.steps;
  e.plane = a.plane;
  e.dmax = a.dmax;
  e.deps = a.deps;
  e.order = a.order;
  e.release = a.release;

  if (a.flags & FX_FLAG_INIT) {
    for (uint32_t q = 0; q < T::NSRC * T::CLKS; ++q) e.w(T::CLK + q) = 0;
    if (a.init_frontier && active) {
      for (uint32_t p = 0; p < T::NSRC && p < 8; ++p) e.w(T::CLK + p * T::CLKS) = a.init_frontier[(size_t)s * 8 + p];
    }
  } else {
    if constexpr (!T::GLOBAL) {
      for (uint32_t q = 0; q < T::REG; ++q) smem[q * WAVE + lane] = gblock[q * WAVE + lane];
    }
    const uint32_t* r = gblock + (size_t)T::REG * WAVE + lane;
    e.occ = (uint64_t)r[0] | ((uint64_t)r[WAVE] << 32);
    e.wmask = (uint64_t)r[2 * WAVE] | ((uint64_t)r[3 * WAVE] << 32);
    e.k = r[4 * WAVE];
    e.err = r[5 * WAVE] & 0xFFFFu;
    e.epoch = r[5 * WAVE] >> 16;
  }
  if (!active) e.err = FX_ERR_INVALID_ARG;  // idle lane (its loads read stream 0)

  const bool at_commit = (a.flags & FX_FLAG_EXECUTE_AT_COMMIT) != 0;
  const uint32_t steps4 = (a.steps + 3) >> 2;
  const size_t lane_off = (size_t)(s >> 6) * steps4 * 256 + ((s & 63u) << 2);
  const uint32_t b_begin = a.step_begin >> 2;
  const uint32_t b_end = (a.step_end + 3) >> 2;
  const uint32_t dmax = a.dmax;

  // Prefetch: every block issues the same 2 + DCAP 16-byte loads per lane
  // (addresses clamped instead of branched around), so the compiler's
  // s_waitcnt for a block's data is a precise vmcnt(N) and never waits for
  // the next block's loads or for this block's scattered stores.
  const uint32_t* dotp = a.dot + lane_off;
  const uint32_t* hdrp = a.hdr + lane_off;
  const uint32_t* depp = (dmax ? a.deps : a.dot) + lane_off;
  const size_t plane = dmax ? a.plane : 0;
  const uint32_t jlast = dmax ? dmax - 1 : 0;
  const uint32_t b_last = b_end ? b_end - 1 : 0;
#define FX_LOAD(B, D, H, DP)                                                                 \
  do {                                                                                       \
    const size_t off_ = (size_t)min((B), b_last) * 256;                                      \
    D = *reinterpret_cast<const uint4*>(dotp + off_);                                        \
    H = *reinterpret_cast<const uint4*>(hdrp + off_);                                        \
    _Pragma("unroll") for (uint32_t j = 0; j < DCAP; ++j)                                    \
      DP[j] = *reinterpret_cast<const uint4*>(depp + (size_t)min(j, jlast) * plane + off_); \
  } while (0)

  uint4 cd, ch, nd_, nh;
  uint4 d0[DCAP], d1[DCAP];
  if (b_begin < b_end) FX_LOAD(b_begin, cd, ch, d0);

  for (uint32_t b = b_begin; b < b_end; ++b) {
    FX_LOAD(b + 1, nd_, nh, d1);
    const uint32_t base = b * 4;
    const uint32_t q0 = base < a.step_begin ? a.step_begin - base : 0u;
    const uint32_t q1 = a.step_end - base < 4u ? a.step_end - base : 4u;
    // Steps are consumed from component x; the block is rotated one step per
    // iteration so every register index stays static (no scratch).
    for (uint32_t q = 0; q < q1; ++q) {
      const uint32_t i = base + q;
      if (q >= q0 && !e.err && i < len) e.handle(i, cd.x, ch.x, d0, at_commit);
      cd = make_uint4(cd.y, cd.z, cd.w, 0u);
      ch = make_uint4(ch.y, ch.z, ch.w, 0u);
#pragma unroll
      for (uint32_t j = 0; j < DCAP; ++j) d0[j] = make_uint4(d0[j].y, d0[j].z, d0[j].w, 0u);
    }
    cd = nd_;
    ch = nh;
#pragma unroll
    for (uint32_t j = 0; j < DCAP; ++j) d0[j] = d1[j];
  }
#undef FX_LOAD

  if (!active) return;
  // Vertices still pending have no release step (yet).
  for (uint64_t m = e.occ; m; m &= m - 1) {
    const int sl = __builtin_ctzll(m);
    a.release[e.at(e.w(T::REC + sl) & 0x03FFFFFFu)] = FX_RELEASE_NONE;
  }
  a.nexec[s] = e.k;
  a.err[s] = e.err;
  if (a.flags & FX_FLAG_SAVE_STATE) {
    if constexpr (!T::GLOBAL) {
      for (uint32_t q = 0; q < T::REG; ++q) gblock[q * WAVE + lane] = smem[q * WAVE + lane];
    }
    uint32_t* r = gblock + (size_t)T::REG * WAVE + lane;
    r[0] = (uint32_t)e.occ;
    r[WAVE] = (uint32_t)(e.occ >> 32);
    r[2 * WAVE] = (uint32_t)e.wmask;
    r[3 * WAVE] = (uint32_t)(e.wmask >> 32);
    r[4 * WAVE] = e.k;
    r[5 * WAVE] = (e.err & 0xFFFFu) | (e.epoch << 16);
  }
}

// ------------------------------------------------------------- metrics
// Metrics::collect for ChainSize (one sample per SCC, mod.rs:492-493) and
// ExecutionDelay (t(release) - t(add), mod.rs:514-518).  One 256-thread block
// per (tile, 4-row block): thread t reads order word t of that 1 KiB granule.
__global__ __launch_bounds__(256) void k_metrics(const uint32_t* __restrict__ hdr,
                                                 const uint32_t* __restrict__ order,
                                                 const uint32_t* __restrict__ release,
                                                 const uint32_t* __restrict__ nexec, uint32_t S,
                                                 uint32_t steps, unsigned long long* chain,
                                                 uint32_t nbc, unsigned long long* delay,
                                                 uint32_t nbd, uint32_t use_lds) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // [nbc + nbd]
  const uint32_t steps4 = (steps + 3) >> 2;
  const uint32_t tiles = (S + 63) >> 6;
  const size_t nblocks = (size_t)tiles * steps4;
  if (use_lds) {
    for (uint32_t q = threadIdx.x; q < nbc + nbd; q += blockDim.x) hist[q] = 0;
    __syncthreads();
  }
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t >> 2, kq = t & 3;
  for (size_t blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const uint32_t tile = (uint32_t)(blk / steps4), kb = (uint32_t)(blk % steps4);
    const uint32_t s = tile * 64 + lane;
    const uint32_t k = kb * 4 + kq;
    if (s >= S || k >= nexec[s]) continue;
    const uint32_t ne = nexec[s];
    const size_t tile_base = (size_t)tile * steps4 * 256 + (lane << 2);
    const uint32_t o = order[tile_base + (size_t)kb * 256 + kq];
    const uint32_t rec = o & 0x7FFFFFFFu;
    const uint32_t rs = release[fx_index(rec, s, steps)];
    if (rec >= steps || rs >= steps) continue;  // not executed (errored stream)
    const uint32_t dl = FX_HDR_T(hdr[fx_index(rs, s, steps)]) - FX_HDR_T(hdr[fx_index(rec, s, steps)]);
    const uint32_t db = dl < nbd - 1 ? dl : nbd - 1;
    if (use_lds) atomicAdd(&hist[nbc + db], 1u);
    else atomicAdd(&delay[db], 1ull);
    if (o & FX_ORDER_SCC_START) {
      uint32_t size = 1;
      while (k + size < ne && !(order[fx_index(k + size, s, steps)] & FX_ORDER_SCC_START)) ++size;
      const uint32_t cb = size < nbc - 1 ? size : nbc - 1;
      if (use_lds) atomicAdd(&hist[cb], 1u);
      else atomicAdd(&chain[cb], 1ull);
    }
  }
  if (use_lds) {
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nbc + nbd; q += blockDim.x) {
      const uint32_t v = hist[q];
      if (v) {
        if (q < nbc) atomicAdd(&chain[q], (unsigned long long)v);
        else atomicAdd(&delay[q - nbc], (unsigned long long)v);
      }
    }
  }
}

// ----------------------------------------------------------- synthesis
__global__ __launch_bounds__(256) void k_synth(fx_synth_params p, uint32_t S, uint32_t steps,
                                               uint32_t* dot, uint32_t* hdr, uint32_t* deps) {
  const uint32_t N = p.n * p.cmds_per_process;
  const size_t total = (size_t)p.instances * N;
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (size_t)gridDim.x * blockDim.x) {
    synth_emit(p, (uint32_t)(x / N), (uint32_t)(x % N), S, steps, dot, hdr, deps);
  }
}

// ------------------------------------------------------------ host side
static int g_device_count = -1;

static int device_count() {
  if (g_device_count < 0) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    g_device_count = c;
  }
  return g_device_count;
}

template <class T>
static size_t state_bytes(uint32_t lanes) {
  return (size_t)((lanes + WAVE - 1) / WAVE) * T::WORDS * WAVE * 4;
}

template <class T>
static int launch_exec(const KArgs& a, hipStream_t stream) {
  if (T::GLOBAL && !a.state) return FX_ERR_INVALID_ARG;
  const uint32_t blocks = (a.num_lanes + WAVE - 1) / WAVE;
  if (blocks == 0) return FX_OK;
  const size_t lds = T::GLOBAL ? 0 : (size_t)T::REG * WAVE * 4;
  static bool configured = false;
  if (!configured && lds > 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)k_graph_exec<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    configured = true;
  }
  hipLaunchKernelGGL(k_graph_exec<T>, dim3(blocks), dim3(WAVE), lds, stream, a);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

template <class T>
static uint32_t decode_pending_t(const uint32_t* block, uint32_t lane, uint32_t* dots,
                                 uint32_t* waits, uint32_t cap) {
  const uint32_t* r = block + (size_t)T::REG * WAVE + lane;
  const uint64_t occ = (uint64_t)r[0] | ((uint64_t)r[WAVE] << 32);
  const uint64_t wm = (uint64_t)r[2 * WAVE] | ((uint64_t)r[3 * WAVE] << 32);
  uint32_t c = 0;
  for (uint64_t m = occ; m; m &= m - 1) {
    const int sl = __builtin_ctzll(m);
    if (c < cap) {
      dots[c] = block[(T::DOT + sl) * WAVE + lane];
      waits[c] = ((wm >> sl) & 1) ? block[(T::WAIT + sl) * WAVE + lane] : 0u;
    }
    ++c;
  }
  return c;
}

uint32_t decode_pending(uint32_t tier, const uint32_t* block, uint32_t lane, uint32_t* dots,
                        uint32_t* waits, uint32_t cap) {
  switch (tier) {
    case 0: return decode_pending_t<Tier0>(block, lane, dots, waits, cap);
    case 1: return decode_pending_t<Tier1>(block, lane, dots, waits, cap);
    case 2: return decode_pending_t<Tier2>(block, lane, dots, waits, cap);
    default: return 0;
  }
}

static bool g_profile = false;
static hipEvent_t g_ev0 = nullptr, g_ev1 = nullptr;
static bool g_ev_valid = false;

}  // namespace fx

using namespace fx;

extern "C" {

int fx_device_count(void) { return device_count(); }

const char* fx_version(void) { return "fantoch_amd 0.1.0 (gfx950)"; }

const char* fx_status_string(int s) {
  switch (s) {
    case FX_OK: return "ok";
    case FX_ERR_INVALID_ARG: return "invalid argument";
    case FX_ERR_CAPACITY: return "tier capacity exceeded";
    case FX_ERR_DOUBLE_INDEX: return "tried to index already indexed dot";
    case FX_ERR_DEPS_UNSORTED: return "deps not strictly ascending";
    case FX_ERR_DOT_RANGE: return "dot out of range";
    case FX_ERR_HIP: return "HIP runtime error";
    case FX_ERR_UNSUPPORTED: return "unsupported (partial replication)";
    case FX_ERR_ORDER_OVERFLOW: return "order plane overflow";
    case FX_ERR_TIME_RANGE: return "time out of range";
    case FX_ERR_NO_DEVICE: return "no GPU device";
    default: return "unknown";
  }
}

int fx_tier_query(uint32_t tier, uint32_t n, fx_tier_info* out) {
  if (!out) return FX_ERR_INVALID_ARG;
  switch (tier) {
    case 0: *out = {Tier0::NSRC, Tier0::P, 32 * Tier0::XW, Tier0::WORDS}; break;
    case 1: *out = {Tier1::NSRC, Tier1::P, 32 * Tier1::XW, Tier1::WORDS}; break;
    case 2: *out = {Tier2::NSRC, Tier2::P, 32 * Tier2::XW, Tier2::WORDS}; break;
    default: return FX_ERR_INVALID_ARG;
  }
  return n >= 1 && n <= out->max_sources ? FX_OK : FX_ERR_INVALID_ARG;
}

size_t fx_batch_state_bytes(uint32_t tier, uint32_t n, uint32_t lanes) {
  (void)n;
  switch (tier) {
    case 0: return state_bytes<Tier0>(lanes);
    case 1: return state_bytes<Tier1>(lanes);
    case 2: return state_bytes<Tier2>(lanes);
    default: return 0;
  }
}

static int check_batch(const fx_stream_batch* in, const fx_order_batch* out) {
  if (!in || !out || !in->dot || !in->hdr || (in->dmax && !in->deps) || !out->order ||
      !out->release || !out->nexec || !out->err)
    return FX_ERR_INVALID_ARG;
  if (in->n < 1 || in->n > 8 || in->steps >= (1u << 26) || in->dmax > 31) return FX_ERR_INVALID_ARG;
  if (device_count() <= 0) return FX_ERR_NO_DEVICE;
  return FX_OK;
}

int fx_batch_execute(const fx_stream_batch* in, const fx_order_batch* out, uint32_t tier,
                     const uint32_t* stream_map, uint32_t num_lanes, void* state,
                     uint32_t step_begin, uint32_t step_end, uint32_t flags,
                     const uint32_t* init_frontier, void* hip_stream) {
  int st = check_batch(in, out);
  if (st) return st;
  if (step_end > in->steps || step_begin > step_end) return FX_ERR_INVALID_ARG;
  if (!(flags & FX_FLAG_INIT) && !state) return FX_ERR_INVALID_ARG;
  if ((flags & FX_FLAG_SAVE_STATE) && !state) return FX_ERR_INVALID_ARG;
  if (!stream_map && num_lanes > in->num_streams) return FX_ERR_INVALID_ARG;
  KArgs a;
  a.dot = in->dot;
  a.hdr = in->hdr;
  a.deps = in->deps;
  a.lengths = in->lengths;
  a.S = in->num_streams;
  a.steps = in->steps;
  a.dmax = in->dmax;
  a.n = in->n;
  a.plane = fx_plane_words(in->num_streams, in->steps);
  a.order = out->order;
  a.release = out->release;
  a.nexec = out->nexec;
  a.err = out->err;
  a.stream_map = stream_map;
  a.num_lanes = num_lanes;
  a.state = (uint32_t*)state;
  a.step_begin = step_begin;
  a.step_end = step_end;
  a.flags = flags;
  a.init_frontier = init_frontier;
  hipStream_t hs = (hipStream_t)hip_stream;
  if (g_profile) {
    if (!g_ev0) {
      if (hipEventCreate(&g_ev0) != hipSuccess || hipEventCreate(&g_ev1) != hipSuccess) return FX_ERR_HIP;
    }
    (void)hipEventRecord(g_ev0, hs);
  }
  switch (tier) {
    case 0: st = launch_exec<Tier0>(a, hs); break;
    case 1: st = launch_exec<Tier1>(a, hs); break;
    case 2: st = launch_exec<Tier2>(a, hs); break;
    default: return FX_ERR_INVALID_ARG;
  }
  if (g_profile) {
    (void)hipEventRecord(g_ev1, hs);
    g_ev_valid = st == FX_OK;
  }
  return st;
}

int fx_profile_enable(int on) {
  g_profile = on != 0;
  g_ev_valid = false;
  return FX_OK;
}

int fx_profile_last_exec_ms(float* ms) {
  if (!ms || !g_ev_valid) return FX_ERR_INVALID_ARG;
  if (hipEventSynchronize(g_ev1) != hipSuccess) return FX_ERR_HIP;
  return hipEventElapsedTime(ms, g_ev0, g_ev1) == hipSuccess ? FX_OK : FX_ERR_HIP;
}

int fx_dev_alloc(void** ptr, size_t bytes) {
  if (!ptr) return FX_ERR_INVALID_ARG;
  if (device_count() <= 0) return FX_ERR_NO_DEVICE;
  return hipMalloc(ptr, bytes ? bytes : 16) == hipSuccess ? FX_OK : FX_ERR_HIP;
}
int fx_dev_free(void* ptr) { return hipFree(ptr) == hipSuccess ? FX_OK : FX_ERR_HIP; }
int fx_dev_memset(void* ptr, int value, size_t bytes, void* hs) {
  return hipMemsetAsync(ptr, value, bytes, (hipStream_t)hs) == hipSuccess ? FX_OK : FX_ERR_HIP;
}
int fx_dev_h2d(void* dst, const void* src, size_t bytes, void* hs) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)hs) == hipSuccess ? FX_OK : FX_ERR_HIP;
}
int fx_dev_d2h(void* dst, const void* src, size_t bytes, void* hs) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)hs) == hipSuccess ? FX_OK : FX_ERR_HIP;
}
int fx_dev_synchronize(void* hs) {
  return hipStreamSynchronize((hipStream_t)hs) == hipSuccess ? FX_OK : FX_ERR_HIP;
}

int fx_batch_metrics(const fx_stream_batch* in, const fx_order_batch* out, const fx_hist_batch* h,
                     void* hip_stream) {
  if (!in || !out || !h || !h->chain_size || !h->execution_delay || h->nbins_chain < 2 ||
      h->nbins_delay < 2)
    return FX_ERR_INVALID_ARG;
  if (device_count() <= 0) return FX_ERR_NO_DEVICE;
  const uint32_t steps4 = (in->steps + 3) >> 2;
  const size_t nblocks = (size_t)((in->num_streams + 63) / 64) * steps4;
  if (nblocks == 0) return FX_OK;
  const uint32_t grid = (uint32_t)std::min<size_t>(nblocks, 256 * 8);
  const size_t lds_bytes = (size_t)(h->nbins_chain + h->nbins_delay) * 4;
  const uint32_t use_lds = lds_bytes <= 48 * 1024 ? 1u : 0u;
  hipLaunchKernelGGL(k_metrics, dim3(grid), dim3(256), use_lds ? lds_bytes : 0, (hipStream_t)hip_stream,
                     in->hdr, out->order, out->release, out->nexec, in->num_streams, in->steps,
                     (unsigned long long*)h->chain_size, h->nbins_chain,
                     (unsigned long long*)h->execution_delay, h->nbins_delay, use_lds);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

static int check_synth(const fx_synth_params* p) {
  if (!p || p->n < 1 || p->n > 8 || p->cmds_per_process < 1 || p->instances < 1 ||
      p->num_conflicts > 8)
    return FX_ERR_INVALID_ARG;
  const uint64_t N = (uint64_t)p->n * p->cmds_per_process;
  if (p->cmds_per_process >= (1u << FX_SEQ_BITS) || N + p->window >= (1u << 24) ||
      N >= (1u << 26))
    return FX_ERR_INVALID_ARG;
  if ((uint64_t)p->instances * p->n >= (1ull << 32)) return FX_ERR_INVALID_ARG;
  return FX_OK;
}

int fx_synth_shape(const fx_synth_params* p, uint32_t* S, uint32_t* steps, uint32_t* dmax) {
  int st = check_synth(p);
  if (st) return st;
  if (S) *S = p->instances * p->n;
  if (steps) *steps = p->n * p->cmds_per_process;
  if (dmax) *dmax = p->n;
  return FX_OK;
}

int fx_synth_generate(const fx_synth_params* p, uint32_t* dot, uint32_t* hdr, uint32_t* deps,
                      void* hip_stream) {
  int st = check_synth(p);
  if (st) return st;
  if (!dot || !hdr || !deps) return FX_ERR_INVALID_ARG;
  if (device_count() <= 0) return FX_ERR_NO_DEVICE;
  const uint32_t S = p->instances * p->n, steps = p->n * p->cmds_per_process;
  hipStream_t hs = (hipStream_t)hip_stream;
  // zero the padding of the planes (tiles of 64 streams x 4 steps)
  const size_t plane = fx_plane_words(S, steps);
  if (hipMemsetAsync(dot, 0, plane * 4, hs) != hipSuccess) return FX_ERR_HIP;
  if (hipMemsetAsync(hdr, 0, plane * 4, hs) != hipSuccess) return FX_ERR_HIP;
  if (hipMemsetAsync(deps, 0, plane * 4 * p->n, hs) != hipSuccess) return FX_ERR_HIP;
  const size_t total = (size_t)p->instances * steps;
  const uint32_t grid = (uint32_t)std::min<size_t>((total + 255) / 256, 256 * 64);
  hipLaunchKernelGGL(k_synth, dim3(grid), dim3(256), 0, hs, *p, S, steps, dot, hdr, deps);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

int fx_synth_generate_host(const fx_synth_params* p, uint32_t* dot, uint32_t* hdr, uint32_t* deps) {
  int st = check_synth(p);
  if (st) return st;
  if (!dot || !hdr || !deps) return FX_ERR_INVALID_ARG;
  const uint32_t S = p->instances * p->n, steps = p->n * p->cmds_per_process;
  const size_t plane = fx_plane_words(S, steps);
  memset(dot, 0, plane * 4);
  memset(hdr, 0, plane * 4);
  memset(deps, 0, plane * 4 * p->n);
  for (uint32_t inst = 0; inst < p->instances; ++inst)
    for (uint32_t g = 0; g < steps; ++g) synth_emit(*p, inst, g, S, steps, dot, hdr, deps);
  return FX_OK;
}

// Synchronous tiered driver: tier 0 for all, then reruns of the streams that
// ran out of capacity at tiers 1 and 2.
int fx_batch_run_tiered(const fx_stream_batch* in, const fx_order_batch* out, uint32_t flags,
                        void* hip_stream, uint32_t* tier_counts) {
  int st = check_batch(in, out);
  if (st) return st;
  hipStream_t hs = (hipStream_t)hip_stream;
  const uint32_t S = in->num_streams;
  flags |= FX_FLAG_INIT;
  flags &= ~FX_FLAG_SAVE_STATE;
  st = fx_batch_execute(in, out, 0, nullptr, S, nullptr, 0, in->steps, flags, nullptr, hip_stream);
  if (st) return st;
  if (tier_counts) tier_counts[0] = S;
  std::vector<uint32_t> err(S);
  if (hipMemcpyAsync(err.data(), out->err, (size_t)S * 4, hipMemcpyDeviceToHost, hs) != hipSuccess)
    return FX_ERR_HIP;
  if (hipStreamSynchronize(hs) != hipSuccess) return FX_ERR_HIP;
  for (uint32_t tier = 1; tier < FX_NUM_TIERS; ++tier) {
    std::vector<uint32_t> redo;
    for (uint32_t s = 0; s < S; ++s)
      if (err[s] == FX_ERR_CAPACITY) redo.push_back(s);
    if (tier_counts) tier_counts[tier] = (uint32_t)redo.size();
    if (redo.empty()) break;
    uint32_t* dmap = nullptr;
    void* dstate = nullptr;
    const uint32_t L = (uint32_t)redo.size();
    if (hipMalloc(&dmap, (size_t)L * 4) != hipSuccess) return FX_ERR_HIP;
    const size_t sb = fx_batch_state_bytes(tier, in->n, L);
    if (tier == 2 && hipMalloc(&dstate, sb) != hipSuccess) {
      (void)hipFree(dmap);
      return FX_ERR_HIP;
    }
    (void)hipMemcpyAsync(dmap, redo.data(), (size_t)L * 4, hipMemcpyHostToDevice, hs);
    st = fx_batch_execute(in, out, tier, dmap, L, dstate, 0, in->steps, flags, nullptr, hip_stream);
    if (!st) {
      for (uint32_t x = 0; x < L; ++x)
        (void)hipMemcpyAsync(&err[redo[x]], out->err + redo[x], 4, hipMemcpyDeviceToHost, hs);
      if (hipStreamSynchronize(hs) != hipSuccess) st = FX_ERR_HIP;
    }
    (void)hipFree(dmap);
    if (dstate) (void)hipFree(dstate);
    if (st) return st;
  }
  for (uint32_t s = 0; s < S; ++s)
    if (err[s]) return (int)err[s];
  return FX_OK;
}

}  // extern "C"
