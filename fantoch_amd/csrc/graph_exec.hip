// graph_exec.hip — batched GraphExecutor for gfx950 (MI355X).
//
// One lane = one commit stream = one (instance, process) executor of the
// reference (fantoch_ps/src/executor/graph/executor.rs:19-29 owns one
// DependencyGraph each).  A 64-thread workgroup is one wavefront running 64
// independent executors; there is no inter-lane communication, so nothing
// here depends on dispatch order or XCD placement.
//
// State restates the reference's containers as fixed tables (SURVEY §8(a)
// rows a4-a10):
//   executed clock AEClock (threshold 0.9.1; tarjan.rs:131-132,293):
//     per source a u32 frontier + an XW-word bitmap of executed seqs above it
//   VertexIndex (index.rs:18-51): P pending-vertex slots {dot, rec, wait,
//     tarjan id/low/visited-epoch, cached deps}
//   PendingIndex (index.rs:145-208): slot.wait = the missing dot the vertex is
//     registered on (a vertex is registered on at most one dot at a time)
//   TarjanSCCFinder (tarjan.rs:25-33): explicit DFS frame stack + Tarjan stack
//   check_pending's `dots` (mod.rs:556-587): LIFO worklist
// Tier 0 keeps the small hot fields (clock, slot dots/waits/recs) in VGPRs
// (unrolled selects, so a lookup is P parallel compares) and the rest in LDS
// in a lane-interleaved layout: word w of lane l at LDS dword (w * 64 + l),
// so whatever slot a lane touches the bank is (l mod 32) — conflict-free.
// Larger tiers keep everything in LDS (tier 1) or HBM (tier 2).
//
// Divergence: the slow path (Tarjan search, check_pending, try_pending) is a
// flat state machine — every iteration each lane performs ONE micro-op (one
// DFS edge or frame pop, one waiter pick, one worklist pop) — so a wavefront's
// cost per Add is the max over its lanes of their micro-op counts instead of
// the product of nested divergent loop trip counts.
//
// Records stream through a double-buffered register pipeline (a block = 4
// steps = one 16-byte load per lane per plane, see fx_index in fantoch_amd.h)
// whose loads have a static count, so waits are precise vmcnt(N).  Within a
// block lanes advance through their 4 steps independently.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <type_traits>
#include <vector>

#include "fantoch_amd.h"
#include "fx_internal.h"
#include "fx_synth.h"

namespace fx {

constexpr uint32_t WAVE = 64;

template <uint32_t NSRC_, uint32_t P_, uint32_t XW_, uint32_t C_, bool GLOBAL_, bool REGS_>
struct Tier {
  static constexpr uint32_t NSRC = NSRC_;  // sources (processes) supported
  static constexpr uint32_t P = P_;        // pending-vertex slots
  static constexpr uint32_t XW = XW_;      // clock window words per source
  static constexpr uint32_t C = C_;        // cached not-yet-executed deps per vertex
  static constexpr bool GLOBAL = GLOBAL_;  // state in HBM instead of LDS
  static constexpr bool REGS = REGS_;      // clock + slot dot/wait/rec in VGPRs
  static constexpr bool SMALL = P <= 15;   // u16 tarjan words, slot hints in cached deps
  using Mask = typename std::conditional<(P <= 32), uint32_t, uint64_t>::type;
  // memory-resident words per lane (register-resident fields are absent)
  static constexpr uint32_t CLKS = 1 + XW;
  static constexpr uint32_t CLK = 0;
  static constexpr uint32_t DOT = CLK + (REGS ? 0 : NSRC * CLKS);
  static constexpr uint32_t WAIT = DOT + (REGS ? 0 : P);
  static constexpr uint32_t REC = WAIT + (REGS ? 0 : P);  // arrival index | ncached << 26
  static constexpr uint32_t TL = REC + (REGS ? 0 : P);    // tarjan id | low | visited epoch
  static constexpr uint32_t DEP = TL + (SMALL ? (P + 1) / 2 : P);  // [C][P] dot | hint << 28
  static constexpr uint32_t TS = DEP + C * P;        // Tarjan stack, u8 slots
  static constexpr uint32_t FR = TS + (P + 3) / 4;   // DFS parent frames, u16 slot | dep idx << 8
  static constexpr uint32_t WL = FR + (P + 1) / 2;   // worklist, P + 1 packed dots
  static constexpr uint32_t MEM = WL + P + 1;        // words in LDS (or HBM)
  static constexpr uint32_t RSAVE = REGS ? 2 * NSRC + 3 * P : 0;  // saved VGPR arrays
  static constexpr uint32_t WORDS = MEM + RSAVE + 6;  // + occ(2) wmask(2) k err|epoch
  static_assert(P <= 64, "slot masks are at most u64");
  static_assert(P < 256, "slots are u8");
  static_assert(C < 32, "ncached is 5 bits");
  static_assert(!REGS || (XW == 1 && SMALL), "register tier: 32-bit windows, <= 15 slots");
};

// Lane-per-stream tiers (tier 0 is the 16-lanes-per-stream group tier,
// graph_group.hip).  LDS bytes / wave: TierLane 35,840 -> 4 waves / CU;
// Tier1 123,136 -> 1 wave / CU.
using TierLane = Tier<8, 12, 1, 5, false, false>;
using Tier1 = Tier<8, 32, 4, 8, false, false>;
using Tier2 = Tier<8, 64, 32, 16, true, false>;  // HBM-resident, 1024-bit clock windows


__device__ __forceinline__ uint32_t hdr_nd(uint32_t h) { return (h >> 24) & 31u; }

// Register arrays indexed by a per-lane value.  Arithmetic masks instead of
// selects: LLVM folds `i == k ? a[k] : r` chains back into a dynamically
// indexed load, which demotes the whole array (and the executor) to scratch.
__device__ __forceinline__ uint32_t lmask(bool c) { return 0u - (uint32_t)c; }
template <uint32_t N>
__device__ __forceinline__ uint32_t rsel(const uint32_t (&a)[N], uint32_t i) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t k = 0; k < N; ++k) r |= a[k] & lmask(i == k);
  return r;
}
template <uint32_t N>
__device__ __forceinline__ void rput(uint32_t (&a)[N], uint32_t i, uint32_t v) {
#pragma unroll
  for (uint32_t k = 0; k < N; ++k) {
    const uint32_t m = lmask(i == k);
    a[k] = (v & m) | (a[k] & ~m);
  }
}

enum : uint32_t { PH_IDLE = 0, PH_DFS = 1, PH_TRY = 2, PH_CHECK = 3 };

template <class T, uint32_t DCAP>
struct Exec {
  using Mask = typename T::Mask;
  static constexpr uint32_t RN = T::REGS ? T::NSRC : 1;
  static constexpr uint32_t RP = T::REGS ? T::P : 1;
  static constexpr Mask ONE = 1;

  uint32_t* st;  // this lane's memory state: word w at st[w * WAVE]
  uint32_t cf[RN], cw[RN];           // clock frontier / window (REGS)
  uint32_t sd[RP], sw[RP], sr[RP];   // slot dot / wait / rec (REGS)
  Mask occ = 0, wmask = 0, tmask = 0;
  uint32_t k = 0, err = 0, epoch = 1, nwl = 0, cur = 0;
  uint32_t stream = 0, n = 0, steps = 0, dmax = 0;
  size_t plane = 0;
  const uint32_t* deps = nullptr;
  uint32_t* order = nullptr;
  uint32_t* release = nullptr;
  // find_scc context
  uint32_t phase = PH_IDLE, root = 0, idc = 0, nts = 0, nfr = 0, missing = 0;
  uint32_t fv = 0, fdi = 0, fnc = 0;
  bool in_try = false, emitted = false;

  __device__ __forceinline__ uint32_t& w(uint32_t i) { return st[i * WAVE]; }
  __device__ __forceinline__ uint8_t& ts(uint32_t i) {
    return reinterpret_cast<uint8_t*>(&w(T::TS + (i >> 2)))[i & 3];
  }
  __device__ __forceinline__ uint16_t& fr(uint32_t i) {
    return reinterpret_cast<uint16_t*>(&w(T::FR + (i >> 1)))[i & 1];
  }
  __device__ __forceinline__ uint32_t& wl(uint32_t i) { return w(T::WL + i); }
  __device__ __forceinline__ size_t at(uint32_t step) const { return fx_index(step, stream, steps); }

  // ------------------------------------------------------- slot fields
  __device__ __forceinline__ uint32_t dot_of(uint32_t sl) {
    if constexpr (T::REGS) return rsel(sd, sl); else return w(T::DOT + sl);
  }
  __device__ __forceinline__ void set_dot(uint32_t sl, uint32_t v) {
    if constexpr (T::REGS) rput(sd, sl, v); else w(T::DOT + sl) = v;
  }
  __device__ __forceinline__ uint32_t wait_of(uint32_t sl) {
    if constexpr (T::REGS) return rsel(sw, sl); else return w(T::WAIT + sl);
  }
  __device__ __forceinline__ void set_wait(uint32_t sl, uint32_t v) {
    if constexpr (T::REGS) rput(sw, sl, v); else w(T::WAIT + sl) = v;
  }
  __device__ __forceinline__ uint32_t rec_of(uint32_t sl) {
    if constexpr (T::REGS) return rsel(sr, sl); else return w(T::REC + sl);
  }
  __device__ __forceinline__ void set_rec(uint32_t sl, uint32_t v) {
    if constexpr (T::REGS) rput(sr, sl, v); else w(T::REC + sl) = v;
  }
  // Tarjan word: id | low | visited epoch (u16 4|4|8 on small tiers, u32 12|12|8)
  static constexpr uint32_t IDB = T::SMALL ? 4 : 12;
  static constexpr uint32_t IDM = (1u << IDB) - 1;
  __device__ __forceinline__ uint32_t tl_of(uint32_t sl) {
    if constexpr (T::SMALL) return reinterpret_cast<uint16_t*>(&w(T::TL + (sl >> 1)))[sl & 1];
    else return w(T::TL + sl);
  }
  __device__ __forceinline__ void set_tl(uint32_t sl, uint32_t v) {
    if constexpr (T::SMALL) reinterpret_cast<uint16_t*>(&w(T::TL + (sl >> 1)))[sl & 1] = (uint16_t)v;
    else w(T::TL + sl) = v;
  }
  static __device__ __forceinline__ uint32_t tid(uint32_t t) { return t & IDM; }
  static __device__ __forceinline__ uint32_t tlow(uint32_t t) { return (t >> IDB) & IDM; }
  static __device__ __forceinline__ uint32_t tep(uint32_t t) { return t >> (2 * IDB); }
  static __device__ __forceinline__ uint32_t tmk(uint32_t id, uint32_t low, uint32_t ep) {
    return id | (low << IDB) | (ep << (2 * IDB));
  }

  // ---------------------------------------------- executed clock (AEClock)
  // AEClock::contains (tarjan.rs:131-132)
  __device__ __forceinline__ bool clk_contains(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) return false;
    const uint32_t seq = d & FX_SEQ_MASK;
    if constexpr (T::REGS) {
      uint32_t f = 0, wv = 0;
#pragma unroll
      for (uint32_t q = 0; q < T::NSRC; ++q) {
        const uint32_t m = lmask(si == q);
        f |= cf[q] & m;
        wv |= cw[q] & m;
      }
      const uint32_t off = seq - f - 1u;
      return seq <= f || (off < 32u && ((wv >> off) & 1u));
    } else {
      const uint32_t b = T::CLK + si * T::CLKS;
      const uint32_t f = w(b);
      if (seq <= f) return true;
      const uint32_t off = seq - f - 1u;
      if (off >= 32u * T::XW) return false;
      return (w(b + 1 + (off >> 5)) >> (off & 31u)) & 1u;
    }
  }
  // AEClock::add (tarjan.rs:293): frontier + exception window
  __device__ __forceinline__ void clk_add(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) { err = FX_ERR_DOT_RANGE; return; }
    const uint32_t seq = d & FX_SEQ_MASK;
    if constexpr (T::REGS) {
      uint32_t f = 0, wv = 0;
#pragma unroll
      for (uint32_t q = 0; q < T::NSRC; ++q) {
        const uint32_t m = lmask(si == q);
        f |= cf[q] & m;
        wv |= cw[q] & m;
      }
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
#pragma unroll
      for (uint32_t q = 0; q < T::NSRC; ++q) {
        const uint32_t m = lmask(si == q);
        cf[q] = (f & m) | (cf[q] & ~m);
        cw[q] = (wv & m) | (cw[q] & ~m);
      }
    } else {
      const uint32_t b = T::CLK + si * T::CLKS;
      const uint32_t f = w(b);
      if (seq <= f) return;
      const uint32_t off = seq - f - 1u;
      if (off >= 32u * T::XW) { err = FX_ERR_CAPACITY; return; }
      if (off != 0) {
        w(b + 1 + (off >> 5)) |= 1u << (off & 31u);
        return;
      }
      uint32_t t = 1;  // 1 + trailing ones of the window from bit 1
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
    if constexpr (T::REGS) {
      Mask m = 0;
#pragma unroll
      for (uint32_t q = 0; q < T::P; ++q) m |= (Mask)(sd[q] == d) << q;
      m &= occ;
      return m ? (int)__builtin_ctzll((uint64_t)m) : -1;
    } else {
      for (Mask m = occ; m; m &= m - 1) {
        const int sl = __builtin_ctzll((uint64_t)m);
        if (w(T::DOT + sl) == d) return sl;
      }
      return -1;
    }
  }
  // registered waiters of x: PendingIndex::remove(x) (index.rs:205-207)
  __device__ __forceinline__ Mask waiters(uint32_t x) {
    Mask t = 0;
    if constexpr (T::REGS) {
#pragma unroll
      for (uint32_t q = 0; q < T::P; ++q) t |= (Mask)(sw[q] == x) << q;
      return t & wmask;
    } else {
      for (Mask m = wmask; m; m &= m - 1) {
        const int sl = __builtin_ctzll((uint64_t)m);
        if (w(T::WAIT + sl) == x) t |= ONE << sl;
      }
      return t;
    }
  }
  // slot with the smallest dot among `m` (canonical C2 order)
  __device__ __forceinline__ int argmin_dot(Mask m) {
    int best = -1;
    uint32_t bd = 0xFFFFFFFFu;
    if constexpr (T::REGS) {
#pragma unroll
      for (uint32_t q = 0; q < T::P; ++q) {
        const uint32_t tk = lmask(((m >> q) & 1) && sd[q] < bd);
        bd = (sd[q] & tk) | (bd & ~tk);
        best = (int)((q & tk) | ((uint32_t)best & ~tk));
      }
    } else {
      for (; m; m &= m - 1) {
        const int sl = __builtin_ctzll((uint64_t)m);
        const uint32_t dd = w(T::DOT + sl);
        if (dd < bd) { bd = dd; best = sl; }
      }
    }
    return best;
  }
  __device__ __forceinline__ int pt_insert(uint32_t d, uint32_t rec) {
    constexpr Mask full = T::P == 8 * sizeof(Mask) ? ~(Mask)0 : ((ONE << T::P) - 1);
    const Mask fre = ~occ & full;
    if (!fre) { err = FX_ERR_CAPACITY; return -1; }
    const uint32_t sl = __builtin_ctzll((uint64_t)fre);
    occ |= ONE << sl;
    set_dot(sl, d);
    set_rec(sl, rec);
    set_wait(sl, 0);
    set_tl(sl, 0);
    return (int)sl;
  }
  __device__ __forceinline__ void pt_free(uint32_t sl) {
    const Mask keep = ~(ONE << sl);
    occ &= keep;
    wmask &= keep;
    tmask &= keep;
  }
  // Vertex::deps restricted to the deps not executed at insertion (executed
  // deps are ignored by every later search, tarjan.rs:128-145, and the
  // executed clock only grows), ascending; a dep pending at insertion carries
  // its slot + 1 (it can only leave that slot by being executed).
  __device__ __forceinline__ void pt_cache_dep(uint32_t sl, uint32_t d, uint32_t dep, uint32_t& nc) {
    if (dep == d || clk_contains(dep)) return;
    if ((dep >> FX_SEQ_BITS) > 15u) { err = FX_ERR_DOT_RANGE; return; }
    if (nc >= T::C) { err = FX_ERR_CAPACITY; return; }
    uint32_t hint = 0;
    if constexpr (T::SMALL) hint = (uint32_t)(pt_find(dep) + 1);
    w(T::DEP + nc * T::P + sl) = dep | (hint << 28);
    ++nc;
  }
  // VertexIndex::index(Vertex::new(dot, cmd, deps, time)) (index.rs:33-37):
  // deps j < DCAP come from the prefetched registers, the rest from HBM.
  __device__ __forceinline__ int insert_vertex(uint32_t i, uint32_t d, uint32_t nd, const uint32_t* rdeps) {
    const int sl = pt_insert(d, i);
    if (sl < 0) return -1;
    uint32_t nc = 0;
#pragma unroll
    for (uint32_t j = 0; j < DCAP; ++j)
      if (j < nd) pt_cache_dep((uint32_t)sl, d, rdeps[j], nc);
    for (uint32_t j = DCAP; j < nd; ++j) pt_cache_dep((uint32_t)sl, d, deps[(size_t)j * plane + at(i)], nc);
    if (err) return -1;
    set_rec((uint32_t)sl, i | (nc << 26));
    return sl;
  }

  // try_pending's `visited` set (mod.rs:598): an epoch stamp per slot
  __device__ __forceinline__ void new_epoch() {
    epoch = (epoch + 1) & 0xFFu;
    if (epoch == 0) {
      for (Mask m = occ; m; m &= m - 1) {
        const uint32_t sl = __builtin_ctzll((uint64_t)m);
        const uint32_t t = tl_of(sl);
        set_tl(sl, tmk(tid(t), tlow(t), 0));
      }
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

  // ------------------------------ find_scc as a micro-op state machine
  // find_scc (mod.rs:409-486) = TarjanSCCFinder::strong_connect
  // (tarjan.rs:96-316) run iteratively + save_scc + finalize (tarjan.rs:60-93)
  __device__ __forceinline__ void dfs_start(uint32_t r, bool intry) {
    root = r;
    in_try = intry;
    emitted = false;
    missing = 0;
    idc = 1;
    set_tl(r, tmk(1, 1, tep(tl_of(r))));
    ts(0) = (uint8_t)r;
    nts = 1;
    nfr = 0;
    fv = r;
    fdi = 0;
    fnc = rec_of(r) >> 26;
    phase = PH_DFS;
  }

  // SCC rooted at fv: members are TS[pos..nts), saved in ascending dot order
  // (SCC = BTreeSet<Dot>, tarjan.rs:15); executed clock updated per member.
  __device__ __forceinline__ void save_scc() {
    uint32_t pos = nts - 1;
    while (ts(pos) != fv) --pos;
    for (uint32_t a = pos + 1; a < nts; ++a) {
      const uint8_t key = ts(a);
      const uint32_t kd = dot_of(key);
      uint32_t b = a;
      while (b > pos && dot_of(ts(b - 1)) > kd) {
        ts(b) = ts(b - 1);
        --b;
      }
      ts(b) = key;
    }
    for (uint32_t a = pos; a < nts; ++a) {
      const uint32_t sl = ts(a);
      const uint32_t d = dot_of(sl);
      emit(rec_of(sl) & 0x03FFFFFFu, d, a == pos);
      wl(nwl++) = d;
      pt_free(sl);
    }
    nts = pos;
    emitted = true;
  }

  __device__ __forceinline__ void dfs_finish() {
    // finalize: reset ids of the vertices left on the stack; in try_pending a
    // failed search that saved no SCC adds them to `visited` (mod.rs:621-629)
    const bool mark = in_try && missing != 0 && !emitted;
    for (uint32_t a = 0; a < nts; ++a) {
      const uint32_t sl = ts(a);
      set_tl(sl, tmk(0, 0, mark ? epoch : tep(tl_of(sl))));
    }
    nts = 0;
    if (missing) {  // index_pending(dot, missing) (mod.rs:525-554)
      set_wait(root, missing);
      wmask |= ONE << root;
    }
    if (in_try) {
      if (!missing || emitted) new_epoch();  // visited.clear() (mod.rs:607, 621-623)
      phase = PH_TRY;
    } else {
      phase = PH_CHECK;
    }
  }

  // one DFS edge or one frame pop
  __device__ __forceinline__ void dfs_iter() {
    if (fdi < fnc) {
      const uint32_t cwd = w(T::DEP + fdi * T::P + fv);
      ++fdi;
      const uint32_t dep = cwd & 0x0FFFFFFFu;
      if (clk_contains(dep)) return;  // executed (tarjan.rs:128-145)
      int x = -1;
      if constexpr (T::SMALL) {
        const uint32_t h = cwd >> 28;
        if (h) x = (int)h - 1;
      }
      if (x < 0) x = pt_find(dep);
      if (x < 0) {  // missing: give up (tarjan.rs:148-157, shard_count == 1)
        missing = dep;
        dfs_finish();
        return;
      }
      const uint32_t tx = tl_of((uint32_t)x);
      if (tid(tx) == 0) {  // not visited: recurse (tarjan.rs:172-214)
        ++idc;
        set_tl((uint32_t)x, tmk(idc, idc, tep(tx)));
        ts(nts++) = (uint8_t)x;
        fr(nfr++) = (uint16_t)(fv | (fdi << 8));
        fv = (uint32_t)x;
        fdi = 0;
        fnc = rec_of(fv) >> 26;
      } else {  // visited and on the stack (tarjan.rs:215-225)
        const uint32_t tv = tl_of(fv);
        if (tid(tx) < tlow(tv)) set_tl(fv, tmk(tid(tv), tid(tx), tep(tv)));
      }
    } else {
      const uint32_t tv = tl_of(fv);
      const uint32_t lowv = tlow(tv);
      if (tid(tv) == lowv) {  // SCC root (tarjan.rs:233-312)
        save_scc();
        if (err) { phase = PH_IDLE; return; }
      }
      if (nfr == 0) {  // root done: Found
        dfs_finish();
        return;
      }
      const uint32_t f = fr(--nfr);  // back in the parent: low = min(low, dep.low) (tarjan.rs:211)
      fv = f & 0xFFu;
      fdi = f >> 8;
      fnc = rec_of(fv) >> 26;
      const uint32_t tp = tl_of(fv);
      if (lowv < tlow(tp)) set_tl(fv, tmk(tid(tp), lowv, tep(tp)));
    }
  }

  // try_pending (mod.rs:589-642): next waiter of the snapshot, ascending (C2)
  __device__ __forceinline__ void try_iter() {
    if (!tmask) { phase = PH_CHECK; return; }
    const int best = argmin_dot(tmask);
    tmask &= ~(ONE << best);
    if (tep(tl_of((uint32_t)best)) == epoch) return;  // visited: skipped, not re-registered
    dfs_start((uint32_t)best, true);
  }

  // check_pending (mod.rs:556-587): pop one released dot (LIFO)
  __device__ __forceinline__ void check_iter() {
    if (nwl == 0 || !wmask) {
      nwl = 0;
      phase = PH_IDLE;
      return;
    }
    const uint32_t x = wl(--nwl);
    const Mask t = waiters(x);
    if (!t) return;
    wmask &= ~t;  // PendingIndex::remove(x): the waiters are no longer registered
    tmask = t;
    new_epoch();  // try_pending's fresh `visited`
    phase = PH_TRY;
  }

  __device__ __forceinline__ void slow_iter() {
    if (phase == PH_DFS) dfs_iter();
    if (phase == PH_TRY) try_iter();
    if (phase == PH_CHECK) check_iter();
    if (err) phase = PH_IDLE;
  }

  // GraphExecutor::handle(Add) (executor.rs:69-80) -> handle_add (mod.rs:213-275):
  // the fast path completes here; otherwise the lane enters the state machine.
  __device__ __forceinline__ void step_start(uint32_t i, uint32_t d, uint32_t h, const uint32_t* rdeps,
                                             bool at_commit) {
    cur = i;
    nwl = 0;
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
        const uint32_t dep = rdeps[j];
        if (dep <= prev) err = FX_ERR_DEPS_UNSORTED;
        prev = dep;
        if (dep != d && !clk_contains(dep)) fast = false;
      }
    }
    if (err) return;
    if (fast) {
      emit(i, d, true);
      if (wmask && !err) {  // check_pending([dot])
        wl(0) = d;
        nwl = 1;
        phase = PH_CHECK;
      }
    } else {
      const int sl = insert_vertex(i, d, nd, rdeps);
      if (sl >= 0) dfs_start((uint32_t)sl, false);
    }
  }
};

template <class T, uint32_t DCAP>
__global__ __launch_bounds__(64) void k_graph_exec(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t lane = threadIdx.x;
  const uint32_t gl = blockIdx.x * WAVE + lane;
  const bool active = gl < a.num_lanes;
  const uint32_t s = active ? (a.stream_map ? a.stream_map[gl] : gl) : 0u;
  const uint32_t len = active ? (a.lengths ? min(a.lengths[s], a.steps) : a.steps) : 0u;
  uint32_t* gblock = a.state ? a.state + (size_t)blockIdx.x * T::WORDS * WAVE : nullptr;

  Exec<T, DCAP> e;
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
#pragma unroll
  for (uint32_t q = 0; q < Exec<T, DCAP>::RN; ++q) e.cf[q] = e.cw[q] = 0;
#pragma unroll
  for (uint32_t q = 0; q < Exec<T, DCAP>::RP; ++q) e.sd[q] = e.sw[q] = e.sr[q] = 0;

  if (a.flags & FX_FLAG_INIT) {
    if constexpr (!T::REGS) {
      for (uint32_t q = 0; q < T::NSRC * T::CLKS; ++q) e.w(T::CLK + q) = 0;
    }
    if (a.init_frontier && active) {
#pragma unroll
      for (uint32_t p = 0; p < T::NSRC && p < 8; ++p) {
        const uint32_t f = a.init_frontier[(size_t)s * 8 + p];
        if constexpr (T::REGS) e.cf[p] = f;
        else e.w(T::CLK + p * T::CLKS) = f;
      }
    }
  } else {
    if constexpr (!T::GLOBAL) {
      for (uint32_t q = 0; q < T::MEM; ++q) smem[q * WAVE + lane] = gblock[q * WAVE + lane];
    }
    const uint32_t* r = gblock + (size_t)T::MEM * WAVE + lane;
    if constexpr (T::REGS) {
#pragma unroll
      for (uint32_t q = 0; q < T::NSRC; ++q) {
        e.cf[q] = r[q * WAVE];
        e.cw[q] = r[(T::NSRC + q) * WAVE];
      }
#pragma unroll
      for (uint32_t q = 0; q < T::P; ++q) {
        e.sd[q] = r[(2 * T::NSRC + q) * WAVE];
        e.sw[q] = r[(2 * T::NSRC + T::P + q) * WAVE];
        e.sr[q] = r[(2 * T::NSRC + 2 * T::P + q) * WAVE];
      }
    }
    r += (size_t)T::RSAVE * WAVE;
    e.occ = (typename T::Mask)((uint64_t)r[0] | ((uint64_t)r[WAVE] << 32));
    e.wmask = (typename T::Mask)((uint64_t)r[2 * WAVE] | ((uint64_t)r[3 * WAVE] << 32));
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
    // Lanes progress through the block's steps independently: a lane starts
    // its next step as soon as its previous one (fast path or micro-op state
    // machine) is done, so the wavefront waits once per block for its slowest
    // lane instead of once per step.
    uint32_t q = q0;
    while (true) {
      const bool want = e.phase == PH_IDLE && q < q1 && !e.err && base + q < len;
      if (!__any(want || e.phase != PH_IDLE)) break;
      if (want) {
        const uint32_t m0 = lmask(q == 0), m1 = lmask(q == 1), m2 = lmask(q == 2), m3 = lmask(q == 3);
#define FX_PICK(V) (((V).x & m0) | ((V).y & m1) | ((V).z & m2) | ((V).w & m3))
        uint32_t rd[DCAP];
#pragma unroll
        for (uint32_t j = 0; j < DCAP; ++j) rd[j] = FX_PICK(d0[j]);
        e.step_start(base + q, FX_PICK(cd), FX_PICK(ch), rd, at_commit);
#undef FX_PICK
        ++q;
      }
      if (e.phase != PH_IDLE) e.slow_iter();
    }
    cd = nd_;
    ch = nh;
#pragma unroll
    for (uint32_t j = 0; j < DCAP; ++j) d0[j] = d1[j];
  }
#undef FX_LOAD

  if (!active) return;
  // Vertices still pending have no release step (yet).
  for (typename T::Mask m = e.occ; m; m &= m - 1) {
    const uint32_t sl = __builtin_ctzll((uint64_t)m);
    a.release[e.at(e.rec_of(sl) & 0x03FFFFFFu)] = FX_RELEASE_NONE;
  }
  a.nexec[s] = e.k;
  a.err[s] = e.err;
  if (a.flags & FX_FLAG_SAVE_STATE) {
    if constexpr (!T::GLOBAL) {
      for (uint32_t q = 0; q < T::MEM; ++q) gblock[q * WAVE + lane] = smem[q * WAVE + lane];
    }
    uint32_t* r = gblock + (size_t)T::MEM * WAVE + lane;
    if constexpr (T::REGS) {
#pragma unroll
      for (uint32_t q = 0; q < T::NSRC; ++q) {
        r[q * WAVE] = e.cf[q];
        r[(T::NSRC + q) * WAVE] = e.cw[q];
      }
#pragma unroll
      for (uint32_t q = 0; q < T::P; ++q) {
        r[(2 * T::NSRC + q) * WAVE] = e.sd[q];
        r[(2 * T::NSRC + T::P + q) * WAVE] = e.sw[q];
        r[(2 * T::NSRC + 2 * T::P + q) * WAVE] = e.sr[q];
      }
    }
    r += (size_t)T::RSAVE * WAVE;
    r[0] = (uint32_t)(uint64_t)e.occ;
    r[WAVE] = (uint32_t)((uint64_t)e.occ >> 32);
    r[2 * WAVE] = (uint32_t)(uint64_t)e.wmask;
    r[3 * WAVE] = (uint32_t)((uint64_t)e.wmask >> 32);
    r[4 * WAVE] = e.k;
    r[5 * WAVE] = (e.err & 0xFFFFu) | (e.epoch << 16);
  }
}

// ------------------------------------------------------------- metrics
// Metrics::collect for ChainSize (one sample per SCC, mod.rs:492-493) and
// ExecutionDelay (t(release) - t(add), mod.rs:514-518).  One 256-thread block
// per (tile, 4-row block): thread t reads order word t of that 1 KiB granule.
// With one tile column of streams (S <= 64; configs[4]: 5) a block takes 256
// consecutive used words instead (4 S per 4-row block), not 4 S of 256 threads.
// Wave-aggregated histogram increment: one atomic per distinct bin in the wave
// (the leader lane adds the popcount of the lanes sharing its bin).  Most Adds
// of a wave land in one or two bins (ChainSize 1, small delays), so per-lane
// atomics serialised on one LDS address (PMC: 96 % of k_metrics' LDS cycles
// were bank-conflict cycles).  Called in wave-uniform control flow; bin ==
// kNoBin means "nothing to add" for that lane.
constexpr uint32_t kNoBin = 0xFFFFFFFFu;
__device__ inline void wave_hist_add(uint32_t* lds, unsigned long long* glob, uint32_t bin,
                                     uint32_t use_lds) {
  unsigned long long active = __ballot(bin != kNoBin);
  while (active) {
    const int leader = __ffsll((long long)active) - 1;
    const uint32_t b = (uint32_t)__shfl((int)bin, leader);
    const unsigned long long same = __ballot(bin == b);
    if ((int)__lane_id() == leader) {
      const uint32_t c = (uint32_t)__popcll(same);
      if (use_lds) atomicAdd(&lds[b], c);
      else atomicAdd(&glob[b], (unsigned long long)c);
    }
    active &= ~same;
  }
}

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
  const bool narrow = S <= 64;
  const uint32_t w = 4u * S;  // narrow: used words per 4-row block
  const size_t nblocks = narrow ? ((size_t)w * steps4 + 255) / 256 : (size_t)tiles * steps4;
  if (use_lds) {
    for (uint32_t q = threadIdx.x; q < nbc + nbd; q += blockDim.x) hist[q] = 0;
    __syncthreads();
  }
  const uint32_t t = threadIdx.x;
  // blk is block-uniform, so every wave runs the aggregated adds together
  // XCD-aware order (narrow batches): the hardware deals blocks to the 8 XCDs
  // round robin; each XCD taking a contiguous eighth of every grid pass keeps
  // the release / hdr lines its rows look up (nearby steps) in its own L2
  const size_t b0 = narrow && gridDim.x % 8u == 0 ? (size_t)(blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u
                                                  : blockIdx.x;
  for (size_t blk = b0; blk < nblocks; blk += gridDim.x) {
    uint32_t s, k;
    if (narrow) {
      const size_t it = blk * 256 + t;
      s = it < (size_t)w * steps4 ? (uint32_t)(it % w) >> 2 : S;
      k = (uint32_t)(it / w) * 4 + (t & 3);
    } else {
      s = (uint32_t)(blk / steps4) * 64 + (t >> 2);
      k = (uint32_t)(blk % steps4) * 4 + (t & 3);
    }
    uint32_t db = kNoBin, cb = kNoBin;
    const uint32_t ne = s < S ? nexec[s] : 0;
    if (k < ne) {
      const uint32_t o = order[fx_index(k, s, steps)];
      const uint32_t rec = o & 0x7FFFFFFFu;
      const uint32_t rs = rec < steps ? release[fx_index(rec, s, steps)] : FX_RELEASE_NONE;
      if (rs < steps) {  // else not executed (errored stream)
        const uint32_t dl =
            FX_HDR_T(hdr[fx_index(rs, s, steps)]) - FX_HDR_T(hdr[fx_index(rec, s, steps)]);
        db = dl < nbd - 1 ? dl : nbd - 1;
        if (o & FX_ORDER_SCC_START) {
          uint32_t size = 1;
          while (k + size < ne && !(order[fx_index(k + size, s, steps)] & FX_ORDER_SCC_START)) ++size;
          cb = size < nbc - 1 ? size : nbc - 1;
        }
      }
    }
    wave_hist_add(use_lds ? hist + nbc : nullptr, delay, db, use_lds);
    wave_hist_add(hist, chain, cb, use_lds);
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

// ------------------------------------------------ single-stream gather
__global__ __launch_bounds__(256) void k_gather_release(const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ release,
                                                        uint32_t steps, uint32_t k0, uint32_t k1,
                                                        uint32_t* __restrict__ out) {
  const uint32_t k = k0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= k1) return;
  const uint32_t rec = FX_ORDER_REC(order[fx_index(k, 0, steps)]);
  out[k - k0] = rec < steps ? release[fx_index(rec, 0, steps)] : FX_RELEASE_NONE;
}

int gather_release(const uint32_t* order, const uint32_t* release, uint32_t steps, uint32_t k0,
                   uint32_t k1, uint32_t* out, hipStream_t stream) {
  if (k1 <= k0) return FX_OK;
  const uint32_t n = k1 - k0;
  hipLaunchKernelGGL(k_gather_release, dim3((n + 255) / 256), dim3(256), 0, stream, order, release,
                     steps, k0, k1, out);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

// ---------------------------------------- single-stream handle transfers
// The handle's uploads arrive as one contiguous staging block (plane-major:
// rows [r0, r0 + rows) of dot, hdr, then each dep plane) and are scattered
// into the stream's words of each 64-stream tile on the device.
__global__ __launch_bounds__(256) void k_scatter_rows(const uint32_t* __restrict__ stage, uint32_t nplanes,
                                                      uint32_t r0, uint32_t rows, uint32_t cap, uint32_t* dot,
                                                      uint32_t* hdr, uint32_t* deps, size_t plane) {
  const size_t total = (size_t)nplanes * rows;
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (size_t)gridDim.x * blockDim.x) {
    const uint32_t pl = (uint32_t)(x / rows), t = (uint32_t)(x % rows);
    uint32_t* dst = pl == 0 ? dot : pl == 1 ? hdr : deps + (size_t)(pl - 2) * plane;
    dst[fx_index(r0 + t, 0, cap)] = stage[x];
  }
}

int scatter_rows(const uint32_t* stage, uint32_t nplanes, uint32_t r0, uint32_t rows, uint32_t cap, uint32_t* dot,
                 uint32_t* hdr, uint32_t* deps, hipStream_t stream) {
  if (!rows || !nplanes) return FX_OK;
  const size_t total = (size_t)nplanes * rows;
  const uint32_t blocks = (uint32_t)std::min<size_t>((total + 255) / 256, 1024);
  hipLaunchKernelGGL(k_scatter_rows, dim3(blocks), dim3(256), 0, stream, stage, nplanes, r0, rows, cap, dot, hdr,
                     deps, fx_plane_words(1, cap));
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

// After a handle's flush: out[0] = nexec, out[1] = err, then for each new
// order entry k in [k0, nexec) its order word and its release step, written
// straight into host-mapped memory (one synchronisation per flush, and only
// the words a flush produced cross the bus).
__global__ __launch_bounds__(256) void k_flush_pack(const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ release,
                                                    const uint32_t* __restrict__ nexec,
                                                    const uint32_t* __restrict__ err, uint32_t cap, uint32_t k0,
                                                    uint32_t* out) {
  const uint32_t ne = *nexec;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = ne;
    out[1] = *err;
  }
  const uint32_t cnt = ne > k0 ? min(ne, cap) - k0 : 0u;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < cnt; t += gridDim.x * blockDim.x) {
    const uint32_t o = order[fx_index(k0 + t, 0, cap)];
    const uint32_t rec = FX_ORDER_REC(o);
    out[2 + 2 * t] = o;
    out[3 + 2 * t] = rec < cap ? release[fx_index(rec, 0, cap)] : FX_RELEASE_NONE;
  }
}

int flush_pack(const uint32_t* order, const uint32_t* release, const uint32_t* nexec, const uint32_t* err,
               uint32_t cap, uint32_t k0, uint32_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_flush_pack, dim3(4), dim3(256), 0, stream, order, release, nexec, err, cap, k0, out);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
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

template <class T, uint32_t DCAP>
static int launch_exec_d(const KArgs& a, hipStream_t stream) {
  if (T::GLOBAL && !a.state) return FX_ERR_INVALID_ARG;
  const uint32_t blocks = (a.num_lanes + WAVE - 1) / WAVE;
  if (blocks == 0) return FX_OK;
  const size_t lds = T::GLOBAL ? 0 : (size_t)T::MEM * WAVE * 4;
  static bool configured = false;
  if (!configured && lds > 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)k_graph_exec<T, DCAP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    configured = true;
  }
  hipLaunchKernelGGL((k_graph_exec<T, DCAP>), dim3(blocks), dim3(WAVE), lds, stream, a);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

// deps of the incoming Add prefetched into registers: the smallest of 3/5/8
// that covers the batch's dep planes (more than 8 are read on demand)
template <class T>
static int launch_exec(const KArgs& a, hipStream_t stream) {
  if (a.dmax <= 3) return launch_exec_d<T, 3>(a, stream);
  if (a.dmax <= 5) return launch_exec_d<T, 5>(a, stream);
  return launch_exec_d<T, 8>(a, stream);
}

template <class T>
static uint32_t decode_pending_t(const uint32_t* block, uint32_t lane, uint32_t* dots,
                                 uint32_t* waits, uint32_t cap) {
  const uint32_t* r = block + (size_t)(T::MEM + T::RSAVE) * WAVE + lane;
  const uint64_t occ = (uint64_t)r[0] | ((uint64_t)r[WAVE] << 32);
  const uint64_t wm = (uint64_t)r[2 * WAVE] | ((uint64_t)r[3 * WAVE] << 32);
  const uint32_t dot_w = T::REGS ? T::MEM + 2 * T::NSRC : T::DOT;
  const uint32_t wait_w = T::REGS ? T::MEM + 2 * T::NSRC + T::P : T::WAIT;
  uint32_t c = 0;
  for (uint64_t m = occ; m; m &= m - 1) {
    const int sl = __builtin_ctzll(m);
    if (c < cap) {
      dots[c] = block[(dot_w + sl) * WAVE + lane];
      waits[c] = ((wm >> sl) & 1) ? block[(wait_w + sl) * WAVE + lane] : 0u;
    }
    ++c;
  }
  return c;
}

uint32_t decode_pending(uint32_t tier, const uint32_t* block, uint32_t lane, uint32_t* dots,
                        uint32_t* waits, uint32_t cap) {
  switch (tier) {
    case 0: return group_decode_pending(block, lane, dots, waits, cap);
    case 1: return decode_pending_t<Tier1>(block, lane, dots, waits, cap);
    case 2: return decode_pending_t<Tier2>(block, lane, dots, waits, cap);
    case 3: return decode_pending_t<TierLane>(block, lane, dots, waits, cap);
    case 4: return wave_decode_pending(block, lane, dots, waits, cap);
    case 5: return lane_decode_pending(block, lane, dots, waits, cap);
    default: return 0;
  }
}

static bool g_profile = false;
static hipEvent_t g_ev0 = nullptr, g_ev1 = nullptr;
static bool g_ev_valid = false;
// split-tier kernels: [1] group kernel (caller's stream), [2] lane kernel (aux stream)
static hipEvent_t g_kev[3][2] = {};
static bool g_kev_valid[3] = {};

bool profile_on() { return g_profile; }

// per-slot kernel events (fx_profile_slot_ms): slot = executor tier
// (fx_batch_execute), FX_PROFILE_SLOT_PRED + tier (fx_pred_execute); each
// holds its slot's last launch
static hipEvent_t g_sev[FX_PROFILE_SLOTS][2] = {};
static bool g_sev_valid[FX_PROFILE_SLOTS] = {};
void profile_slot_record(uint32_t slot, bool end, hipStream_t s) {
  if (!g_profile || slot >= FX_PROFILE_SLOTS) return;
  hipEvent_t& e = g_sev[slot][end ? 1 : 0];
  if (!e && hipEventCreate(&e) != hipSuccess) return;
  (void)hipEventRecord(e, s);
  g_sev_valid[slot] = end;
}

void split_profile_record(int which, bool end, hipStream_t s) {
  if (!g_profile || which < 1 || which > 2) return;
  hipEvent_t& e = g_kev[which][end ? 1 : 0];
  if (!e && hipEventCreate(&e) != hipSuccess) return;
  (void)hipEventRecord(e, s);
  g_kev_valid[which] = end;
}

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
    case FX_ERR_LOG_FORMAT: return "malformed execution log";
    case FX_ERR_SIM_CAPACITY: return "simulated instance outgrew its launch geometry";
    case FX_ERR_SIM_LATE: return "simulated message found no state for its dot";
    case FX_ERR_SIM_EVENTS: return "simulated instance exceeded its event budget";
    case FX_ERR_TIMEOUT: return "a drop-in handle's wait for its resident kernel passed the deadline";
    default: return "unknown";
  }
}

int fx_tier_query(uint32_t tier, uint32_t n, fx_tier_info* out) {
  if (!out) return FX_ERR_INVALID_ARG;
  switch (tier) {
    case 0: *out = {GROUP_LANES, GROUP_SLOTS, GROUP_WINDOW_BITS, group_state_words_per_stream()}; break;
    case 1: *out = {Tier1::NSRC, Tier1::P, 32 * Tier1::XW, Tier1::WORDS}; break;
    case 2: *out = {Tier2::NSRC, Tier2::P, 32 * Tier2::XW, Tier2::WORDS}; break;
    case 3: *out = {TierLane::NSRC, TierLane::P, 32 * TierLane::XW, TierLane::WORDS}; break;
    case 4: *out = {8, WAVE_SLOTS, WAVE_WINDOW_BITS, wave_state_words_per_stream()}; break;
    case 5: *out = {8, LANE_SLOTS, LANE_WINDOW_BITS, lane_state_words_per_stream()}; break;
    case 6: *out = {8, std::min(LANE_SLOTS, GROUP_SLOTS), std::min(LANE_WINDOW_BITS, GROUP_WINDOW_BITS), 0}; break;
    case FX_TIER_WIDE: *out = {8, 512, 1024, 0}; break;
    case FX_TIER_WIDE_HBM: *out = {8, 16384, 32768, (uint32_t)(wide_state_bytes(FX_TIER_WIDE_HBM, n, 1) / 4)}; break;
    default: return FX_ERR_INVALID_ARG;
  }
  return n >= 1 && n <= out->max_sources ? FX_OK : FX_ERR_INVALID_ARG;
}

size_t fx_batch_state_bytes(uint32_t tier, uint32_t n, uint32_t lanes) {
  switch (tier) {
    case 0: return group_state_bytes(lanes);
    case 1: return state_bytes<Tier1>(lanes);
    case 2: return state_bytes<Tier2>(lanes);
    case 3: return state_bytes<TierLane>(lanes);
    case 4: return wave_state_bytes(lanes);
    case 5: return lane_state_bytes(lanes);
    case 6: return split_scratch_bytes(lanes);  // scheduling scratch, not resumable state
    case FX_TIER_WIDE:
    case FX_TIER_WIDE_HBM: return wide_state_bytes(tier, n, lanes);  // working tables (HBM tier)
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
  // the split tier schedules whole batches: no map, no resumable state
  if (tier == FX_TIER_SPLIT &&
      (stream_map || num_lanes != in->num_streams || !state || !(flags & FX_FLAG_INIT) ||
       (flags & FX_FLAG_SAVE_STATE)))
    return FX_ERR_INVALID_ARG;
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
  a.dbg = nullptr;
  a.lanes_dev = nullptr;
  a.req = nullptr;
  a.req_cap = 0;
  if (flags & FX_FLAG_PARTIAL) return FX_ERR_INVALID_ARG;  // fx_batch_execute_partial
  hipStream_t hs = (hipStream_t)hip_stream;
  if (g_profile) {
    if (!g_ev0) {
      if (hipEventCreate(&g_ev0) != hipSuccess || hipEventCreate(&g_ev1) != hipSuccess) return FX_ERR_HIP;
    }
    (void)hipEventRecord(g_ev0, hs);
    g_kev_valid[1] = g_kev_valid[2] = false;
  }
  profile_slot_record(tier, false, hs);
  switch (tier) {
    case 0: st = launch_group(a, hs); break;
    case 1: st = launch_exec<Tier1>(a, hs); break;
    case 2: st = launch_exec<Tier2>(a, hs); break;
    case 3: st = launch_exec<TierLane>(a, hs); break;
    case 4: st = launch_wave(a, hs); break;
    case 5: st = launch_lane(a, hs); break;
    case 6: st = launch_split(a, state, hs); break;
    case FX_TIER_WIDE: st = launch_wide(a, false, hs); break;
    case FX_TIER_WIDE_HBM: st = launch_wide(a, true, hs); break;
    default: return FX_ERR_INVALID_ARG;
  }
  if (g_profile) {
    (void)hipEventRecord(g_ev1, hs);
    g_ev_valid = st == FX_OK;
    if (st == FX_OK) profile_slot_record(tier, true, hs);
  }
  return st;
}

size_t fx_partial_state_bytes(uint32_t n, uint32_t num_streams) { return wide_partial_state_bytes(n, num_streams); }

int fx_batch_execute_partial(const fx_stream_batch* in, const fx_order_batch* out, void* state,
                             uint32_t step_begin, uint32_t step_end, uint32_t flags,
                             const uint32_t* init_frontier, uint32_t* req, uint32_t req_cap, void* hip_stream) {
  int st = check_batch(in, out);
  if (st) return st;
  if (step_end > in->steps || step_begin > step_end || !state || !req || req_cap == 0) return FX_ERR_INVALID_ARG;
  if (flags & ~(FX_FLAG_INIT | FX_FLAG_SAVE_STATE)) return FX_ERR_INVALID_ARG;
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
  a.stream_map = nullptr;
  a.num_lanes = in->num_streams;
  a.state = (uint32_t*)state;
  a.step_begin = step_begin;
  a.step_end = step_end;
  a.flags = flags | FX_FLAG_PARTIAL;
  a.init_frontier = init_frontier;
  a.dbg = nullptr;
  a.lanes_dev = nullptr;
  a.drift = 0;
  a.req = req;
  a.req_cap = req_cap;
  return launch_wide(a, true, (hipStream_t)hip_stream);
}

int fx_profile_enable(int on) {
  g_profile = on != 0;
  g_ev_valid = false;
  g_kev_valid[1] = g_kev_valid[2] = false;
  for (uint32_t i = 0; i < FX_PROFILE_SLOTS; ++i) g_sev_valid[i] = false;
  return FX_OK;
}

int fx_profile_slot_ms(uint32_t slot, float* ms) {
  if (!ms || slot >= FX_PROFILE_SLOTS) return FX_ERR_INVALID_ARG;
  if (!g_sev_valid[slot]) return FX_ERR_INVALID_ARG;
  if (hipEventSynchronize(g_sev[slot][1]) != hipSuccess) return FX_ERR_HIP;
  return hipEventElapsedTime(ms, g_sev[slot][0], g_sev[slot][1]) == hipSuccess ? FX_OK : FX_ERR_HIP;
}

int fx_profile_last_kernel_ms(uint32_t which, float* ms) {
  if (!ms) return FX_ERR_INVALID_ARG;
  if (which == 0) return fx_profile_last_exec_ms(ms);
  if (which > 2 || !g_kev_valid[which]) return FX_ERR_INVALID_ARG;
  if (hipEventSynchronize(g_kev[which][1]) != hipSuccess) return FX_ERR_HIP;
  return hipEventElapsedTime(ms, g_kev[which][0], g_kev[which][1]) == hipSuccess ? FX_OK : FX_ERR_HIP;
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
  const size_t nblocks = in->num_streams <= 64 ? ((size_t)4 * in->num_streams * steps4 + 255) / 256
                                               : (size_t)((in->num_streams + 63) / 64) * steps4;
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
  if (p->clients > 1 && p->cmds_per_process % p->clients) return FX_ERR_INVALID_ARG;
  if (p->key_pool == 1 || (p->key_pool > 1 && p->clients > 1)) return FX_ERR_INVALID_ARG;
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
  // every command writes its own words of the planes: commands split over threads
  const size_t total = (size_t)p->instances * steps;
  const uint32_t nt = total < 4096 ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (size_t i = t; i < total; i += nt)
        synth_emit(*p, (uint32_t)(i / steps), (uint32_t)(i % steps), S, steps, dot, hdr, deps);
    });
  for (auto& x : th) x.join();
  return FX_OK;
}

}  // extern "C"

namespace fx {

static void* g_scratch[SCRATCH_SLOTS] = {};
static size_t g_scratch_cap[SCRATCH_SLOTS] = {};

void* scratch(uint32_t slot, size_t bytes) {
  if (slot >= SCRATCH_SLOTS) return nullptr;
  bytes = std::max<size_t>(bytes, 256);
  if (g_scratch_cap[slot] >= bytes) return g_scratch[slot];
  if (g_scratch[slot]) (void)hipFree(g_scratch[slot]);
  g_scratch[slot] = nullptr;
  g_scratch_cap[slot] = 0;
  const size_t grown = bytes + bytes / 4;
  if (hipMalloc(&g_scratch[slot], grown) != hipSuccess) return nullptr;
  g_scratch_cap[slot] = grown;
  return g_scratch[slot];
}

std::recursive_mutex& scratch_mutex() {
  static std::recursive_mutex m;
  return m;
}

// Escalation chain of fx_batch_run_tiered (FX_NUM_TIERS = none).
static uint32_t escalate(uint32_t tier) {
  switch (tier) {
    case FX_TIER_GROUP: return FX_TIER_LDS_LARGE;
    case FX_TIER_LANE: return FX_TIER_LDS_LARGE;
    case FX_TIER_LDS_LARGE: return FX_TIER_GLOBAL;
    case FX_TIER_GLOBAL: return FX_TIER_WIDE;
    case FX_TIER_WIDE: return FX_TIER_WIDE_HBM;
    case FX_TIER_WAVE: return FX_TIER_GLOBAL;
    case FX_TIER_LANE_REG: return FX_TIER_LDS_LARGE;
    case FX_TIER_SPLIT: return FX_TIER_LDS_LARGE;
    default: return FX_NUM_TIERS;
  }
}

// Synchronous tiered driver: the first tier for all (or for the streams in
// `only`), then reruns of the streams that ran out of capacity up the
// escalation chain.  The error plane comes back with one copy per tier.
// Streams of a launch (list, or 0..L-1 when list is null) that stopped with
// FX_ERR_CAPACITY, appended to out_list (order arbitrary: the next tier's
// stream map; results do not depend on it); cnt[0] = how many.
__global__ __launch_bounds__(256) void k_collect_capacity(const uint32_t* __restrict__ err,
                                                          const uint32_t* __restrict__ list, uint32_t L,
                                                          uint32_t* __restrict__ out_list, uint32_t* cnt) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t s = i < L ? (list ? list[i] : i) : 0u;
  const bool cap = i < L && err[s] == FX_ERR_CAPACITY;
  const uint64_t b = __ballot(cap);
  if (!b) return;
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t base = 0;
  if (lane == (uint32_t)__builtin_ctzll(b)) base = atomicAdd(cnt, (uint32_t)__builtin_popcountll(b));
  base = (uint32_t)__shfl((int)base, (int)__builtin_ctzll(b), 64);
  if (cap) out_list[base + (uint32_t)__builtin_popcountll(b & ((1ull << lane) - 1ull))] = s;
}

// cnt[1] = lowest stream index (of list, or 0..L-1) with a nonzero status
__global__ __launch_bounds__(256) void k_first_error(const uint32_t* __restrict__ err,
                                                     const uint32_t* __restrict__ list, uint32_t L, uint32_t* cnt) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t s = i < L ? (list ? list[i] : i) : 0u;
  const bool bad = i < L && err[s] != 0;
  const uint64_t b = __ballot(bad);
  if (!b) return;
  uint32_t m = bad ? s : 0xFFFFFFFFu;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) m = min(m, (uint32_t)__shfl_xor((int)m, (int)o, 64));
  if ((threadIdx.x & 63u) == 0) atomicMin(&cnt[1], m);
}

// The escalation driver.  Every decision stays on the device except one
// 8-byte read per tier: the streams that ran out of capacity are compacted
// into the next tier's stream map by k_collect_capacity, and the status to
// return is the lowest failing stream's (k_first_error) -- no per-stream host
// work, which at 4.4 M segments (configs[4]) had cost ~10 ms per call.
int run_tiered(const fx_stream_batch* in, const fx_order_batch* out, uint32_t flags, void* hip_stream,
               const std::vector<uint32_t>* only, uint32_t* tier_counts) {
  std::lock_guard<std::recursive_mutex> lock(scratch_mutex());
  int st = check_batch(in, out);
  if (st) return st;
  hipStream_t hs = (hipStream_t)hip_stream;
  const uint32_t S = in->num_streams;
  flags |= FX_FLAG_INIT;
  flags &= ~FX_FLAG_SAVE_STATE;
  const uint32_t ft = (flags >> FX_FLAG_TIER_SHIFT) & 15u;
  flags &= ~(15u << FX_FLAG_TIER_SHIFT);
  uint32_t first = ft ? ft - 1u : (uint32_t)FX_TIER_DEFAULT;
  if (first >= FX_NUM_TIERS) return FX_ERR_INVALID_ARG;
  if (only && first == FX_TIER_SPLIT) first = FX_TIER_GROUP;  // the split tier takes whole batches
  // tiers that cannot hold the widest Add start one step up the chain
  if ((first == FX_TIER_WAVE && in->dmax > WAVE_MAX_DEPS) ||
      ((first == FX_TIER_GROUP || first == FX_TIER_SPLIT) && in->dmax > GROUP_LANES) ||
      (first == FX_TIER_LANE_REG && in->dmax > LANE_MAX_DEPS))
    first = FX_TIER_LDS_LARGE;
  if (tier_counts)
    for (uint32_t t = 0; t < FX_NUM_TIERS; ++t) tier_counts[t] = 0;
  const uint32_t L0 = only ? (uint32_t)only->size() : S;
  if (L0 == 0) return FX_OK;
  uint32_t* maps[2] = {(uint32_t*)scratch(SCRATCH_TIERED_MAP, (size_t)L0 * 4),
                       (uint32_t*)scratch(SCRATCH_TIERED_MAP2, (size_t)L0 * 4)};
  uint32_t* cnt = (uint32_t*)scratch(SCRATCH_TIERED_CNT, 8);
  if (!maps[0] || !maps[1] || !cnt) return FX_ERR_HIP;
  const uint32_t* list0 = nullptr;  // the launch's streams: null = all S
  if (only && hipMemcpyAsync(maps[0], only->data(), (size_t)L0 * 4, hipMemcpyHostToDevice, hs) != hipSuccess)
    return FX_ERR_HIP;
  if (only) list0 = maps[0];
  const uint32_t* list = list0;
  uint32_t L = L0, side = only ? 1u : 0u;
  uint32_t h[2] = {0, 0};
  for (uint32_t tier = first; tier < FX_NUM_TIERS && L; tier = escalate(tier)) {
    if (tier == FX_TIER_WIDE && !wide_lds_fits(in->n, in->dmax)) continue;  // straight to the HBM tables
    if (tier_counts) tier_counts[tier] = L;
    void* dstate = nullptr;
    if ((tier == FX_TIER_GLOBAL || tier == FX_TIER_SPLIT || tier == FX_TIER_WIDE_HBM) &&
        !(dstate = scratch(SCRATCH_TIERED_STATE, fx_batch_state_bytes(tier, in->n, L))))
      return FX_ERR_HIP;
    st = fx_batch_execute(in, out, tier, list, L, dstate, 0, in->steps, flags, nullptr, hip_stream);
    if (st) return st;
    uint32_t* next = maps[side];
    if (next == list) next = maps[side ^ 1u];
    if (hipMemsetAsync(cnt, 0, 4, hs) != hipSuccess) return FX_ERR_HIP;
    hipLaunchKernelGGL(k_collect_capacity, dim3((L + 255) / 256), dim3(256), 0, hs, out->err, list, L, next, cnt);
    if (hipMemcpyAsync(h, cnt, 4, hipMemcpyDeviceToHost, hs) != hipSuccess || hipStreamSynchronize(hs) != hipSuccess)
      return FX_ERR_HIP;
    L = h[0];
    list = next;
    side = (next == maps[0]) ? 1u : 0u;
  }
  // status: the lowest failing stream's (streams still at FX_ERR_CAPACITY
  // after the last tier included)
  const uint32_t init[2] = {0, 0xFFFFFFFFu};
  if (hipMemcpyAsync(cnt, init, 8, hipMemcpyHostToDevice, hs) != hipSuccess) return FX_ERR_HIP;
  if (only && hipMemcpyAsync(maps[0], only->data(), (size_t)L0 * 4, hipMemcpyHostToDevice, hs) != hipSuccess)
    return FX_ERR_HIP;
  hipLaunchKernelGGL(k_first_error, dim3((L0 + 255) / 256), dim3(256), 0, hs, out->err, only ? maps[0] : nullptr,
                     L0, cnt);
  uint32_t e = 0;
  if (hipMemcpyAsync(h, cnt, 8, hipMemcpyDeviceToHost, hs) != hipSuccess || hipStreamSynchronize(hs) != hipSuccess)
    return FX_ERR_HIP;
  if (h[1] != 0xFFFFFFFFu &&
      (hipMemcpyAsync(&e, out->err + h[1], 4, hipMemcpyDeviceToHost, hs) != hipSuccess ||
       hipStreamSynchronize(hs) != hipSuccess))
    return FX_ERR_HIP;
  return h[1] == 0xFFFFFFFFu ? FX_OK : (int)e;
}

}  // namespace fx

extern "C" {

int fx_batch_run_tiered(const fx_stream_batch* in, const fx_order_batch* out, uint32_t flags,
                        void* hip_stream, uint32_t* tier_counts) {
  return fx::run_tiered(in, out, flags, hip_stream, nullptr, tier_counts);
}

}  // extern "C"
