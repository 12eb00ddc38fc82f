// graph_wave.hip — the wavefront-per-stream tier of the batched GraphExecutor.
//
// Same algorithm as graph_exec.hip / graph_group.hip (DependencyGraph::handle_add,
// fantoch_ps/src/executor/graph/mod.rs:213-642, canonical orders C1 and C2),
// laid out so that ONE 64-lane wavefront runs ONE executor and every control
// decision is wave-uniform (scalar branches, no divergence at all):
//   * lane l owns pending-vertex slot l (VertexIndex, index.rs:18-51): its dot,
//     arrival index, registered-on dot (PendingIndex, index.rs:145-208), Tarjan
//     id/low/visited-epoch word and one DFS frame sit in lane l's VGPRs; a
//     lookup by dot is one compare + ballot, a field read is one v_readlane;
//   * lane l < n owns the executed clock of source l + 1 (AEClock, threshold
//     0.9.1: frontier + 32-bit exception window);
//   * the deps of an incoming Add are checked in parallel (lane j: dep j);
//   * the Tarjan stack is implicit: the vertices on it are exactly the pending
//     slots with a non-zero id, in id order (tarjan.rs:96-316), so an SCC pop
//     is one ballot (id >= id(root));
//   * the deps of each pending vertex that were not yet executed when it was
//     indexed, the check_pending worklist and a 16-step chunk of the input
//     planes live in LDS.
// The input chunk for steps [16c, 16c+16) is fetched one chunk ahead by one
// 16-byte load per lane (lane 4p+b: plane p, 4-step block b of the chunk), so
// HBM latency is covered by 16 steps of work and the vmcnt wait is static.
// A stream that outgrows 64 pending vertices, 8 cached deps per vertex or the
// 32-bit clock window stops with FX_ERR_CAPACITY and is rerun at tier 2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace wav {

constexpr uint32_t P = WAVE_SLOTS;      // pending slots (one per lane)
constexpr uint32_t C = WAVE_CACHE;      // cached deps per slot
constexpr uint32_t WLC = P + 1;         // check_pending worklist capacity
constexpr uint32_t CH = 16;             // steps per input chunk
constexpr uint32_t NPL = 16;            // input planes per chunk: dot, hdr, 14 dep planes
constexpr uint32_t MAXD = NPL - 2;      // deps per Add this tier reads
constexpr uint32_t WPB = 4;             // wavefronts (streams) per workgroup
constexpr uint32_t L_CACHE = 0;         // LDS words per stream: [P][C] cached deps
constexpr uint32_t L_WL = P * C;        //                        [WLC] worklist
constexpr uint32_t L_IN = (L_WL + WLC + 3) & ~3u;  //            [NPL][CH] input chunk
constexpr uint32_t LW = L_IN + NPL * CH;
constexpr uint32_t RREGS = 7;           // saved per-lane registers
constexpr uint32_t S_LDS = 64 * RREGS;  // saved state: regs | LDS cache + worklist | scalars
constexpr uint32_t S_SCAL = S_LDS + L_IN;
constexpr uint32_t WPS = S_SCAL + 8;

enum : uint32_t { PH_IDLE = 0, PH_DFS = 1, PH_TRY = 2, PH_CHECK = 3 };

// Tarjan word: id (7 bits) | low (7 bits) | visited epoch (16 bits)
__device__ __forceinline__ uint32_t tid(uint32_t t) { return t & 127u; }
__device__ __forceinline__ uint32_t tlow(uint32_t t) { return (t >> 7) & 127u; }
__device__ __forceinline__ uint32_t tep(uint32_t t) { return t >> 14; }
__device__ __forceinline__ uint32_t tmk(uint32_t id, uint32_t low, uint32_t ep) {
  return id | (low << 7) | (ep << 14);
}
constexpr uint32_t EPOCH_MAX = 0xFFFFu;

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)src);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint32_t gather(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ uint64_t bal(bool p) { return (uint64_t)__ballot(p); }
__device__ __forceinline__ uint32_t ctz64(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }
__device__ __forceinline__ uint32_t pop64(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }

// Where an executed command goes.  PlaneOut: the batch tiers' order plane
// (row k = the k-th executed command) and release plane (row rec = the step
// that executed arrival rec).  The persistent handle kernel (handle_persist.hip)
// writes the same (order word, release step) pairs into a host-mapped ring.
struct PlaneOut {
  uint32_t* order = nullptr;
  uint32_t* release = nullptr;
  uint32_t stream = 0, steps = 0;
  __device__ __forceinline__ void put(uint32_t k, uint32_t word, uint32_t rec, uint32_t cur) const {
    order[fx_index(k, stream, steps)] = word;
    release[fx_index(rec, stream, steps)] = cur;
  }
};

template <class Out>
struct Wave {
  uint32_t lid;
  uint64_t lbit;  // 1 << lid
  // lane-owned slot fields (slot = lid), DFS frame (depth = lid), clock (source = lid + 1)
  uint32_t sdot = 0, srec = 0, swait = 0, stl = 0, sfr = 0;
  uint32_t cf = 0, cw = 0;
  uint32_t fdep = 0;  // lane j < C: cached dep j of the DFS's current vertex fv
  // wave-uniform state
  uint64_t occ = 0, wmask = 0, tmask = 0;
  uint32_t k = 0, err = 0, epoch = 1, nwl = 0, cur = 0;
  uint32_t phase = PH_IDLE, root = 0, idc = 0, nfr = 0, missing = 0;
  uint32_t fv = 0, fdi = 0, fnc = 0, in_try = 0, emitted = 0;
  // stream context; kcap: order entries the output holds
  uint32_t stream = 0, n = 0, steps = 0, kcap = 0;
  uint32_t* lds = nullptr;
  Out out;

  __device__ __forceinline__ size_t at(uint32_t step) const { return fx_index(step, stream, steps); }
  __device__ __forceinline__ bool mine(uint64_t m) const { return (m & lbit) != 0; }

  // ------------------------------------------------------------ clock
  // AEClock::contains for a per-lane dot (tarjan.rs:131-132)
  __device__ __forceinline__ bool contains_v(uint32_t d) const {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    const uint32_t f = gather(cf, si & 63u), w = gather(cw, si & 63u);
    const uint32_t seq = d & FX_SEQ_MASK, off = seq - f - 1u;
    return si < n && (seq <= f || (off < 32u && ((w >> (off & 31u)) & 1u)));
  }
  // AEClock::contains for a wave-uniform dot
  __device__ __forceinline__ bool contains_u(uint32_t d) const {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) return false;
    const uint32_t f = rl(cf, si), w = rl(cw, si);
    const uint32_t seq = d & FX_SEQ_MASK, off = seq - f - 1u;
    return seq <= f || (off < 32u && ((w >> off) & 1u));
  }
  // AEClock::add for a wave-uniform dot (tarjan.rs:293)
  __device__ __forceinline__ void clk_add(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) { err = FX_ERR_DOT_RANGE; return; }
    uint32_t f = rl(cf, si), w = rl(cw, si);
    const uint32_t seq = d & FX_SEQ_MASK;
    if (seq <= f) return;
    const uint32_t off = seq - f - 1u;
    if (off >= 32u) { err = FX_ERR_CAPACITY; return; }
    if (off != 0) {
      w |= 1u << off;
    } else {
      const uint32_t win = w >> 1;               // bit j <-> seq f + 2 + j
      const uint32_t ones = __builtin_ctz(~win);  // top bit of win is 0 -> <= 31
      f = f + 1 + ones;
      w = win >> ones;
    }
    if (lid == si) {
      cf = f;
      cw = w;
    }
  }

  // ------------------------------------------------------ slot table
  __device__ __forceinline__ int find(uint32_t d) const {
    const uint64_t m = bal(mine(occ) && sdot == d);
    return m ? (int)ctz64(m) : -1;
  }
  __device__ __forceinline__ uint32_t& cache(uint32_t sl, uint32_t j) { return lds[L_CACHE + sl * C + j]; }
  __device__ __forceinline__ uint32_t& wl(uint32_t i) { return lds[L_WL + i]; }

  __device__ __forceinline__ void new_epoch() {
    epoch = epoch + 1;
    if (epoch > EPOCH_MAX) {
      if (mine(occ)) stl = tmk(tid(stl), tlow(stl), 0);
      epoch = 1;
    }
  }

  // VertexIndex::index(Vertex::new(dot, cmd, deps, time)) (index.rs:33-37);
  // keep = lane j holds dep j of the Add and it is not executed (executed deps
  // are ignored by every later search, tarjan.rs:128-145, and the executed
  // clock only grows); they are cached in ascending order.
  __device__ __forceinline__ int insert_vertex(uint32_t i, uint32_t d, bool keep, uint32_t depj) {
    const uint64_t fre = ~occ;
    if (!fre) { err = FX_ERR_CAPACITY; return -1; }
    const uint32_t sl = ctz64(fre);
    const uint64_t km = bal(keep);
    const uint32_t nc = pop64(km);
    if (nc > C) { err = FX_ERR_CAPACITY; return -1; }
    if (keep) cache(sl, pop64(km & (lbit - 1u))) = depj;
    if (lid == sl) {
      sdot = d;
      srec = i | (nc << 26);
      swait = 0;
      stl = 0;
    }
    occ |= 1ull << sl;
    return (int)sl;
  }

  // save_scc (mod.rs:488-523) for a singleton: to_execute + executed clock
  __device__ __forceinline__ void emit_one(uint32_t rec, uint32_t d) {
    if (k >= kcap) { err = FX_ERR_ORDER_OVERFLOW; return; }
    if (lid == 0) out.put(k, rec | FX_ORDER_SCC_START, rec, cur);
    ++k;
    clk_add(d);
  }

  // the current vertex's cached deps into lanes 0..C-1 (one LDS read per
  // vertex entered or returned to; its latency overlaps the rest of the step)
  __device__ __forceinline__ void load_fdep() { fdep = lid < C ? cache(fv, lid) : 0u; }

  __device__ __forceinline__ void dfs_start(uint32_t r, bool intry) {
    root = r;
    in_try = intry;
    emitted = 0;
    missing = 0;
    idc = 1;
    const uint32_t tr = rl(stl, r);
    if (lid == r) stl = tmk(1, 1, tep(tr));
    nfr = 0;
    fv = r;
    load_fdep();
    fdi = 0;
    fnc = rl(srec, r) >> 26;
    phase = PH_DFS;
  }

  // The SCC rooted at fv = the stack vertices with id >= id(fv), saved in
  // ascending dot order (SCC = BTreeSet<Dot>, tarjan.rs:15), clock updated.
  __device__ __forceinline__ void save_scc() {
    const uint32_t idv = tid(rl(stl, fv));
    const bool mem = mine(occ) && tid(stl) >= idv;
    const uint64_t mm = bal(mem);
    const uint32_t cnt = pop64(mm);
    if (cnt > kcap - k) { err = FX_ERR_ORDER_OVERFLOW; return; }
    if (nwl + cnt > WLC) { err = FX_ERR_CAPACITY; return; }
    uint32_t rank = 0;
    if (cnt == 1) {
      const uint32_t d = rl(sdot, fv);
      if (lid == 0) {
        const uint32_t rec = rl(srec, fv) & 0x03FFFFFFu;
        out.put(k, rec | FX_ORDER_SCC_START, rec, cur);
        wl(nwl) = d;
      }
      ++k;
      ++nwl;
      clk_add(d);
    } else {
      for (uint64_t m = mm; m; m &= m - 1) rank += rl(sdot, ctz64(m)) < sdot ? 1u : 0u;
      if (mem) {
        const uint32_t rec = srec & 0x03FFFFFFu;
        out.put(k + rank, rec | (rank == 0 ? FX_ORDER_SCC_START : 0u), rec, cur);
        wl(nwl + rank) = sdot;
      }
      k += cnt;
      nwl += cnt;
      for (uint32_t r = 0; r < cnt; ++r) {  // clock in ascending dot order
        const uint32_t lr = ctz64(bal(mem && rank == r));
        clk_add(rl(sdot, lr));
      }
    }
    occ &= ~mm;
    wmask &= ~mm;
    tmask &= ~mm;
    emitted = 1;
  }

  __device__ __forceinline__ void dfs_finish() {
    // finalize (tarjan.rs:60-93): reset ids of the vertices left on the stack;
    // in try_pending a failed search that saved no SCC marks them visited
    const bool mark = in_try && missing != 0 && !emitted;
    if (mine(occ) && tid(stl) != 0) stl = tmk(0, 0, mark ? epoch : tep(stl));
    if (missing) {  // index_pending(dot, missing) (mod.rs:525-554)
      if (lid == root) swait = missing;
      wmask |= 1ull << root;
    }
    if (in_try) {
      if (!missing || emitted) new_epoch();  // visited.clear() (mod.rs:607, 621-623)
      phase = PH_TRY;
    } else {
      phase = PH_CHECK;
    }
  }

  // one DFS edge or one frame pop (TarjanSCCFinder::strong_connect, iterative)
  __device__ __forceinline__ void dfs_iter() {
    if (fdi < fnc) {
      const uint32_t dep = rl(fdep, fdi);
      ++fdi;
      if (contains_u(dep)) return;  // executed (tarjan.rs:128-145)
      const int x = find(dep);
      if (x < 0) {  // missing: give up (tarjan.rs:148-157, shard_count == 1)
        missing = dep;
        dfs_finish();
        return;
      }
      const uint32_t tx = rl(stl, (uint32_t)x);
      if (tid(tx) == 0) {  // not visited: recurse (tarjan.rs:172-214)
        ++idc;
        if (lid == (uint32_t)x) stl = tmk(idc, idc, tep(tx));
        if (lid == nfr) sfr = fv | (fdi << 8);
        ++nfr;
        fv = (uint32_t)x;
        load_fdep();
        fdi = 0;
        fnc = rl(srec, fv) >> 26;
      } else {  // visited and on the stack (tarjan.rs:215-225)
        const uint32_t tv = rl(stl, fv);
        if (tid(tx) < tlow(tv) && lid == fv) stl = tmk(tid(tv), tid(tx), tep(tv));
      }
    } else {
      const uint32_t tv = rl(stl, fv);
      const uint32_t lowv = tlow(tv);
      if (tid(tv) == lowv) {  // SCC root (tarjan.rs:233-312)
        save_scc();
        if (err) return;
      }
      if (nfr == 0) {  // root done: Found
        dfs_finish();
        return;
      }
      --nfr;
      const uint32_t f = rl(sfr, nfr);  // back in the parent (tarjan.rs:211)
      fv = f & 0xFFu;
      load_fdep();
      fdi = f >> 8;
      fnc = rl(srec, fv) >> 26;
      const uint32_t tp = rl(stl, fv);
      if (lowv < tlow(tp) && lid == fv) stl = tmk(tid(tp), lowv, tep(tp));
    }
  }

  // try_pending (mod.rs:589-642): next waiter of the snapshot, ascending (C2)
  __device__ __forceinline__ void try_iter() {
    if (!tmask) { phase = PH_CHECK; return; }
    uint32_t best = ctz64(tmask), best_dot = rl(sdot, best);
    for (uint64_t m = tmask & (tmask - 1); m; m &= m - 1) {
      const uint32_t b = ctz64(m), v = rl(sdot, b);
      if (v < best_dot) {
        best_dot = v;
        best = b;
      }
    }
    tmask &= ~(1ull << best);
    if (tep(rl(stl, best)) == epoch) return;  // visited: skipped, not re-registered
    dfs_start(best, true);
  }

  // check_pending (mod.rs:556-587): pop one released dot (LIFO)
  __device__ __forceinline__ void check_iter() {
    if (nwl == 0 || !wmask) {
      nwl = 0;
      phase = PH_IDLE;
      return;
    }
    --nwl;
    const uint32_t x = uni(wl(nwl));
    const uint64_t t = bal(mine(wmask) && swait == x);
    if (!t) return;
    wmask &= ~t;  // PendingIndex::remove(x)
    tmask = t;
    new_epoch();  // try_pending's fresh `visited`
    phase = PH_TRY;
  }

  // GraphExecutor::handle(Add) (executor.rs:69-80) -> handle_add (mod.rs:213-275)
  __device__ __forceinline__ void step_start(uint32_t i, uint32_t d, uint32_t h, uint32_t depj,
                                             uint32_t dmax, bool at_commit) {
    cur = i;
    nwl = 0;
    const uint32_t nd = (h >> 24) & 31u, kind = h >> 29;
    if (nd > dmax || nd > MAXD) { err = FX_ERR_INVALID_ARG; return; }
    if ((d >> FX_SEQ_BITS) - 1u >= n || (d & FX_SEQ_MASK) == 0) { err = FX_ERR_DOT_RANGE; return; }
    if (at_commit) {  // execute_at_commit bypass (executor.rs:72-73)
      if (k >= kcap) { err = FX_ERR_ORDER_OVERFLOW; return; }
      if (lid == 0) out.put(k, i | FX_ORDER_SCC_START, i, i);
      ++k;
      return;
    }
    // the clock lookups (two ds_bpermute) are issued first so that their LDS
    // latency overlaps the checks; lane j - 1's dep comes by DPP (wave_shr:1)
    const bool exd = contains_v(depj);  // every lane active: ds_bpermute reads 0 from inactive lanes
    const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)depj, 0x138, 0xF, 0xF, false);
    if (occ && find(d) >= 0) { err = FX_ERR_DOUBLE_INDEX; return; }  // mod.rs:233-237
    const bool valid = lid < nd;
    if (bal(valid && lid > 0 && depj <= prev)) { err = FX_ERR_DEPS_UNSORTED; return; }
    const bool keep = valid && depj != d && !exd;
    if (kind == FX_KIND_INDEX_ONLY) {
      insert_vertex(i, d, keep, depj);
      return;
    }
    // fast path: every dep is self or executed -> a singleton SCC
    if (!bal(keep)) {
      emit_one(i, d);
      if (wmask && !err) {  // check_pending([dot])
        if (lid == 0) wl(0) = d;
        nwl = 1;
        phase = PH_CHECK;
      }
      return;
    }
    const int sl = insert_vertex(i, d, keep, depj);
    if (sl >= 0) dfs_start((uint32_t)sl, false);
  }

  // the wave-uniform state back into scalar registers (readfirstlane of a
  // value the compiler keeps in a VGPR; a no-op for one already scalar), so the
  // step loop's branches are scalar compares and its state is not copied
  // between VGPR versions on every iteration
  __device__ __forceinline__ void canon() {
    phase = uni(phase);
    root = uni(root);
    idc = uni(idc);
    nfr = uni(nfr);
    missing = uni(missing);
    fv = uni(fv);
    fdi = uni(fdi);
    fnc = uni(fnc);
    in_try = uni(in_try);
    emitted = uni(emitted);
    k = uni(k);
    err = uni(err);
    epoch = uni(epoch);
    nwl = uni(nwl);
  }

  __device__ __forceinline__ void run_slow() {
    while (phase != PH_IDLE) {
      canon();
      if (phase == PH_DFS) dfs_iter();
      else if (phase == PH_TRY) try_iter();
      else check_iter();
      if (err) phase = PH_IDLE;
    }
  }
};

// workgroup index -> logical workgroup: two consecutive logical workgroups
// (8 streams = one 128-byte line of every input tile row) share an XCD
// (hardware dispatch is round-robin over the 8 XCDs).
__device__ __forceinline__ uint32_t logical_block(uint32_t b) {
  const uint32_t x = b & 7u, j = b >> 3;
  return 16u * (j >> 1) + 2u * x + (j & 1u);
}

__global__ __launch_bounds__(64 * WPB) void k_graph_wave(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[WPB * LW];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = uni(threadIdx.x >> 6);
  const uint32_t gg = logical_block(blockIdx.x) * WPB + w;  // stream index within the launch
  if (gg >= a.num_lanes) return;  // whole wavefront
  const uint32_t s = a.stream_map ? uni(a.stream_map[gg]) : gg;
  const uint32_t len = a.lengths ? min(uni(a.lengths[s]), a.steps) : a.steps;
  uint32_t* gst = a.state ? a.state + (size_t)gg * WPS : nullptr;

  Wave<PlaneOut> e;
  e.lid = lane;
  e.lbit = 1ull << lane;
  e.stream = s;
  e.n = a.n;
  e.steps = a.steps;
  e.kcap = a.steps;
  e.lds = smem + w * LW;
  e.out.order = a.order;
  e.out.release = a.release;
  e.out.stream = s;
  e.out.steps = a.steps;

  if (a.flags & FX_FLAG_INIT) {
    if (a.init_frontier && lane < 8) e.cf = a.init_frontier[(size_t)s * 8 + lane];
  } else {
    const uint32_t* r = gst + lane * RREGS;
    e.sdot = r[0];
    e.srec = r[1];
    e.swait = r[2];
    e.stl = r[3];
    e.sfr = r[4];
    e.cf = r[5];
    e.cw = r[6];
    for (uint32_t q = lane; q < L_IN; q += 64) e.lds[q] = gst[S_LDS + q];
    e.occ = (uint64_t)uni(gst[S_SCAL + 0]) | ((uint64_t)uni(gst[S_SCAL + 1]) << 32);
    e.wmask = (uint64_t)uni(gst[S_SCAL + 2]) | ((uint64_t)uni(gst[S_SCAL + 3]) << 32);
    e.k = uni(gst[S_SCAL + 4]);
    e.err = uni(gst[S_SCAL + 5]);
    e.epoch = uni(gst[S_SCAL + 6]);
  }

  const bool at_commit = (a.flags & FX_FLAG_EXECUTE_AT_COMMIT) != 0;
  const uint32_t dmax = a.dmax;
  const uint32_t steps4 = (a.steps + 3) >> 2;
  const size_t soff = (size_t)(s >> 6) * steps4 * 256 + ((s & 63u) << 2);
  // lane 4p+b fetches plane p (0 dot, 1 hdr, 2+j dep j) of block b of a chunk
  const uint32_t pl = lane >> 2, bq = lane & 3u;
  const uint32_t* src = pl == 0 ? a.dot
                      : pl == 1 ? a.hdr
                      : (dmax ? a.deps + (size_t)min(pl - 2u, dmax - 1u) * a.plane : a.dot);
  src += soff;
  const uint32_t b_last = steps4 ? steps4 - 1 : 0;
  uint32_t* in = e.lds + L_IN;
  const uint32_t c_begin = a.step_begin / CH;
  const uint32_t c_end = (min(a.step_end, len) + CH - 1) / CH;

  uint4 nxt = make_uint4(0, 0, 0, 0);
  if (c_begin < c_end)
    nxt = *reinterpret_cast<const uint4*>(src + (size_t)min(c_begin * 4 + bq, b_last) * 256);
  for (uint32_t c = c_begin; c < c_end && !e.err; ++c) {
    *reinterpret_cast<uint4*>(in + pl * CH + bq * 4) = nxt;
    nxt = *reinterpret_cast<const uint4*>(src + (size_t)min((c + 1) * 4 + bq, b_last) * 256);
    __builtin_amdgcn_wave_barrier();
    const uint32_t base = c * CH;
    const uint32_t q0 = base < a.step_begin ? a.step_begin - base : 0u;
    const uint32_t q1 = min(min(a.step_end, len) - base, CH);
    for (uint32_t q = q0; q < q1; ++q) {
      const uint32_t d = uni(in[q]);
      const uint32_t h = uni(in[CH + q]);
      const uint32_t depj = in[(2 + (lane < MAXD ? lane : 0u)) * CH + q];
      e.step_start(base + q, d, h, depj, dmax, at_commit);
      if (e.phase != PH_IDLE) e.run_slow();
      if (e.err) break;
    }
    __builtin_amdgcn_wave_barrier();
  }

  // vertices still pending have no release step (yet)
  if (e.mine(e.occ)) a.release[e.at(e.srec & 0x03FFFFFFu)] = FX_RELEASE_NONE;
  if (lane == 0) {
    a.nexec[s] = e.k;
    a.err[s] = e.err;
  }
  if (a.flags & FX_FLAG_SAVE_STATE) {
    uint32_t* r = gst + lane * RREGS;
    r[0] = e.sdot;
    r[1] = e.srec;
    r[2] = e.swait;
    r[3] = e.stl;
    r[4] = e.sfr;
    r[5] = e.cf;
    r[6] = e.cw;
    for (uint32_t q = lane; q < L_IN; q += 64) gst[S_LDS + q] = e.lds[q];
    if (lane == 0) {
      gst[S_SCAL + 0] = (uint32_t)e.occ;
      gst[S_SCAL + 1] = (uint32_t)(e.occ >> 32);
      gst[S_SCAL + 2] = (uint32_t)e.wmask;
      gst[S_SCAL + 3] = (uint32_t)(e.wmask >> 32);
      gst[S_SCAL + 4] = e.k;
      gst[S_SCAL + 5] = e.err;
      gst[S_SCAL + 6] = e.epoch;
    }
  }
}

// ---------------------------------------------------------------------------
// The persistent single-executor kernel of the drop-in handle (executor_host.cpp,
// "persistent mode").  The reference's simulator calls the executor once per
// Add and drains it right after (fantoch/src/sim/runner.rs:406-424); a launch
// plus a synchronisation per Add costs tens of microseconds, so instead ONE
// wavefront stays resident and runs the wave tier's executor (the Wave above)
// over Adds the host publishes in host-mapped memory:
//   ctl[PUB]     rows published by the host (written after the rows)
//   ctl[EXIT]    host asks the kernel to stop
//   ctl[MB..]    mailbox: tag (= row index + 1), dot, hdr, 12 deps, checksum of the row of
//                a one-Add flush, read in the same round trip as the doorbell
//   ctl[DONE..]  rows processed, executed count, status: tagged 64-bit words
//   ctl[PAIRS..] the flush's pairs when there are at most PERSIST_INLINE of
//                them (tagged 64-bit words: no fence), else the out ring and
//                one release fence before the status
//   ctl[RUN]     1 while the kernel is resident
// (fx_internal.h has the layout.)
// rows: a ring of PR rows of PRW words (dot, hdr, up to 14 deps), row i in slot
// i mod PR; out: a ring of PO (order word, release step) pairs, pair k in slot
// k mod PO.  The kernel polls; with nothing published for 20 ms (or on an
// error, or when asked) it saves the executor state in the wave tier's state
// layout and exits, and the host relaunches it on the next flush, so no
// kernel outlives an idle or vanished host (a device-wide synchronisation
// waits for it at most that long).
namespace persist {
enum : uint32_t { P_PUB = PERSIST_PUB, P_EXIT = PERSIST_EXIT, P_MB = PERSIST_MB, P_DONE = PERSIST_DONE,
                  P_DONE2 = PERSIST_DONE2, P_TCOMP = PERSIST_TCOMP, P_RUN = PERSIST_RUN, P_PAIRS = PERSIST_PAIRS };
constexpr uint32_t PRW = 16;                     // words per published row
constexpr uint32_t MBD = PERSIST_MB_DEPS;        // deps a mailbox row carries (tag, dot, hdr, deps, checksum)
constexpr uint64_t IDLE_TICKS = 2000000ull;      // s_memrealtime runs at 100 MHz: 20 ms
// Poller waves: a poll of host memory takes a round trip (~1.25 us), so one
// wave that polls and then waits samples the doorbell once per round trip.
// NPOLL waves of the workgroup poll instead, each in its own time slot of
// SLOT_TICKS (100 MHz ticks; NPOLL slots > one round trip, so no poller misses
// its slot), and hand what they read to the executor wave through LDS: the
// doorbell is sampled every SLOT_TICKS (0.2 us) and the executor waits on LDS.
// Cost: 8 reads of two 64-byte lines per 1.6 us, ~0.6 GB/s of PCIe reads
// while the kernel is resident (it exits after 20 ms without work).
constexpr uint32_t NPOLL = 8;
constexpr uint64_t SLOT_TICKS = 20;

// The pairs of one flush are staged in LDS (the wave tier's unused input-chunk
// words) and copied to the host ring by one lane-parallel store before the
// fence; a flush with more than STAGE pairs writes the rest straight through.
constexpr uint32_t STAGE = NPL * CH / 2;
struct RingOut {
  uint32_t* ring = nullptr;  // host-mapped pairs
  uint32_t mask = 0;         // PO - 1
  uint32_t* stage = nullptr;
  uint32_t k0 = 0;           // the flush's first pair
  __device__ __forceinline__ void put(uint32_t k, uint32_t word, uint32_t rec, uint32_t cur) const {
    const uint32_t j = k - k0;
    if (j < STAGE) {  // separate stores keep the LDS one an LDS store
      stage[2u * j] = word;
      stage[2u * j + 1u] = cur;
    } else {
      ring[2u * (k & mask)] = word;
      ring[2u * (k & mask) + 1u] = cur;
    }
  }
};

// one lane-parallel load with system coherence (the host's latest writes)
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// a tagged 64-bit word {tag, v}: one single-copy-atomic system-scope store
__device__ __forceinline__ void st_tag(uint32_t* p, uint32_t tag, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), (uint64_t)tag | ((uint64_t)v << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

// Poller wave i: in each of its slots, one load of the doorbell and mailbox
// lines; a new doorbell value goes to LDS slot i and then into `latest`
// (doorbell << 3 | i, an LDS max), an exit request into `stop`.  Leaves when the
// executor sets `stop`.
__device__ void poller(uint32_t i, uint32_t lane, const uint32_t* ctl, uint32_t* slot, uint32_t* stamp,
                       uint32_t* latest, uint32_t* stop) {
  uint32_t last = 0xFFFFFFFFu;
  auto slot_of = [](uint64_t t) { return (uint32_t)((t / SLOT_TICKS) % NPOLL); };
  while (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
    uint64_t t = __builtin_amdgcn_s_memrealtime();
    while (slot_of(t) != i) {
      __builtin_amdgcn_s_sleep(1);
      t = __builtin_amdgcn_s_memrealtime();
    }
    const uint32_t v = lane < 32u ? ld_sys(ctl + lane) : 0u;
    const uint32_t pub = rl(v, P_PUB);
    if (rl(v, P_EXIT)) {
      __hip_atomic_store(stop, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
    if (pub != last) {
      if (lane < 32u) slot[lane] = v;
      if (lane == 0) {
        *stamp = (uint32_t)t;
        __hip_atomic_fetch_max(latest, (pub << 3) | i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      last = pub;
    }
    do {  // one poll per slot
      __builtin_amdgcn_s_sleep(1);
      t = __builtin_amdgcn_s_memrealtime();
    } while (slot_of(t) == i);
  }
}

__global__ __launch_bounds__(64 * (1 + NPOLL)) void k_handle_persist(PersistArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[LW];
  __shared__ uint32_t ps_slot[NPOLL * 32], ps_stamp[NPOLL], ps_latest, ps_stop;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = uni(threadIdx.x >> 6);
  uint32_t* ctl = a.ctl;
  uint32_t done = a.done0;
  if (threadIdx.x == 0) {
    ps_latest = done << 3;
    ps_stop = 0;
  }
  __syncthreads();
  if (wv != 0) {
    poller(wv - 1u, lane, ctl, ps_slot + (wv - 1u) * 32u, ps_stamp + (wv - 1u), &ps_latest, &ps_stop);
    return;
  }
  Wave<RingOut> e;
  e.lid = lane;
  e.lbit = 1ull << lane;
  e.stream = 0;
  e.n = a.n;
  e.steps = 0xFFFFFFFFu;
  e.kcap = 0xFFFFFFFFu;
  e.lds = smem;
  e.out.ring = a.out;
  e.out.mask = a.out_slots - 1u;
  e.out.stage = smem + L_IN;
  uint32_t* gst = a.state;
  if (a.init) {
    for (uint32_t q = lane; q < L_IN; q += 64) e.lds[q] = 0;
  } else {  // the layout k_graph_wave saves
    const uint32_t* r = gst + lane * RREGS;
    e.sdot = r[0];
    e.srec = r[1];
    e.swait = r[2];
    e.stl = r[3];
    e.sfr = r[4];
    e.cf = r[5];
    e.cw = r[6];
    for (uint32_t q = lane; q < L_IN; q += 64) e.lds[q] = gst[S_LDS + q];
    e.occ = (uint64_t)uni(gst[S_SCAL + 0]) | ((uint64_t)uni(gst[S_SCAL + 1]) << 32);
    e.wmask = (uint64_t)uni(gst[S_SCAL + 2]) | ((uint64_t)uni(gst[S_SCAL + 3]) << 32);
    e.k = uni(gst[S_SCAL + 4]);
    e.err = uni(gst[S_SCAL + 5]);
    e.epoch = uni(gst[S_SCAL + 6]);
  }
  uint64_t idle0 = __builtin_amdgcn_s_memrealtime();
  // timing words for tools/handle_latency (100 MHz ticks): the age of the
  // sample that carried the last doorbell, the LDS checks before it, the last
  // flush's compute and its publish
  uint32_t t_rtt = 0, t_polls = 0, t_fence = 0, t_iter = 0, t_step = 0;
  uint32_t nflush = 0, t_mb = 0;
  while (!e.err) {
    const uint32_t lv = __hip_atomic_load(&ps_latest, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t pub = uni(lv) >> 3;
    const uint64_t tp1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t cy1 = __builtin_amdgcn_s_memtime();
    ++t_polls;
    if (pub == done) {
      const uint64_t idle = tp1 - idle0;
      if (idle >= a.debug_hold_ticks) {  // (the test hook holds the kernel resident a bounded time)
        if (__hip_atomic_load(&ps_stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        if (idle > IDLE_TICKS) break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint32_t si = uni(lv) & 7u;
    const uint32_t v = lane < 32u ? ps_slot[si * 32u + lane] : 0u;
    t_rtt = (uint32_t)tp1 - ps_stamp[si];
    e.out.k0 = e.k;
    // the mailbox line's checksum (fx_internal.h persist_mb_mix): lanes
    // P_MB .. P_MB + 14 mix their word, an XOR over the 16 lanes of the line
    // compares with word P_MB + 15 (a line mixed from two flushes fails)
    uint32_t mbx = 0;
    if (pub == done + 1u && rl(v, P_MB) == pub) {
      const uint32_t k = lane - P_MB;
      mbx = k < 15u ? persist_mb_mix(v, k) : k == 15u ? v : 0u;
      mbx ^= __shfl_xor(mbx, 1);
      mbx ^= __shfl_xor(mbx, 2);
      mbx ^= __shfl_xor(mbx, 4);
      mbx ^= __shfl_xor(mbx, 8);
    }
    if (pub == done + 1u && rl(v, P_MB) == pub && rl(mbx, P_MB) == 0u) {
      // a one-Add flush: its row came with the doorbell (the host writes the
      // mailbox line before the doorbell; a load that saw the new doorbell but
      // an older mailbox tag, or a torn line, falls back to the ring)
      const uint32_t d = rl(v, P_MB + 1u), h = rl(v, P_MB + 2u);
      t_mb = 1;
      const uint32_t depj = gather(v, (P_MB + 3u + lane) & 63u);
      e.step_start(done, d, h, lane < MBD ? depj : 0u, MBD, a.at_commit != 0);
      t_step = (uint32_t)(__builtin_amdgcn_s_memtime() - cy1);
      while (e.phase != PH_IDLE) {  // run_slow, counted
        e.canon();
        if (e.phase == PH_DFS) e.dfs_iter();
        else if (e.phase == PH_TRY) e.try_iter();
        else e.check_iter();
        if (e.err) e.phase = PH_IDLE;
        ++t_iter;
      }
    } else {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the rows after the doorbell
      // rows [done, pub) from the ring, four per load: lane 16 r + w reads word w of row i + r
      for (uint32_t i = done; i < pub && !e.err; i += 4) {
        const uint32_t r4 = lane >> 4, w = lane & 15u;
        const uint32_t row = i + r4;
        const uint32_t rv = row < pub ? a.rows[(size_t)(row & (a.row_slots - 1u)) * PRW + w] : 0u;
        for (uint32_t r = 0; r < 4 && i + r < pub && !e.err; ++r) {
          const uint32_t d = rl(rv, 16u * r), h = rl(rv, 16u * r + 1u);
          const uint32_t depj = gather(rv, (16u * r + 2u + lane) & 63u);
          e.step_start(i + r, d, h, lane < MAXD ? depj : 0u, MAXD, a.at_commit != 0);
          if (e.phase != PH_IDLE) e.run_slow();
        }
      }
    }
    // the flush's pairs: at most PERSIST_INLINE go into the control words as
    // tagged words (lane 2j: {pub, order word j}, lane 2j + 1: {pub, release
    // step j}) and need no fence; more go to the out ring (lane j: pair j of
    // the staged ones) and one release fence orders them before the status
    const uint32_t np = e.k - e.out.k0;
    const uint64_t tc = __builtin_amdgcn_s_memrealtime();
    const uint32_t cyc = (uint32_t)(__builtin_amdgcn_s_memtime() - cy1);
    if (np > PERSIST_INLINE) {
      const uint32_t ns = min(np, STAGE);
      for (uint32_t j = lane; j < ns; j += 64) {
        const uint2 pr = *reinterpret_cast<const uint2*>(e.out.stage + 2u * j);
        *reinterpret_cast<uint2*>(a.out + 2u * ((e.out.k0 + j) & e.out.mask)) = pr;
      }
      __threadfence_system();
    }
    {  // one store: lane 0 the status, lane 1 the error word, lanes 2.. the inline pairs
      const uint32_t m = lane - 2u;
      const bool pair = lane >= 2u && np <= PERSIST_INLINE && m < 2u * np;
      const uint32_t val = lane == 0 ? (e.k | (e.err ? PERSIST_ERR_BIT : 0u)) : lane == 1 ? e.err
                         : pair ? e.out.stage[m] : 0u;
      uint32_t* dst = lane == 0 ? ctl + P_DONE : lane == 1 ? ctl + P_DONE2 : ctl + P_PAIRS + 2u * m;
      ++nflush;
      const bool skip = a.debug_skip_status != 0u && nflush == a.debug_skip_status;  // test hook
      if ((lane < 2u && !skip) || pair) st_tag(dst, pub, val);
    }
    if (lane >= 2u && lane < 10u)  // timing words (diagnostics) and the mailbox flag
      st_sys(ctl + P_TCOMP + lane - 2u, lane == 2 ? (uint32_t)(tc - tp1) : lane == 3 ? t_fence
                                      : lane == 4 ? t_polls : lane == 5 ? t_rtt : lane == 6 ? cyc
                                      : lane == 7 ? t_iter : lane == 8 ? t_step : t_mb);
    t_iter = 0;
    t_step = 0;
    t_mb = 0;
    done = pub;
    idle0 = __builtin_amdgcn_s_memrealtime();
    t_fence = (uint32_t)(idle0 - tc);
    t_polls = 0;
  }
  uint32_t* r = gst + lane * RREGS;
  r[0] = e.sdot;
  r[1] = e.srec;
  r[2] = e.swait;
  r[3] = e.stl;
  r[4] = e.sfr;
  r[5] = e.cf;
  r[6] = e.cw;
  for (uint32_t q = lane; q < L_IN; q += 64) gst[S_LDS + q] = e.lds[q];
  if (lane == 0) {
    gst[S_SCAL + 0] = (uint32_t)e.occ;
    gst[S_SCAL + 1] = (uint32_t)(e.occ >> 32);
    gst[S_SCAL + 2] = (uint32_t)e.wmask;
    gst[S_SCAL + 3] = (uint32_t)(e.wmask >> 32);
    gst[S_SCAL + 4] = e.k;
    gst[S_SCAL + 5] = e.err;
    gst[S_SCAL + 6] = e.epoch;
  }
  __hip_atomic_store(&ps_stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // the pollers leave
  __threadfence_system();
  if (lane == 0) st_sys(ctl + P_RUN, 0u);
}
}  // namespace persist

}  // namespace wav

int persist_launch(const PersistArgs& a, hipStream_t stream) {
  if ((a.row_slots & (a.row_slots - 1u)) || (a.out_slots & (a.out_slots - 1u)) || !a.ctl || !a.rows || !a.out ||
      !a.state)
    return FX_ERR_INVALID_ARG;
  hipLaunchKernelGGL(wav::persist::k_handle_persist, dim3(1), dim3(64 * (1 + wav::persist::NPOLL)), 0, stream, a);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

int launch_wave(const KArgs& a, hipStream_t stream) {
  if (a.num_lanes == 0) return FX_OK;
  if (a.dmax > wav::MAXD) return FX_ERR_INVALID_ARG;
  const uint32_t lb = (a.num_lanes + wav::WPB - 1) / wav::WPB;  // logical workgroups
  const uint32_t blocks = (lb + 15u) & ~15u;                     // whole XCD pairs
  hipLaunchKernelGGL(wav::k_graph_wave, dim3(blocks), dim3(64 * wav::WPB), 0, stream, a);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

uint32_t wave_state_words_per_stream() { return wav::WPS; }

size_t wave_state_bytes(uint32_t streams) {
  const uint32_t lb = (streams + wav::WPB - 1) / wav::WPB;
  return (size_t)(((lb + 15u) & ~15u) * wav::WPB) * wav::WPS * 4;
}

uint32_t wave_decode_pending(const uint32_t* st, uint32_t stream_in_launch, uint32_t* dots,
                             uint32_t* waits, uint32_t cap) {
  const uint32_t* b = st + (size_t)stream_in_launch * wav::WPS;
  const uint64_t occ = (uint64_t)b[wav::S_SCAL + 0] | ((uint64_t)b[wav::S_SCAL + 1] << 32);
  const uint64_t wm = (uint64_t)b[wav::S_SCAL + 2] | ((uint64_t)b[wav::S_SCAL + 3] << 32);
  uint32_t c = 0;
  for (uint32_t sl = 0; sl < wav::P; ++sl) {
    if (!((occ >> sl) & 1u)) continue;
    if (c < cap) {
      dots[c] = b[sl * wav::RREGS + 0];
      waits[c] = ((wm >> sl) & 1u) ? b[sl * wav::RREGS + 2] : 0u;
    }
    ++c;
  }
  return c;
}

}  // namespace fx
