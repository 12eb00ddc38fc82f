// graph_group.hip — tier 0 of the batched GraphExecutor: 16 lanes per stream.
//
// Same algorithm as graph_exec.hip (DependencyGraph::handle_add,
// fantoch_ps/src/executor/graph/mod.rs:213-642, with the canonical orders C1
// and C2), laid out for SIMT: a 64-lane wavefront runs 4 streams, and the 16
// lanes of a stream's group share the work of that one executor:
//   * lane l owns pending-vertex slot l (VertexIndex, index.rs:18-51): its dot,
//     arrival index, registered-on dot (PendingIndex, index.rs:145-208) and
//     Tarjan id/low/visited-epoch word sit in lane l's VGPRs, so a lookup by
//     dot is one compare + ballot and a slot field read is one __shfl;
//   * lane l < n owns the executed clock of source l + 1 (AEClock, threshold
//     0.9.1: a frontier + a 32-bit exception window);
//   * the deps of an incoming Add are checked in parallel (lane j: dep j);
//   * the Tarjan DFS (tarjan.rs:96-316), check_pending and try_pending run in
//     group-uniform control flow, one micro-op per iteration (DFS edge, frame
//     pop, waiter pick, worklist pop), so the wavefront only diverges between
//     its 4 streams — never inside one executor;
//   * the deps of each pending vertex (those not yet executed when it was
//     indexed) and the check_pending worklist live in LDS.
// A stream that outgrows 16 pending vertices, 8 cached deps per vertex or the
// 32-bit clock window stops with FX_ERR_CAPACITY and is rerun at tier 1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace grp {

constexpr uint32_t G = GROUP_LANES;   // lanes per stream
constexpr uint32_t SPW = 64 / G;      // streams per wavefront
constexpr uint32_t P = GROUP_SLOTS;   // pending slots (one per lane)
constexpr uint32_t C = GROUP_CACHE;   // cached deps per slot
constexpr uint32_t WLC = P + 1;       // check_pending worklist capacity
constexpr uint32_t L_CACHE = 0;       // LDS words per stream: [P][C] cached deps
constexpr uint32_t L_WL = P * C;      //                        [WLC] worklist
constexpr uint32_t LW = L_WL + WLC;   // 145 words
constexpr uint32_t RREGS = 6;         // saved per-lane registers
constexpr uint32_t S_LDS = G * RREGS; // saved state per stream: regs | LDS words | scalars
constexpr uint32_t S_SCAL = S_LDS + LW;
constexpr uint32_t WPS = S_SCAL + 4;  // 245 words per stream

enum : uint32_t { PH_IDLE = 0, PH_DFS = 1, PH_TRY = 2, PH_CHECK = 3 };

// Tarjan word: id (5 bits) | low (5 bits) | visited epoch (8 bits)
__device__ __forceinline__ uint32_t tid(uint32_t t) { return t & 31u; }
__device__ __forceinline__ uint32_t tlow(uint32_t t) { return (t >> 5) & 31u; }
__device__ __forceinline__ uint32_t tep(uint32_t t) { return t >> 10; }
__device__ __forceinline__ uint32_t tmk(uint32_t id, uint32_t low, uint32_t ep) {
  return id | (low << 5) | (ep << 10);
}
// component q of v; arithmetic masks (a select chain is folded into a
// dynamically indexed load, which sends the vector to scratch)
__device__ __forceinline__ uint32_t pick4(const uint4& v, uint32_t q) {
  return (v.x & (0u - (uint32_t)(q == 0))) | (v.y & (0u - (uint32_t)(q == 1))) |
         (v.z & (0u - (uint32_t)(q == 2))) | (v.w & (0u - (uint32_t)(q == 3)));
}

struct Group {
  // lane identity
  uint32_t lid, gbase;
  // lane-owned slot fields (slot = lid) and clock (source = lid + 1)
  uint32_t sdot = 0, srec = 0, swait = 0, stl = 0;
  uint32_t sts = 0, sfr = 0;  // Tarjan stack entry lid, DFS frame entry lid
  uint32_t cf = 0, cw = 0;
  // group-uniform state
  uint32_t occ = 0, wmask = 0, tmask = 0;
  uint32_t k = 0, err = 0, epoch = 1, nwl = 0, cur = 0;
  uint32_t phase = PH_IDLE, root = 0, idc = 0, nts = 0, nfr = 0, missing = 0;
  uint32_t fv = 0, fdi = 0, fnc = 0, in_try = 0, emitted = 0;
  // stream context
  uint32_t stream = 0, n = 0, steps = 0;
  uint32_t* lds = nullptr;  // this stream's LDS words
  uint32_t* order = nullptr;
  uint32_t* release = nullptr;

  __device__ __forceinline__ size_t at(uint32_t step) const { return fx_index(step, stream, steps); }
  // group ballot of pred (bit i = lane gbase + i)
  __device__ __forceinline__ uint32_t gb(bool pred) const {
    return (uint32_t)(__ballot(pred) >> gbase) & 0xFFFFu;
  }
  // value of v in group lane src
  __device__ __forceinline__ uint32_t bc(uint32_t v, uint32_t src) const {
    return (uint32_t)__shfl((int)v, (int)(gbase + (src & (G - 1))), 64);
  }
  __device__ __forceinline__ uint32_t g_or(uint32_t v) const {
#pragma unroll
    for (uint32_t o = 1; o < G; o <<= 1) v |= (uint32_t)__shfl_xor((int)v, (int)o, (int)G);
    return v;
  }
  __device__ __forceinline__ uint32_t g_min(uint32_t v) const {
#pragma unroll
    for (uint32_t o = 1; o < G; o <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, (int)o, (int)G));
    return v;
  }

  // ------------------------------------------------------------ clock
  // AEClock::contains for a per-lane dot (tarjan.rs:131-132)
  __device__ __forceinline__ bool contains(uint32_t d) const {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    const uint32_t f = bc(cf, si), w = bc(cw, si);
    const uint32_t seq = d & FX_SEQ_MASK, off = seq - f - 1u;
    return si < n && (seq <= f || (off < 32u && ((w >> (off & 31u)) & 1u)));
  }
  // AEClock::add for a group-uniform dot (tarjan.rs:293)
  __device__ __forceinline__ void clk_add(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) { err = FX_ERR_DOT_RANGE; return; }
    uint32_t f = bc(cf, si), w = bc(cw, si);
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
    const uint32_t m = gb(((occ >> lid) & 1u) && sdot == d);
    return m ? (int)__builtin_ctz(m) : -1;
  }
  __device__ __forceinline__ uint32_t& cache(uint32_t sl, uint32_t j) { return lds[L_CACHE + sl * C + j]; }
  __device__ __forceinline__ uint32_t& wl(uint32_t i) { return lds[L_WL + i]; }

  __device__ __forceinline__ void new_epoch() {
    epoch = (epoch + 1) & 0xFFu;
    if (epoch == 0) {
      if ((occ >> lid) & 1u) stl = tmk(tid(stl), tlow(stl), 0);
      epoch = 1;
    }
  }

  // VertexIndex::index(Vertex::new(dot, cmd, deps, time)) (index.rs:33-37);
  // depj = dep `lid` of the Add (valid for lid < nd).  Only deps not yet
  // executed are kept (executed deps are ignored by every later search,
  // tarjan.rs:128-145, and the executed clock only grows), in ascending order.
  __device__ __forceinline__ int insert_vertex(uint32_t i, uint32_t d, uint32_t nd, uint32_t depj) {
    const uint32_t fre = ~occ & 0xFFFFu;
    if (!fre) { err = FX_ERR_CAPACITY; return -1; }
    const uint32_t sl = __builtin_ctz(fre);
    const bool exd = contains(depj);  // every lane active (see step_start)
    const bool keep = lid < nd && depj != d && !exd;
    const uint32_t km = gb(keep);
    const uint32_t nc = __builtin_popcount(km);
    if (nc > C) { err = FX_ERR_CAPACITY; return -1; }
    if (keep) cache(sl, __builtin_popcount(km & ((1u << lid) - 1u))) = depj;
    if (lid == sl) {
      sdot = d;
      srec = i | (nc << 26);
      swait = 0;
      stl = 0;
    }
    occ |= 1u << sl;
    return (int)sl;
  }

  // save_scc (mod.rs:488-523) for one member: to_execute + executed clock
  __device__ __forceinline__ void emit_one(uint32_t rec, uint32_t d) {
    if (k >= steps) { err = FX_ERR_ORDER_OVERFLOW; return; }
    if (lid == 0) {
      order[at(k)] = rec | FX_ORDER_SCC_START;
      release[at(rec)] = cur;
    }
    ++k;
    clk_add(d);
  }

  __device__ __forceinline__ void dfs_start(uint32_t r, bool intry) {
    root = r;
    in_try = intry;
    emitted = 0;
    missing = 0;
    idc = 1;
    const uint32_t tr = bc(stl, r);
    if (lid == r) stl = tmk(1, 1, tep(tr));
    if (lid == 0) sts = r;
    nts = 1;
    nfr = 0;
    fv = r;
    fdi = 0;
    fnc = bc(srec, r) >> 26;
    phase = PH_DFS;
  }

  // SCC rooted at fv = Tarjan stack entries [pos, nts): saved in ascending
  // dot order (SCC = BTreeSet<Dot>, tarjan.rs:15), executed clock updated.
  __device__ __forceinline__ void save_scc() {
    const uint32_t pos = __builtin_ctz(gb(lid < nts && sts == fv));
    const bool mem = lid >= pos && lid < nts;
    const uint32_t mdot = bc(sdot, sts), mrec = bc(srec, sts) & 0x03FFFFFFu;
    const uint32_t cnt = nts - pos;
    uint32_t rank = 0;
    for (uint32_t b = pos; b < nts; ++b) rank += bc(mdot, b) < mdot ? 1u : 0u;
    if (k + cnt > steps) { err = FX_ERR_ORDER_OVERFLOW; return; }
    if (nwl + cnt > WLC) { err = FX_ERR_CAPACITY; return; }
    if (mem) {
      order[at(k + rank)] = mrec | (rank == 0 ? FX_ORDER_SCC_START : 0u);
      release[at(mrec)] = cur;
      wl(nwl + rank) = mdot;
    }
    k += cnt;
    nwl += cnt;
    for (uint32_t r = 0; r < cnt; ++r) {  // clock in ascending dot order
      const uint32_t lr = __builtin_ctz(gb(mem && rank == r));
      clk_add(bc(mdot, lr));
    }
    const uint32_t fm = g_or(mem ? 1u << sts : 0u);
    occ &= ~fm;
    wmask &= ~fm;
    tmask &= ~fm;
    nts = pos;
    emitted = 1;
  }

  __device__ __forceinline__ void dfs_finish() {
    // finalize (tarjan.rs:60-93): reset ids of the vertices left on the stack;
    // in try_pending a failed search that saved no SCC marks them visited
    const bool mark = in_try && missing != 0 && !emitted;
    const uint32_t tsm = g_or(lid < nts ? 1u << sts : 0u);
    if ((tsm >> lid) & 1u) stl = tmk(0, 0, mark ? epoch : tep(stl));
    nts = 0;
    if (missing) {  // index_pending(dot, missing) (mod.rs:525-554)
      if (lid == root) swait = missing;
      wmask |= 1u << root;
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
      const uint32_t dep = cache(fv, fdi);
      ++fdi;
      if (contains(dep)) return;  // executed (tarjan.rs:128-145)
      const int x = find(dep);
      if (x < 0) {  // missing: give up (tarjan.rs:148-157, shard_count == 1)
        missing = dep;
        dfs_finish();
        return;
      }
      const uint32_t tx = bc(stl, (uint32_t)x);
      if (tid(tx) == 0) {  // not visited: recurse (tarjan.rs:172-214)
        ++idc;
        if (lid == (uint32_t)x) stl = tmk(idc, idc, tep(tx));
        if (lid == nts) sts = (uint32_t)x;
        ++nts;
        if (lid == nfr) sfr = fv | (fdi << 8);
        ++nfr;
        fv = (uint32_t)x;
        fdi = 0;
        fnc = bc(srec, fv) >> 26;
      } else {  // visited and on the stack (tarjan.rs:215-225)
        const uint32_t tv = bc(stl, fv);
        if (tid(tx) < tlow(tv) && lid == fv) stl = tmk(tid(tv), tid(tx), tep(tv));
      }
    } else {
      const uint32_t tv = bc(stl, fv);
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
      const uint32_t f = bc(sfr, nfr);  // back in the parent (tarjan.rs:211)
      fv = f & 0xFFu;
      fdi = f >> 8;
      fnc = bc(srec, fv) >> 26;
      const uint32_t tp = bc(stl, fv);
      if (lowv < tlow(tp) && lid == fv) stl = tmk(tid(tp), lowv, tep(tp));
    }
  }

  // try_pending (mod.rs:589-642): next waiter of the snapshot, ascending (C2)
  __device__ __forceinline__ void try_iter() {
    if (!tmask) { phase = PH_CHECK; return; }
    const bool in = (tmask >> lid) & 1u;
    const uint32_t best_dot = g_min(in ? sdot : 0xFFFFFFFFu);
    const uint32_t best = __builtin_ctz(gb(in && sdot == best_dot));
    tmask &= ~(1u << best);
    if (tep(bc(stl, best)) == epoch) return;  // visited: skipped, not re-registered
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
    const uint32_t x = wl(nwl);
    const uint32_t t = gb(((wmask >> lid) & 1u) && swait == x);
    if (!t) return;
    wmask &= ~t;  // PendingIndex::remove(x)
    tmask = t;
    new_epoch();  // try_pending's fresh `visited`
    phase = PH_TRY;
  }

  __device__ __forceinline__ void slow_iter() {
    if (phase == PH_DFS) dfs_iter();
    if (!err && phase == PH_TRY) try_iter();
    if (!err && phase == PH_CHECK) check_iter();
    if (err) phase = PH_IDLE;
  }

  // GraphExecutor::handle(Add) (executor.rs:69-80) -> handle_add (mod.rs:213-275)
  __device__ __forceinline__ void step_start(uint32_t i, uint32_t d, uint32_t h, uint32_t depj,
                                             uint32_t dmax, bool at_commit) {
    cur = i;
    nwl = 0;
    const uint32_t nd = (h >> 24) & 31u, kind = h >> 29;
    if (nd > dmax || nd > G) { err = FX_ERR_INVALID_ARG; return; }
    if ((d >> FX_SEQ_BITS) - 1u >= n || (d & FX_SEQ_MASK) == 0) { err = FX_ERR_DOT_RANGE; return; }
    if (at_commit) {  // execute_at_commit bypass (executor.rs:72-73)
      if (lid == 0) {
        order[at(k)] = i | FX_ORDER_SCC_START;
        release[at(i)] = i;
      }
      ++k;
      return;
    }
    if (occ && find(d) >= 0) { err = FX_ERR_DOUBLE_INDEX; return; }  // mod.rs:233-237
    const bool valid = lid < nd;
    const uint32_t prev = (uint32_t)__shfl((int)depj, (int)(gbase + ((lid - 1) & (G - 1))), 64);
    if (gb(valid && lid > 0 && depj <= prev)) { err = FX_ERR_DEPS_UNSORTED; return; }
    if (kind == FX_KIND_INDEX_ONLY) {
      insert_vertex(i, d, nd, depj);
      return;
    }
    // fast path: every dep is self or executed -> a singleton SCC.  The clock
    // shuffle runs with every lane active: a __shfl (ds_bpermute) from an
    // inactive lane reads 0, and the clock of source s sits in lane s, often
    // outside [0, nd) (inside `&&` it would run in the masked branch)
    const bool exd = contains(depj);
    if (!gb(valid && depj != d && !exd)) {
      emit_one(i, d);
      if (wmask && !err) {  // check_pending([dot])
        if (lid == 0) wl(0) = d;
        nwl = 1;
        phase = PH_CHECK;
      }
      return;
    }
    const int sl = insert_vertex(i, d, nd, depj);
    if (sl >= 0) dfs_start((uint32_t)sl, false);
  }
};

__global__ __launch_bounds__(64) void k_graph_group(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[SPW * LW];
  const uint32_t lane = threadIdx.x;
  const uint32_t g = lane / G;
  const uint32_t gg = blockIdx.x * SPW + g;  // stream index within the launch
  const uint32_t nl = a.lanes_dev ? min(a.num_lanes, *a.lanes_dev) : a.num_lanes;
  if (blockIdx.x * SPW >= nl) return;  // wavefront past a device-side lane count
  // map entries >= S are padding lanes (FX_TIER_SPLIT's ragged last tile)
  const uint32_t s0 = gg < nl ? (a.stream_map ? a.stream_map[gg] : gg) : 0xFFFFFFFFu;
  const bool active = s0 < a.S;
  const uint32_t s = active ? s0 : 0u;
  const uint32_t len = active ? (a.lengths ? min(a.lengths[s], a.steps) : a.steps) : 0u;
  uint32_t* gst = a.state ? a.state + (size_t)gg * WPS : nullptr;

  Group e;
  e.lid = lane & (G - 1);
  e.gbase = lane & ~(G - 1);
  e.stream = s;
  e.n = a.n;
  e.steps = a.steps;
  e.lds = smem + g * LW;
  e.order = a.order;
  e.release = a.release;

  if (a.flags & FX_FLAG_INIT) {
    if (a.init_frontier && active && e.lid < 8) e.cf = a.init_frontier[(size_t)s * 8 + e.lid];
  } else if (active) {
    const uint32_t* r = gst + e.lid * RREGS;
    e.sdot = r[0];
    e.srec = r[1];
    e.swait = r[2];
    e.stl = r[3];
    e.cf = r[4];
    e.cw = r[5];
    for (uint32_t q = e.lid; q < LW; q += G) e.lds[q] = gst[S_LDS + q];
    e.occ = gst[S_SCAL + 0];
    e.wmask = gst[S_SCAL + 1];
    e.k = gst[S_SCAL + 2];
    e.err = gst[S_SCAL + 3] & 0xFFFFu;
    e.epoch = gst[S_SCAL + 3] >> 16;
  }
  if (!active) e.err = FX_ERR_INVALID_ARG;  // idle group (its loads read stream 0)

  const bool at_commit = (a.flags & FX_FLAG_EXECUTE_AT_COMMIT) != 0;
  const uint32_t steps4 = (a.steps + 3) >> 2;
  const size_t soff = (size_t)(s >> 6) * steps4 * 256 + ((s & 63u) << 2);
  const uint32_t b_begin = a.step_begin >> 2;
  const uint32_t b_end = (a.step_end + 3) >> 2;
  const uint32_t b_last = b_end ? b_end - 1 : 0;
  const uint32_t dmax = a.dmax;
  // lane j streams dep plane j of its stream (clamped: a static load count)
  const uint32_t* dotp = a.dot + soff;
  const uint32_t* hdrp = a.hdr + soff;
  const uint32_t* depp = (dmax ? a.deps + (size_t)min(e.lid, dmax - 1) * a.plane : a.dot) + soff;

  uint4 cd = make_uint4(0, 0, 0, 0), ch = cd, cp = cd, nd_ = cd, nh = cd, np = cd;
  if (b_begin < b_end) {
    cd = *reinterpret_cast<const uint4*>(dotp + (size_t)b_begin * 256);
    ch = *reinterpret_cast<const uint4*>(hdrp + (size_t)b_begin * 256);
    cp = *reinterpret_cast<const uint4*>(depp + (size_t)b_begin * 256);
  }
  for (uint32_t b = b_begin; b < b_end; ++b) {
    const size_t off = (size_t)min(b + 1, b_last) * 256;
    nd_ = *reinterpret_cast<const uint4*>(dotp + off);
    nh = *reinterpret_cast<const uint4*>(hdrp + off);
    np = *reinterpret_cast<const uint4*>(depp + off);
    const uint32_t base = b * 4;
    const uint32_t q0 = base < a.step_begin ? a.step_begin - base : 0u;
    const uint32_t q1 = a.step_end - base < 4u ? a.step_end - base : 4u;
    // each group advances through the block's steps on its own
    uint32_t q = q0;
    while (true) {
      const bool want = e.phase == PH_IDLE && q < q1 && !e.err && base + q < len;
      if (!__any(want || e.phase != PH_IDLE)) break;
      if (want) {
        e.step_start(base + q, pick4(cd, q), pick4(ch, q), pick4(cp, q), dmax, at_commit);
        ++q;
      }
      if (e.phase != PH_IDLE) e.slow_iter();
    }
    cd = nd_;
    ch = nh;
    cp = np;
  }

  if (!active) return;
  // vertices still pending have no release step (yet)
  if ((e.occ >> e.lid) & 1u) a.release[e.at(e.srec & 0x03FFFFFFu)] = FX_RELEASE_NONE;
  if (e.lid == 0) {
    a.nexec[s] = e.k;
    a.err[s] = e.err;
  }
  if (a.flags & FX_FLAG_SAVE_STATE) {
    uint32_t* r = gst + e.lid * RREGS;
    r[0] = e.sdot;
    r[1] = e.srec;
    r[2] = e.swait;
    r[3] = e.stl;
    r[4] = e.cf;
    r[5] = e.cw;
    for (uint32_t q = e.lid; q < LW; q += G) gst[S_LDS + q] = e.lds[q];
    if (e.lid == 0) {
      gst[S_SCAL + 0] = e.occ;
      gst[S_SCAL + 1] = e.wmask;
      gst[S_SCAL + 2] = e.k;
      gst[S_SCAL + 3] = (e.err & 0xFFFFu) | (e.epoch << 16);
    }
  }
}

}  // namespace grp

int launch_group(const KArgs& a, hipStream_t stream) {
  const uint32_t blocks = (a.num_lanes + grp::SPW - 1) / grp::SPW;
  if (blocks == 0) return FX_OK;
  if (a.dmax > grp::G) return FX_ERR_INVALID_ARG;
  hipLaunchKernelGGL(grp::k_graph_group, dim3(blocks), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? FX_OK : FX_ERR_HIP;
}

uint32_t group_state_words_per_stream() { return grp::WPS; }

size_t group_state_bytes(uint32_t streams) {
  return (size_t)(streams + grp::SPW) * grp::WPS * 4;
}

uint32_t group_decode_pending(const uint32_t* st, uint32_t stream_in_launch, uint32_t* dots,
                              uint32_t* waits, uint32_t cap) {
  const uint32_t* b = st + (size_t)stream_in_launch * grp::WPS;
  const uint32_t occ = b[grp::S_SCAL + 0], wm = b[grp::S_SCAL + 1];
  uint32_t c = 0;
  for (uint32_t sl = 0; sl < grp::P; ++sl) {
    if (!((occ >> sl) & 1u)) continue;
    if (c < cap) {
      dots[c] = b[sl * grp::RREGS + 0];
      waits[c] = ((wm >> sl) & 1u) ? b[sl * grp::RREGS + 2] : 0u;
    }
    ++c;
  }
  return c;
}

}  // namespace fx
