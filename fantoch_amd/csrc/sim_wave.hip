// sim_wave.hip — the batched simulator: ONE wavefront runs ONE simulated
// instance of fantoch's discrete-event simulator (fantoch/src/sim/runner.rs)
// with Atlas or EPaxos processes and their GraphExecutors, all state in LDS and
// VGPRs, thousands of instances per launch.
//
// Event queue.  The reference keeps every pending action in one BinaryHeap
// ordered by time (schedule.rs:6-61; ties FIFO here, canonical C3).  Every
// action travels on a "link" whose delay is a constant (runner.rs:507-530,
// distance = ping / 2, no reordering), so each link delivers in send order
// and the heap is exactly a k-way merge of per-link FIFO queues:
//   P(p,q)  process p -> process q messages (a ring of entries in LDS)
//   S(c)    client c -> its process (SubmitToProc; one in flight: closed loop)
//   R(c)    process -> client c (SendToClient; one in flight)
//   G(p)    process p's periodic GarbageCollection event (runner.rs:179-183)
//   E(p)    process p's periodic executed notification (runner.rs:184-187);
//           GraphExecutor::executed is None (executor/mod.rs:74-79), so E
//           events only matter for where a run with extra time stops, and are
//           simulated only then
// Lane l holds the head (time, insertion seq) of links l, l + 64, ...; the
// next action is a wave-wide min-reduction over those heads.
//
// Handlers follow the reference's recursion exactly: a handler's actions
// (Vec, popped LIFO, runner.rs:403) and execution infos are processed by
// send_to_processes_and_executors (runner.rs:395-441), self-deliveries recurse
// at their position in the target iteration (ascending ids, C4), and ready
// command results are scheduled after the actions.  The recursion is an
// explicit frame stack in LDS.
//
// Per-dot protocol state (SequentialCommandsInfo, info/sequential.rs) lives in
// a per-instance dot table indexed by (source, seq mod W); a slot also holds
// the payloads of every message about that dot (MCollect deps, each
// MCollectAck's deps, the committed value), so a queued message is just
// (time, seq, kind, dot).  A slot is freed once all n processes executed the
// dot: by then no message about it can be in flight (every process needed
// MCollect and MCommit to execute it, and the coordinator needed every
// MCollectAck / MConsensusAck before committing).
//
// Executors: the wavefront-per-stream GraphExecutor of graph_wave.hip
// (DependencyGraph::handle_add, graph/mod.rs:213-642, canonical C1/C2), one
// state per process: lane l owns pending slot l (dot, start time, waited-on
// dot, Tarjan word, DFS frame) and lane l < n the executed clock of source
// l + 1; vertex deps are read from the dot table.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace sim {

constexpr uint32_t NMAX = FX_SIM_MAX_N;  // processes
constexpr uint32_t CMAX = 32;            // clients per instance
constexpr uint32_t KMAX = 2;             // keys per command
constexpr uint32_t VMAX = 16;            // deps of a committed value (per-launch: K (n + 1))
// GC log entries per (process, source), per launch (Geo::rt, Geo::rc): the
// tick log needs one entry per GC interval in which the frontier moved over the
// last max-distance + interval, the change log the moves of the last interval
constexpr uint32_t FMAX = 12;            // frame stack depth
constexpr uint32_t RDMAX = 16;           // ready results per frame (at most one per client: min(16, C))
constexpr uint32_t HC_BINS = 64;         // ChainSize values counted per instance in lanes
constexpr uint32_t HD_BINS = 224;        // ExecutionDelay values counted per instance in LDS (p95 of configs[1]: 198 ms)
constexpr uint32_t HMAX = 2;             // link heads per lane (links <= 128; a template parameter)
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t LNIL = 0xFFFFu;  // end of a link's message list
// per-process tables packed in one VGPR (lane PT_x + p)
constexpr uint32_t PT_SEQ = 0, PT_FAST = 8, PT_SLOW = 16, PT_EXEC = 24, PT_OCC = 32, PT_WAIT = 48;

// FX_SIM_PROFILE builds (make prof): shader-clock cycles per event phase in
// the stats rows (slots 0-15 cycles, 16-23 counts) instead of the counters
#ifdef FX_SIM_PROFILE
#define PROF_T0() const uint64_t prof_t0_ = __builtin_amdgcn_s_memtime()
#define PROF_ADD(cat) prof[cat] += __builtin_amdgcn_s_memtime() - prof_t0_
#else
#define PROF_T0() (void)0
#define PROF_ADD(cat) (void)0
#endif

// message kinds (numbering of the oracle's trace, sim_oracle.cpp MK)
enum : uint32_t { M_COLLECT = 0, M_COLLECT_ACK = 1, M_COMMIT = 2, M_CONSENSUS = 3, M_CONSENSUS_ACK = 4,
                  M_COMMIT_DOT = 5, M_GC = 6, M_STABLE = 7,
                  // Basic (basic.rs:363-385; run-time geometry builds only)
                  M_STORE = 8, M_STORE_ACK = 9, M_COMMIT_BASIC = 10,
                  M_SUBMIT = 15 /* SubmitToProc (handle_submit_to_proc), not a message */ };
enum : uint32_t { ST_START = 0, ST_PAYLOAD = 1, ST_COLLECT = 2, ST_COMMIT = 3 };
enum : uint32_t { PH_IDLE = 0, PH_DFS = 1, PH_TRY = 2, PH_CHECK = 3 };

// dot-table slot (u32 words): fixed header, then (per-launch sizes, Geo)
// collect deps [K] | value [vmax] | ack deps [n][amax]
constexpr uint32_t SL_CLIENT = 0,  // (the slot's dot lives in lane `slot`, sdv)
    SL_IDX = 1, SL_KEYS = 2, SL_PST = 3,  // 3,4: per-process state bytes
    SL_MASKS = 5, SL_CNT = 6, SL_COLLECT = 7;
// per-process state byte: status(2) | buffered commit(1) | accepted(1) | buffered-from(4)
// SL_MASKS: participants(8) | proposer accepts(8) | committed count(8) | executed count(8)
// SL_CNT:   value count(8) | collect count(8) | proposer ballot set(1) << 16 | nkeys << 20


struct Geo {  // launch-uniform geometry
  uint32_t n, C, K, W, R, L, NP, ncli_keys, rt, rc, rdm;
  uint32_t amax, vmax, sl_value, sl_ack, slotw;  // dot-slot layout (MCollectAck deps <= 2K, value <= K(n+1))
  uint32_t off_pool, off_free, off_gct, off_gcc, off_gcr, off_slot, off_kd, off_frame, off_wl, off_hist, words;
};

__host__ __device__ constexpr uint32_t cmin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__host__ __device__ constexpr uint32_t cmax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// the launch geometry of n processes, C clients, K keys per command and a
// conflict pool of `pool` keys; ring / wslots = 0: the defaults.  constexpr:
// the fixed-geometry kernels (GeoCT) fold it into immediates
__host__ __device__ constexpr bool geo_make(uint32_t n, uint32_t C, uint32_t K, uint32_t pool, uint32_t ring,
                                            uint32_t wslots, Geo& g) {
  if (n < 2 || n > NMAX) return false;
  if (C < 1 || C > CMAX) return false;
  g.n = n;
  g.C = C;
  g.K = K;
  // table sizes: small by default (LDS decides how many instances share a CU);
  // fx_sim_run_tiered reruns the instances that outgrow them with 256 dots
  const uint32_t cpr = (C + n - 1) / n;  // clients per process region
  // live dots per instance: 8 per client, at most 64; 32 for n > 5 with one
  // client per region (configs[2]'s n = 7: 12.4 KB instead of 15.4 KB, 13
  // instances per CU instead of 10, the same reruns; 24 reran more, 16 lost 4x)
  g.W = wslots ? wslots : (n > 5 && C <= 8 ? 32u : cmin(64u, 8u * C));
  if (g.W > 256u) return false;
  // messages in flight per instance: 16 per process and client; at least 192
  // for n > 5, where a lagging far replica overflowed the smaller pool often
  // enough (reruns at 4x) that the larger table wins despite fewer instances
  // per CU (configs[2] sweep)
  g.R = ring ? ring : cmin(4096u, cmax(16u * n * cpr, n > 5 ? 192u : 0u));
  if (g.R > 65534u) return false;
  g.NP = n * (n - 1);
  g.L = g.NP + n + 2 * C;
  if (g.L > 64 * HMAX) return false;
  g.ncli_keys = pool + C + 1;
  // an MCollectAck carries the coordinator's deps plus the replica's latest
  // write per key (<= 2K); a committed value is their union over the fast
  // quorum (<= K (n + 1): the coordinator's past plus one latest per member)
  g.amax = 2 * g.K;
  g.vmax = cmin(VMAX, g.K * (n + 1));
  g.sl_value = SL_COLLECT + g.K;
  g.sl_ack = g.sl_value + g.vmax;
  g.slotw = g.sl_ack + n * g.amax;
  if (n * g.amax > 64 || g.slotw > 64) return false;
  uint32_t o = 0;
  // messages in flight: one pool per instance, a FIFO list per process link
  g.off_pool = o; o += g.R * 4;
  g.off_free = o; o += g.R;
  // GC logs: 4 / 2 entries per client per region (commits of one source
  // arrive about once per client round trip), 32 / 16 in the rerun geometry
  g.rt = 4;
  while (g.rt < 4 * cpr && g.rt < 64) g.rt <<= 1;
  if (g.W > 64u) g.rt = cmax(g.rt, 32u);
  g.rc = g.rt / 2;
  g.off_gct = o; o += n * n * g.rt * 2;
  g.off_gcc = o; o += n * n * g.rc * 2;
  // the final GC summaries (gc_finish, after the run) reuse the message pool
  if (g.R >= n * n) {
    g.off_gcr = g.off_pool;
  } else {
    g.off_gcr = o; o += n * n * 4;
  }
  g.off_slot = o; o += g.W * g.slotw;
  g.off_kd = o; o += n * g.ncli_keys;
  g.rdm = cmin(RDMAX, C);  // a client's command completes once per frame at most
  g.off_frame = o; o += FMAX * g.rdm;
  g.off_wl = o; o += 68;  // released dots: nwl + cnt <= 65
  g.off_hist = o; o += HD_BINS;
  g.words = (o + 3) & ~3u;
  return true;
}
__host__ __device__ constexpr Geo geo_fixed(uint32_t n, uint32_t C) {
  Geo g{};
  geo_make(n, C, 1, 1, 0, 0, g);
  return g;
}

// Geometry policy of a kernel build.  GeoRT: the launch's geometry arrives in
// the kernel arguments (any batch the all-on-chip kernel takes).  GeoCT: one
// BASELINE geometry (protocol, n, f, one client per region, one key per
// command, a one-key conflict pool, default tables) compiled in, so table
// offsets, link arithmetic and quorum sizes are immediates and their scalar
// registers and instructions go away (the kernel is bound by scalar issue).
// xp_lanes: the executors' slot tables.  0: one 64-lane table per process
// (xdot / xrec / xwait[NX]), swapped into the working registers for each Add.
// > 0: ONE table whose lanes are split between the processes, xp_lanes each
// (process p owns lanes [p xp_lanes, (p + 1) xp_lanes)), so an Add works on
// the table in place: no swap, and occupancy / waiting masks are ballots of
// the lanes (a slot is occupied iff its dot is non-zero, waiting iff its
// waited-on dot is).  A process that needs more pending slots fails with
// FX_ERR_SIM_CAPACITY and fx_sim_run_tiered reruns the instance on the
// run-time build's larger tables.
constexpr uint32_t FANY = 0xFFu;  // f: per instance
struct GeoRT {
  static constexpr bool fixed = false;
  static constexpr uint32_t proto = 0xFFu, fc = FANY, xp_lanes = 0;
  Geo g;
};
template <uint32_t PR, uint32_t N, uint32_t F, uint32_t CC>
struct GeoCT {
  static constexpr bool fixed = true;
#ifdef FX_XSWAP
  static constexpr uint32_t proto = PR, fc = F, xp_lanes = 0;
#else
  static constexpr uint32_t proto = PR, fc = F, xp_lanes = 64u / N;
#endif
  static constexpr Geo g = geo_fixed(N, CC);
};

struct SimArgs {
  const fx_sim_spec* specs;
  uint32_t instances;
  Geo g;
  const uint16_t* ping;  // [RP][RP]
  const uint8_t* rank;   // [RP][RP]
  uint32_t RP;           // planet row stride
  uint32_t exec_cap, lat_cap, max_events, sim_exec_notif;
  uint32_t* executed;
  uint32_t* executed_len;
  uint32_t* latency_log;
  unsigned long long* lat_hist;
  uint32_t lat_bins;
  unsigned long long* chain_hist;
  uint32_t chain_bins;
  unsigned long long* delay_hist;
  uint32_t delay_bins;
  unsigned long long* stats;
  uint32_t* err;
  uint32_t* dot_client;  // [instances][n][exec_cap]: the client (1-based) that submitted dot (p, s)
};

// The kernel's arguments, read where a rarely taken path needs them through
// the kernarg segment (scalar loads, scalar-cache hits) instead of being held
// in scalar registers for the whole run: the simulator is short of SGPRs, and
// every spilled one costs a v_readlane / v_writelane pair on the hot path.
// The empty asm makes the pointer opaque so the loads are not hoisted.
typedef __attribute__((address_space(4))) const SimArgs KSimArgs;
__device__ __forceinline__ KSimArgs* kargs() {
  KSimArgs* p = (KSimArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
// a copy of a uniform value the compiler must treat as per-lane: arithmetic
// on it runs on the (mostly idle) vector unit instead of the scalar unit
__device__ __forceinline__ uint32_t vdiv(uint32_t x) {
  uint32_t r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)src);
}
__device__ __forceinline__ uint32_t gather(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ uint64_t bal(bool p) { return (uint64_t)__ballot(p); }
__device__ __forceinline__ uint32_t ctz64(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }
__device__ __forceinline__ uint32_t pop64(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }
__device__ __forceinline__ uint32_t pop32(uint32_t m) { return (uint32_t)__builtin_popcount(m); }

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finalizer (C6)
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ uint64_t sim_rand(uint64_t seed, uint64_t inst, uint64_t client, uint64_t idx,
                                             uint64_t purpose) {
  return mix64(mix64(mix64(mix64(seed ^ 0x5851F42D4C957F2Dull) + inst) + client) + ((idx << 8) | purpose));
}

// register arrays indexed by a wave-uniform value: arithmetic selects keep
// them in VGPRs (a dynamically indexed private array goes to scratch)
template <uint32_t N>
__device__ __forceinline__ uint32_t rsel(const uint32_t (&a)[N], uint32_t i) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t k = 0; k < N; ++k) r = (i == k) ? a[k] : r;
  return r;
}
template <uint32_t N>
__device__ __forceinline__ void rput(uint32_t (&a)[N], uint32_t i, uint32_t v) {
#pragma unroll
  for (uint32_t k = 0; k < N; ++k) a[k] = (i == k) ? v : a[k];
}

// Tarjan word: id (7 bits) | low (7 bits) | visited epoch (16 bits)
__device__ __forceinline__ uint32_t tid(uint32_t t) { return t & 127u; }
__device__ __forceinline__ uint32_t tlow(uint32_t t) { return (t >> 7) & 127u; }
__device__ __forceinline__ uint32_t tep(uint32_t t) { return t >> 14; }
__device__ __forceinline__ uint32_t tmk(uint32_t id, uint32_t low, uint32_t ep) { return id | (low << 7) | (ep << 14); }
constexpr uint32_t EPOCH_MAX = 0xFFFFu;

// NX: processes the executor slot tables are sized for (n <= NX)
template <uint32_t HM, uint32_t DS, uint32_t NX, class GP>
struct Sim : GP {
  using GP::g;
  // ---------------------------------------------------------------- context
  // the lane id, opaque at every use: expressions of it are recomputed where
  // they are used instead of being hoisted out of the event loop and held --
  // or spilled -- for the whole run
  uint32_t lid_;
  __device__ __forceinline__ uint32_t lidv() const {
    uint32_t x = lid_;
    asm volatile("" : "+v"(x));
    return x;
  }
  uint32_t* lds;
  uint32_t protocol, n, f, synod_f, fq, wq;
  // Per-instance parameters and rarely changed values in lanes of one VGPR
  // (lane P_*), read with v_readlane where they are used: kept in scalar
  // registers for the whole run they pushed hot values into spill slots.
  enum : uint32_t { P_SEED = 0, P_RNG = 2, P_GC = 4, P_EN = 5, P_CMDS = 6, P_CONFLICT = 7, P_POOL = 8, P_EXTRA = 9,
                    P_HAS_EXTRA = 10, P_FINAL = 11, P_CDONE = 12, P_ERRSITE = 13, P_INST = 14 };
  uint32_t pv = 0;
  // one v_readlane at each use (volatile: not hoisted into a scalar register
  // for the whole loop); it reads the lane whatever the exec mask, so it is
  // also right inside lane-divergent code
  __device__ __forceinline__ uint32_t prm(uint32_t k) const {
    uint32_t r;
    // The hazard recognizer does not look inside inline asm, so the asm
    // carries the wait states of both of its hazards itself:
    //  * before: a VALU write of a VGPR followed by a v_readlane of it needs
    //    one wait state on gfx940 / gfx950 (the compiler emits `s_nop 0`
    //    between its own v_cndmask and v_readlane).  Without it the
    //    readlane returns the VGPR's previous contents: under the iterative-
    //    ILP schedule the compiler put the v_cndmask that builds pv directly
    //    before prm(P_CMDS), the kernel read whatever an earlier kernel had
    //    left in that register as the command count, a client never started
    //    and the run ended in FX_ERR_SIM_LATE (round-3 open item, located in
    //    round 4 by tools/sim_stale_repro.py: divergence at the first event;
    //    vector-register poisoning hid it, scalar poisoning did not);
    //  * after: the asm's SGPR write read by a VALU lane select / VMEM needs
    //    wait states.
    asm volatile("s_nop 1\n\tv_readlane_b32 %0, %1, %2\n\ts_nop 4" : "=s"(r) : "v"(pv), "i"(k));
    return r;
  }
  __device__ __forceinline__ uint64_t prm64(uint32_t k) const {
    return (uint64_t)prm(k) | ((uint64_t)prm(k + 1) << 32);
  }
  __device__ __forceinline__ void prm_set(uint32_t k, uint32_t x) {
    if (lidv() == k) pv = x;
  }
  uint32_t C;
  uint32_t err = 0;
  // source line of the first capacity failure (diagnostics): lane P_ERRSITE
  __device__ __forceinline__ void fail_cap(uint32_t line) {
    if (!err) prm_set(P_ERRSITE, line);
    err = FX_ERR_SIM_CAPACITY;
  }
  // a simulated message that found no state for its dot (the reference
  // panics): the site is recorded like a capacity failure's
  __device__ __forceinline__ void fail_late(uint32_t line) {
    if (!err) prm_set(P_ERRSITE, line);
    err = FX_ERR_SIM_LATE;
  }
  uint32_t now = 0;       // ms
  uint32_t seq = 0;       // insertion counter (C3)
  uint32_t events = 0;  // <= max_events < 2^32
  // per-lane (vector-unit) bookkeeping, every lane holds the same value: the
  // action trace hash, deps and latency sums
  uint64_t trace, deps_total, lat_sum;
  // histogram samples counted per instance: ChainSize value v < 64 in lane v
  // of hcv, ExecutionDelay value v < 256 in LDS word v of the instance's
  // table, client latencies in a direct-mapped cache keyed by (region,
  // latency): lane h holds key + 1 (hlk) and its count (hlc); everything else
  // goes to the global bins directly; the bins are clamped when the counts are
  // flushed (exact)
  uint32_t hcv = 0, hlk = 0, hlc = 0;
  bool done = false, in_extra = false;

  // link heads owned by this lane: time, seq (time NONE = empty)
  uint32_t ht[HM], hs[HM];
  // GC state of lane 8 p + s (see h_mcommitdot): committed frontier + window
  // of source s + 1 at process p, tick-log and change-log counters
  uint32_t gf = 0, gw = 0, gnt = 0, glk = 0, gkm = 0, gnc = 0;
  // Small per-process / per-client tables live in lanes (a wave-uniform
  // index reads them with v_readlane instead of an LDS round trip):
  // lane p: proposal seq, Fast / Slow counters, executed count, the
  // executor's occupancy and waiting masks, fast | write quorum << 8
  // lane 8 k + p of `pt`: table k of process p (proposal seq, Fast, Slow,
  // executed count, the executor's occupancy and waiting masks, two words
  // each) — eight small tables in one VGPR; lane p of `pq`: fast | write quorum << 8
  uint32_t pt = 0, pq = 0;
  // lane c: process | region << 8, commands issued, start time, results pending
  // lane c / 32 + c of `ca`, `cb`, `cd` (C <= 32): process | region << 8 /
  // commands issued; start time / results pending; the client -> process
  // delay / the process -> client delay
  uint32_t ca = 0, cb = 0, cd = 0;
  // link delays (runner.rs:575-595): lane 8 p + q for p -> q (the client
  // links' delays are in cd)
  uint32_t dpq = 0;
  // handler frame stack, frame fi in lane fi: action (0 none, 1 ToSend) |
  // kind << 2 | targets << 8 | next target << 16 | ready results << 20; dot
  uint32_t frw = 0, frd = 0;
  // message ring of process link l (< n (n - 1) <= 56): head | tail << 16 in lane l
  uint32_t rhv = 0xFFFFFFFFu;
  uint32_t nfree = 0;  // free message-pool entries (a stack of indices in LDS)
  uint32_t sdv[DS];  // dot of dot-table slot 64 k + lane in sdv[k] (0 = free)
  // executed clocks of the executors: lane 8 p + s = source s + 1 at process p
  uint32_t ecf = 0, ecw = 0;

  // executor state of every process (lane-owned slot l / clock of source l + 1)
  uint32_t xdot[NX], xrec[NX], xwait[NX];
  // executor working copy (the process being run); the Tarjan words and the
  // DFS frames only live during one handle_add
  uint32_t sdot, srec, swait, stl, sfr;
  uint64_t occ, wmask, tmask;
  static constexpr uint32_t XPL = GP::xp_lanes;
  uint64_t pmask = ~0ull;  // lanes of the running process's slots
  uint32_t xk, epoch, nwl, phase, root, idc, nfr, missing, fv, fdi, fnc, in_try, emitted, xp;
#ifdef FX_SIM_PROFILE
  uint64_t prof[24] = {};
#endif

  // ------------------------------------------------------------ LDS views
  __device__ __forceinline__ uint32_t& W(uint32_t i) { return lds[i]; }
  // message pool entry e: time | kind << 28, insertion seq, dot, next entry of its link
  __device__ __forceinline__ uint32_t& msg(uint32_t e, uint32_t w) {
    return lds[g.off_pool + e * 4 + w];
  }
  // GC logs of (process p, source s): tick log entry i = (tick count, frontier
  // before the change), change log entry i = (time, frontier after)
  __device__ __forceinline__ uint32_t* gct(uint32_t p, uint32_t s) { return &lds[g.off_gct + (p * g.n + s) * g.rt * 2]; }
  __device__ __forceinline__ uint32_t* gcc(uint32_t p, uint32_t s) { return &lds[g.off_gcc + (p * g.n + s) * g.rc * 2]; }
  __device__ __forceinline__ uint32_t* gcr(uint32_t p, uint32_t s) { return &lds[g.off_gcr + (p * g.n + s) * 4]; }
  // dot table: a pool of g.W <= 64 DS slots shared by every coordinator of
  // the instance (a coordinator far ahead of a lagging replica holds many live
  // dots); slot 64 k + l is lane l of sdv[k]; look-up = DS ballots
  __device__ __forceinline__ uint32_t slot_find(uint32_t d) const {
    uint32_t r = NONE;
#pragma unroll
    for (uint32_t k = 0; k < DS; ++k) {
      const uint64_t m = bal(sdv[k] == d && d != 0u);
      if (m && r == NONE) r = k * 64u + ctz64(m);
    }
    return r;
  }
  __device__ __forceinline__ void slot_set(uint32_t sl, uint32_t d) {
#pragma unroll
    for (uint32_t k = 0; k < DS; ++k)
      if ((sl >> 6) == k && lidv() == (sl & 63u)) sdv[k] = d;
  }
  __device__ __forceinline__ uint32_t slot_alloc() const {
#pragma unroll
    for (uint32_t k = 0; k < DS; ++k) {
      const uint32_t lo = k * 64u;
      if (lo >= g.W) break;
      const uint64_t pool = g.W - lo >= 64u ? ~0ull : ((1ull << (g.W - lo)) - 1ull);
      const uint64_t fre = ~bal(sdv[k] != 0u) & pool;
      if (fre) return lo + ctz64(fre);
    }
    return NONE;
  }
  __device__ __forceinline__ uint32_t& S(uint32_t sl, uint32_t w) { return lds[g.off_slot + sl * g.slotw + w]; }
  // GC deliveries p -> q: base insertion seq of p's tick k (the tick's sends
  // take consecutive seqs in ascending target order) and the next tick index
  // link (p, q) delivers
  __device__ __forceinline__ uint32_t& kd(uint32_t p, uint32_t key) { return lds[g.off_kd + p * g.ncli_keys + key]; }
  __device__ __forceinline__ uint32_t& FRR(uint32_t fi, uint32_t r) { return lds[g.off_frame + fi * g.rdm + r]; }
  __device__ __forceinline__ uint32_t& wl(uint32_t i) { return lds[g.off_wl + i]; }
  // Histogram samples are counted per instance in LDS (ChainSize bins
  // [0, HC_BINS), ExecutionDelay bins [0, HD_BINS)) and added to the global
  // histograms once at the end: one global atomic per sample made every
  // executed command a device-scope atomic on the same few bins.
  __device__ __forceinline__ void hist_chain(uint32_t v) {
    if (v < HC_BINS) {
      hcv += lidv() == v ? 1u : 0u;
    } else if (lidv() == 0) {
      KSimArgs* k = kargs();
      if (k->chain_hist) atomicAdd(&k->chain_hist[min(v, k->chain_bins - 1u)], 1ull);
    }
  }
  // client latency samples: a direct-mapped per-instance cache of (region,
  // bin) -> count (a region's latencies take few distinct values); a sample
  // whose entry is taken by another bin goes to the global bin directly
  __device__ __forceinline__ void hist_lat(uint32_t region, uint32_t lat) {
    const uint32_t key = (region << 24) | min(lat, 0xFFFFFFu);
    const uint32_t h = (key * 2654435761u) >> 26;
    const uint32_t k = rl(hlk, h);
    if (k == key + 1u || k == 0) {
      if (lidv() == h) {
        hlk = key + 1u;
        ++hlc;
      }
    } else {
      flush_lat(key, 1u);
    }
  }
  __device__ __forceinline__ void flush_lat(uint32_t key, uint32_t cnt) {
    if (lidv() == 0) {
      KSimArgs* k = kargs();
      const uint32_t lat = key & 0xFFFFFFu, bins = k->lat_bins;
      if (k->lat_hist) atomicAdd(&k->lat_hist[(key >> 24) * bins + min(lat, bins - 1u)], (unsigned long long)cnt);
    }
  }
  __device__ __forceinline__ void hist_delay(uint32_t v) {
#ifdef FX_ABL_HIST  // measurement-only ablation (wrong histograms)
    return;
#endif
    if (v < HD_BINS) {
      if (lidv() == 0) atomicAdd(&lds[g.off_hist + v], 1u);
    } else if (lidv() == 0) {
      KSimArgs* k = kargs();
      if (k->delay_hist) atomicAdd(&k->delay_hist[min(v, k->delay_bins - 1u)], 1ull);
    }
  }

  __device__ __forceinline__ uint32_t pst(uint32_t sl, uint32_t p) {
    return (uni(S(sl, SL_PST + (p >> 2))) >> ((p & 3u) * 8u)) & 0xFFu;
  }
  __device__ __forceinline__ void set_pst(uint32_t sl, uint32_t p, uint32_t v) {
    const uint32_t w = uni(S(sl, SL_PST + (p >> 2)));
    const uint32_t sh = (p & 3u) * 8u;
    const uint32_t nw = (w & ~(0xFFu << sh)) | ((v & 0xFFu) << sh);
    S(sl, SL_PST + (p >> 2)) = nw;
  }
  // store a uniform value to an LDS word: every lane computed the same value
  // and stores it (one ds_write; no exec-mask save / restore around a
  // lane-0-only store, which costs scalar issue slots — the kernel's bound)
  __device__ __forceinline__ void put(uint32_t& dst, uint32_t v) { dst = v; }
  // set lane `lane` of a lane table
  __device__ __forceinline__ void lset(uint32_t& reg, uint32_t lane, uint32_t v) {
    if (lidv() == lane) reg = v;
  }

  // ------------------------------------------------------------- links
  __device__ __forceinline__ uint32_t link_p(uint32_t p, uint32_t q) const {  // 0-based p != q
    return p * (g.n - 1) + (q < p ? q : q - 1);
  }
  __device__ __forceinline__ uint32_t link_e(uint32_t p) const { return g.NP + p; }
  __device__ __forceinline__ uint32_t link_s(uint32_t c) const { return g.NP + g.n + c; }
  __device__ __forceinline__ uint32_t link_r(uint32_t c) const { return g.NP + g.n + g.C + c; }

  __device__ __forceinline__ void head_set(uint32_t link, uint32_t t, uint32_t s) {
    const uint32_t ln = link & 63u, h = link >> 6;
    if (lidv() == ln) {
#pragma unroll
      for (uint32_t k = 0; k < HM; ++k)
        if (h == k) {
          ht[k] = t;
          hs[k] = s;
        }
    }
  }

  // Schedule::schedule on a link (schedule.rs:38-49): insertion seq = C3 tie-break
  __device__ __forceinline__ void schedule_timer(uint32_t link, uint32_t delay) {
    head_set(link, now + delay, seq);
    ++seq;
  }
  __device__ __forceinline__ void send_p(uint32_t from, uint32_t to, uint32_t kind, uint32_t w2) {
    PROF_T0();
    send_p_(from, to, kind, w2);
    PROF_ADD(3);
  }
  __device__ __forceinline__ void send_p_(uint32_t from, uint32_t to, uint32_t kind, uint32_t w2) {  // 0-based processes
    const uint32_t link = link_p(from, to);
    const uint32_t t = now + rl(dpq, from * 8u + to);
    if (nfree == 0) {
      fail_cap(__LINE__);
      return;
    }
    if (t >= (1u << 28)) {
      err = FX_ERR_TIME_RANGE;
      return;
    }
    const uint32_t e = uni(lds[g.off_free + --nfree]);
    put(msg(e, 0), t | (kind << 28));
    put(msg(e, 1), seq);
    put(msg(e, 2), w2);
    put(msg(e, 3), LNIL);
    const uint32_t ht_ = rl(rhv, link);
    const uint32_t head = ht_ & 0xFFFFu, tail = ht_ >> 16;
    if (head == LNIL) {
      lset(rhv, link, e | (e << 16));
      head_set(link, t, seq);
    } else {
      put(msg(tail, 3), e);
      lset(rhv, link, head | (e << 16));
    }
    ++seq;
  }

  // the sends of one ToSend action to the targets in `mask` (p excluded), in
  // ascending target order (C4), as one lane-parallel step: lane q builds the
  // message to q with the insertion seq and the pool entry the one-by-one
  // loop would give it (seq + rank, the rank-th pop of the free stack) and
  // appends it to link (p, q); the link lanes then take their new list words
  // and heads from the target lanes
  __device__ __forceinline__ void send_batch(uint32_t p, uint32_t mask, uint32_t kind, uint32_t w2) {
    PROF_T0();
    send_batch_(p, mask, kind, w2);
    PROF_ADD(3);
  }
  __device__ __forceinline__ void send_batch_(uint32_t p, uint32_t mask, uint32_t kind, uint32_t w2) {
    const uint32_t k = pop32(mask);
    if (k == 0) return;
    if (nfree < k) {
      fail_cap(__LINE__);
      return;
    }
    const bool tq = lidv() < 8u && ((mask >> lidv()) & 1u);
    const uint32_t r = pop32(mask & (lidv() < 8u ? (1u << lidv()) - 1u : 0u));
    const uint32_t t = now + gather(dpq, (p * 8u + lidv()) & 63u);  // lane q: now + d(p, q)
    if (bal(tq && t >= (1u << 28))) {
      err = FX_ERR_TIME_RANGE;
      return;
    }
    const uint32_t base = p * (g.n - 1u);
    const uint32_t rh = gather(rhv, (base + (lidv() < p ? lidv() : lidv() - 1u)) & 63u);  // lane q: link (p, q)'s list
    const uint32_t head = rh & 0xFFFFu;
    uint32_t e = 0;
    if (tq) {
      e = lds[g.off_free + nfree - 1u - r];
      // one 16-byte store of the entry's four words; the vector type may
      // alias the u32 words the message is read back through (msg)
      typedef uint32_t u32x4_alias __attribute__((ext_vector_type(4), may_alias));
      u32x4_alias v4 = {t | (kind << 28), seq + r, w2, LNIL};
      *reinterpret_cast<u32x4_alias*>(&lds[g.off_pool + e * 4u]) = v4;
      if (head != LNIL) msg(rh >> 16, 3) = e;  // after the tail
    }
    const uint32_t nrh = head == LNIL ? (e | (e << 16)) : (head | (e << 16));
    // lane base + i = link (p, q(i)) takes lane q(i)'s values: the new list
    // word, and time (28 bits) | rank << 28 | link was empty << 31 in one word
    const uint32_t tw = t | (r << 28) | (head == LNIL ? 1u << 31 : 0u);
    const uint32_t i = lidv() - base;
    const bool ll = lidv() >= base && i < g.n - 1u;
    const uint32_t q = (ll ? (i < p ? i : i + 1u) : 0u) & 63u;
    const uint32_t v_nrh = gather(nrh, q), v_tw = gather(tw, q);
    if (ll && ((mask >> q) & 1u)) {
      rhv = v_nrh;
      if (v_tw >> 31) {  // the link was empty: the message is its head (P links are lanes < 64)
        ht[0] = v_tw & 0x0FFFFFFFu;
        hs[0] = seq + ((v_tw >> 28) & 7u);
      }
    }
    nfree -= k;
    seq += k;
  }

  // -------------------------------------------------------------- trace
  __device__ __forceinline__ void note(uint64_t kind, uint64_t a, uint64_t b, uint64_t c) {
    PROF_T0();
    note_(kind, a, b, c);
    PROF_ADD(6);
  }
  __device__ __forceinline__ void note_(uint64_t kind, uint64_t a, uint64_t b, uint64_t c) {
    ++events;
#ifdef FX_ABL_NOTE  // measurement-only ablation (wrong trace): the cost of the trace hash
    return;
#endif
    trace = mix64(trace ^ ((uint64_t)now << 24) ^ (kind << 20) ^ (a << 12) ^ (b << 4)) + c;
  }

  // ------------------------------------------------------------ workload
  // Workload::gen_cmd (workload.rs:142-197) keys of command idx of client c
  // (1-based id), canonical C6/C7/C11: packed key0 | key1 << 16, count
  __device__ __forceinline__ uint32_t gen_keys(uint32_t cid, uint32_t idx, uint32_t& nk) {
    const uint64_t seed = prm64(P_SEED), rng_inst = prm64(P_RNG);
    const uint32_t conflict_ = prm(P_CONFLICT), pool = prm(P_POOL);
    uint32_t k0 = 0xFFFFu, k1 = 0xFFFFu;
    nk = 0;
    for (uint32_t draw = 0; nk < g.K && draw < 65536u; ++draw) {  // gen_unique_keys draws until distinct
      bool conflict;
      if (conflict_ == 0) conflict = false;
      else if (conflict_ >= 100) conflict = true;
      else conflict = sim_rand(seed, rng_inst, cid, (uint64_t)idx * 64 + draw, 1) % 100ull < conflict_;
      uint32_t key;
      if (conflict) key = pool <= 1 ? 0u : (uint32_t)(sim_rand(seed, rng_inst, cid, (uint64_t)idx * 64 + draw, 2) % pool);
      else key = pool + cid;
      if (nk == 0) { k0 = key; nk = 1; }
      else if (key != k0) { k1 = key; nk = 2; }
    }
    if (nk != g.K) fail_cap(__LINE__);
    if (nk == 2 && k1 < k0) { const uint32_t t = k0; k0 = k1; k1 = t; }  // C11
    return k0 | (k1 << 16);
  }

  // ------------------------------------------------------- frame stack
  uint32_t nfrm = 0;  // frames in use
  uint32_t xinfo = 0; // execution info pushed by the current handler (dot, 0 = none)

  __device__ __forceinline__ void act_send(uint32_t kind, uint32_t dot, uint32_t tgt) {
    const uint32_t fi = nfrm - 1;
    const uint32_t w = rl(frw, fi);
    lset(frw, fi, (w & (31u << 20)) | 1u | (kind << 2) | (tgt << 8));
    lset(frd, fi, dot);
  }

  // ============================================================ protocol
  // key_deps.add_cmd (sequential.rs:74-118): latest write per key (no reads,
  // no noops in these workloads); `past` merged; returns sorted unique deps in
  // lanes [0, cnt) of `out` (a per-lane value)
  __device__ __forceinline__ uint32_t add_cmd(uint32_t p, uint32_t dot, uint32_t keys, uint32_t nk, uint32_t pastv, uint32_t npast,
                              uint32_t& outv) {
    const uint32_t key0 = keys & 0xFFFFu, key1 = keys >> 16;
    const uint32_t d0 = uni(kd(p, key0));
    put(kd(p, key0), dot);
    uint32_t d1 = 0;
    if (nk > 1) {
      d1 = uni(kd(p, key1));
      put(kd(p, key1), dot);
    }
    // candidates: lanes [0, npast) the past deps, lane npast / npast + 1 the
    // latest writes of the keys; the result is their sorted distinct set
    const uint32_t v = lidv() < npast ? pastv : (lidv() == npast ? d0 : (lidv() == npast + 1 ? d1 : 0u));
    const bool valid = v != 0;
    bool first = valid;
    const uint64_t vm = bal(valid);
    for (uint64_t m = vm; m; m &= m - 1) {
      const uint32_t j = ctz64(m);
      if (j < lidv() && rl(v, j) == v) first = false;
    }
    const uint64_t fm = bal(first);
    uint32_t rank = 0;
    for (uint64_t m = fm; m; m &= m - 1) rank += rl(v, ctz64(m)) < v ? 1u : 0u;
    outv = 0;
    for (uint64_t m = fm; m; m &= m - 1) {
      const uint32_t j = ctz64(m);
      const uint32_t vj = rl(v, j), rj = rl(rank, j);
      if (lidv() == rj) outv = vj;
    }
    return pop64(fm);
  }

  // Protocol::submit (atlas.rs:210-249, epaxos.rs:199-221)
  __device__ __forceinline__ void h_submit(uint32_t p, uint32_t c) {
    const uint32_t s = rl(pt, PT_SEQ + p) + 1u;
    lset(pt, PT_SEQ + p, s);
    if (s > FX_SEQ_MASK) { err = FX_ERR_DOT_RANGE; return; }
    const uint32_t dot = FX_PACK_DOT(p + 1, s);
    const uint32_t sl = slot_alloc();
    if (sl == NONE) { fail_cap(__LINE__); return; }
    const uint32_t idx = rl(ca, 32u + c) - 1u;
    // the rifl of the dot (Result.rifls / monitors): dot (p, s) was
    // submitted by client c + 1, whose k-th dot is its command k
    const uint32_t inst = prm(P_INST);
    if (lidv() == 0) {
      KSimArgs* k = kargs();
      if (k->dot_client && s <= k->exec_cap) k->dot_client[((size_t)inst * n + p) * k->exec_cap + s - 1u] = c + 1u;
    }
    uint32_t nk = 0;
    const uint32_t keys = gen_keys(c + 1, idx, nk);
    // fresh slot
    if (lidv() < g.slotw) S(sl, lidv()) = 0;
    slot_set(sl, dot);
    put(S(sl, SL_CLIENT), c);
    put(S(sl, SL_IDX), idx);
    put(S(sl, SL_KEYS), keys);
    if (!GP::fixed && protocol == FX_PROTOCOL_BASIC) {  // basic.rs:171-185: MStore to all
      put(S(sl, SL_CNT), nk << 20);
      act_send(M_STORE, dot, (1u << n) - 1u);
      return;
    }
    uint32_t depv = 0;
    const uint32_t nd = add_cmd(p, dot, keys, nk, 0, 0, depv);
    if (lidv() < nd) S(sl, SL_COLLECT + lidv()) = depv;
    put(S(sl, SL_CNT), (nd << 8) | (nk << 20));
    act_send(M_COLLECT, dot, (1u << n) - 1u);
  }

  // ------------------------------------------------------------- Basic
  // basic.rs:187-211 handle_mstore: the command arrives; a member of the
  // coordinator's quorum acks; a commit that arrived first is applied now
  __device__ __forceinline__ void h_mstore(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    const uint32_t ps = pst(sl, p);
    set_pst(sl, p, (ps & ~7u) | ST_PAYLOAD);
    const uint32_t src = (dot >> FX_SEQ_BITS) - 1u;
    if ((rl(pq, src) >> p) & 1u) act_send(M_STORE_ACK, dot, 1u << from);
    if (ps & 4u) h_bcommit(p, dot);  // buffered_mcommits.remove
  }
  // basic.rs:213-230 handle_mstoreack: f + 1 acks commit
  __device__ __forceinline__ void h_mstoreack(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    const uint32_t masks = uni(S(sl, SL_MASKS));
    const uint32_t acks = (masks & 0xFFu) | (1u << from);
    put(S(sl, SL_MASKS), (masks & ~0xFFu) | acks);
    if (pop32(acks) == f + 1u) act_send(M_COMMIT_BASIC, dot, (1u << n) - 1u);
  }
  // basic.rs:232-257 handle_mcommit: BasicExecutor::handle runs one
  // BasicExecutionInfo per key at once (executor/basic.rs:39-53): the dot is
  // logged once per key (the oracle's execution log) and the key results go
  // to AggregatePending; no ExecutionDelay / ChainSize samples
  __device__ __forceinline__ void h_bcommit(uint32_t p, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    const uint32_t ps = pst(sl, p);
    if ((ps & 3u) == ST_START) {  // buffered_mcommits.insert
      set_pst(sl, p, ps | 4u);
      return;
    }
    set_pst(sl, p, (ps & ~7u) | ST_COMMIT);
    const uint32_t c = uni(S(sl, SL_CLIENT));
    const uint32_t nk = (uni(S(sl, SL_CNT)) >> 20) & 3u;
    const uint32_t inst = prm(P_INST);
    const uint32_t x0 = rl(pt, PT_EXEC + p);
    if (lidv() == 0) {
      KSimArgs* k = kargs();
      for (uint32_t j = 0; j < nk; ++j)
        if (x0 + j < k->exec_cap && k->executed) k->executed[((size_t)inst * n + p) * k->exec_cap + x0 + j] = dot;
    }
    lset(pt, PT_EXEC + p, x0 + nk);
    if ((rl(ca, c) & 0xFFu) == p) {  // pending.wait_for registered this rifl at p
      const uint32_t pend = rl(cb, 32u + c);
      if (pend < nk) { fail_late(__LINE__); return; }
      lset(cb, 32u + c, pend - nk);
      if (pend == nk) {
        const uint32_t fi = nfrm - 1;
        const uint32_t w = rl(frw, fi);
        const uint32_t nr = (w >> 20) & 31u;
        if (nr >= g.rdm) { fail_cap(__LINE__); return; }
        put(FRR(fi, nr), c);
        lset(frw, fi, w + (1u << 20));
      }
    }
    const uint32_t masks = uni(S(sl, SL_MASKS));
    if (((masks >> 24) & 0xFFu) + 1u == n) {
      slot_set(sl, 0u);  // executed everywhere: nothing about the dot is in flight
    } else {
      put(S(sl, SL_MASKS), masks + (1u << 24));
    }
    if (prm(P_GC)) h_mcommitdot(p, dot);  // Forward(MCommitDot) (basic.rs:246-251)
  }

  // atlas.rs:251-325 / epaxos.rs:223-301
  __device__ __forceinline__ void h_mcollect(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    const uint32_t ps = pst(sl, p);
    if ((ps & 3u) != ST_START) return;
    const uint32_t src = (dot >> FX_SEQ_BITS) - 1u;
    const uint32_t quorum = rl(pq, src) & 0xFFu;
    if (!((quorum >> p) & 1u)) {
      set_pst(sl, p, (ps & ~3u) | ST_PAYLOAD);
      if (ps & 4u) {  // buffered commit (atlas.rs:288-292)
        set_pst(sl, p, ((ps & ~3u) | ST_PAYLOAD) & ~4u);
        h_mcommit(p, ps >> 4, dot);
      }
      return;
    }
    const bool from_self = from == p;
    const uint32_t cnt = uni(S(sl, SL_CNT));
    const uint32_t ncol = (cnt >> 8) & 0xFFu, nk = (cnt >> 20) & 3u;
    uint32_t depv = 0, nd = 0;
    const uint32_t colv = lidv() < ncol ? S(sl, SL_COLLECT + lidv()) : 0u;
    if (from_self) {
      depv = colv;
      nd = ncol;
    } else {
      nd = add_cmd(p, dot, uni(S(sl, SL_KEYS)), nk, colv, ncol, depv);
    }
    if (nd > g.amax) { fail_cap(__LINE__); return; }
    set_pst(sl, p, (ps & ~3u) | ST_COLLECT);
    // the ack's deps travel in the slot: ack deps of p
    if (lidv() < g.amax) S(sl, g.sl_ack + p * g.amax + lidv()) = lidv() < nd ? depv : 0u;
    if (protocol == FX_PROTOCOL_EPAXOS && from_self) return;  // epaxos.rs:290-300
    act_send(M_COLLECT_ACK, dot, 1u << from);
  }

  // atlas.rs:327-402 / epaxos.rs:303-368
  __device__ __forceinline__ void h_mcollectack(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    if ((pst(sl, p) & 3u) != ST_COLLECT) return;
    const uint32_t masks = uni(S(sl, SL_MASKS));
    const uint32_t part = (masks & 0xFFu) | (1u << from);
    put(S(sl, SL_MASKS), (masks & ~0xFFu) | part);
    const uint32_t fq_eff = protocol == FX_PROTOCOL_EPAXOS ? fq - 1u : fq;
    if (pop32(part) != fq_eff) return;
    // QuorumDeps: union + per-dep report counts over the participants' acks.
    // lane j of a participant block holds one reported dep: lanes
    // [q*amax, q*amax + amax) for process q (<= 32 lanes)
    const uint32_t q = lidv() / g.amax, j = lidv() % g.amax;
    uint32_t v = 0;
    if (q < n && ((part >> q) & 1u)) v = S(sl, g.sl_ack + q * g.amax + j);
    const bool valid = v != 0;
    // count and first occurrence
    uint32_t cnt = 0;
    bool first = valid;
    const uint64_t vm = bal(valid);
    for (uint64_t m = vm; m; m &= m - 1) {
      const uint32_t l2 = ctz64(m);
      const uint32_t v2 = rl(v, l2);
      if (valid && v2 == v) {
        ++cnt;
        if (l2 < lidv()) first = false;
      }
    }
    const uint64_t um = bal(first);  // one lane per distinct dep
    const uint32_t nu = pop64(um);
    if (nu > g.vmax) { fail_cap(__LINE__); return; }
    bool fast;
    if (protocol == FX_PROTOCOL_ATLAS) {
      // threshold = |quorum| - minority (atlas.rs:361-368)
      const uint32_t threshold = fq - (n / 2u);
      fast = !bal(first && cnt < threshold);
    } else {
      // check_equal (quorum.rs:72-103): every dep reported by every participant
      fast = nu == 0 || !bal(first && cnt != fq_eff);
    }
    // value = union, ascending
    uint32_t rank = 0;
    for (uint64_t m = um; m; m &= m - 1) rank += rl(v, ctz64(m)) < v ? 1u : 0u;
    if (first) S(sl, g.sl_value + rank) = v;
    const uint32_t c0 = uni(S(sl, SL_CNT));
    put(S(sl, SL_CNT), (c0 & ~0xFFu) | nu | (fast ? 0u : (1u << 16)));  // slow: proposer ballot set
    if (lidv() == (fast ? PT_FAST : PT_SLOW) + p) ++pt;
    if (fast) {
      act_send(M_COMMIT, dot, (1u << n) - 1u);
    } else {
      // synod.skip_prepare (single.rs:208-213): ballot = coordinator id
      act_send(M_CONSENSUS, dot, rl(pq, p) >> 8);
    }
  }

  // atlas.rs:404-475 / epaxos.rs:370-428
  __device__ __forceinline__ void h_mcommit(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    const uint32_t ps = pst(sl, p);
    if ((ps & 3u) == ST_START) {  // buffered_commits.insert
      set_pst(sl, p, (ps & 0x0Bu) | 4u | (from << 4));
      return;
    }
    if ((ps & 3u) == ST_COMMIT) return;
    xinfo = dot;  // to_executors.push(GraphExecutionInfo::add(dot, cmd, value.deps))
    set_pst(sl, p, (ps & ~3u) | ST_COMMIT);
    const uint32_t masks = uni(S(sl, SL_MASKS));
    put(S(sl, SL_MASKS), masks + (1u << 16));  // committed count
    // Forward(MCommitDot) to self: it only moves the GC track's committed
    // clock (gc/clock.rs:43-48), which nothing but the GC evaluation reads,
    // so it is applied in place
    if (prm(P_GC)) h_mcommitdot(p, dot);
  }

  // atlas.rs:477-524 / epaxos.rs:430-477
  __device__ __forceinline__ void h_mconsensus(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    const uint32_t ps = pst(sl, p);
    if ((ps & 3u) == ST_COMMIT) {  // chosen: reply with the chosen value
      act_send(M_COMMIT, dot, 1u << from);
      return;
    }
    set_pst(sl, p, ps | 8u);  // acceptor accepts (b >= ballot)
    act_send(M_CONSENSUS_ACK, dot, 1u << from);
  }

  // atlas.rs:526-558 / epaxos.rs:479-517
  __device__ __forceinline__ void h_mconsensusack(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = slot_find(dot);
    if (sl == NONE) { fail_late(__LINE__); return; }
    if (!((uni(S(sl, SL_CNT)) >> 16) & 1u)) return;  // proposer ballot != b
    const uint32_t masks = uni(S(sl, SL_MASKS));
    const uint32_t acc = ((masks >> 8) & 0xFFu) | (1u << from);
    if (pop32(acc) == synod_f + 1u) {
      put(S(sl, SL_MASKS), masks & ~0xFF00u);  // reset_state
      if (!(pst(sl, p) & 8u)) { fail_late(__LINE__); return; }  // single.rs:346-349 panic
      act_send(M_COMMIT, dot, (1u << n) - 1u);
    } else {
      put(S(sl, SL_MASKS), (masks & ~0xFF00u) | (acc << 8));
    }
  }

  // ------------------------------------------------------------------ GC
  // The GC traffic (periodic GarbageCollection, atlas.rs:699-714, and the
  // MGarbageCollection / MStable it causes, atlas.rs:657-697, gc/clock.rs:
  // 21-138) only feeds the GC track, which nothing else reads, and under C3 it
  // follows every other action of its millisecond.  Its only output, the
  // Stable count, is therefore a function of the committed frontiers'
  // history, evaluated once at the end (gc_finish) instead of as ~90 % of the
  // events:
  //  * tick k of process p (time (k + 1) gc) reports p's committed frontier
  //    as of that millisecond; it reaches q at (k + 1) gc + d(p, q);
  //  * every reported frontier only grows and q's own frontier only grows, so
  //    q's Stable count = sum over sources of min(q's frontier at its last
  //    delivery, the frontier in the last delivery from each other process),
  //    or 0 if some process has not reported yet.
  // Lane 8 p + s keeps the committed clock of source s + 1 at p (AEClock:
  // frontier + 32-bit exception window) and two logs of its frontier: one
  // entry per tick interval in which it moved (the value a tick before the
  // move reports) and its last moves with their times (Geo::rt, Geo::rc entries).
  __device__ __forceinline__ bool gc_lane(uint32_t p) const { return (lidv() >> 3) == p && (lidv() & 7u) < n; }

  // MCommitDot: add_to_clock (gc/clock.rs:43-48)
  __device__ __forceinline__ void h_mcommitdot(uint32_t p, uint32_t dot) {
    const uint32_t gc_ms = prm(P_GC);
#ifdef FX_ABL_GC
    return;
#endif
    const uint32_t si = (dot >> FX_SEQ_BITS) - 1u, sq = dot & FX_SEQ_MASK;
    bool bad = false;
    if (lidv() == p * 8u + si && sq > gf) {
      const uint32_t off = sq - gf - 1u;
      if (off >= 32u) {
        bad = true;
      } else if (off) {
        gw |= 1u << off;
      } else {
        const uint32_t old = gf;
        const uint32_t win = gw >> 1;
        const uint32_t ones = __builtin_ctz(~win);
        gf = gf + 1 + ones;
        gw = win >> ones;
        if (gc_ms) {
          const uint32_t kt = now ? (now - 1u) / gc_ms : 0u;  // ticks strictly before now
          if (gnt == 0 || kt != glk) {
            uint32_t* tl = gct(p, si);
            const uint32_t e = gnt & (g.rt - 1u);
            if (gnt >= g.rt) gkm = tl[e * 2];  // newest dropped entry
            tl[e * 2] = kt;
            tl[e * 2 + 1] = old;
            ++gnt;
            glk = kt;
          }
          uint32_t* cl = gcc(p, si);
          const uint32_t e2 = gnc & (g.rc - 1u);
          cl[e2 * 2] = now;
          cl[e2 * 2 + 1] = gf;
          ++gnc;
        }
      }
    }
    if (bal(bad)) fail_cap(__LINE__);
  }

  // frontier of source s at p reported by tick k; false if the log lost it
  __device__ __forceinline__ bool gc_tick_value(uint32_t p, uint32_t s, uint32_t k, uint32_t& v) {
    const uint32_t* r = gcr(p, s);
    const uint32_t nt = r[1], km = r[2];
    if (nt > g.rt && k < km) return false;
    const uint32_t* tl = gct(p, s);
    const uint32_t cnt = min(nt, g.rt);
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint32_t e = (nt - cnt + i) & (g.rt - 1u);
      if (tl[e * 2] > k) {
        v = tl[e * 2 + 1];
        return true;
      }
    }
    v = r[0];
    return true;
  }
  // frontier of source s at p after every action up to time x
  __device__ __forceinline__ bool gc_value_at(uint32_t p, uint32_t s, uint32_t x, uint32_t& v) {
    const uint32_t nc = gcr(p, s)[3];
    const uint32_t* cl = gcc(p, s);
    const uint32_t cnt = min(nc, g.rc);
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint32_t e = (nc - 1u - i) & (g.rc - 1u);
      if (cl[e * 2] <= x) {
        v = cl[e * 2 + 1];
        return true;
      }
    }
    v = 0;
    return nc <= g.rc;
  }

  // first GC action after time x: its time, and (ticks first, then
  // deliveries by (from, to)) the delivery it is, or NONE for a tick
  __device__ __forceinline__ uint32_t gc_next_after(uint32_t x, uint32_t& pair) {
    const uint32_t gc_ms = prm(P_GC);
    const uint32_t tick = (x / gc_ms + 1u) * gc_ms;
    uint32_t tv = NONE;
    const uint32_t p = lidv() >> 3, q = lidv() & 7u;
    if (p < n && q < n && p != q) {
      const uint32_t d = dpq;
      tv = x < gc_ms + d ? gc_ms + d : ((x - d) / gc_ms + 1u) * gc_ms + d;
    }
    uint32_t tmin = tv;
    for (uint32_t o = 1; o < 64; o <<= 1) tmin = min(tmin, (uint32_t)__shfl_xor((int)tmin, (int)o));
    tmin = uni(tmin);
    if (tick <= tmin) {
      pair = NONE;
      return tick;
    }
    pair = ctz64(bal(tv == tmin));
    return tmin;
  }

  // Stable counts at the end of the run: the GC actions processed are those
  // before time tc, plus the delivery `pair` (8 from + to) at tc if the run
  // stopped on it
  __device__ __forceinline__ void gc_finish(uint32_t tc, uint32_t pair, unsigned long long* st) {
    const uint32_t gc_ms = prm(P_GC);
    if (gc_lane(lidv() >> 3)) {
      uint32_t* r = gcr(lidv() >> 3, lidv() & 7u);
      r[0] = gf;
      r[1] = gnt;
      r[2] = gkm;
      r[3] = gnc;
    }
    for (uint32_t q = 0; q < n; ++q) {
      // lane p: deliveries p -> q processed, m
      uint32_t m = 0;
      const bool pl = lidv() < n && lidv() != q;
      const uint32_t dq = gather(dpq, (lidv() * 8u + q) & 63u);  // lane p: d(p, q)
      if (pl) {
        const uint32_t d = dq;
        if (tc > d) m = (tc - d - 1u) / gc_ms;
        if (pair == lidv() * 8u + q && tc >= d + gc_ms && (tc - d) % gc_ms == 0) ++m;
      }
      uint32_t stable = 0;
      if (!bal(pl && m == 0)) {
        uint32_t tl = pl ? m * gc_ms + dq : 0u;
        for (uint32_t o = 1; o < 64; o <<= 1) tl = max(tl, (uint32_t)__shfl_xor((int)tl, (int)o));
        tl = uni(tl);
        uint32_t cur = 0;
        bool ok = true;
        if (lidv() < n) ok = gc_value_at(q, lidv(), tl, cur);
        for (uint32_t p = 0; p < n; ++p) {
          if (p == q) continue;
          const uint32_t kl = rl(m, p) - 1u;
          uint32_t v = 0;
          if (lidv() < n) {
            ok = ok && gc_tick_value(p, lidv(), kl, v);
            cur = min(cur, v);
          }
        }
        if (bal(lidv() < n && !ok)) fail_cap(__LINE__);
        for (uint32_t s2 = 0; s2 < n; ++s2) stable += rl(cur, s2);
      }
      if (st && lidv() == 0) st[FX_SIM_STAT_STABLE + q] = stable;
    }
  }

  // ===================================================== GraphExecutor
  // lane bit of a wave-uniform 64-bit mask (no per-lane 64-bit lane mask kept live)
  __device__ __forceinline__ bool mine(uint64_t m) const {
    const uint32_t half = lidv() < 32u ? (uint32_t)m : (uint32_t)(m >> 32);
    return (half >> (lidv() & 31u)) & 1u;
  }
  __device__ __forceinline__ uint32_t vcount_of(uint32_t d) { return uni(S(slot_find(d), SL_CNT)) & 0xFFu; }
  __device__ __forceinline__ uint32_t value_at(uint32_t d, uint32_t j) { return uni(S(slot_find(d), g.sl_value + j)); }

  __device__ __forceinline__ void x_load(uint32_t p) {
    xp = p;
    // the search state is written before it is read in every Add; fixing it
    // here makes its values dead between Adds (no scalar registers held
    // across the event loop)
    root = idc = nfr = missing = fv = fdi = fnc = in_try = emitted = nwl = 0;
    // Tarjan ids are reset at the end of every search (finalize) and the
    // visited marks only matter inside one try_pending: a fresh epoch per call
    stl = 0;
    sfr = 0;
    epoch = 1;
    if constexpr (XPL != 0) {
      pmask = ((1ull << XPL) - 1ull) << (p * XPL);
      occ = bal(sdot != 0u) & pmask;
      wmask = bal(swait != 0u) & pmask;
    } else {
      sdot = rsel(xdot, p); srec = rsel(xrec, p); swait = rsel(xwait, p);
      occ = (uint64_t)rl(pt, PT_OCC + p) | ((uint64_t)rl(pt, PT_OCC + 8u + p) << 32);
      wmask = (uint64_t)rl(pt, PT_WAIT + p) | ((uint64_t)rl(pt, PT_WAIT + 8u + p) << 32);
    }
    xk = rl(pt, PT_EXEC + p);
    tmask = 0;
    phase = PH_IDLE;
  }
  __device__ __forceinline__ void x_store() {
    const uint32_t p = xp;
    if constexpr (XPL != 0) {
      lset(pt, PT_EXEC + p, xk);
      return;
    }
    rput(xdot, p, sdot); rput(xrec, p, srec); rput(xwait, p, swait);
    if ((lidv() & 7u) == p) {
      const uint32_t k = lidv() >> 3;
      if (k == PT_OCC / 8u) pt = (uint32_t)occ;
      else if (k == PT_OCC / 8u + 1u) pt = (uint32_t)(occ >> 32);
      else if (k == PT_WAIT / 8u) pt = (uint32_t)wmask;
      else if (k == PT_WAIT / 8u + 1u) pt = (uint32_t)(wmask >> 32);
      else if (k == PT_EXEC / 8u) pt = xk;
    }
  }

  // AEClock::contains for a per-lane dot / a uniform dot (tarjan.rs:131-132)
  __device__ __forceinline__ bool contains_v(uint32_t d) const {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    const uint32_t ln = (xp * 8u + si) & 63u;
    const uint32_t fr = gather(ecf, ln), w = gather(ecw, ln);
    const uint32_t sq = d & FX_SEQ_MASK, off = sq - fr - 1u;
    return si < n && (sq <= fr || (off < 32u && ((w >> (off & 31u)) & 1u)));
  }
  __device__ __forceinline__ bool contains_u(uint32_t d) const {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) return false;
    const uint32_t fr = rl(ecf, xp * 8u + si), w = rl(ecw, xp * 8u + si);
    const uint32_t sq = d & FX_SEQ_MASK, off = sq - fr - 1u;
    return sq <= fr || (off < 32u && ((w >> off) & 1u));
  }
  // AEClock::add (tarjan.rs:293)
  __device__ __forceinline__ void clk_add(uint32_t d) {
    const uint32_t si = (d >> FX_SEQ_BITS) - 1u;
    if (si >= n) { err = FX_ERR_DOT_RANGE; return; }
    uint32_t fr = rl(ecf, xp * 8u + si), w = rl(ecw, xp * 8u + si);
    const uint32_t sq = d & FX_SEQ_MASK;
    if (sq <= fr) return;
    const uint32_t off = sq - fr - 1u;
    if (off >= 32u) { fail_cap(__LINE__); return; }
    if (off != 0) {
      w |= 1u << off;
    } else {
      const uint32_t win = w >> 1;
      const uint32_t ones = __builtin_ctz(~win);
      fr = fr + 1 + ones;
      w = win >> ones;
    }
    if (lidv() == xp * 8u + si) {
      ecf = fr;
      ecw = w;
    }
  }
  __device__ __forceinline__ int find(uint32_t d) const {
    const uint64_t m = bal(mine(occ) && sdot == d);
    return m ? (int)ctz64(m) : -1;
  }
  __device__ __forceinline__ void new_epoch() {
    epoch = epoch + 1;
    if (epoch > EPOCH_MAX) {
      if (mine(occ)) stl = tmk(tid(stl), tlow(stl), 0);
      epoch = 1;
    }
  }

  // one executed command: to_execute -> Command::execute -> to_clients ->
  // AggregatePending (runner.rs:406-424), executor metrics, execution log
  __device__ __forceinline__ void on_execute(uint32_t d, uint32_t start) {
    const uint32_t p = xp;
    // lane reads (prm, rl) only outside lane-divergent code: a VGPR the
    // compiler reloads or copies under a partial exec mask holds garbage in the
    // inactive lanes
    const uint32_t inst = prm(P_INST);
    if (lidv() == 0) {
      KSimArgs* k = kargs();
      if (xk < k->exec_cap && k->executed) k->executed[((size_t)inst * n + p) * k->exec_cap + xk] = d;
    }
    ++xk;
    const uint32_t delay = now - start;  // ExecutionDelay (graph/mod.rs:514-518)
    hist_delay(delay);
    const uint32_t sl = slot_find(d);
    if (sl == NONE) { fail_late(__LINE__); return; }
    const uint32_t c = uni(S(sl, SL_CLIENT));
    const uint32_t nk = (uni(S(sl, SL_CNT)) >> 20) & 3u;
    if ((rl(ca, c) & 0xFFu) == p) {  // pending.wait_for registered this rifl at p
      const uint32_t pend = rl(cb, 32u + c);
      if (pend < nk) { fail_late(__LINE__); return; }
      lset(cb, 32u + c, pend - nk);  // one ExecutorResult per key
      if (pend == nk) {
        const uint32_t fi = nfrm - 1;
        const uint32_t w = rl(frw, fi);
        const uint32_t nr = (w >> 20) & 31u;
        if (nr >= g.rdm) { fail_cap(__LINE__); return; }
        put(FRR(fi, nr), c);
        lset(frw, fi, w + (1u << 20));
      }
    }
    const uint32_t masks = uni(S(sl, SL_MASKS));
    if (((masks >> 24) & 0xFFu) + 1u == n) {
      slot_set(sl, 0u);  // executed everywhere: free the slot
    } else {
      put(S(sl, SL_MASKS), masks + (1u << 24));
    }
  }

  __device__ __forceinline__ void emit_one(uint32_t d, uint32_t start) {
    hist_chain(1u);
    clk_add(d);
    on_execute(d, start);
  }

  __device__ __forceinline__ int insert_vertex(uint32_t d) {
    const uint64_t fre = ~occ & pmask;
    if (!fre) { fail_cap(__LINE__); return -1; }
    const uint32_t sl = ctz64(fre);
    if (lidv() == sl) {
      sdot = d;
      srec = now;  // Vertex::start_time_ms (tarjan.rs:332-348)
      swait = 0;
      stl = 0;
    }
    occ |= 1ull << sl;
    return (int)sl;
  }

  __device__ __forceinline__ void dfs_start(uint32_t r, bool intry) {
    root = r;
    in_try = intry;
    emitted = 0;
    missing = 0;
    idc = 1;
    const uint32_t tr = rl(stl, r);
    if (lidv() == r) stl = tmk(1, 1, tep(tr));
    nfr = 0;
    fv = r;
    fdi = 0;
    fnc = vcount_of(rl(sdot, r));
    phase = PH_DFS;
  }

  // SCC rooted at fv: stack vertices with id >= id(fv), saved in ascending
  // dot order (SCC = BTreeSet<Dot>, tarjan.rs:15)
  __device__ __forceinline__ void save_scc() {
    const uint32_t idv = tid(rl(stl, fv));
    const bool mem = mine(occ) && tid(stl) >= idv;
    const uint64_t mm = bal(mem);
    const uint32_t cnt = pop64(mm);
    if (nwl + cnt > 65u) { fail_cap(__LINE__); return; }
    hist_chain(cnt);
    uint32_t rank = 0;
    for (uint64_t m = mm; m; m &= m - 1) rank += rl(sdot, ctz64(m)) < sdot ? 1u : 0u;
    for (uint32_t r = 0; r < cnt; ++r) {
      const uint32_t lr = ctz64(bal(mem && rank == r));
      const uint32_t d = rl(sdot, lr);
      const uint32_t st = rl(srec, lr);
      put(wl(nwl + r), d);
      clk_add(d);
      on_execute(d, st);
      if (err) return;
    }
    nwl += cnt;
    if constexpr (XPL != 0) {
      if (mem) {  // the slots are free again
        sdot = 0;
        swait = 0;
      }
    }
    occ &= ~mm;
    wmask &= ~mm;
    tmask &= ~mm;
    emitted = 1;
  }

  __device__ __forceinline__ void dfs_finish() {
    // finalize (tarjan.rs:60-93); in try_pending a failed search that saved no
    // SCC marks the stack vertices visited (mod.rs:621-629)
    const bool mark = in_try && missing != 0 && !emitted;
    if (mine(occ) && tid(stl) != 0) stl = tmk(0, 0, mark ? epoch : tep(stl));
    if (missing) {  // index_pending (mod.rs:525-554)
      if (lidv() == root) swait = missing;
      wmask |= 1ull << root;
    }
    if (in_try) {
      if (!missing || emitted) new_epoch();
      phase = PH_TRY;
    } else {
      phase = PH_CHECK;
    }
  }

  // one DFS edge or one frame pop (TarjanSCCFinder::strong_connect, iterative)
  __device__ __forceinline__ void dfs_iter() {
    if (fdi < fnc) {
      const uint32_t vd = rl(sdot, fv);
      const uint32_t dep = value_at(vd, fdi);
      ++fdi;
      if (dep == vd || contains_u(dep)) return;  // self or executed (tarjan.rs:128-145)
      const int x = find(dep);
      if (x < 0) {  // missing (tarjan.rs:148-157, shard_count == 1)
        missing = dep;
        dfs_finish();
        return;
      }
      const uint32_t tx = rl(stl, (uint32_t)x);
      if (tid(tx) == 0) {  // recurse (tarjan.rs:172-214)
        ++idc;
        if (idc > 127u) { fail_cap(__LINE__); return; }
        if (lidv() == (uint32_t)x) stl = tmk(idc, idc, tep(tx));
        if (lidv() == nfr) sfr = fv | (fdi << 8);
        ++nfr;
        fv = (uint32_t)x;
        fdi = 0;
        fnc = vcount_of(rl(sdot, fv));
      } else {  // on the stack (tarjan.rs:215-225)
        const uint32_t tv = rl(stl, fv);
        if (tid(tx) < tlow(tv) && lidv() == fv) stl = tmk(tid(tv), tid(tx), tep(tv));
      }
    } else {
      const uint32_t tv = rl(stl, fv);
      const uint32_t lowv = tlow(tv);
      if (tid(tv) == lowv) {  // SCC root (tarjan.rs:233-312)
        save_scc();
        if (err) return;
      }
      if (nfr == 0) {
        dfs_finish();
        return;
      }
      --nfr;
      const uint32_t fw = rl(sfr, nfr);
      fv = fw & 0xFFu;
      fdi = fw >> 8;
      fnc = vcount_of(rl(sdot, fv));
      const uint32_t tp = rl(stl, fv);
      if (lowv < tlow(tp) && lidv() == fv) stl = tmk(tid(tp), lowv, tep(tp));
    }
  }

  // try_pending (mod.rs:589-642): next waiter, ascending (C2)
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
    if (tep(rl(stl, best)) == epoch) return;
    dfs_start(best, true);
  }

  // check_pending (mod.rs:556-587): LIFO over released dots
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
    wmask &= ~t;
    if constexpr (XPL != 0) {
      if (mine(t)) swait = 0;
    }
    tmask = t;
    new_epoch();
    phase = PH_TRY;
  }

  // GraphExecutor::handle(Add) (executor.rs:69-80) -> handle_add (mod.rs:213-275)
  __device__ __forceinline__ void x_add(uint32_t p, uint32_t d) {
    PROF_T0();
    x_load(p);
    nwl = 0;
    if (find(d) >= 0) { err = FX_ERR_DOUBLE_INDEX; x_store(); return; }
    const uint32_t vc = vcount_of(d);
    deps_total += vc;
    const uint32_t dsl = slot_find(d);
    const uint32_t depj = lidv() < vc ? S(dsl, g.sl_value + lidv()) : 0u;
    // the clock gather runs with every lane active: ds_bpermute reads 0 from a
    // lane that is inactive, and the clock words sit in lanes 8 p + s, mostly
    // outside [0, vc) (inside `&&` the call would run in the masked branch)
    const bool exd = contains_v(depj);
    const bool keep = lidv() < vc && depj != d && !exd;
    PROF_ADD(5);
    if (!bal(keep)) {  // fast path: a singleton SCC
#ifdef FX_SIM_PROFILE
      const uint64_t pe0 = __builtin_amdgcn_s_memtime();
#endif
      emit_one(d, now);
#ifdef FX_SIM_PROFILE
      prof[13] += __builtin_amdgcn_s_memtime() - pe0;
      prof[21] += 1;
#endif
      if (wmask && !err) {
        put(wl(0), d);
        nwl = 1;
        phase = PH_CHECK;
      }
    } else {
      const int sl = insert_vertex(d);
      if (sl >= 0) dfs_start((uint32_t)sl, false);
    }
    uint32_t guard = 0;
    while (phase != PH_IDLE && !err) {
      if (phase == PH_DFS) dfs_iter();
      else if (phase == PH_TRY) try_iter();
      else check_iter();
      if (++guard > (1u << 22)) fail_cap(__LINE__);
    }
#ifdef FX_SIM_PROFILE
    const uint64_t ps0 = __builtin_amdgcn_s_memtime();
#endif
    x_store();
#ifdef FX_SIM_PROFILE
    prof[14] += __builtin_amdgcn_s_memtime() - ps0;
    prof[22] += 1;
#endif
  }

  // =========================================== send_to_processes_and_executors
  __device__ __forceinline__ void frame_push() {
    if (nfrm >= FMAX) { fail_cap(__LINE__); return; }
    const uint32_t fi = nfrm++;
    lset(frw, fi, 0);
    xinfo = 0;
  }

  // handle_send_to_proc(from, p, msg) / handle_submit_to_proc, each followed
  // by send_to_processes_and_executors(p) (runner.rs:351-377, 395-488), with
  // every self-delivery they cause, in the reference's recursion order.  One
  // call site for the handlers and one for the executor keep the inlined
  // kernel small: the loop either runs the pending handler (pushing its frame
  // and running the executor on what it committed), or advances the top
  // frame's action, or schedules the frame's ready results and pops it.
  __device__ __forceinline__ void run_handlers(uint32_t p, uint32_t from, uint32_t kind, uint32_t w2) {
    PROF_T0();
    run_handlers_(p, from, kind, w2);
    PROF_ADD(7);
  }
  __device__ __forceinline__ void run_handlers_(uint32_t p, uint32_t from, uint32_t kind, uint32_t w2) {
    bool pend = true;
    uint32_t guard = 0;
    while (!err) {
      if (++guard > 4096u) { fail_cap(__LINE__); return; }
      if (pend) {
        pend = false;
        frame_push();
        if (err) return;
        PROF_T0();
        switch (kind) {
          case M_SUBMIT: h_submit(p, w2); break;
          case M_COLLECT: h_mcollect(p, from, w2); break;
          case M_COLLECT_ACK: h_mcollectack(p, from, w2); break;
          case M_COMMIT: h_mcommit(p, from, w2); break;
          case M_CONSENSUS: h_mconsensus(p, from, w2); break;
          case M_CONSENSUS_ACK: h_mconsensusack(p, from, w2); break;
          default:
            if constexpr (!GP::fixed) {
              if (kind == M_STORE) { h_mstore(p, from, w2); break; }
              if (kind == M_STORE_ACK) { h_mstoreack(p, from, w2); break; }
              if (kind == M_COMMIT_BASIC) { h_bcommit(p, w2); break; }
            }
            err = FX_ERR_INVALID_ARG;
        }
#ifdef FX_SIM_PROFILE
        prof[8 + min(kind, 7u)] += __builtin_amdgcn_s_memtime() - prof_t0_;
        prof[16 + min(kind, 7u)] += 1;
#endif
        if (xinfo && !err) {  // to_executors (<= 1 per handler), LIFO
          const uint32_t d = xinfo;
          xinfo = 0;
          PROF_T0();
          x_add(p, d);
          PROF_ADD(2);
        }
        continue;
      }
      if (nfrm == 0) return;
      const uint32_t fi = nfrm - 1;
      const uint32_t w = rl(frw, fi);
      if (w & 3u) {  // ToSend: targets ascending (C4), self recurses in place
        const uint32_t tgt = (w >> 8) & 0xFFu, k2 = (w >> 2) & 15u, dot = rl(frd, fi);
        const uint32_t nx = (w >> 16) & 15u;
        // the targets before the self-delivery (or all of them) in one batch
        const bool self = ((tgt >> p) & 1u) && p >= nx;
        const uint32_t hi = self ? p : n;
        send_batch(p, tgt & ((1u << hi) - 1u) & ~((1u << nx) - 1u) & ~(1u << p), k2, dot);
        if (err) return;
        if (self) {
          lset(frw, fi, (w & ~(15u << 16)) | ((p + 1u) << 16));
          from = p;
          kind = k2;
          w2 = dot;
          pend = true;
          continue;
        }
      }
      // ready results -> schedule_to_client (runner.rs:434-440)
      const uint32_t nr = (w >> 20) & 31u;
      for (uint32_t r = 0; r < nr; ++r) {
        const uint32_t c = uni(FRR(fi, r));
        schedule_timer(link_r(c), rl(cd, 32u + c));
      }
      --nfrm;
    }
  }

  // ======================================================= event loop
  // Client::cmd_send: next command of client c (0-based) -> SubmitToProc
  __device__ __forceinline__ bool client_send(uint32_t c) {
    const uint32_t issued = rl(ca, 32u + c);
    if (issued >= prm(P_CMDS)) return false;
    lset(ca, 32u + c, issued + 1u);
    lset(cb, c, now);  // Pending::start
    schedule_timer(link_s(c), rl(cd, c));
    return true;
  }

  __device__ __forceinline__ void run_event(uint32_t link) {
    if (link < g.NP) {  // P(p, q): SendToProc
      const uint32_t p = link / (g.n - 1u), qi = link % (g.n - 1u);
      const uint32_t q = qi < p ? qi : qi + 1u;
      const uint32_t ht_ = rl(rhv, link);
      const uint32_t e = ht_ & 0xFFFFu, tail = ht_ >> 16;
      const uint32_t w0 = uni(msg(e, 0)), w2 = uni(msg(e, 2)), nx = uni(msg(e, 3));
      const uint32_t kind = w0 >> 28;
      put(lds[g.off_free + nfree++], e);
      if (nx != LNIL) {
        lset(rhv, link, nx | (tail << 16));
        head_set(link, uni(msg(nx, 0)) & 0x0FFFFFFFu, uni(msg(nx, 1)));
      } else {
        lset(rhv, link, 0xFFFFFFFFu);
        head_set(link, NONE, NONE);
      }
      note(3, q + 1, p + 1, ((uint64_t)kind << 32) | w2);
      run_handlers(q, p, kind, w2);
      return;
    }
    uint32_t x = link - g.NP;
    if (x < g.n) {  // E(p): executed notification (a no-op for the GraphExecutor)
      schedule_timer(link_e(x), prm(P_EN));
      return;
    }
    x -= g.n;
    if (x < g.C) {  // S(c): SubmitToProc
      const uint32_t c = x;
      head_set(link, NONE, NONE);
      const uint32_t p = rl(ca, c) & 0xFFu;
      note(2, p + 1, c + 1, rl(ca, 32u + c));
      lset(cb, 32u + c, g.K);  // AggregatePending::wait_for: key_count results
      run_handlers(p, p, M_SUBMIT, c);
      return;
    }
    x -= g.C;
    PROF_T0();
    {  // R(c): SendToClient -> Client::cmd_recv + cmd_send (simulation.rs:132-149)
      const uint32_t c = x;
      head_set(link, NONE, NONE);
      const uint32_t issued = rl(ca, 32u + c);
      note(4, c + 1, 0, issued);
      const uint32_t lat = now - rl(cb, c);  // latency.as_millis()
      lat_sum += lat;
      const uint32_t region = rl(ca, c) >> 8;
      const uint32_t inst = prm(P_INST);
      if (lidv() == 0) {
        KSimArgs* k = kargs();
        if (k->latency_log && issued - 1u < k->lat_cap)
          k->latency_log[((size_t)inst * g.C + c) * k->lat_cap + issued - 1u] = lat;
      }
      hist_lat(region, lat);
      if (!client_send(c)) {
        const uint32_t cdone = prm(P_CDONE) + 1u;
        prm_set(P_CDONE, cdone);
        if (cdone == g.C) {
          if (prm(P_HAS_EXTRA)) {
            prm_set(P_FINAL, now + prm(P_EXTRA));
            in_extra = true;
          } else {
            done = true;
          }
        }
      }
    }
    PROF_ADD(4);
  }

  // wave-wide min over the link heads, (time, seq) lexicographic: each lane's
  // local minimum, then two DPP min-scans (time, then seq among the lanes at
  // that time); the link is unique because insertion seqs are
  __device__ __forceinline__ static uint32_t dpp_min(uint32_t v) {
    // inclusive min-scan over the wavefront (row_shr 1/2/4/8, row_bcast 15/31);
    // lane 63 ends with the minimum
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x111, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x112, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x114, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x118, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x142, 0xA, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x143, 0xC, 0xF, false));
    return rl(v, 63);
  }
  __device__ __forceinline__ uint32_t pop_min(uint32_t& t_out) {
    uint32_t bt = ht[0], bs = hs[0], bk = 0;
#pragma unroll
    for (uint32_t k = 1; k < HM; ++k) {
      const bool lt = ht[k] < bt || (ht[k] == bt && hs[k] < bs);
      bt = lt ? ht[k] : bt;
      bs = lt ? hs[k] : bs;
      bk = lt ? k : bk;
    }
    const uint32_t tmin = dpp_min(bt);
    const uint32_t smin = dpp_min(bt == tmin ? bs : NONE);
    t_out = tmin;
    if (tmin == NONE) return NONE;
    const uint64_t w = bal(bt == tmin && bs == smin);
    const uint32_t l = ctz64(w);
    return rl(bk, l) * 64u + l;
  }
};

// WPS = waves per SIMD the register budget targets: 4 for launches whose LDS
// lets 16 instances share a CU (the default configs[1] geometry: 10.0 KB at
// n = 5 — 4 waves issue more of the scalar unit's slots than 3 even with a few
// spilled registers, +14 %), 3 otherwise, 2 for the 256-slot dot tables
// WPB: instances per workgroup (a CU holds at most 16 workgroups; each
// instance's wavefront works on its own LDS block, no workgroup barrier)
template <uint32_t HM, uint32_t DS, uint32_t WPS, uint32_t NX, class GP = GeoRT, uint32_t WPB = 1>
__global__ __launch_bounds__(64 * WPB, WPS) void k_sim(SimArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_all[];
  const uint32_t wv = WPB > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0u;
  const uint32_t inst = blockIdx.x * WPB + wv;
  if (inst >= a.instances) return;  // whole wavefront
  Sim<HM, DS, NX, GP> s;
#pragma unroll
  for (uint32_t k = 0; k < DS; ++k) s.sdv[k] = 0;
  s.lid_ = threadIdx.x & 63u;
  s.trace = ((uint64_t)vdiv(0) << 32) | vdiv(0);
  s.deps_total = s.trace;
  s.lat_sum = s.trace;
  if constexpr (!GP::fixed) s.g = a.g;
  uint32_t* smem = smem_all + wv * s.g.words;  // this instance's block (g.words per instance)
  s.lds = smem;
  const fx_sim_spec& sp = a.specs[inst];
  s.protocol = GP::fixed ? GP::proto : sp.protocol;
  s.n = s.g.n;
  s.f = GP::fc != FANY ? GP::fc : sp.f;
  s.C = s.g.C;
  const bool has_extra = sp.extra_sim_time_ms >= 0;
  {
    const uint32_t l = s.lidv();
    uint32_t v = 0;
    v = l == Sim<HM, DS, NX, GP>::P_SEED ? (uint32_t)sp.seed : v;
    v = l == Sim<HM, DS, NX, GP>::P_SEED + 1 ? (uint32_t)(sp.seed >> 32) : v;
    v = l == Sim<HM, DS, NX, GP>::P_RNG ? (uint32_t)sp.instance : v;
    v = l == Sim<HM, DS, NX, GP>::P_RNG + 1 ? (uint32_t)(sp.instance >> 32) : v;
    v = l == Sim<HM, DS, NX, GP>::P_GC ? sp.gc_interval_ms : v;
    v = l == Sim<HM, DS, NX, GP>::P_EN ? sp.executed_notification_ms : v;
    v = l == Sim<HM, DS, NX, GP>::P_CMDS ? sp.commands_per_client : v;
    v = l == Sim<HM, DS, NX, GP>::P_CONFLICT ? sp.conflict_rate : v;
    v = l == Sim<HM, DS, NX, GP>::P_POOL ? sp.pool_size : v;
    v = l == Sim<HM, DS, NX, GP>::P_EXTRA ? (has_extra ? (uint32_t)sp.extra_sim_time_ms : 0u) : v;
    v = l == Sim<HM, DS, NX, GP>::P_HAS_EXTRA ? (has_extra ? 1u : 0u) : v;
    v = l == Sim<HM, DS, NX, GP>::P_INST ? inst : v;
    s.pv = v;
  }
  const uint32_t gc_ms = sp.gc_interval_ms, en_ms = sp.executed_notification_ms;
  const uint32_t n = s.n;
  if (s.protocol == FX_PROTOCOL_ATLAS) {
    s.fq = n / 2 + s.f;
    s.wq = s.f + 1;
    s.synod_f = s.f;
  } else if (!GP::fixed && s.protocol == FX_PROTOCOL_BASIC) {
    s.fq = s.f + 1;  // basic_quorum_size (config.rs:285-287); no write quorum
    s.wq = 0;
    s.synod_f = 0;
  } else {
    const uint32_t fe = n / 2;
    s.fq = fe + (fe + 1) / 2;
    s.wq = fe + 1;
    s.synod_f = fe;  // EPaxos::allowed_faults
  }
  // ---------------------------------------------------------------- init
  for (uint32_t i = s.lidv(); i < s.g.words; i += 64) smem[i] = 0;
  for (uint32_t i = s.lidv(); i < s.g.R; i += 64) smem[s.g.off_free + i] = s.g.R - 1u - i;  // free stack
  s.nfree = s.g.R;
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (uint32_t k = 0; k < HM; ++k) s.ht[k] = s.hs[k] = NONE;
#pragma unroll
  for (uint32_t k = 0; k < NX; ++k) s.xdot[k] = s.xrec[k] = s.xwait[k] = 0;
  s.sdot = s.srec = s.swait = 0;
  const uint32_t RP = a.RP;
  // process regions, quorums (BaseProcess::discover over
  // sort_processes_by_distance, base.rs:62-154, util.rs:153-185)
  for (uint32_t p = 0; p < n; ++p) {
    const uint32_t rp = sp.process_regions[p];
    // lane q < n: position of process q in p's distance order
    uint32_t pos = 0;
    if (s.lidv() < n) {
      const uint32_t rq = sp.process_regions[s.lidv()];
      const uint32_t kq = a.rank[rp * RP + rq];
      for (uint32_t q2 = 0; q2 < n; ++q2) {
        const uint32_t r2 = sp.process_regions[q2];
        const uint32_t k2 = a.rank[rp * RP + r2];
        if (k2 < kq || (k2 == kq && q2 < s.lidv())) ++pos;
      }
    }
    const uint32_t fqm = (uint32_t)bal(s.lidv() < n && pos < s.fq);
    const uint32_t wqm = (uint32_t)bal(s.lidv() < n && pos < s.wq);
    s.lset(s.pq, p, fqm | (wqm << 8));
    if (s.lidv() >= p * 8u && s.lidv() < p * 8u + n) s.dpq = a.ping[rp * RP + sp.process_regions[s.lidv() - p * 8u]] / 2u;
  }
  // clients: for region in client_regions, clients_per_region each (runner.rs:143-163)
  {
    uint32_t c = 0;
    for (uint32_t r = 0; r < sp.num_client_regions; ++r) {
      const uint32_t rc = sp.client_regions[r];
      // closest process: minimal (rank, id)
      uint32_t best = 0, bk = 0xFFFFFFFFu;
      for (uint32_t p = 0; p < n; ++p) {
        const uint32_t k = a.rank[rc * RP + sp.process_regions[p]];
        if (k < bk) {
          bk = k;
          best = p;
        }
      }
      for (uint32_t i = 0; i < sp.clients_per_region; ++i, ++c) {
        if (s.lidv() == c) {
          s.ca = best | (rc << 8);
          s.cd = a.ping[rc * RP + sp.process_regions[best]] / 2u;
        }
        if (s.lidv() == 32u + c) s.cd = a.ping[sp.process_regions[best] * RP + rc] / 2u;
      }
    }
  }
  __builtin_amdgcn_s_barrier();
  // periodic events (runner.rs:179-187), then clients (run(), C5 ascending)
  // (the periodic GC events are evaluated in gc_finish; their insertion
  // seqs only shift the numbering, C3)
  const bool sim_en = a.sim_exec_notif || has_extra;
  for (uint32_t p = 0; p < n; ++p) {
    if (sim_en) s.schedule_timer(s.link_e(p), en_ms);
    else ++s.seq;  // keep the insertion numbering of the reference
  }
  for (uint32_t c = 0; c < s.C; ++c) {
    s.client_send(c);
    if (sp.commands_per_client == 0) s.err = FX_ERR_INVALID_ARG;
  }
  // ------------------------------------------------------------ loop
  const uint32_t max_events = a.max_events ? a.max_events : 0xFFFFFFFFu;
  uint32_t gc_pair = NONE;
  while (!s.done && !s.err) {
    uint32_t t = 0;
#ifdef FX_SIM_PROFILE
    const uint64_t pt0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t link = s.pop_min(t);
#ifdef FX_SIM_PROFILE
    const uint64_t pt1 = __builtin_amdgcn_s_memtime();
    s.prof[0] += pt1 - pt0;
#endif
    if (link == NONE || t == NONE) {
      s.err = FX_ERR_SIM_LATE;  // "there should be a new action"
      break;
    }
    if (t < s.now) {
      s.err = FX_ERR_TIME_RANGE;
      break;
    }
    if (s.in_extra && t > s.prm(s.P_FINAL) && gc_ms) {
      // the run stops at the first action after final_ms: a GC action
      // before t (C3: at t, t's other actions go first) ends it instead
      uint32_t pair = NONE;
      const uint32_t tg = s.gc_next_after(s.prm(s.P_FINAL), pair);
      if (tg < t) {
        s.now = tg;
        gc_pair = pair;
        break;
      }
    }
    s.now = t;
    s.run_event(link);
#ifdef FX_SIM_PROFILE
    s.prof[1] += __builtin_amdgcn_s_memtime() - pt1;
#endif
    if (s.in_extra && s.now > s.prm(s.P_FINAL)) s.done = true;
    if (s.events >= max_events) s.err = FX_ERR_SIM_EVENTS;
  }
  // ----------------------------------------------------------- outputs
  __builtin_amdgcn_s_barrier();
  const uint32_t o_exec = gather(s.pt, (PT_EXEC + s.lidv()) & 63u), o_fast = gather(s.pt, (PT_FAST + s.lidv()) & 63u),
                 o_slow = gather(s.pt, (PT_SLOW + s.lidv()) & 63u);
  if (s.lidv() < n && a.executed_len) a.executed_len[(size_t)inst * n + s.lidv()] = o_exec;
  if (a.stats) {
    unsigned long long* st = a.stats + (size_t)inst * FX_SIM_STATS;
    if (s.lidv() < NMAX) {
      const bool v = s.lidv() < n;
      st[FX_SIM_STAT_FAST + s.lidv()] = v ? o_fast : 0u;
      st[FX_SIM_STAT_SLOW + s.lidv()] = v ? o_slow : 0u;
      st[FX_SIM_STAT_STABLE + s.lidv()] = 0u;
      st[FX_SIM_STAT_FAST_READS + s.lidv()] = 0u;  // no read-only commands on this kernel
      st[FX_SIM_STAT_SLOW_READS + s.lidv()] = 0u;
    }
    if (gc_ms && !s.err) s.gc_finish(s.now, gc_pair, st);
    const uint32_t err_site = s.prm(s.P_ERRSITE);
    if (s.lidv() == 0) {
      st[FX_SIM_STAT_EVENTS] = s.events;
#ifdef FX_SIM_PROFILE
      for (uint32_t i = 0; i < 24; ++i) st[i] = s.prof[i];
#endif
      st[FX_SIM_STAT_END_MS] = s.now;
      st[FX_SIM_STAT_TRACE] = s.trace;
      st[FX_SIM_STAT_SEQ] = s.seq;
      st[FX_SIM_STAT_DEPS] = s.deps_total;
      st[FX_SIM_STAT_LAT_SUM] = s.lat_sum;
      st[FX_SIM_STAT_ERR_SITE] = err_site;
    }
  }
  // the instance's histogram counts held in lanes (exact: a sample either
  // went there or straight to its global bin), clamped into the bins here
  if (s.hcv && a.chain_hist) atomicAdd(&a.chain_hist[min(s.lidv(), a.chain_bins - 1u)], (unsigned long long)s.hcv);
  for (uint32_t i = s.lidv(); i < HD_BINS; i += 64) {
    const uint32_t c = smem[s.g.off_hist + i];
    if (c && a.delay_hist) atomicAdd(&a.delay_hist[min(i, a.delay_bins - 1u)], (unsigned long long)c);
  }
  if (s.hlk && a.lat_hist) {
    const uint32_t key = s.hlk - 1u, lat = key & 0xFFFFFFu;
    atomicAdd(&a.lat_hist[(key >> 24) * a.lat_bins + min(lat, a.lat_bins - 1u)], (unsigned long long)s.hlc);
  }
  if (s.lidv() == 0) a.err[inst] = s.err;
}

}  // namespace sim

using namespace sim;

// the large-instance kernel (sim_big.hip)
size_t simx_arena_bytes(const fx_sim_spec& sp, uint32_t ring, uint32_t dots);
bool simx_table_sizes(const fx_sim_spec& sp, uint32_t ring, uint32_t dots, uint32_t* R, uint32_t* NS);
int simx_launch(const fx_sim_batch* b, const fx_sim_output* o, hipStream_t hs);

// the fixed-geometry builds: BASELINE configs[1] (EPaxos n = 5 f = 2, one
// client in each of the 5 process regions) and configs[0] (Atlas n = 3 f = 1)
using GeoC1 = GeoCT<FX_PROTOCOL_EPAXOS, 5, 2, 5>;
#ifdef FX_XSWAP
constexpr uint32_t XNX = 5;
#else
constexpr uint32_t XNX = 1;
#endif
using GeoC0 = GeoCT<FX_PROTOCOL_ATLAS, 3, 1, 3>;
// configs[2]: Atlas over region subsets, one client per region, f = 1 and 2
// in one batch (f per instance)
using GeoC2a = GeoCT<FX_PROTOCOL_ATLAS, 5, FANY, 5>;
using GeoC2b = GeoCT<FX_PROTOCOL_ATLAS, 7, FANY, 7>;
template <class GP>
static bool geo_is(const Geo& g, const fx_sim_spec& s0) {
  const Geo c = GP::g;
  return s0.protocol == GP::proto && (GP::fc == FANY || s0.f == GP::fc) && std::memcmp(&g, &c, sizeof(Geo)) == 0;
}

static bool sim_geometry(const fx_sim_spec& sp, uint32_t ring, uint32_t wslots, Geo& g) {
  return geo_make(sp.n, sp.clients_per_region * sp.num_client_regions, sp.keys_per_command, sp.pool_size, ring,
                  wslots, g);
}

}  // namespace fx

using namespace fx;

extern "C" {

int fx_sim_plan(const fx_sim_spec* sp, uint32_t ring_entries, uint32_t dot_slots, uint32_t* lds_bytes) {
  if (!sp || !lds_bytes) return FX_ERR_INVALID_ARG;
  Geo g;
  if (!sim_geometry(*sp, ring_entries, dot_slots, g)) return FX_ERR_UNSUPPORTED;
  *lds_bytes = g.words * 4;
  return FX_OK;
}

int fx_sim_plan_large(const fx_sim_spec* sp, uint32_t ring_entries, uint32_t dot_slots, uint64_t* arena_bytes) {
  if (!sp || !arena_bytes) return FX_ERR_INVALID_ARG;
  const size_t b = simx_arena_bytes(*sp, ring_entries, dot_slots);
  if (!b) return FX_ERR_UNSUPPORTED;
  *arena_bytes = b;
  return FX_OK;
}

int fx_sim_run(const fx_sim_batch* b, const fx_sim_output* o, void* hip_stream) {
  if (!b || !o || !b->specs || !b->host_specs || !o->err || !b->planet_ping || !b->planet_rank) return FX_ERR_INVALID_ARG;
  if (b->instances == 0) return FX_OK;
  int dc = 0;
  if (hipGetDeviceCount(&dc) != hipSuccess || dc <= 0) return FX_ERR_NO_DEVICE;
  const uint32_t ring = b->ring_entries;  // 0 = the default of the kernel's geometry
  const uint32_t W = b->dot_slots;
  if (ring > 65534 || W > 8u * 65536u) return FX_ERR_INVALID_ARG;
  const fx_sim_spec& s0 = b->host_specs[0];
  // the all-on-chip kernel unless the batch needs the large-instance one
  bool large = (b->flags & FX_SIM_FLAG_LARGE) != 0 || W > 256;
  // one protocol and f over the batch: a fixed-geometry build may take it
  bool one_p = true, one_f = true;
  // every instance of a launch shares the geometry (protocol, n, clients, keys)
  for (uint32_t i = 0; i < b->instances; ++i) {
    const fx_sim_spec& s = b->host_specs[i];
    if (s.protocol != s0.protocol) one_p = false;
    if (s.f != s0.f) one_f = false;
    if (s.protocol != FX_PROTOCOL_ATLAS && s.protocol != FX_PROTOCOL_EPAXOS && s.protocol != FX_PROTOCOL_BASIC)
      return FX_ERR_UNSUPPORTED;
    if (s.n != s0.n || s.clients_per_region != s0.clients_per_region ||
        s.num_client_regions != s0.num_client_regions || s.keys_per_command != s0.keys_per_command ||
        s.pool_size != s0.pool_size)
      return FX_ERR_INVALID_ARG;
    if (s.read_only_pct > 100) return FX_ERR_INVALID_ARG;
    if (s.read_only_pct != 0 || s.reorder_messages || s.nfr) large = true;
    if (s.keys_per_command < 1 || s.keys_per_command > KMAX || s.pool_size < 1) return FX_ERR_INVALID_ARG;
    if (s.f > s.n / 2) return FX_ERR_INVALID_ARG;
    if (s.keys_per_command == 2 && s.conflict_rate >= 100) return FX_ERR_INVALID_ARG;  // workload.rs:49-51
    // two distinct keys from {client key} U pool: the reference's draw loop never ends
    if (s.keys_per_command == 2 && s.conflict_rate == 0) return FX_ERR_INVALID_ARG;
    for (uint32_t p = 0; p < s.n; ++p)
      if (s.process_regions[p] >= b->planet_regions) return FX_ERR_INVALID_ARG;
    for (uint32_t r = 0; r < s.num_client_regions; ++r)
      if (s.client_regions[r] >= b->planet_regions) return FX_ERR_INVALID_ARG;
    if (s.executed_notification_ms == 0 && s.extra_sim_time_ms >= 0) return FX_ERR_INVALID_ARG;
  }
  SimArgs a{};
  if (!large && (!sim_geometry(s0, ring, W, a.g) || (size_t)a.g.words * 4 > 160 * 1024 || a.g.ncli_keys > 0xFFFFu))
    large = true;
  if (large) {
    if (s0.pool_size + s0.clients_per_region * s0.num_client_regions + 1 > 0xFFFFu) return FX_ERR_UNSUPPORTED;
    return simx_launch(b, o, (hipStream_t)hip_stream);
  }
  const size_t lds = (size_t)a.g.words * 4;
  a.specs = b->specs;
  a.instances = b->instances;
  a.ping = b->planet_ping;
  a.rank = b->planet_rank;
  a.RP = b->planet_stride;
  a.exec_cap = b->exec_cap;
  a.lat_cap = b->lat_cap;
  a.max_events = b->max_events;
  a.sim_exec_notif = b->flags & FX_SIM_FLAG_EXEC_NOTIFICATIONS;
  a.executed = o->executed;
  a.executed_len = o->executed_len;
  a.latency_log = o->latency_log;
  a.lat_hist = (unsigned long long*)o->latency_hist;
  a.lat_bins = o->lat_bins ? o->lat_bins : 1;
  a.chain_hist = (unsigned long long*)o->chain_hist;
  a.chain_bins = o->chain_bins ? o->chain_bins : 1;
  a.delay_hist = (unsigned long long*)o->delay_hist;
  a.delay_bins = o->delay_bins ? o->delay_bins : 1;
  a.stats = (unsigned long long*)o->stats;
  a.err = o->err;
  a.dot_client = o->dot_client;
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 4, 5>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 4, NMAX>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 3, NMAX>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<2, 1, 3, NMAX>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 4, 2, NMAX>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<2, 4, 2, NMAX>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 4, XNX, GeoC1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 5, XNX, GeoC1, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 5, 1, GeoC2a>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 4, 1, GeoC2a>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 3, 1, GeoC2b>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void*)sim::k_sim<1, 1, 4, 1, GeoC0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    configured = true;
  }
  // link heads per lane: one when every link fits a lane
  // and one dot-table VGPR when the pool fits a lane each
  const dim3 grid(b->instances), block(64);
  hipStream_t hs = (hipStream_t)hip_stream;
  const bool four = lds <= 160u * 1024u / 16u;  // 16 instances per CU: 4 waves per SIMD
  // the BASELINE geometries compiled in (same results as the run-time build)
  const bool fixed_ok = one_p && !(b->flags & FX_SIM_FLAG_GENERIC) && a.g.L <= 64;
  // 5 waves per SIMD (a 102-VGPR budget) for the compiled-in configs[1] / [2]
  // n = 5 geometry (8,192 B of LDS) is opt-in: a CU holds at most 16
  // single-wave workgroups, so it still runs 4 per SIMD, with more spills
  // (configs[1] 416 vs 418 M cmds/s at 4; two instances per 128-lane
  // workgroup, 20 waves per CU, 399 M — r03f A/B; again in round 5, 408.4 vs
  // 429.3 M, profiles/archive/calls/r5_s5.sh: the scalar unit, not waiting, bounds k_sim)
#ifdef FX_SIM_WPS5
  const bool five = lds <= 160u * 1024u / 20u;
#else
  const bool five = false;
#endif
  if (fixed_ok && one_f && five && geo_is<GeoC1>(a.g, s0)) {
    // two instances per workgroup: 20 per CU (a CU holds at most 16 workgroups)
    hipLaunchKernelGGL((sim::k_sim<1, 1, 5, XNX, GeoC1, 2>), dim3((b->instances + 1) / 2), dim3(128), lds * 2, hs,
                       a);
  } else if (fixed_ok && five && geo_is<GeoC2a>(a.g, s0)) {
    hipLaunchKernelGGL((sim::k_sim<1, 1, 5, 1, GeoC2a>), grid, block, lds, hs, a);
  } else if (fixed_ok && one_f && four && geo_is<GeoC1>(a.g, s0)) {
    hipLaunchKernelGGL((sim::k_sim<1, 1, 4, XNX, GeoC1>), grid, block, lds, hs, a);
  } else if (fixed_ok && one_f && four && geo_is<GeoC0>(a.g, s0)) {
    hipLaunchKernelGGL((sim::k_sim<1, 1, 4, 1, GeoC0>), grid, block, lds, hs, a);
  } else if (fixed_ok && four && geo_is<GeoC2a>(a.g, s0)) {
    hipLaunchKernelGGL((sim::k_sim<1, 1, 4, 1, GeoC2a>), grid, block, lds, hs, a);
  } else if (fixed_ok && !four && geo_is<GeoC2b>(a.g, s0)) {
    hipLaunchKernelGGL((sim::k_sim<1, 1, 3, 1, GeoC2b>), grid, block, lds, hs, a);
  } else if (a.g.W <= 64) {
    // n <= 5 (configs[0], configs[1], half of configs[2]): executor tables
    // for 5 processes, 9 VGPRs fewer under the 4-wave budget
    if (a.g.L <= 64 && four && a.g.n <= 5) hipLaunchKernelGGL((sim::k_sim<1, 1, 4, 5>), grid, block, lds, hs, a);
    else if (a.g.L <= 64 && four) hipLaunchKernelGGL((sim::k_sim<1, 1, 4, NMAX>), grid, block, lds, hs, a);
    else if (a.g.L <= 64) hipLaunchKernelGGL((sim::k_sim<1, 1, 3, NMAX>), grid, block, lds, hs, a);
    else hipLaunchKernelGGL((sim::k_sim<2, 1, 3, NMAX>), grid, block, lds, hs, a);
  } else {
    if (a.g.L <= 64) hipLaunchKernelGGL((sim::k_sim<1, 4, 2, NMAX>), grid, block, lds, hs, a);
    else hipLaunchKernelGGL((sim::k_sim<2, 4, 2, NMAX>), grid, block, lds, hs, a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::fprintf(stderr, "fx_sim_run: launch failed: %s\n", hipGetErrorString(e));
    return FX_ERR_HIP;
  }
  return FX_OK;
}

// ------------------------------------------------------ escalation driver
// Instances that outgrow the launch's message pool or dot table
// (FX_ERR_SIM_CAPACITY) are rerun with larger tables.  Their histogram
// contributions before the failure are removed exactly: the kernel is
// deterministic per instance, so a rerun of just those instances at the
// first geometry reproduces the same partial samples, which are subtracted.

}  // extern "C"

namespace fx {
namespace sim {

__global__ void k_hist_sub(unsigned long long* dst, const unsigned long long* src, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] -= src[i];
}
template <typename T>
__global__ void k_rows_scatter(T* dst, const T* src, const uint32_t* map, uint32_t rows, uint32_t width) {
  const uint64_t total = (uint64_t)rows * width;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = t / width, c = t % width;
    dst[(uint64_t)map[r] * width + c] = src[t];
  }
}

struct Tmp {
  std::vector<void*> ptrs;
  ~Tmp() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  T* alloc(size_t count, hipStream_t hs, bool zero) {
    void* p = nullptr;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 8);
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    if (zero) (void)hipMemsetAsync(p, 0, bytes, hs);
    return (T*)p;
  }
};

}  // namespace sim
}  // namespace fx

// whether fx_sim_run runs the batch on the large-instance kernel
static bool sim_runs_large(const fx_sim_batch* b) {
  if ((b->flags & FX_SIM_FLAG_LARGE) || b->dot_slots > 256) return true;
  for (uint32_t i = 0; i < b->instances; ++i) {
    const fx_sim_spec& s = b->host_specs[i];
    if (s.read_only_pct != 0 || s.reorder_messages || s.nfr) return true;
  }
  Geo g;
  return !sim_geometry(b->host_specs[0], b->ring_entries, b->dot_slots, g) || (size_t)g.words * 4 > 160 * 1024 ||
         g.ncli_keys > 0xFFFFu;
}

extern "C" int fx_sim_run_tiered(const fx_sim_batch* b, const fx_sim_output* o, void* hip_stream,
                                 uint32_t* reruns) {
  if (reruns) *reruns = 0;
  int st = fx_sim_run(b, o, hip_stream);
  if (st || b->instances == 0) return st;
  hipStream_t hs = (hipStream_t)hip_stream;
  const uint32_t N = b->instances;
  std::vector<uint32_t> err(N);
  if (hipMemcpyAsync(err.data(), o->err, (size_t)N * 4, hipMemcpyDeviceToHost, hs) != hipSuccess ||
      hipStreamSynchronize(hs) != hipSuccess)
    return FX_ERR_HIP;
  std::vector<uint32_t> fail;  // indices into the original batch
  for (uint32_t i = 0; i < N; ++i)
    if (err[i] == FX_ERR_SIM_CAPACITY) fail.push_back(i);
  if (fail.empty()) return FX_OK;
  // the tier ladder (flags, events, dots): the caller's geometry, then larger tables
  const uint32_t f0 = b->flags & ~FX_SIM_FLAG_LARGE;
  uint32_t geo_flags[3], geo_ring[3], geo_dots[3];
  geo_flags[0] = b->flags;
  geo_ring[0] = b->ring_entries;
  geo_dots[0] = b->dot_slots;
  if (!sim_runs_large(b)) {
    Geo g0;
    if (!sim_geometry(b->host_specs[0], b->ring_entries, b->dot_slots, g0)) return FX_ERR_UNSUPPORTED;
    const uint32_t r1 = std::min<uint32_t>(65534u, std::max<uint32_t>(4u * g0.R, 256u * g0.n));
    geo_flags[1] = f0;
    geo_ring[1] = r1;
    geo_dots[1] = 256u;
    geo_flags[2] = f0 | FX_SIM_FLAG_LARGE;  // then the large-instance kernel
    geo_ring[2] = std::min<uint32_t>(16384u, std::max<uint32_t>(2u * r1, 1024u));
    geo_dots[2] = 2048u;
  } else {
    uint32_t R0 = 0, NS0 = 0;
    if (!simx_table_sizes(b->host_specs[0], b->ring_entries, b->dot_slots, &R0, &NS0)) return FX_ERR_UNSUPPORTED;
    for (uint32_t t = 1; t < 3; ++t) {
      geo_flags[t] = f0 | FX_SIM_FLAG_LARGE;
      geo_ring[t] = std::min<uint32_t>(16384u, R0 << t);
      geo_dots[t] = std::min<uint32_t>(8u * 65536u, NS0 << (2 * t));
    }
  }
  const uint32_t C = b->host_specs[0].clients_per_region * b->host_specs[0].num_client_regions;
  const uint32_t n = b->host_specs[0].n;
  const size_t nh_lat = o->latency_hist ? (size_t)b->planet_regions * o->lat_bins : 0;
  const size_t nh_chain = o->chain_hist ? o->chain_bins : 0, nh_delay = o->delay_hist ? o->delay_bins : 0;
  for (uint32_t tier = 1; tier <= 3 && !fail.empty(); ++tier) {
    Tmp tmp;
    const uint32_t F = (uint32_t)fail.size();
    std::vector<fx_sim_spec> sub(F);
    for (uint32_t j = 0; j < F; ++j) sub[j] = b->host_specs[fail[j]];
    fx_sim_spec* dspec = tmp.alloc<fx_sim_spec>(F, hs, false);
    uint32_t* dmap = tmp.alloc<uint32_t>(F, hs, false);
    uint32_t* terr = tmp.alloc<uint32_t>(F, hs, true);
    uint64_t* nlat = tmp.alloc<uint64_t>(nh_lat, hs, true);
    uint64_t* nchain = tmp.alloc<uint64_t>(nh_chain, hs, true);
    uint64_t* ndelay = tmp.alloc<uint64_t>(nh_delay, hs, true);
    if (!dspec || !dmap || !terr || !nlat || !nchain || !ndelay) return FX_ERR_HIP;
    (void)hipMemcpyAsync(dspec, sub.data(), (size_t)F * sizeof(fx_sim_spec), hipMemcpyHostToDevice, hs);
    (void)hipMemcpyAsync(dmap, fail.data(), (size_t)F * 4, hipMemcpyHostToDevice, hs);
    // 1. replay the failed runs at the geometry they failed with: their partial
    //    histogram samples, to subtract
    fx_sim_batch nb = *b;
    nb.specs = dspec;
    nb.host_specs = sub.data();
    nb.instances = F;
    nb.flags = geo_flags[tier - 1];
    nb.ring_entries = geo_ring[tier - 1];
    nb.dot_slots = geo_dots[tier - 1];
    fx_sim_output no{};
    no.latency_hist = o->latency_hist ? nlat : nullptr;
    no.chain_hist = o->chain_hist ? nchain : nullptr;
    no.delay_hist = o->delay_hist ? ndelay : nullptr;
    no.err = terr;
    no.lat_bins = o->lat_bins;
    no.chain_bins = o->chain_bins;
    no.delay_bins = o->delay_bins;
    if ((st = fx_sim_run(&nb, &no, hip_stream))) return st;
    const dim3 hg(64), hb(256);
    if (nh_lat) hipLaunchKernelGGL(k_hist_sub, hg, hb, 0, hs, (unsigned long long*)o->latency_hist,
                                   (const unsigned long long*)nlat, (uint32_t)nh_lat);
    if (nh_chain) hipLaunchKernelGGL(k_hist_sub, hg, hb, 0, hs, (unsigned long long*)o->chain_hist,
                                     (const unsigned long long*)nchain, (uint32_t)nh_chain);
    if (nh_delay) hipLaunchKernelGGL(k_hist_sub, hg, hb, 0, hs, (unsigned long long*)o->delay_hist,
                                     (const unsigned long long*)ndelay, (uint32_t)nh_delay);
    if (tier == 3) {  // no larger geometry: these stay failed, without histogram samples
      if (hipStreamSynchronize(hs) != hipSuccess) return FX_ERR_HIP;
      break;
    }
    // 2. rerun them with larger tables into temporaries, histograms straight into the caller's
    fx_sim_batch pb = nb;
    pb.flags = geo_flags[tier];
    pb.ring_entries = geo_ring[tier];
    pb.dot_slots = geo_dots[tier];
    fx_sim_output po = *o;
    po.executed = o->executed ? tmp.alloc<uint32_t>((size_t)F * n * b->exec_cap, hs, false) : nullptr;
    po.executed_len = o->executed_len ? tmp.alloc<uint32_t>((size_t)F * n, hs, true) : nullptr;
    po.latency_log = o->latency_log && b->lat_cap ? tmp.alloc<uint32_t>((size_t)F * C * b->lat_cap, hs, false)
                                                  : nullptr;
    po.stats = o->stats ? tmp.alloc<uint64_t>((size_t)F * FX_SIM_STATS, hs, true) : nullptr;
    po.dot_client = o->dot_client ? tmp.alloc<uint32_t>((size_t)F * n * b->exec_cap, hs, true) : nullptr;
    po.err = tmp.alloc<uint32_t>(F, hs, true);
    if (!po.err || (o->executed && !po.executed) || (o->executed_len && !po.executed_len) ||
        (o->stats && !po.stats))
      return FX_ERR_HIP;
    if ((st = fx_sim_run(&pb, &po, hip_stream))) return st;
    const dim3 sg(256), sb(256);
    if (po.executed) hipLaunchKernelGGL(k_rows_scatter<uint32_t>, sg, sb, 0, hs, o->executed, po.executed, dmap, F,
                                        n * b->exec_cap);
    if (po.executed_len) hipLaunchKernelGGL(k_rows_scatter<uint32_t>, sg, sb, 0, hs, o->executed_len,
                                            po.executed_len, dmap, F, n);
    if (po.latency_log) hipLaunchKernelGGL(k_rows_scatter<uint32_t>, sg, sb, 0, hs, o->latency_log, po.latency_log,
                                           dmap, F, C * b->lat_cap);
    if (po.dot_client) hipLaunchKernelGGL(k_rows_scatter<uint32_t>, sg, sb, 0, hs, o->dot_client, po.dot_client,
                                          dmap, F, n * b->exec_cap);
    if (po.stats) hipLaunchKernelGGL(k_rows_scatter<uint64_t>, sg, sb, 0, hs, o->stats, po.stats, dmap, F,
                                     FX_SIM_STATS);
    hipLaunchKernelGGL(k_rows_scatter<uint32_t>, sg, sb, 0, hs, o->err, po.err, dmap, F, 1u);
    std::vector<uint32_t> e2(F);
    if (hipMemcpyAsync(e2.data(), po.err, (size_t)F * 4, hipMemcpyDeviceToHost, hs) != hipSuccess ||
        hipStreamSynchronize(hs) != hipSuccess)
      return FX_ERR_HIP;
    if (reruns) *reruns += F;
    std::vector<uint32_t> next;
    for (uint32_t j = 0; j < F; ++j)
      if (e2[j] == FX_ERR_SIM_CAPACITY) next.push_back(fail[j]);
    fail.swap(next);
  }
  return FX_OK;
}
