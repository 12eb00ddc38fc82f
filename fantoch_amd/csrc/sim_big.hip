// sim_big.hip — the batched simulator for the instances the all-on-chip
// kernel (sim_wave.hip) cannot hold: many clients per instance (BASELINE
// configs[3]: 64 clients per region, 320 per instance at n = 5, hundreds of
// commands pending at every executor), message reordering
// (Runner::reorder_messages, runner.rs:519-524), NFR (keys/mod.rs:44-75,
// maybe_adjust_fast_quorum) and read-only commands (workload.rs:158-160) —
// the shapes of the reference's own protocol simulations (protocol/mod.rs:
// 702-768 sim_test: 10 clients per process, reordering, GC every 100 ms).
//
// Still ONE wavefront per simulated instance, wave-uniform control flow; the
// per-instance state moves from LDS to an HBM arena (about 1 MB at configs[3]),
// so many instances per CU hide the memory latency:
//   dot table   one slot per live dot, direct-mapped per source (seq mod Q):
//               the command (client, keys, read-only), the protocol state
//               shared by its messages (collect deps, every MCollectAck's deps,
//               the committed value, quorum, participants / accepts / commit /
//               execution counts) and, per process, an 8-word record: protocol
//               status byte, and the GraphExecutor's vertex (start time, the
//               dot it waits on, Tarjan id / low, on-stack + visited epoch, its
//               links in the waiter list of the dot it waits on, the head of
//               its own waiter list).  A slot is freed once every process
//               executed its dot; a dep whose slot no longer holds it is
//               therefore executed everywhere (the AEClock test of tarjan.rs:
//               128-145 needs no clock).
//   events      every scheduled action (messages, client submits and replies,
//               the periodic GC and executed-notification events, the
//               MGarbageCollection deliveries) is a pool entry keyed
//               (time, class, seq) — the oracle's Schedule order (C3) — and the
//               next action is found by a two-level 64-ary min tree: the group
//               minima live in lanes (lane g = group g), the leaves in HBM.
//               Per pop: one DPP min over the group minima, one coalesced
//               64-leaf read and a DPP min over it.  With reordering the links
//               are no longer FIFO, so the per-link merge of sim_wave.hip does
//               not apply; the tree is exact for any delays.
//   GC          simulated, not evaluated: with reordering the MGarbageCollection
//               delays are random draws of the shared reorder stream (runner.rs:
//               519-524), so sim_wave.hip's closed-form Stable count does not
//               hold.  The committed frontier per (process, source) lives in
//               lane 8 p + s and advances over the dot table.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace fx {
namespace simx {

constexpr uint32_t NMAX = FX_SIM_MAX_N;
constexpr uint32_t KMAX = 2;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t FMAX = 12;       // handler frame stack depth
constexpr uint32_t HC_BINS = 64;    // ChainSize bins counted per instance in LDS
constexpr uint32_t HD_BINS = 256;   // ExecutionDelay bins counted per instance in LDS
constexpr uint32_t HL_LOG = 6, HL_SLOTS = 1u << HL_LOG;  // client-latency cache
constexpr uint32_t TIME_LIMIT = 1u << 24;  // ms; the event key holds time << 8
// per-instance LDS: the histogram caches, then lane tables kept out of the
// register file (the 5-wave configs[3] build spills what does not fit): at
// 8 p + s, p's committed GC frontier of source s + 1, its previous stable
// frontier, the link delay p -> s; and two 64-bit sums (the executor Adds'
// deps, the client latencies)
constexpr uint32_t L_GCF = HC_BINS + HD_BINS + 2 * HL_SLOTS, L_GPS = L_GCF + 64, L_DPQ = L_GPS + 64;
constexpr uint32_t L_DEPS = L_DPQ + 64, L_LATSUM = L_DEPS + 2;
// the top of the free event stack (FC entries): a push takes an entry with an
// LDS read instead of a dependent HBM one; spilled / refilled FC / 2 at a time
constexpr uint32_t FC = 64, L_FC = L_LATSUM + 2;
// each process's table of the frontiers the others reported (GC, n x n x n <= 512)
constexpr uint32_t L_GCO = L_FC + FC;
constexpr uint32_t LDS_WORDS = L_GCO + NMAX * NMAX * NMAX;

// event kinds (protocol kinds numbered as the oracle's trace, sim_oracle.cpp MK)
enum : uint32_t {
  M_COLLECT = 0, M_COLLECT_ACK = 1, M_COMMIT = 2, M_CONSENSUS = 3, M_CONSENSUS_ACK = 4,
  M_GC = 6,        // MGarbageCollection delivery (payload: the sender's committed frontier)
  M_STORE = 8, M_STORE_ACK = 9, M_COMMIT_BASIC = 10,  // Basic (basic.rs:363-385)
  M_SUBMIT = 12,   // SubmitToProc
  E_CLIENT = 13,   // SendToClient
  E_TICK = 14,     // PeriodicProcessEvent (GarbageCollection)
  E_NOTIF = 15     // PeriodicExecutedNotification
};
enum : uint32_t { ST_START = 0, ST_PAYLOAD = 1, ST_COLLECT = 2, ST_COMMIT = 3 };
// per-process record word R_PST: status (2) | buffered commit | accepted |
// buffered-commit sender (4) | in the executor's graph | executed
constexpr uint32_t PS_BUF = 4u, PS_ACC = 8u, PS_INGRAPH = 1u << 8, PS_EXEC = 1u << 9;
// dot-slot words (then collect deps [2K] | value [vmax] | ack deps [n][amax])
enum : uint32_t { SL_DOT = 0, SL_CLIENT = 1, SL_IDX = 2, SL_KEYS = 3, SL_CNT = 4, SL_MASKS = 5,
                  SL_QUORUM = 6, SL_COLLECT = 8 };
// SL_CNT:    collect count (8) | value count (8) << 8 | nkeys (2) << 16 | read-only << 18 |
//            proposer ballot set << 19
// SL_MASKS:  participants (8) | proposer accepts (8) << 8 | committed (8) << 16 | executed (8) << 24
// SL_QUORUM: the MCollect's quorum mask (8) | its size << 8
// per-(slot, process) record words
enum : uint32_t { R_PST = 0, R_START = 1, R_WAIT = 2, R_TL = 3, R_MARK = 4, R_NEXT = 5, R_PREV = 6,
                  R_HEAD = 7, R_CMISS = 8, R_CEPOCH = 9, RW = 16 };
// R_TL:   Tarjan id (16) | low (16) << 16
// R_MARK: on the Tarjan stack | visited epoch << 1 (try_pending's skip rule)
// R_WAIT / R_NEXT / R_PREV / R_HEAD: slot + 1 (0 = none) — the PendingIndex
//         entry of a waited-on dot is a doubly linked list through its waiters
// R_CMISS / R_CEPOCH: the missing dep the last search rooted at this vertex
//         stopped at, and the process's execution epoch then (0 = none); see
//         x_add_ for why a still-valid one stands in for a whole search

struct GeoX {  // launch-uniform geometry (words)
  uint32_t n, C, K, Q, qlog, NS, R, ncli_keys;
  uint32_t amax, vmax, sl_value, sl_ack, SW;
  uint32_t o_slot, o_rec, o_kd, o_cl, o_kh, o_kl, o_inf, o_arg, o_gp, o_free, o_gco, o_tstk, o_fv, o_fi, o_fp, o_wl,
      o_tmp, o_tl, o_tw, o_rdy;
  uint32_t words;  // per instance
};

// the geometry of n processes, C clients, K keys per command, a key pool of
// `pool`, `ring` events in flight and `dots` live dots (0: the defaults); a
// constant expression, so a kernel can compile one in (GS below)
__host__ __device__ constexpr bool geo_build(uint32_t n, uint32_t C, uint32_t K, uint32_t pool, uint32_t ring,
                                             uint32_t dots, GeoX& g) {
  if (n < 2 || n > NMAX || C < 1 || C > 65535u || K < 1 || K > KMAX) return false;
  g.n = n;
  g.C = C;
  g.K = K;
  const uint32_t cpr = (C + n - 1) / n;
  const uint32_t want = dots ? (dots + n - 1) / n : (8u * cpr > 32u ? 8u * cpr : 32u);
  uint32_t Q = 16, qlog = 4;
  while (Q < want && Q < (1u << 16)) {
    Q <<= 1;
    ++qlog;
  }
  if (Q < want) return false;
  g.Q = Q;
  g.qlog = qlog;
  g.NS = n * Q;
  const uint32_t rdef = 16u * C + 8u * n * n + 256u;
  uint32_t R = ring ? ring : (rdef < 16384u ? rdef : 16384u);
  R = (R + 63u) & ~63u;
  if (R > 16384u) return false;
  g.R = R;
  g.ncli_keys = pool + C + 1;
  // an MCollectAck carries the coordinator's deps (<= 2K: a write and a read
  // per key) plus the replica's own (<= 2K); a committed value is their union
  // over the quorum (<= 2K (n + 1))
  g.amax = 4 * K;
  g.vmax = 2 * K * (n + 1);
  if (n * g.amax > 64 || g.vmax > 64) return false;
  g.sl_value = SL_COLLECT + 2 * K;
  g.sl_ack = g.sl_value + g.vmax;
  g.SW = g.sl_ack + n * g.amax;
  uint64_t o = 0;
  auto take = [&o](uint32_t& off, uint64_t words) {
    off = (uint32_t)o;
    o += (words + 15u) & ~15ull;  // 64-byte aligned tables
  };
  take(g.o_slot, (uint64_t)g.NS * g.SW);
  take(g.o_rec, (uint64_t)g.NS * n * RW);
  take(g.o_kd, (uint64_t)n * g.ncli_keys * 2u);
  take(g.o_cl, (uint64_t)C * 8u);
  take(g.o_kh, R);
  take(g.o_kl, R);
  take(g.o_inf, R);
  take(g.o_arg, R);
  take(g.o_gp, (uint64_t)R * n);
  take(g.o_free, R);
  take(g.o_gco, (uint64_t)n * n * n);
  take(g.o_tstk, g.NS);
  take(g.o_fv, g.NS);
  take(g.o_fi, g.NS);
  take(g.o_fp, g.NS);
  take(g.o_wl, 2ull * g.NS);
  take(g.o_tmp, g.NS);
  take(g.o_tl, g.NS);
  take(g.o_tw, g.NS);
  take(g.o_rdy, C + 64u);
  if (o > 0x7FFFFFFFull) return false;
  g.words = (uint32_t)o;
  return true;
}
// GS = 1: BASELINE configs[3] (n = 5, 64 clients per region in the 5 process
// regions, one key per command, a one-key pool, default ring and dots)
__host__ __device__ constexpr GeoX geo_compiled(uint32_t gs) {
  GeoX g{};
  if (gs == 1) geo_build(5, 320, 1, 1, 0, 0, g);
  return g;
}

struct ArgsX {
  const fx_sim_spec* specs;
  uint32_t instances;
  GeoX g;
  uint32_t* arena;
  const uint16_t* ping;
  const uint8_t* rank;
  uint32_t RP;
  uint32_t exec_cap, lat_cap, max_events, sim_exec_notif;
  uint32_t* executed;
  uint32_t* executed_len;
  uint32_t* latency_log;
  uint32_t* dot_client;
  unsigned long long* lat_hist;
  uint32_t lat_bins;
  unsigned long long* chain_hist;
  uint32_t chain_bins;
  unsigned long long* delay_hist;
  uint32_t delay_bins;
  unsigned long long* stats;
  uint32_t* err;
};

// the kernel's arguments and the instance's spec, read where they are needed
// (scalar loads through the constant address space, scalar-cache hits); the
// empty asm makes the pointer opaque so the loads are not hoisted into scalar
// registers held for the whole run
typedef __attribute__((address_space(4))) const ArgsX KArgsX;
typedef __attribute__((address_space(4))) const fx_sim_spec KSpec;
__device__ __forceinline__ KArgsX* kx() {
  KArgsX* p = (KArgsX*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
__device__ __forceinline__ KSpec* kspec(uint32_t inst) { return (KSpec*)(kx()->specs + inst); }

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
enum : uint64_t { R_CONFLICT = 1, R_POOL = 2, R_READ_ONLY = 3, R_REORDER = 4 };

// inclusive min-scan over the wavefront (row_shr 1/2/4/8, row_bcast 15/31);
// every lane gets the minimum
__device__ __forceinline__ uint32_t dpp_min(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x111, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x112, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x114, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x118, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x142, 0xA, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x143, 0xC, 0xF, false));
  return rl(v, 63);
}

enum : uint32_t { FOUND = 0, MISSING = 1 };

// FX_SIM_PROFILE builds (make prof): shader-clock cycles and counts per phase
// in the stats rows (slots 0-23) instead of the counters (tools/simx_phase.py)
#ifdef FX_SIM_PROFILE
#define XPROF_T0() const uint64_t xprof_t0_ = __builtin_amdgcn_s_memtime()
#define XPROF_ADD(cat) prof[cat] += __builtin_amdgcn_s_memtime() - xprof_t0_
#define XPROF_CNT(cat, v) prof[cat] += (v)
#else
#define XPROF_T0() (void)0
#define XPROF_ADD(cat) (void)0
#define XPROF_CNT(cat, v) (void)0
#endif
enum : uint32_t { PF_POP = 0, PF_EVENT = 1, PF_XADD = 2, PF_FIND = 3, PF_CHECK = 4, PF_SORT = 5, PF_EMIT = 6,
                  PF_HANDLER = 7, PF_SEND = 8, PF_GC = 9, PF_CLIENT = 10, PF_READY = 12, PF_HLOAD = 13,
                  PF_PUSH = 14, PF_DEPST = 15,
                  PC_EDGES = 16, PC_RECURSE = 17, PC_XADD = 18, PC_FIND = 19, PC_WAITERS = 20, PC_FAST = 21,
                  PC_EVENTS = 22, PC_SEND = 23, PC_CACHE = 11 };

// NG: registers of group minima per lane (message pool <= 4096 NG entries)
template <uint32_t NG>
struct Big {
  // ---------------------------------------------------------------- context
  // the lane id, opaque at every use: expressions of it (lane offsets of the
  // lane-parallel loads) are recomputed where they are used instead of being
  // hoisted out of the event loop and held -- or spilled -- for the whole run
  uint32_t lid_;
  __device__ __forceinline__ uint32_t lidv() const {
    uint32_t x = lid_;
    asm volatile("" : "+v"(x));
    return x;
  }

  GeoX g;
  uint32_t* M;    // this instance's arena
  uint32_t* lds;  // histogram caches
  uint32_t inst;
  uint32_t protocol, n, f, synod_f;
  // the instance's other workload parameters are read from its spec where
  // they are used (scalar loads, scalar-cache hits) instead of being held in
  // scalar registers for the whole run (the kernel is short of SGPRs)
  __device__ __forceinline__ KSpec* spec_() const { return kspec(inst); }
  __device__ __forceinline__ uint64_t seed_() const { return spec_()->seed; }
  __device__ __forceinline__ uint64_t rng_inst_() const { return spec_()->instance; }
  __device__ __forceinline__ uint32_t conflict_() const { return spec_()->conflict_rate; }
  __device__ __forceinline__ uint32_t pool_() const { return spec_()->pool_size; }
  __device__ __forceinline__ uint32_t ro_pct_() const { return spec_()->read_only_pct; }
  __device__ __forceinline__ uint32_t cmds_() const { return spec_()->commands_per_client; }
  __device__ __forceinline__ uint32_t gc_ms_() const { return spec_()->gc_interval_ms; }
  __device__ __forceinline__ uint32_t en_ms_() const { return spec_()->executed_notification_ms; }
  __device__ __forceinline__ uint32_t extra_() const {
    const int32_t e = spec_()->extra_sim_time_ms;
    return e >= 0 ? (uint32_t)e : 0u;
  }
  bool has_extra, reorder, nfr;
  uint32_t C, K;
  uint32_t err = 0, err_site = 0;
  __device__ __forceinline__ void fail_cap(uint32_t line) {
    if (!err) err_site = line;
    err = FX_ERR_SIM_CAPACITY;
  }
  // FX_ERR_SIM_LATE with its source line in the stats row (as capacity failures)
  __device__ __forceinline__ void fail_late(uint32_t line) {
#ifdef FX_SIMX_DIAG
    if (!err) {
      dput(0, line | (0xD1A6ull << 32));
      dput(1, now | ((uint64_t)(uint32_t)events << 32));
      dput(2, seq | ((uint64_t)nfree << 32));
      dput(3, xp | (rtop << 8) | (nfrm << 16) | ((uint64_t)cur_info << 32));
      dput(4, cur_arg | ((uint64_t)cur_hi << 32));
    }
#endif
    if (!err) err_site = line;
    err = FX_ERR_SIM_LATE;
  }
#ifdef FX_SIMX_DIAG
  // diagnostics build (make fvariant V=diag F=sim_big D=-DFX_SIMX_DIAG,
  // tools/simx_diag.py): the first failure's state goes to stats slots 0..23
  // of the instance (the protocol counters are not written in this build)
  uint32_t cur_info = 0, cur_arg = 0, cur_hi = 0;
  __device__ __forceinline__ void dput(uint32_t i, uint64_t v) {
    if (lidv() == 0 && kx()->stats) kx()->stats[(size_t)inst * FX_SIM_STATS + i] = v;
  }
#endif
  uint32_t now = 0;  // ms
  // the clock read at a cold use without a vector copy of it kept live
  __device__ __forceinline__ uint32_t nowv() const {
    uint32_t x = now;
    asm volatile("" : "+s"(x));
    return x;
  }
  uint32_t seq = 0;  // insertion counter (C3)
  uint32_t rdraws = 0, events = 0;  // (32 bits: bounded by max_events; 64-bit counters live in LDS)
  uint64_t trace = 0;
  __device__ __forceinline__ void lds_add64(uint32_t off, uint32_t v) {
    const uint64_t x = (uint64_t)uni(lds[off]) | ((uint64_t)uni(lds[off + 1]) << 32);
    const uint64_t y = x + v;
    put(lds[off], (uint32_t)y);
    put(lds[off + 1], (uint32_t)(y >> 32));
  }
  __device__ __forceinline__ uint64_t lds64(uint32_t off) const {
    return (uint64_t)uni(lds[off]) | ((uint64_t)uni(lds[off + 1]) << 32);
  }
  uint32_t clients_done = 0;
  bool done = false, in_extra = false;
  uint32_t final_ms = 0;

  // event pool: minimum (key hi, key lo) of group 64 k + lane in gh[k], gl[k]
  uint32_t gh[NG], gl[NG];
  uint32_t nfree = 0;  // entries in the HBM part of the free stack
  uint32_t fcn = 0;    // entries in its LDS top (lds[L_FC + 0 .. fcn))
  // lane p: proposal seq, Fast / Slow (and their read-only shares), executed
  // count, Stable, quorums (fast | write << 8 | majority << 16), GC reporters
  // (packed into two VGPRs, 8 lanes a field: pa lane A_x + p, pb lane B_x + p)
  uint32_t pa = 0, pb = 0;
  enum : uint32_t { A_SEQ = 0, A_FAST = 8, A_SLOW = 16, A_FR = 24, A_SR = 32, A_EXEC = 40, A_STAB = 48, A_Q = 56 };
  enum : uint32_t { B_REP = 0, B_XE = 8, B_FRW = 16, B_FRD = 32, B_FRB = 48 };  // frames: lanes B_FR* + fi (fi < 16)
  // lane p: executions so far at p, in SCCs (the epoch of the search-result cache)

  // lane 8 p + s: p's committed frontier of source s + 1 (GC track), its
  // previous stable frontier, and the link delay p -> s
  __device__ __forceinline__ uint32_t dpq_(uint32_t i) { return uni(lds[L_DPQ + i]); }
  // handler frames, frame fi in lane fi: action (0 none, 1 ToSend) | kind << 2 |
  // targets << 8 | next target << 16; dot; base of its ready results

  uint32_t nfrm = 0, xinfo = NONE, rtop = 0;
  // executor (the process being run)
  uint32_t xp = 0, xk = 0, xe = 0, epoch = 0, nwl = 0, idc = 0, tsp = 0, fsp = 0;
#ifdef FX_SIM_PROFILE
  uint64_t prof[24] = {};
#endif

  // ------------------------------------------------------------ arena views
  __device__ __forceinline__ uint32_t& S(uint32_t sl, uint32_t w) { return M[g.o_slot + sl * g.SW + w]; }
  __device__ __forceinline__ uint32_t& RC(uint32_t sl, uint32_t p, uint32_t w) {
    return M[g.o_rec + (sl * g.n + p) * RW + w];
  }
  __device__ __forceinline__ uint32_t& CL(uint32_t c, uint32_t w) { return M[g.o_cl + c * 8u + w]; }
  __device__ __forceinline__ uint32_t& KD(uint32_t p, uint32_t key, uint32_t w) {
    return M[g.o_kd + (p * g.ncli_keys + key) * 2u + w];
  }
  __device__ __forceinline__ uint32_t& W(uint32_t off, uint32_t i) { return M[off + i]; }
  __device__ __forceinline__ uint32_t rd(uint32_t& x) { return uni(x); }
  __device__ __forceinline__ void put(uint32_t& dst, uint32_t v) {
    if (lidv() == 0) dst = v;
  }
  __device__ __forceinline__ void lset(uint32_t& reg, uint32_t lane, uint32_t v) {
    if (lidv() == lane) reg = v;
  }
  // dot table slot of a dot (direct-mapped per source)
  __device__ __forceinline__ uint32_t hslot(uint32_t d) const {
    return ((FX_DOT_SRC(d) - 1u) << g.qlog) | (FX_DOT_SEQ(d) & (g.Q - 1u));
  }
  __device__ __forceinline__ bool src_ok(uint32_t d) const {
    const uint32_t s = FX_DOT_SRC(d);
    return s >= 1u && s <= n;
  }
  // slot of a live dot, NONE if its slot no longer holds it
  __device__ __forceinline__ uint32_t slot_of(uint32_t d) {
    if (!src_ok(d)) return NONE;
    const uint32_t sl = hslot(d);
    return rd(S(sl, SL_DOT)) == d ? sl : NONE;
  }

  // ------------------------------------------------- handler row prefetch
  // A handler reads many words of one dot slot and of its record at the
  // handling process, one dependent HBM round trip each.  Instead the slot's
  // first HR_S words (lanes 0 .. HR_S - 1) and the record (lanes HR_S ..
  // HR_S + 15) come in ONE lane-parallel load when the handler starts; the
  // handler reads them with readlanes and writes through sput / rput, which
  // keep the copy current.  Words past HR_S (the ack deps of high processes
  // in large geometries) are read from the arena.  x_add, run right after
  // the handler that committed the slot, reuses the copy.
  static constexpr uint32_t HR_S = 48;
  uint32_t hsl = NONE, hpp = NONE, hrow = 0;
  __device__ __forceinline__ void hload(uint32_t sl, uint32_t p) {
    XPROF_T0();
    hsl = sl;
    hpp = p;
    hrow = lidv() < HR_S ? (lidv() < g.SW ? S(sl, lidv()) : 0u) : RC(sl, p, lidv() - HR_S);
#ifdef FX_SIM_PROFILE
    hrow = uni(hrow) == 0xFFFFFFFFu ? hrow + 1u : hrow;  // (waits for the load inside the bracket)
#endif
    XPROF_ADD(PF_HLOAD);
  }
  // the slot of a live dot with its row and p's record loaded (always from
  // the arena: other events wrote it since); NONE if the slot no longer holds
  // the dot
  __device__ __forceinline__ uint32_t hslot_of(uint32_t d, uint32_t p) {
    if (!src_ok(d)) return NONE;
    const uint32_t sl = hslot(d);
    hload(sl, p);
    return rl(hrow, SL_DOT) == d ? sl : NONE;
  }
  __device__ __forceinline__ uint32_t sv(uint32_t w) { return w < HR_S ? rl(hrow, w) : rd(S(hsl, w)); }
  __device__ __forceinline__ void sput(uint32_t w, uint32_t v) {
    put(S(hsl, w), v);
    if (w < HR_S) lset(hrow, w, v);
  }
  __device__ __forceinline__ uint32_t rv(uint32_t w) { return rl(hrow, HR_S + w); }
  __device__ __forceinline__ void rput(uint32_t w, uint32_t v) {
    put(RC(hsl, hpp, w), v);
    lset(hrow, HR_S + w, v);
  }
  // lane-parallel read of slot words w0 + lidv() for lanes with lidv() < cnt
  __device__ __forceinline__ uint32_t svl(uint32_t w0, uint32_t cnt) {
    const uint32_t w = w0 + lidv();
    const uint32_t gv = gather(hrow, w & 63u);
    if (lidv() >= cnt) return 0u;
    return w < HR_S ? gv : S(hsl, w);
  }
  // the copy is valid from a handler's hslot_of to the end of the x_add that
  // follows it (run_handlers drops it after that)
  __device__ __forceinline__ void hforget() { hsl = hpp = NONE; }

  // ------------------------------------------------------------- histograms
  __device__ __forceinline__ void hist_chain(uint32_t v) {
    if (!kx()->chain_hist) return;
    const uint32_t b = min(v, kx()->chain_bins - 1u);
    if (lidv() == 0) {
      if (b < HC_BINS) atomicAdd(&lds[b], 1u);
      else atomicAdd(&kx()->chain_hist[b], 1ull);
    }
  }
  __device__ __forceinline__ void hist_delay(uint32_t v) {
    if (!kx()->delay_hist) return;
    const uint32_t b = min(v, kx()->delay_bins - 1u);
    if (lidv() == 0) {
      if (b < HD_BINS) atomicAdd(&lds[HC_BINS + b], 1u);
      else atomicAdd(&kx()->delay_hist[b], 1ull);
    }
  }
  __device__ __forceinline__ void hist_lat(uint32_t region, uint32_t lat) {
    if (!kx()->lat_hist) return;
    const uint32_t key = region * kx()->lat_bins + min(lat, kx()->lat_bins - 1u);
    const uint32_t h = (key * 2654435761u) >> (32 - HL_LOG);
    uint32_t* lc = lds + HC_BINS + HD_BINS;
    const uint32_t k = uni(lc[h]);
    if (lidv() == 0) {
      if (k == key + 1u) {
        atomicAdd(&lc[HL_SLOTS + h], 1u);
      } else if (k == 0) {
        lc[h] = key + 1u;
        lc[HL_SLOTS + h] = 1u;
      } else {
        atomicAdd(&kx()->lat_hist[key], 1ull);
      }
    }
  }

  // ------------------------------------------------------------------ trace
  __device__ __forceinline__ void note(uint64_t kind, uint64_t a, uint64_t b, uint64_t c) {
    ++events;
    trace = mix64(trace ^ ((uint64_t)now << 24) ^ (kind << 20) ^ (a << 12) ^ (b << 4)) + c;
  }

  // ----------------------------------------------------------------- events
  // key hi = time << 8 | class << 6 | a << 3 | b (class 0 protocol / client /
  // executed notification; 1 the GC event of process a; 2 the GC delivery
  // a -> b), key lo = insertion seq: the oracle's (time, class, seq) order
  __device__ __forceinline__ uint32_t push_event(uint32_t t, uint32_t cls, uint32_t info, uint32_t arg) {
    XPROF_T0();
    const uint32_t e = push_event_(t, cls, info, arg);
    XPROF_ADD(PF_PUSH);
    return e;
  }
  __device__ __forceinline__ uint32_t push_event_(uint32_t t, uint32_t cls, uint32_t info, uint32_t arg) {
    if (t >= TIME_LIMIT) {
      err = FX_ERR_TIME_RANGE;
      return NONE;
    }
    if (fcn == 0) {  // refill the LDS top from the HBM stack: its top FC / 2 entries, in order
      if (nfree == 0) {
        fail_cap(__LINE__);
        return NONE;
      }
      const uint32_t k = min(nfree, FC / 2u);
      if (lidv() < k) lds[L_FC + lidv()] = W(g.o_free, nfree - k + lidv());
      nfree -= k;
      fcn = k;
    }
    const uint32_t e = uni(lds[L_FC + --fcn]);
    const uint32_t hi = (t << 8) | cls, lo = seq++;
    put(W(g.o_kh, e), hi);
    put(W(g.o_kl, e), lo);
    put(W(g.o_inf, e), info);
    put(W(g.o_arg, e), arg);
    const uint32_t grp = e >> 6;
    if (lidv() == (grp & 63u)) {
#pragma unroll
      for (uint32_t k = 0; k < NG; ++k)
        if ((grp >> 6) == k && (hi < gh[k] || (hi == gh[k] && lo < gl[k]))) {
          gh[k] = hi;
          gl[k] = lo;
        }
    }
    return e;
  }
  // removes the minimum event; returns its entry (NONE if the queue is empty)
  // and its info / arg words, read with the group's keys (one round trip: the
  // event loop's next loads depend on them)
  __device__ __forceinline__ uint32_t pop_event(uint32_t& hi_out, uint32_t& info_out, uint32_t& arg_out) {
    uint32_t bh = gh[0], bl = gl[0], bk = 0;
#pragma unroll
    for (uint32_t k = 1; k < NG; ++k) {
      const bool lt = gh[k] < bh || (gh[k] == bh && gl[k] < bl);
      bh = lt ? gh[k] : bh;
      bl = lt ? gl[k] : bl;
      bk = lt ? k : bk;
    }
    const uint32_t th = dpp_min(bh);
    hi_out = th;
    if (th == NONE) return NONE;
    const uint32_t tl = dpp_min(bh == th ? bl : NONE);
    const uint32_t ln = ctz64(bal(bh == th && bl == tl));
    const uint32_t grp = rl(bk, ln) * 64u + ln;
    const uint32_t e0 = grp * 64u + lidv();
    uint32_t kh = W(g.o_kh, e0), kl = W(g.o_kl, e0);
    const uint32_t vi = W(g.o_inf, e0), va = W(g.o_arg, e0);
    const uint64_t hit = bal(kh == th && kl == tl);
    if (!hit) {  // the group's minimum is not among its leaves: a broken event tree
#ifdef FX_SIMX_DIAG
      if (!err) diag_tree(th, tl, grp, ln, bk, kh, kl);
#endif
      fail_late(__LINE__);
      hi_out = NONE;
      return NONE;
    }
    const uint32_t j = ctz64(hit);
    info_out = rl(vi, j);
    arg_out = rl(va, j);
    if (lidv() == j) {
      kh = NONE;
      kl = NONE;
      W(g.o_kh, e0) = NONE;
    }
    const uint32_t nh = dpp_min(kh);
    const uint32_t nl = dpp_min(kh == nh ? kl : NONE);
    if (lidv() == (grp & 63u)) {
#pragma unroll
      for (uint32_t k = 0; k < NG; ++k)
        if ((grp >> 6) == k) {
          gh[k] = nh;
          gl[k] = nl;
        }
    }
    return grp * 64u + j;
  }
  __device__ __forceinline__ void free_event(uint32_t e) {
    if (fcn == FC) {  // spill the LDS top's lower half to the HBM stack, in order
      const uint32_t v = lds[L_FC + lidv()];  // (lanes < FC)
      const uint32_t hi = lds[L_FC + ((lidv() + FC / 2u) & (FC - 1u))];
      if (lidv() < FC / 2u) {
        W(g.o_free, nfree + lidv()) = v;
        lds[L_FC + lidv()] = hi;
      }
      nfree += FC / 2u;
      fcn = FC / 2u;
    }
    put(lds[L_FC + fcn++], e);
  }
#ifdef FX_SIMX_DIAG
  // the broken group, its leaves, and every group whose lane minimum differs
  // from the minimum of its leaves
  __device__ void diag_tree(uint32_t th, uint32_t tl, uint32_t grp, uint32_t ln, uint32_t bk, uint32_t kh,
                            uint32_t kl) {
    dput(8, th | ((uint64_t)tl << 32));
    dput(9, grp | ((uint64_t)ln << 16) | ((uint64_t)rl(bk, ln) << 32));
    const uint32_t nh = dpp_min(kh), nl = dpp_min(kh == nh ? kl : NONE);
    dput(10, nh | ((uint64_t)nl << 32));
    dput(11, pop64(bal(kh == NONE)) | ((uint64_t)pop64(bal(kh == th)) << 8) | ((uint64_t)pop64(bal(kl == tl)) << 16));
    uint32_t bad = 0, first = NONE, fh = 0, fl = 0, ah = 0, al = 0;
    const uint32_t ngr = g.R >> 6;
    for (uint32_t g2 = 0; g2 < ngr; ++g2) {
      const uint32_t h2 = W(g.o_kh, g2 * 64u + lidv()), l2 = W(g.o_kl, g2 * 64u + lidv());
      const uint32_t mh = dpp_min(h2), ml = dpp_min(h2 == mh ? l2 : NONE);
      uint32_t sh = NONE, slo = NONE;
#pragma unroll
      for (uint32_t k = 0; k < NG; ++k)
        if ((g2 >> 6) == k) {
          sh = rl(gh[k], g2 & 63u);
          slo = rl(gl[k], g2 & 63u);
        }
      if (sh != mh || slo != ml) {
        if (!bad) {
          first = g2;
          fh = sh;
          fl = slo;
          ah = mh;
          al = ml;
        }
        ++bad;
      }
    }
    dput(12, bad | ((uint64_t)first << 32));
    dput(13, fh | ((uint64_t)fl << 32));
    dput(14, ah | ((uint64_t)al << 32));
    // lanes of the group-minimum registers beyond the pool's groups must hold NONE
    uint32_t junk = 0, jv = 0, jl = 0;
#pragma unroll
    for (uint32_t k = 0; k < NG; ++k) {
      const bool off = k * 64u + lidv() >= ngr;
      const uint64_t m = bal(off && (gh[k] != NONE || gl[k] != NONE));
      if (m && !junk) {
        jl = k * 64u + ctz64(m);
        jv = rl(gh[k], ctz64(m));
      }
      junk += pop64(m);
    }
    dput(15, junk | ((uint64_t)jl << 16) | ((uint64_t)jv << 32));
  }
  // a message for a dot whose slot no longer holds it
  __device__ void diag_slot(uint32_t d, uint32_t p) {
    dput(8, d | ((uint64_t)p << 32));
    const uint32_t sl = src_ok(d) ? hslot(d) : NONE;
    dput(9, sl | ((uint64_t)rl(pa, A_SEQ + ((FX_DOT_SRC(d) - 1u) & 7u)) << 32));
    if (sl != NONE) {
      dput(10, S(sl, SL_DOT) | ((uint64_t)S(sl, SL_MASKS) << 32));
      dput(11, S(sl, SL_CNT) | ((uint64_t)S(sl, SL_CLIENT) << 32));
      dput(12, RC(sl, p, R_PST) | ((uint64_t)RC(sl, p, R_WAIT) << 32));
      dput(13, rl(hrow, SL_DOT) | ((uint64_t)hsl << 32));
    }
  }
#endif

  // Runner::schedule_message (runner.rs:507-530): distance, times the C6
  // multiplier in [0, 10) when reordering (one draw per message, in schedule order)
  __device__ __forceinline__ uint32_t msg_delay(uint32_t d) {
    if (!reorder) return d;
    const uint64_t u = sim_rand(seed_(), rng_inst_(), 0, rdraws++, R_REORDER);
    const double mult = (double)(u >> 11) * (1.0 / 9007199254740992.0) * 10.0;
    return (uint32_t)(uint64_t)((double)d * mult);
  }

  // ------------------------------------------------------------ workload
  // Workload::gen_cmd (workload.rs:142-197) of command idx of client cid
  // (1-based), canonical C6/C7/C11: keys packed key0 | key1 << 16
  __device__ __forceinline__ uint32_t gen_keys(uint32_t cid, uint32_t idx, uint32_t& nk) {
    uint32_t k0 = 0xFFFFu, k1 = 0xFFFFu;
    nk = 0;
    for (uint32_t draw = 0; nk < K && draw < 65536u; ++draw) {  // gen_unique_keys draws until distinct
      bool conflict;
      if (conflict_() == 0) conflict = false;
      else if (conflict_() >= 100) conflict = true;
      else conflict = sim_rand(seed_(), rng_inst_(), cid, (uint64_t)idx * 64 + draw, R_CONFLICT) % 100ull < conflict_();
      uint32_t key;
      if (conflict)
        key = pool_() <= 1 ? 0u : (uint32_t)(sim_rand(seed_(), rng_inst_(), cid, (uint64_t)idx * 64 + draw, R_POOL) % pool_());
      else
        key = pool_() + cid;
      if (nk == 0) {
        k0 = key;
        nk = 1;
      } else if (key != k0) {
        k1 = key;
        nk = 2;
      }
    }
    if (nk != K) fail_cap(__LINE__);
    if (nk == 2 && k1 < k0) {  // C11
      const uint32_t t = k0;
      k0 = k1;
      k1 = t;
    }
    return k0 | (k1 << 16);
  }
  __device__ __forceinline__ bool gen_read_only(uint32_t cid, uint32_t idx) {  // workload.rs:158-160
    if (ro_pct_() == 0) return false;
    if (ro_pct_() >= 100) return true;
    return sim_rand(seed_(), rng_inst_(), cid, idx, R_READ_ONLY) % 100ull < ro_pct_();
  }

  // ------------------------------------------------------- frame stack
  __device__ __forceinline__ void act_send(uint32_t kind, uint32_t dot, uint32_t tgt) {
    const uint32_t fi = nfrm - 1;
    lset(pb, B_FRW + fi, 1u | (kind << 2) | (tgt << 8));
    lset(pb, B_FRD + fi, dot);
  }

  // ============================================================ protocol
  // SequentialKeyDeps::add_cmd (sequential.rs:74-118, keys/mod.rs:44-75): the
  // latest write per key, and the latest read unless the command is read-only
  // or NFR is on; `past` merged; returns the sorted distinct deps in lanes
  // [0, cnt) of outv
  __device__ __forceinline__ uint32_t add_cmd(uint32_t p, uint32_t dot, uint32_t keys, uint32_t nk, bool ro,
                                              uint32_t pastv, uint32_t npast, uint32_t& outv) {
    const uint32_t key0 = keys & 0xFFFFu, key1 = keys >> 16;
    const uint32_t w0 = rd(KD(p, key0, 0)), r0 = rd(KD(p, key0, 1));
    put(KD(p, key0, ro ? 1u : 0u), dot);
    uint32_t w1 = 0, r1 = 0;
    if (nk > 1) {
      w1 = rd(KD(p, key1, 0));
      r1 = rd(KD(p, key1, 1));
      put(KD(p, key1, ro ? 1u : 0u), dot);
    }
    const bool reads = !ro && !nfr;
    const uint32_t i = lidv() - npast;
    uint32_t v = 0;
    if (lidv() < npast) v = pastv;
    else if (i == 0) v = w0;
    else if (i == 1) v = reads ? r0 : 0u;
    else if (i == 2) v = w1;
    else if (i == 3) v = reads ? r1 : 0u;
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
    const uint32_t s = rl(pa, A_SEQ + p) + 1u;
    lset(pa, A_SEQ + p, s);
    if (s > FX_SEQ_MASK) {
      err = FX_ERR_DOT_RANGE;
      return;
    }
    const uint32_t dot = FX_PACK_DOT(p + 1, s);
    const uint32_t sl = hslot(dot);
    if (rd(S(sl, SL_DOT)) != 0) {  // the dot Q seqs back is still live
      fail_cap(__LINE__);
      return;
    }
    const uint32_t idx = rd(CL(c, 1)) - 1u;
    uint32_t nk = 0;
    const uint32_t keys = gen_keys(c + 1, idx, nk);
    const bool ro = gen_read_only(c + 1, idx);
    const bool basic = protocol == FX_PROTOCOL_BASIC;  // no deps (basic.rs:171-185)
    uint32_t depv = 0;
    const uint32_t nd = basic ? 0u : add_cmd(p, dot, keys, nk, ro, 0, 0, depv);
    // maybe_adjust_fast_quorum: a single-key read under NFR goes to a majority
    const uint32_t qw = rl(pa, A_Q + p);
    const uint32_t qm = (nfr && ro && nk == 1) ? (qw >> 16) & 0xFFu : qw & 0xFFu;
    // the fresh slot in one lane-parallel pass, and its per-process records
    const uint32_t dv = gather(depv, (lidv() - SL_COLLECT) & 63u);
    for (uint32_t i = lidv(); i < g.SW; i += 64) {
      uint32_t v = 0;
      if (i == SL_DOT) v = dot;
      else if (i == SL_CLIENT) v = c;
      else if (i == SL_IDX) v = idx;
      else if (i == SL_KEYS) v = keys;
      else if (i == SL_CNT) v = nd | (nk << 16) | (ro ? 1u << 18 : 0u);
      else if (i == SL_QUORUM) v = qm | (pop32(qm) << 8);
      else if (i >= SL_COLLECT && i < SL_COLLECT + nd) v = dv;
      S(sl, i) = v;
    }
    for (uint32_t i = lidv(); i < g.n * RW; i += 64) M[g.o_rec + sl * g.n * RW + i] = 0;
    if (kx()->dot_client && s <= kx()->exec_cap && lidv() == 0)
      kx()->dot_client[((size_t)inst * n + p) * kx()->exec_cap + s - 1u] = c + 1u;
    act_send(basic ? M_STORE : M_COLLECT, dot, (1u << n) - 1u);
  }

  // ------------------------------------------------------------- Basic
  // basic.rs:187-211 handle_mstore: the command arrives; a member of the
  // coordinator's quorum acks; a commit that arrived first is applied now
  __device__ __forceinline__ void h_mstore(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    const uint32_t ps = rv(R_PST);
    rput(R_PST, (ps & ~(3u | PS_BUF)) | ST_PAYLOAD);
    if ((sv(SL_QUORUM) >> p) & 1u) act_send(M_STORE_ACK, dot, 1u << from);
    if (ps & PS_BUF) h_bcommit(p, dot);  // buffered_mcommits.remove
  }
  // basic.rs:213-230 handle_mstoreack: f + 1 acks commit
  __device__ __forceinline__ void h_mstoreack(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    const uint32_t masks = sv(SL_MASKS);
    const uint32_t acks = (masks & 0xFFu) | (1u << from);
    sput(SL_MASKS, (masks & ~0xFFu) | acks);
    if (pop32(acks) == f + 1u) act_send(M_COMMIT_BASIC, dot, (1u << n) - 1u);
  }
  // basic.rs:232-257 handle_mcommit, and BasicExecutor::handle for each key at
  // once (executor/basic.rs:39-53): the dot is logged once per key (the
  // oracle's execution log), the key results go to AggregatePending; no
  // ExecutionDelay / ChainSize samples
  __device__ __forceinline__ void h_bcommit(uint32_t p, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    const uint32_t ps = rv(R_PST);
    if ((ps & 3u) == ST_START) {  // buffered_mcommits.insert
      rput(R_PST, ps | PS_BUF);
      return;
    }
    rput(R_PST, (ps & ~3u) | ST_COMMIT);
    const uint32_t c = sv(SL_CLIENT);
    const uint32_t nk = (sv(SL_CNT) >> 16) & 3u;
    const uint32_t x0 = rl(pa, A_EXEC + p);
    if (lidv() < nk && kx()->executed && x0 + lidv() < kx()->exec_cap)
      kx()->executed[((size_t)inst * n + p) * kx()->exec_cap + x0 + lidv()] = dot;
    lset(pa, A_EXEC + p, x0 + nk);
    if ((rd(CL(c, 0)) & 0xFFu) == p) client_result(c, nk);  // pending.wait_for registered this rifl at p
    if (err) return;
    if (gc_ms_()) gc_commit(p, dot);  // Forward(MCommitDot) (basic.rs:246-251), before the slot can go
    const uint32_t masks = sv(SL_MASKS);
    if (((masks >> 24) & 0xFFu) + 1u == n) sput(SL_DOT, 0u);  // executed everywhere: free the slot
    else sput(SL_MASKS, masks + (1u << 24));
  }

  // atlas.rs:251-325 / epaxos.rs:223-301
  __device__ __forceinline__ void h_mcollect(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    const uint32_t ps = rv(R_PST);
    if ((ps & 3u) != ST_START) return;
    const uint32_t qm = sv(SL_QUORUM) & 0xFFu;
    if (!((qm >> p) & 1u)) {
      const uint32_t ps2 = (ps & ~3u) | ST_PAYLOAD;
      if (ps & PS_BUF) {  // buffered commit (atlas.rs:288-292)
        rput(R_PST, ps2 & ~PS_BUF);
        h_mcommit(p, (ps >> 4) & 15u, dot);
      } else {
        rput(R_PST, ps2);
      }
      return;
    }
    const bool from_self = from == p;
    const uint32_t cnt = sv(SL_CNT);
    const uint32_t ncol = cnt & 0xFFu, nk = (cnt >> 16) & 3u;
    const bool ro = (cnt >> 18) & 1u;
    const uint32_t colv = svl(SL_COLLECT, ncol);
    uint32_t depv = 0, nd = 0;
    if (from_self) {
      depv = colv;
      nd = ncol;
    } else {
      nd = add_cmd(p, dot, sv(SL_KEYS), nk, ro, colv, ncol, depv);
    }
    if (nd > g.amax) {
      fail_cap(__LINE__);
      return;
    }
    rput(R_PST, (ps & ~3u) | ST_COLLECT);
    if (lidv() < g.amax) S(sl, g.sl_ack + p * g.amax + lidv()) = lidv() < nd ? depv : 0u;
    if (protocol == FX_PROTOCOL_EPAXOS && from_self) return;  // epaxos.rs:290-300
    act_send(M_COLLECT_ACK, dot, 1u << from);
  }

  // atlas.rs:327-402 / epaxos.rs:303-368
  __device__ __forceinline__ void h_mcollectack(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    if ((rv(R_PST) & 3u) != ST_COLLECT) return;
    const uint32_t masks = sv(SL_MASKS);
    const uint32_t part = (masks & 0xFFu) | (1u << from);
    sput(SL_MASKS, (masks & ~0xFFu) | part);
    const uint32_t qs = sv(SL_QUORUM) >> 8;
    const uint32_t fq_eff = protocol == FX_PROTOCOL_EPAXOS ? qs - 1u : qs;  // EPaxosInfo (epaxos.rs:650-662)
    if (pop32(part) != fq_eff) return;
    // QuorumDeps: union + per-dep report counts; lanes [q amax, (q + 1) amax)
    // hold process q's reported deps
    const uint32_t q = lidv() / g.amax, j = lidv() % g.amax;
    const uint32_t aw = g.sl_ack + q * g.amax + j;
    const uint32_t ag = gather(hrow, aw & 63u);
    uint32_t v = 0;
    if (q < n && ((part >> q) & 1u)) v = aw < HR_S ? ag : S(sl, aw);
    const bool valid = v != 0;
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
    const uint64_t um = bal(first);
    const uint32_t nu = pop64(um);
    if (nu > g.vmax) {
      fail_cap(__LINE__);
      return;
    }
    bool fast;
    if (protocol == FX_PROTOCOL_ATLAS) {
      const uint32_t threshold = qs - n / 2u;  // |quorum| - minority (atlas.rs:361-368)
      fast = !bal(first && cnt < threshold);
    } else {
      fast = nu == 0 || !bal(first && cnt != fq_eff);  // check_equal (quorum.rs:72-103)
    }
    uint32_t rank = 0;
    for (uint64_t m = um; m; m &= m - 1) rank += rl(v, ctz64(m)) < v ? 1u : 0u;
    if (first) S(sl, g.sl_value + rank) = v;  // (the copy's value words go stale: not read again here)
    const uint32_t c0 = sv(SL_CNT);
    sput(SL_CNT, (c0 & ~0xFF00u) | (nu << 8) | (fast ? 0u : (1u << 19)));
    const bool ro = (c0 >> 18) & 1u;
    // BaseProcess::path (base.rs:229-243): Fast / Slow at p, and their read-only shares
    if (lidv() == (fast ? A_FAST : A_SLOW) + p || (ro && lidv() == (fast ? A_FR : A_SR) + p)) ++pa;
    if (fast) act_send(M_COMMIT, dot, (1u << n) - 1u);
    else act_send(M_CONSENSUS, dot, (rl(pa, A_Q + p) >> 8) & 0xFFu);  // skip_prepare: ballot = coordinator
  }

  // the GC track's committed clock at p (MCommitDot, gc/clock.rs:43-48): the
  // frontier moves over every contiguous seq committed at p; a dot whose slot
  // was freed was executed, hence committed, everywhere
  __device__ __forceinline__ void gc_commit(uint32_t p, uint32_t dot) {
    const uint32_t si = FX_DOT_SRC(dot) - 1u, sq = FX_DOT_SEQ(dot);
    uint32_t fr = uni(lds[L_GCF + p * 8u + si]);
    if (sq != fr + 1u) return;
    const uint32_t top = rl(pa, A_SEQ + si);
    for (uint32_t guard = 0; guard <= g.NS; ++guard) {
      const uint32_t nx = fr + 1u;
      if (nx > top) break;
      const uint32_t d2 = FX_PACK_DOT(si + 1u, nx);
      const uint32_t sl = hslot(d2);
      if (rd(S(sl, SL_DOT)) == d2 && (rd(RC(sl, p, R_PST)) & 3u) != ST_COMMIT) break;
      fr = nx;
    }
    put(lds[L_GCF + p * 8u + si], fr);
  }

  // atlas.rs:404-475 / epaxos.rs:370-428
  __device__ __forceinline__ void h_mcommit(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    const uint32_t ps = rv(R_PST);
    if ((ps & 3u) == ST_START) {  // buffered_commits.insert
      rput(R_PST, (ps & ~0xF4u) | PS_BUF | (from << 4));
      return;
    }
    if ((ps & 3u) == ST_COMMIT) return;
    xinfo = sl;  // to_executors.push(GraphExecutionInfo::add(dot, cmd, value.deps))
    rput(R_PST, (ps & ~3u) | ST_COMMIT);
    const uint32_t masks = sv(SL_MASKS);
    sput(SL_MASKS, masks + (1u << 16));
    if (gc_ms_()) gc_commit(p, dot);  // Forward(MCommitDot) to self
  }

  // atlas.rs:477-524 / epaxos.rs:430-477
  __device__ __forceinline__ void h_mconsensus(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    const uint32_t ps = rv(R_PST);
    if ((ps & 3u) == ST_COMMIT) {  // chosen: reply with the chosen value
      act_send(M_COMMIT, dot, 1u << from);
      return;
    }
    rput(R_PST, ps | PS_ACC);
    act_send(M_CONSENSUS_ACK, dot, 1u << from);
  }

  // atlas.rs:526-558 / epaxos.rs:479-517
  __device__ __forceinline__ void h_mconsensusack(uint32_t p, uint32_t from, uint32_t dot) {
    const uint32_t sl = hslot_of(dot, p);
    if (sl == NONE) {
#ifdef FX_SIMX_DIAG
      if (!err) diag_slot(dot, p);
#endif
      fail_late(__LINE__);
      return;
    }
    if (!((sv(SL_CNT) >> 19) & 1u)) return;  // proposer ballot != b
    const uint32_t masks = sv(SL_MASKS);
    const uint32_t acc = ((masks >> 8) & 0xFFu) | (1u << from);
    if (pop32(acc) == synod_f + 1u) {
      sput(SL_MASKS, masks & ~0xFF00u);  // reset_state
      if (!(rv(R_PST) & PS_ACC)) {  // single.rs:346-349 panic
        fail_late(__LINE__);
        return;
      }
      act_send(M_COMMIT, dot, (1u << n) - 1u);
    } else {
      sput(SL_MASKS, (masks & ~0xFF00u) | (acc << 8));
    }
  }

  // ------------------------------------------------------------------ GC
  // periodic GarbageCollection at p (atlas.rs:699-714): MGarbageCollection
  // with p's committed frontier to every other process (ascending)
  __device__ __forceinline__ void gc_tick(uint32_t p) {
    const uint32_t fv = lds[L_GCF + ((p * 8u + lidv()) & 63u)];  // lane s: frontier of source s + 1
    for (uint32_t q = 0; q < n && !err; ++q) {
      if (q == p) continue;
      const uint32_t d = msg_delay(dpq_(p * 8u + q));
      const uint32_t e = push_event(now + d, (2u << 6) | (p << 3) | q, M_GC | (p << 4) | (q << 8), 0);
      if (e == NONE) return;
      if (lidv() < n) W(g.o_gp, e * n + lidv()) = fv;
    }
  }
  // MGarbageCollection at q from `from` (gc/clock.rs:50-138): merge the
  // reported frontier; once every other process reported, the stable range of
  // each source is (previous stable, min over all frontiers]; MStable to self
  // erases those dots (all committed at q), counted as Stable
  __device__ __forceinline__ void gc_deliver(uint32_t q, uint32_t from, uint32_t v) {
    // q's table of reported frontiers (row r = the last report from r, lane
    // r n + s = source s + 1) in one lane-parallel load; the report from
    // `from` is merged in registers and written back
    const uint32_t nn = n * n, base = L_GCO + q * nn;
    uint32_t blk = lidv() < nn ? lds[base + lidv()] : 0u;
    const uint32_t row = lidv() / n, src = lidv() - row * n;
    const uint32_t vs = gather(v, src & 63u);
    if (lidv() < nn && row == from) {
      blk = max(blk, vs);
      lds[base + lidv()] = blk;
    }
    const uint32_t rep = rl(pb, B_REP + q) | (1u << from);
    lset(pb, B_REP + q, rep);
    uint32_t cur = 0;
    const uint32_t mine = lds[L_GCF + ((q * 8u + lidv()) & 63u)];
    if (pop32(rep) == n - 1u) {
      cur = lidv() < n ? mine : 0u;
      for (uint32_t r = 0; r < n; ++r) {
        if (r == q) continue;
        const uint32_t o = gather(blk, (r * n + lidv()) & 63u);
        if (lidv() < n) cur = min(cur, o);
      }
    }
    const uint32_t prev = lds[L_GPS + ((q * 8u + lidv()) & 63u)];
    const uint32_t cnt = (lidv() < n && cur > prev) ? cur - prev : 0u;
    const uint32_t np = max(cur, prev);
    const uint32_t t = gather(np, lidv() & 7u);
    if ((lidv() >> 3) == q && (lidv() & 7u) < n) lds[L_GPS + lidv()] = t;
    uint32_t total = 0;
    for (uint32_t s = 0; s < n; ++s) total += rl(cnt, s);
    if (lidv() == A_STAB + q) pa += total;
  }

  // ===================================================== GraphExecutor
  // AEClock::contains at xp for a per-lane dot (tarjan.rs:131-132)
  __device__ __forceinline__ bool contains_v(uint32_t d) {
    if (!src_ok(d)) return false;
    const uint32_t sl = hslot(d);
    if (S(sl, SL_DOT) != d) return true;  // slot freed: executed everywhere
    return (RC(sl, xp, R_PST) & PS_EXEC) != 0;
  }

  // one executed command: to_execute -> Command::execute -> to_clients ->
  // AggregatePending (runner.rs:406-424), executor metrics, execution log
  __device__ __forceinline__ void on_execute(uint32_t sl, uint32_t d, uint32_t start) {
    const uint32_t p = xp;
    if (xk < kx()->exec_cap && kx()->executed && lidv() == 0) kx()->executed[((size_t)inst * n + p) * kx()->exec_cap + xk] = d;
    ++xk;
    hist_delay(now - start);  // ExecutionDelay (graph/mod.rs:514-518)
    if (rd(RC(sl, p, R_WAIT))) unlink(sl);
    const uint32_t c = rd(S(sl, SL_CLIENT));
    const uint32_t nk = (rd(S(sl, SL_CNT)) >> 16) & 3u;
    if ((rd(CL(c, 0)) & 0xFFu) == p) client_result(c, nk);  // pending.wait_for registered this rifl at p
    if (err) return;
    const uint32_t masks = rd(S(sl, SL_MASKS));
    if (((masks >> 24) & 0xFFu) + 1u == n) put(S(sl, SL_DOT), 0u);  // executed everywhere: free the slot
    else put(S(sl, SL_MASKS), masks + (1u << 24));
  }

  // AggregatePending::add_executor_result (aggregate.rs:48-87): one
  // ExecutorResult per key; the rifl is ready once all arrived
  __device__ __forceinline__ void client_result(uint32_t c, uint32_t nk) {
    const uint32_t pend = rd(CL(c, 3));
    if (pend < nk) {
      fail_late(__LINE__);
      return;
    }
    put(CL(c, 3), pend - nk);
    if (pend == nk) {
      if (rtop >= g.C + 64u) {
        fail_cap(__LINE__);
        return;
      }
      put(W(g.o_rdy, rtop++), c);
    }
  }

  // PendingIndex (index.rs:145-208): v waits on the dot in slot m
  __device__ __forceinline__ void unlink(uint32_t v) {
    const uint32_t p = xp;
    const uint32_t w = rd(RC(v, p, R_WAIT)), nx = rd(RC(v, p, R_NEXT)), pv = rd(RC(v, p, R_PREV));
    if (pv) put(RC(pv - 1u, p, R_NEXT), nx);
    else put(RC(w - 1u, p, R_HEAD), nx);
    if (nx) put(RC(nx - 1u, p, R_PREV), pv);
    put(RC(v, p, R_WAIT), 0u);
    put(RC(v, p, R_NEXT), 0u);
    put(RC(v, p, R_PREV), 0u);
  }
  __device__ __forceinline__ void index_pending(uint32_t v, uint32_t missing) {
    const uint32_t p = xp;
    if (rd(RC(v, p, R_WAIT))) unlink(v);
    const uint32_t m = slot_of(missing);
    if (m == NONE) {  // a missing dep is never executed at p, so its slot is live
      fail_late(__LINE__);
      return;
    }
    const uint32_t h = rd(RC(m, p, R_HEAD));
    put(RC(v, p, R_NEXT), h);
    put(RC(v, p, R_PREV), 0u);
    if (h) put(RC(h - 1u, p, R_PREV), v + 1u);
    put(RC(m, p, R_HEAD), v + 1u);
    put(RC(v, p, R_WAIT), m + 1u);
  }

  // sorts the slots W(src, 0 .. cnt) by dot, ascending, into W(dst, ..)
  // (SCC = BTreeSet<Dot>, tarjan.rs:15; waiters in C2 order)
  __device__ __forceinline__ void sort_slots(uint32_t src, uint32_t cnt, uint32_t dst) {
    if (cnt == 1) {
      put(W(dst, 0), rd(W(src, 0)));
      return;
    }
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
      const uint32_t i = i0 + lidv();
      const uint32_t msl = i < cnt ? W(src, i) : 0u;
      const uint32_t md = i < cnt ? S(msl, SL_DOT) : NONE;
      uint32_t rank = 0;
      for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
        const uint32_t k = k0 + lidv();
        const uint32_t kd = k0 == i0 ? md : (k < cnt ? S(W(src, k), SL_DOT) : NONE);
        const uint32_t m = min(64u, cnt - k0);
        for (uint32_t j = 0; j < m; ++j) rank += rl(kd, j) < md ? 1u : 0u;
      }
      if (i < cnt) W(dst, rank) = msl;
    }
  }

  // save_scc (mod.rs:488-523): the members W(o_tstk, base .. base + cnt)
  // (already in the executed clock) in ascending dot order; released dots
  // pushed to the worklist.  Up to 64 members at a time, lane-parallel: each
  // lane loads its member's fields at once, then the log, the ExecutionDelay
  // samples, the worklist and the slots' execution counts are written in
  // parallel; only waiter-list unlinks and the client results at the client's
  // own process go one by one, in order.
  __device__ __forceinline__ void save_scc(uint32_t base, uint32_t cnt) {
    hist_chain(cnt);
    ++xe;  // the graph lost vertices: every cached search result of xp is stale
    {
      XPROF_T0();
      sort_slots(g.o_tstk + base, cnt, g.o_tl);
      XPROF_ADD(PF_SORT);
    }
    XPROF_T0();
    if (nwl + cnt > 2u * g.NS) {
      fail_cap(__LINE__);
      return;
    }
    const uint32_t p = xp;
    for (uint32_t r0 = 0; r0 < cnt && !err; r0 += 64) {
      const uint32_t r = r0 + lidv();
      const bool act = r < cnt;
      uint32_t sl = 0, d = 0, st = 0, wt = 0, c = 0, cw = 0, mk = 0;
      if (act) {
        sl = W(g.o_tl, r);
        d = S(sl, SL_DOT);
        st = RC(sl, p, R_START);
        wt = RC(sl, p, R_WAIT);
        c = S(sl, SL_CLIENT);
        cw = S(sl, SL_CNT);
        mk = S(sl, SL_MASKS);
      }
      const uint32_t cpr = act ? CL(c, 0) : 0u;
      const uint32_t m = min(64u, cnt - r0);
      if (act) {
        if (kx()->executed && xk + lidv() < kx()->exec_cap) kx()->executed[((size_t)inst * n + p) * kx()->exec_cap + xk + lidv()] = d;
        W(g.o_wl, nwl + lidv()) = sl;
        if (kx()->delay_hist) {  // ExecutionDelay (graph/mod.rs:514-518)
          const uint32_t bn = min(now - st, kx()->delay_bins - 1u);
          if (bn < HD_BINS) atomicAdd(&lds[HC_BINS + bn], 1u);
          else atomicAdd(&kx()->delay_hist[bn], 1ull);
        }
        if (((mk >> 24) & 0xFFu) + 1u == n) S(sl, SL_DOT) = 0u;  // executed everywhere: free the slot
        else S(sl, SL_MASKS) = mk + (1u << 24);
      }
      xk += m;
      nwl += m;
      const uint64_t need = bal(act && (wt != 0 || (cpr & 0xFFu) == p));
      for (uint64_t mm = need; mm && !err; mm &= mm - 1) {
        const uint32_t j = ctz64(mm);
        if (rl(wt, j)) unlink(rl(sl, j));
        if ((rl(cpr, j) & 0xFFu) == p) client_result(rl(c, j), (rl(cw, j) >> 16) & 3u);
      }
    }
    XPROF_ADD(PF_EMIT);
  }

  // the per-lane states of the top frame's deps, lanes [ci, cnd): the tag of
  // the dep's slot and its record at xp (status, Tarjan id / low, mark).
  // They stay valid until the search recurses (nothing else writes them).
  __device__ __forceinline__ void dep_states(uint32_t drow, uint32_t ci, uint32_t cnd, uint32_t& ptag,
                                             uint32_t& ppst, uint32_t& ptl, uint32_t& pmk) {
    ptag = ppst = ptl = pmk = 0;
    if (lidv() >= ci && lidv() < cnd && src_ok(drow)) {
      const uint32_t sl = hslot(drow);
      ptag = S(sl, SL_DOT);
      ppst = RC(sl, xp, R_PST);
      ptl = RC(sl, xp, R_TL);
      pmk = RC(sl, xp, R_MARK);
    }
  }
  // a vertex's dot, dep count and dep row (lane j = dep j), loaded together
  __device__ __forceinline__ void frame_row(uint32_t sl, uint32_t& cdot, uint32_t& cnd, uint32_t& drow) {
    const uint32_t t = S(sl, SL_DOT), cw = S(sl, SL_CNT);
    drow = lidv() < g.vmax ? S(sl, g.sl_value + lidv()) : 0u;
    cdot = uni(t);
    cnd = (uni(cw) >> 8) & 0xFFu;
    if (lidv() >= cnd) drow = 0;
  }

  // find_scc (mod.rs:409-486) + strong_connect (tarjan.rs:96-316) + finalize
  // (tarjan.rs:60-93) from the pending vertex in slot rsl.  On a missing dep,
  // *missing = it and the vertices left on the stack are marked visited with
  // mark_epoch (0 = no marks).
  __device__ __forceinline__ uint32_t find_scc(uint32_t rsl, uint32_t* missing, uint32_t mark_epoch, bool* saved) {
    XPROF_T0();
    XPROF_CNT(PC_FIND, 1);
    const uint32_t r = find_scc_(rsl, missing, mark_epoch, saved);
    XPROF_ADD(PF_FIND);
    return r;
  }
  __device__ __forceinline__ uint32_t find_scc_(uint32_t rsl, uint32_t* missing, uint32_t mark_epoch, bool* saved) {
    const uint32_t p = xp;
    *saved = false;
    idc = 1;
    tsp = 0;
    // DFS frames 0..63 in lanes: slot | next dep << 24, and the stack
    // position of the frame's vertex; deeper frames in W(o_fv / o_fi)
    uint32_t frs = 0, frt = 0;
    const uint32_t mk0 = rd(RC(rsl, p, R_MARK));
    put(RC(rsl, p, R_TL), 1u | (1u << 16));
    put(RC(rsl, p, R_MARK), mk0 | 1u);
    put(W(g.o_tstk, tsp++), rsl);
    fsp = 1;
    // the top frame in registers: slot, next dep, id, low, stack position,
    // dot, dep count, dep row and the deps' prefetched states
    uint32_t cv = rsl, ci = 0, cid = 1, clow = 1, ctp = 0, cdot = 0, cnd = 0, drow = 0;
    frame_row(rsl, cdot, cnd, drow);
    uint32_t ptag, ppst, ptl, pmk;
    dep_states(drow, 0, cnd, ptag, ppst, ptl, pmk);
    uint32_t result = FOUND;
    for (uint32_t guard = 0; fsp && !err; ++guard) {
      if (guard > 64u * g.NS + 64u) {
        fail_cap(__LINE__);
        break;
      }
      if (ci < cnd) {
        const uint32_t d = rl(drow, ci), tag = rl(ptag, ci), ps = rl(ppst, ci);
        ++ci;
        XPROF_CNT(PC_EDGES, 1);
        // self (tarjan.rs:128-130); executed everywhere (its slot was freed)
        // or here (tarjan.rs:131-145)
        if (d == cdot || !src_ok(d) || tag != d || (ps & PS_EXEC)) continue;
        if (!(ps & PS_INGRAPH)) {  // missing (tarjan.rs:148-157, shard_count == 1)
          *missing = d;
          result = MISSING;
          break;
        }
        const uint32_t tw = rl(ptl, ci - 1u), mk = rl(pmk, ci - 1u);
        if ((tw & 0xFFFFu) == 0) {  // recurse (tarjan.rs:172-214)
          XPROF_CNT(PC_RECURSE, 1);
          const uint32_t f = fsp - 1u;
          if (f < 64u) {
            lset(frs, f, cv | (ci << 24));
            lset(frt, f, ctp);
          } else {
            put(W(g.o_fv, f), cv | (ci << 24));
            put(W(g.o_fi, f), ctp);
          }
          put(RC(cv, p, R_TL), cid | (clow << 16));
          ++idc;
          if (idc > 0xFFFFu || tsp >= g.NS || fsp >= g.NS) {
            fail_cap(__LINE__);
            break;
          }
          const uint32_t sl = hslot(d);
          put(RC(sl, p, R_TL), idc | (idc << 16));
          put(RC(sl, p, R_MARK), mk | 1u);
          ctp = tsp;
          put(W(g.o_tstk, tsp++), sl);
          ++fsp;
          cv = sl;
          ci = 0;
          cid = idc;
          clow = idc;
          frame_row(sl, cdot, cnd, drow);
          dep_states(drow, 0, cnd, ptag, ppst, ptl, pmk);
        } else if (mk & 1u) {  // on the stack (tarjan.rs:215-225)
          clow = min(clow, tw & 0xFFFFu);
        }
        continue;
      }
      // cv finished
      const uint32_t lowv = clow;
      if (cid == lowv) {  // SCC root: pop the members tstk[ctp, tsp) (tarjan.rs:233-312)
        bool broken = false;
        for (uint32_t i0 = ctp; i0 < tsp; i0 += 64) {
          const uint32_t i = i0 + lidv();
          uint32_t psx = PS_INGRAPH;
          if (i < tsp) {
            const uint32_t x = W(g.o_tstk, i);
            const uint32_t mkx = RC(x, p, R_MARK);
            psx = RC(x, p, R_PST);
            RC(x, p, R_MARK) = mkx & ~1u;
            RC(x, p, R_PST) = psx | PS_EXEC;  // executed_clock.add (tarjan.rs:293)
          }
          // a member in xp's graph and not executed yet (tarjan.rs:245-255 expects)
          broken = broken || bal((psx & (PS_INGRAPH | PS_EXEC)) != PS_INGRAPH);
        }
        if (broken) {
#ifdef FX_SIMX_DIAG
          if (!err) {
            dput(8, rsl | ((uint64_t)tsp << 32));
            dput(9, ctp | ((uint64_t)cv << 32));
            for (uint32_t i0 = ctp; i0 < tsp; i0 += 64) {
              const uint32_t i = i0 + lidv();
              const uint32_t x = i < tsp ? W(g.o_tstk, i) : 0u;
              const uint32_t psx = i < tsp ? RC(x, p, R_PST) : PS_INGRAPH;
              const uint64_t m = bal((psx & (PS_INGRAPH | PS_EXEC)) != PS_INGRAPH);
              if (m) {
                const uint32_t j = ctz64(m), xj = rl(x, j);
                dput(10, xj | ((uint64_t)rl(psx, j) << 32));
                dput(11, S(xj, SL_DOT) | ((uint64_t)S(xj, SL_MASKS) << 32));
                dput(12, RC(xj, p, R_TL) | ((uint64_t)RC(xj, p, R_MARK) << 32));
                dput(13, (i0 + j) | ((uint64_t)pop64(m) << 32));
                break;
              }
            }
          }
#endif
          fail_late(__LINE__);
          break;
        }
        save_scc(ctp, tsp - ctp);
        tsp = ctp;
        *saved = true;
        if (err) break;
      }
      --fsp;
      if (fsp) {  // resume the parent frame (tarjan.rs:211: low = min(low, dep low))
        const uint32_t f = fsp - 1u;
        uint32_t pk, tp;
        if (f < 64u) {
          pk = rl(frs, f);
          tp = rl(frt, f);
        } else {
          pk = rd(W(g.o_fv, f));
          tp = rd(W(g.o_fi, f));
        }
        cv = pk & 0xFFFFFFu;
        ci = pk >> 24;
        ctp = tp;
        const uint32_t tw = RC(cv, p, R_TL);
        frame_row(cv, cdot, cnd, drow);
        cid = uni(tw) & 0xFFFFu;
        clow = min(uni(tw) >> 16, lowv);
        dep_states(drow, ci, cnd, ptag, ppst, ptl, pmk);
      }
    }
    // finalize: ids of the vertices left on the stack; failed searches mark them visited
    const bool markit = mark_epoch && result == MISSING;
    for (uint32_t i0 = 0; i0 < tsp; i0 += 64) {
      const uint32_t i = i0 + lidv();
      if (i < tsp) {
        const uint32_t x = W(g.o_tstk, i);
        RC(x, p, R_TL) = 0u;
        if (markit) RC(x, p, R_MARK) = (RC(x, p, R_MARK) & 1u) | (mark_epoch << 1);
      }
    }
    tsp = 0;
    return result;
  }

  // PendingIndex::remove (index.rs:204-207) of the released dot in slot x:
  // unregisters its waiters and sorts them ascending (C2) into W(o_tw, ..)
  __device__ __forceinline__ uint32_t take_waiters(uint32_t x) {
    const uint32_t p = xp;
    uint32_t v = rd(RC(x, p, R_HEAD));
    if (!v) return 0;
    put(RC(x, p, R_HEAD), 0u);
    uint32_t cnt = 0;
    while (v) {
      const uint32_t sl = v - 1u;
      if (cnt >= g.NS) {
        fail_cap(__LINE__);
        return 0;
      }
      const uint32_t nx = rd(RC(sl, p, R_NEXT));
      put(W(g.o_tmp, cnt++), sl);
      put(RC(sl, p, R_WAIT), 0u);
      put(RC(sl, p, R_NEXT), 0u);
      put(RC(sl, p, R_PREV), 0u);
      v = nx;
    }
    XPROF_CNT(PC_WAITERS, cnt);
    sort_slots(g.o_tmp, cnt, g.o_tw);
    return cnt;
  }

  // GraphExecutor::handle(Add) (executor.rs:69-80) -> handle_add (mod.rs:213-275)
  __device__ __forceinline__ void x_add(uint32_t p, uint32_t sl) {
    XPROF_T0();
    XPROF_CNT(PC_XADD, 1);
    x_add_(p, sl);
    XPROF_ADD(PF_XADD);
  }
  // The searches of one handle_add: the new vertex's first find, then
  // check_pending (mod.rs:556-587) LIFO over the released dots and
  // try_pending (589-642) over each one's waiters in ascending dot order (C2),
  // skipping the ones a failed search of this round visited.  One loop, one
  // find_scc call site.
  __device__ __forceinline__ void x_add_(uint32_t p, uint32_t sl) {
    xp = p;
    xk = rl(pa, A_EXEC + p);
    xe = rl(pb, B_XE + p);
    nwl = 0;
    // the slot's row and p's record: the copy the committing handler loaded
    // (run_handlers calls x_add right after h_mcommit), else one load
    if (hsl != sl || hpp != p) hload(sl, p);
    const uint32_t d = sv(SL_DOT);
    const uint32_t ps = rv(R_PST);
    if (ps & (PS_INGRAPH | PS_EXEC)) {
      err = FX_ERR_DOUBLE_INDEX;
      return;
    }
    const uint32_t vc = (sv(SL_CNT) >> 8) & 0xFFu;
    lds_add64(L_DEPS, vc);
    const uint32_t depj = svl(g.sl_value, vc);
    // every dep's slot tag and record at p in one round trip (lane j: dep j):
    // AEClock::contains (tarjan.rs:131-132: a freed slot was executed
    // everywhere) and the search-result cache words below
    uint32_t dtag = 0, dps = 0, dcm = 0, dce = 0;
    const bool dl = lidv() < vc && depj != d && src_ok(depj);
    if (dl) {
      const uint32_t dsl = hslot(depj);
      dtag = S(dsl, SL_DOT);
      dps = RC(dsl, p, R_PST);
      dcm = RC(dsl, p, R_CMISS);
      dce = RC(dsl, p, R_CEPOCH);
    }
    bool keep = false;
    if (lidv() < vc && depj != d) keep = !src_ok(depj) || (dtag == depj && !(dps & PS_EXEC));
    bool first = bal(keep) != 0;
    if (!first) {  // every dep executed: a singleton SCC
      XPROF_CNT(PC_FAST, 1);
      rput(R_PST, ps | PS_EXEC);
      ++xe;
      hist_chain(1u);
      put(W(g.o_wl, nwl++), sl);
      on_execute(sl, d, now);
    } else {
      rput(R_PST, ps | PS_INGRAPH);
      put(RC(sl, p, R_START), nowv());  // Vertex::start_time_ms (tarjan.rs:332-348)
      // The first search from the new vertex v enters its first dep u that is
      // neither v nor executed (deps ascend, C1).  If u is pending and the last
      // search rooted at u stopped at missing dep m with no execution at p
      // since, and m is still missing and is not v, this search stops at m
      // too, having found no SCC: u's walk meets the same deps in the same
      // states up to m (a vertex that was pending then is still pending; one
      // that was missing then would have stopped that search, so only m can
      // have arrived; v itself is reachable only through a dep that was
      // missing then).  So v just waits on m (index_pending) — no walk; and
      // v's own result is the same cache entry.
      const uint32_t j0 = ctz64(bal(keep));
      const uint32_t u = rl(depj, j0);
      const uint32_t ut = rl(dtag, j0), ups = rl(dps, j0), cm = rl(dcm, j0), uce = rl(dce, j0);
      if (src_ok(u) && ut == u && (ups & (PS_INGRAPH | PS_EXEC)) == PS_INGRAPH && cm && cm != d && uce == xe &&
          src_ok(cm)) {
        // m's tag, its record at p and the head of its waiter list together
        const uint32_t msl = hslot(cm);
        const uint32_t mt = S(msl, SL_DOT), mps = RC(msl, p, R_PST), mh = RC(msl, p, R_HEAD);
        if (uni(mt) == cm && !(uni(mps) & (PS_INGRAPH | PS_EXEC))) {
          XPROF_CNT(PC_CACHE, 1);
          // index_pending (mod.rs:525-554) of the fresh vertex (it waits on
          // nothing yet: its record was zeroed when its dot was proposed)
          const uint32_t h = uni(mh);
          put(RC(sl, p, R_NEXT), h);
          put(RC(sl, p, R_PREV), 0u);
          if (h) put(RC(h - 1u, p, R_PREV), sl + 1u);
          put(RC(msl, p, R_HEAD), sl + 1u);
          put(RC(sl, p, R_WAIT), msl + 1u);
          put(RC(sl, p, R_CMISS), cm);
          put(RC(sl, p, R_CEPOCH), xe);
          first = false;
        }
      }
    }
    hforget();
    XPROF_T0();
    uint32_t wk = 0, wcnt = 0, cur = 0;  // the waiter list being tried
    uint32_t wps = 0, wmk = 0, wbase = NONE;  // lanes: states of waiters [wbase, wbase + 64)
    while (!err) {
      uint32_t root, mark = 0;
      if (first) {
        root = sl;
        first = false;
      } else {
        // the next waiter still pending and not visited in this round
        root = NONE;
        while (wk < wcnt) {
          if (wbase == NONE || wk >= wbase + 64u) {
            wbase = wk;
            wps = wmk = 0;
            if (wbase + lidv() < wcnt) {
              const uint32_t w = W(g.o_tw, wbase + lidv());
              wps = RC(w, p, R_PST);
              wmk = RC(w, p, R_MARK);
            }
          }
          const uint64_t ok = bal(lidv() >= wk - wbase && wbase + lidv() < wcnt && !(wps & PS_EXEC) &&
                                  (wmk >> 1) != cur);
          if (!ok) {
            wk = wbase + 64u;
            continue;
          }
          const uint32_t j = ctz64(ok);
          root = rd(W(g.o_tw, wbase + j));
          wk = wbase + j + 1u;
          break;
        }
        if (root == NONE) {  // this list is done: the next released dot with waiters
          if (!nwl) break;
          wcnt = take_waiters(rd(W(g.o_wl, --nwl)));
          wk = 0;
          wbase = NONE;
          cur = ++epoch;  // try_pending's visited set starts empty
          continue;
        }
        mark = cur;
      }
      uint32_t missing = 0;
      bool saved = false;
      const uint32_t r = find_scc(root, &missing, mark, &saved);
      if (err) break;
      if (r == MISSING) {
        index_pending(root, missing);  // index_pending (mod.rs:525-554)
        if (!saved) {  // a fresh search from root now stops at `missing`
          put(RC(root, p, R_CMISS), missing);
          put(RC(root, p, R_CEPOCH), xe);
        }
      }
      if (mark && (r == FOUND || saved)) {
        cur = ++epoch;  // visited.clear()
        wbase = NONE;   // marks and states changed: reload the waiters' states
      } else if (mark) {
        wbase = NONE;
      }
    }
    XPROF_ADD(PF_CHECK);
    lset(pa, A_EXEC + p, xk);
    lset(pb, B_XE + p, xe);
  }

  // =========================================== send_to_processes_and_executors
  __device__ __forceinline__ void frame_push() {
    if (nfrm >= FMAX) {
      fail_cap(__LINE__);
      return;
    }
    const uint32_t fi = nfrm++;
    lset(pb, B_FRW + fi, 0);
    lset(pb, B_FRB + fi, rtop);
    xinfo = NONE;
  }
  __device__ __forceinline__ void send_p(uint32_t from, uint32_t to, uint32_t kind, uint32_t dot) {
    XPROF_T0();
    XPROF_CNT(PC_SEND, 1);
    const uint32_t d = msg_delay(dpq_(from * 8u + to));
    push_event(now + d, 0u, kind | (from << 4) | (to << 8), dot);
    XPROF_ADD(PF_SEND);
  }

  // handle_send_to_proc / handle_submit_to_proc, then
  // send_to_processes_and_executors (runner.rs:351-377, 395-488) with every
  // self-delivery in the reference's recursion order (sim_wave.hip's loop)
  __device__ __forceinline__ void run_handlers(uint32_t p, uint32_t from, uint32_t kind, uint32_t w2) {
    bool pend = true;
    for (uint32_t guard = 0; !err; ++guard) {
      if (guard > 4096u) {
        fail_cap(__LINE__);
        return;
      }
      if (pend) {
        pend = false;
        frame_push();
        if (err) return;
        XPROF_T0();
        switch (kind) {
          case M_SUBMIT: h_submit(p, w2); break;
          case M_COLLECT: h_mcollect(p, from, w2); break;
          case M_COLLECT_ACK: h_mcollectack(p, from, w2); break;
          case M_COMMIT: h_mcommit(p, from, w2); break;
          case M_CONSENSUS: h_mconsensus(p, from, w2); break;
          case M_CONSENSUS_ACK: h_mconsensusack(p, from, w2); break;
          case M_STORE: h_mstore(p, from, w2); break;
          case M_STORE_ACK: h_mstoreack(p, from, w2); break;
          case M_COMMIT_BASIC: h_bcommit(p, w2); break;
          default: err = FX_ERR_INVALID_ARG;
        }
        XPROF_ADD(PF_HANDLER);
        if (xinfo != NONE && !err) {  // to_executors (<= 1 per handler)
          const uint32_t sl = xinfo;
          xinfo = NONE;
          x_add(p, sl);
        }
        hforget();
        continue;
      }
      if (nfrm == 0) return;
      const uint32_t fi = nfrm - 1;
      const uint32_t w = rl(pb, B_FRW + fi);
      if (w & 3u) {  // ToSend: targets ascending (C4), self recurses in place
        const uint32_t tgt = (w >> 8) & 0xFFu, k2 = (w >> 2) & 15u, dot = rl(pb, B_FRD + fi);
        uint32_t nx = (w >> 16) & 15u;
        while (nx < n) {
          const uint32_t to = nx++;
          if (!((tgt >> to) & 1u)) continue;
          if (to == p) {
            lset(pb, B_FRW + fi, (w & ~(15u << 16)) | (nx << 16));
            from = p;
            kind = k2;
            w2 = dot;
            pend = true;
            break;
          }
          send_p(p, to, k2, dot);
          if (err) return;
        }
        if (pend) continue;
        lset(pb, B_FRW + fi, 0);
      }
      // ready results -> schedule_to_client (runner.rs:434-440, 491-504)
      XPROF_T0();
      const uint32_t b = rl(pb, B_FRB + fi);
      for (uint32_t r = b; r < rtop && !err; ++r) {
        const uint32_t c = rd(W(g.o_rdy, r));
        const uint32_t d = msg_delay(rd(CL(c, 5)));
        push_event(now + d, 0u, E_CLIENT, c);
      }
      rtop = b;
      --nfrm;
      XPROF_ADD(PF_READY);
    }
  }

  // ======================================================= event loop
  // Client::cmd_send: the next command of client c -> SubmitToProc
  __device__ __forceinline__ bool client_send(uint32_t c) {
    const uint32_t issued = rd(CL(c, 1));
    if (issued >= cmds_()) return false;
    put(CL(c, 1), issued + 1u);
    put(CL(c, 2), now);  // Pending::start
    const uint32_t d = msg_delay(rd(CL(c, 4)));
    push_event(now + d, 0u, M_SUBMIT | ((rd(CL(c, 0)) & 0xFFu) << 8), c);
    return true;
  }

  __device__ __forceinline__ void run_event(uint32_t kind, uint32_t from, uint32_t to, uint32_t arg, uint32_t gcv) {
    switch (kind) {
      case M_SUBMIT: {
        const uint32_t c = arg, p = to;
        note(2, p + 1, c + 1, rd(CL(c, 1)));
        put(CL(c, 3), K);  // AggregatePending::wait_for: key_count results
        run_handlers(p, p, M_SUBMIT, c);
        return;
      }
      case E_CLIENT: {  // Client::cmd_recv + cmd_send (simulation.rs:132-149)
        XPROF_T0();
        const uint32_t c = arg;
        const uint32_t issued = rd(CL(c, 1));
        note(4, c + 1, 0, issued);
        const uint32_t lat = now - rd(CL(c, 2));  // latency.as_millis()
        lds_add64(L_LATSUM, lat);
#ifndef FX_SIMX_EVLOG
        if (lidv() == 0 && kx()->latency_log && issued - 1u < kx()->lat_cap)
          kx()->latency_log[((size_t)inst * g.C + c) * kx()->lat_cap + issued - 1u] = lat;
#endif
        hist_lat(rd(CL(c, 0)) >> 8, lat);
        if (!client_send(c)) {
          ++clients_done;
          if (clients_done == g.C) {
            if (has_extra) {
              final_ms = now + extra_();
              in_extra = true;
            } else {
              done = true;
            }
          }
        }
        XPROF_ADD(PF_CLIENT);
        return;
      }
      case E_TICK: {
        XPROF_T0();
        gc_tick(to);
        push_event(now + gc_ms_(), (1u << 6) | (to << 3), E_TICK | (to << 8), 0);
        XPROF_ADD(PF_GC);
        return;
      }
      case E_NOTIF:  // GraphExecutor::executed is None (executor/mod.rs:74-79)
        push_event(now + en_ms_(), 0u, E_NOTIF | (to << 8), 0);
        return;
      case M_GC: {
        XPROF_T0();
        gc_deliver(to, from, gcv);
        XPROF_ADD(PF_GC);
        return;
      }
      default:
        note(3, to + 1, from + 1, ((uint64_t)kind << 32) | arg);
        run_handlers(to, from, kind, arg);
    }
  }
};

// waves per SIMD the register budget is built for (3: 168 VGPRs, no spills).
// The build with configs[3]'s geometry compiled in (GS, HBM Tarjan records)
// holds fewer values in registers: at 4 (128 VGPRs, 52 bytes of spills per
// lane) 16 instances per CU instead of 12, 117 -> 138 M cmds/s at 4,096
// instances (profiles/archive/calls/r5_occ2.sh); at 5 (102 VGPRs, 136 bytes of spills) with
// two instances per workgroup (a CU holds at most 16 workgroups) 20 per CU,
// 139.4 -> 144.3 M at 5,120 instances (profiles/archive/calls/r5_x5.sh)
#ifndef FX_SIMX_WAVES
#define FX_SIMX_WAVES 3
#endif
#ifndef FX_SIMX_WAVES_GS
#define FX_SIMX_WAVES_GS 5
#endif
// instances per workgroup of that build (a CU holds at most 16 workgroups)
#ifndef FX_SIMX_WPB
#define FX_SIMX_WPB 2
#endif
// GS != 0: the geometry geo_compiled(GS) compiled in (the host launches it
// when the batch's geometry equals it word for word): its offsets become
// immediates instead of scalar registers, of which the kernel is short
template <uint32_t NG, uint32_t GS = 0, uint32_t WPB = 1>
__global__ __launch_bounds__(64 * WPB, GS != 0 ? FX_SIMX_WAVES_GS : FX_SIMX_WAVES) void k_simx(ArgsX a) {
  // LDS_WORDS of histogram caches per instance (WPB instances per workgroup)
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_all[];
  const uint32_t wv = WPB > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0u;
  uint32_t* smem = smem_all + wv * LDS_WORDS;
  const uint32_t inst = blockIdx.x * WPB + wv;
  if (inst >= a.instances) return;  // whole wavefront
  Big<NG> s;
  if constexpr (GS != 0) {
    constexpr GeoX gc = geo_compiled(GS);
    static_assert(gc.words != 0, "compiled geometry");
    s.g = gc;
  } else {
    s.g = a.g;
  }
  s.lid_ = threadIdx.x & 63u;
  s.M = a.arena + (size_t)inst * s.g.words;
  s.lds = smem;
  s.inst = inst;
  const fx_sim_spec& sp = a.specs[inst];
  s.protocol = sp.protocol;
  s.n = s.g.n;
  s.f = sp.f;
  s.C = s.g.C;
  s.K = s.g.K;
  s.reorder = sp.reorder_messages != 0;
  s.nfr = sp.nfr != 0;
  s.has_extra = sp.extra_sim_time_ms >= 0;
  const uint32_t n = s.n;
  uint32_t fq, wq;
  if (s.protocol == FX_PROTOCOL_ATLAS) {
    fq = n / 2 + s.f;
    wq = s.f + 1;
    s.synod_f = s.f;
  } else if (s.protocol == FX_PROTOCOL_BASIC) {
    fq = s.f + 1;  // basic_quorum_size (config.rs:285-287); no write quorum
    wq = 0;
    s.synod_f = 0;
  } else {
    const uint32_t fe = n / 2;
    fq = fe + (fe + 1) / 2;
    wq = fe + 1;
    s.synod_f = fe;  // EPaxos::allowed_faults
  }
  const uint32_t maj = n / 2 + 1;
  const GeoX& g = a.g;
  uint32_t* M = s.M;
  // ---------------------------------------------------------------- init
  for (uint32_t i = s.lidv(); i < LDS_WORDS; i += 64) smem[i] = 0;
  for (uint32_t i = s.lidv(); i < g.NS; i += 64) M[g.o_slot + i * g.SW + SL_DOT] = 0;
  for (uint32_t i = s.lidv(); i < g.n * g.ncli_keys * 2u; i += 64) M[g.o_kd + i] = 0;
  for (uint32_t i = s.lidv(); i < g.R; i += 64) {
    M[g.o_kh + i] = NONE;
    M[g.o_kl + i] = NONE;
    M[g.o_free + i] = g.R - 1u - i;  // free stack
  }
  s.nfree = g.R;
#pragma unroll
  for (uint32_t k = 0; k < NG; ++k) s.gh[k] = s.gl[k] = NONE;
  const uint32_t RP = a.RP;
  // process quorums (BaseProcess::discover over sort_processes_by_distance,
  // base.rs:62-154, util.rs:153-185) and link delays
  for (uint32_t p = 0; p < n; ++p) {
    const uint32_t rp = sp.process_regions[p];
    uint32_t pos = 0;
    if (s.lidv() < n) {
      const uint32_t kq = a.rank[rp * RP + sp.process_regions[s.lidv()]];
      for (uint32_t q2 = 0; q2 < n; ++q2) {
        const uint32_t k2 = a.rank[rp * RP + sp.process_regions[q2]];
        if (k2 < kq || (k2 == kq && q2 < s.lidv())) ++pos;
      }
    }
    const uint32_t fqm = (uint32_t)bal(s.lidv() < n && pos < fq);
    const uint32_t wqm = (uint32_t)bal(s.lidv() < n && pos < wq);
    const uint32_t mqm = (uint32_t)bal(s.lidv() < n && pos < maj);
    s.lset(s.pa, s.A_Q + p, fqm | (wqm << 8) | (mqm << 16));
    if (s.lidv() >= p * 8u && s.lidv() < p * 8u + n) smem[L_DPQ + s.lidv()] = a.ping[rp * RP + sp.process_regions[s.lidv() - p * 8u]] / 2u;
  }
  // clients: for region in client_regions, clients_per_region each (runner.rs:143-163)
  {
    uint32_t c0 = 0;
    for (uint32_t r = 0; r < sp.num_client_regions; ++r) {
      const uint32_t rc = sp.client_regions[r];
      uint32_t best = 0, bk = 0xFFFFFFFFu;
      for (uint32_t p = 0; p < n; ++p) {  // closest process: minimal (rank, id)
        const uint32_t k = a.rank[rc * RP + sp.process_regions[p]];
        if (k < bk) {
          bk = k;
          best = p;
        }
      }
      const uint32_t dcs = a.ping[rc * RP + sp.process_regions[best]] / 2u;
      const uint32_t dcr = a.ping[sp.process_regions[best] * RP + rc] / 2u;
      for (uint32_t i = s.lidv(); i < sp.clients_per_region; i += 64) {
        const uint32_t c = c0 + i;
        M[g.o_cl + c * 8u + 0] = best | (rc << 8);
        M[g.o_cl + c * 8u + 1] = 0;
        M[g.o_cl + c * 8u + 2] = 0;
        M[g.o_cl + c * 8u + 3] = 0;
        M[g.o_cl + c * 8u + 4] = dcs;
        M[g.o_cl + c * 8u + 5] = dcr;
      }
      c0 += sp.clients_per_region;
    }
  }
  if constexpr (WPB > 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
#ifdef FX_SIMX_DIAG
  // canaries in arena words the simulation never writes (client words 6 / 7,
  // the ready list's last entry), checked after every event: a write the
  // kernel did not make (or a stray one of its own) shows up at its event
  const uint32_t can_v = 0xC0FFEE00u | (inst & 0xFFu);
  const uint32_t can_a = g.o_cl + 6u, can_b = g.o_cl + (s.C - 1u) * 8u + 7u, can_c = g.o_rdy + s.C + 63u;
  if (s.lidv() == 0) {
    M[can_a] = can_v;
    M[can_b] = can_v;
    M[can_c] = can_v;
  }
  if constexpr (WPB > 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
#endif
  // periodic events (runner.rs:179-187), then clients (run(), C5 ascending)
  if (s.gc_ms_())
    for (uint32_t p = 0; p < n; ++p) s.push_event(s.gc_ms_(), (1u << 6) | (p << 3), E_TICK | (p << 8), 0);
  const bool sim_en = a.sim_exec_notif || s.has_extra;
  for (uint32_t p = 0; p < n; ++p) {
    if (sim_en) s.push_event(s.en_ms_(), 0u, E_NOTIF | (p << 8), 0);
    else ++s.seq;  // keep the insertion numbering of the reference
  }
  for (uint32_t c = 0; c < s.C && !s.err; ++c) {
    if (s.cmds_() == 0) s.err = FX_ERR_INVALID_ARG;
    else s.client_send(c);
  }
  // ------------------------------------------------------------ loop
  const uint32_t max_events = a.max_events ? a.max_events : 0xFFFFFFFFu;
#ifdef FX_SIMX_EVLOG
  uint32_t evn = 0;
#endif
  while (!s.done && !s.err) {
    uint32_t hi = 0;
#ifdef FX_SIM_PROFILE
    const uint64_t pt0 = __builtin_amdgcn_s_memtime();
#endif
    uint32_t info = 0, arg = 0;
    const uint32_t e = s.pop_event(hi, info, arg);
#ifdef FX_SIM_PROFILE
    const uint64_t pt1 = __builtin_amdgcn_s_memtime();
    s.prof[PF_POP] += pt1 - pt0;
    s.prof[PC_EVENTS] += 1;
#endif
    if (e == NONE) {
      if (!s.err) s.fail_late(__LINE__);  // "there should be a new action"
      break;
    }
    const uint32_t t = hi >> 8;
    if (t < s.now) {
      s.err = FX_ERR_TIME_RANGE;
      break;
    }
    s.now = t;
    const uint32_t kind = info & 15u, from = (info >> 4) & 15u, to = (info >> 8) & 15u;
    const uint32_t gcv = kind == M_GC && s.lidv() < n ? M[g.o_gp + e * n + s.lidv()] : 0u;
#ifdef FX_SIMX_DIAG
    s.cur_info = info;
    s.cur_arg = arg;
    s.cur_hi = hi;
#endif
    s.free_event(e);
#ifdef FX_SIMX_DIAG
    {
      const uint32_t ca = uni(M[can_a]), cb = uni(M[can_b]), cc = uni(M[can_c]);
      if ((ca != can_v || cb != can_v || cc != can_v) && !s.err) {
        s.dput(16, ca | ((uint64_t)cb << 32));
        s.dput(17, cc | ((uint64_t)s.events << 32));
        s.fail_late(__LINE__);
        break;
      }
    }
#endif
    s.run_event(kind, from, to, arg, gcv);
#ifdef FX_SIMX_EVLOG
    // debug build (tools/simx_repro.py): every event's key, info, argument and
    // the trace hash after it, into the instance's latency-log region
    if (s.lidv() == 0 && a.latency_log && 4ull * evn + 3ull < (uint64_t)g.C * a.lat_cap) {
      uint32_t* lg = a.latency_log + (size_t)inst * g.C * a.lat_cap + 4ull * evn;
      lg[0] = hi;
      lg[1] = info;
      lg[2] = arg;
      lg[3] = (uint32_t)s.trace ^ (uint32_t)(s.trace >> 32);
    }
    ++evn;
#endif
#ifdef FX_SIM_PROFILE
    s.prof[PF_EVENT] += __builtin_amdgcn_s_memtime() - pt1;
#endif
    if (s.in_extra && s.now > s.final_ms) s.done = true;
    if (s.events >= max_events) s.err = FX_ERR_SIM_EVENTS;
  }
  // ----------------------------------------------------------- outputs
  if constexpr (WPB > 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
  const uint32_t o_exec = gather(s.pa, (s.A_EXEC + s.lidv()) & 63u), o_fast = gather(s.pa, (s.A_FAST + s.lidv()) & 63u),
                 o_slow = gather(s.pa, (s.A_SLOW + s.lidv()) & 63u), o_stab = gather(s.pa, (s.A_STAB + s.lidv()) & 63u),
                 o_fr = gather(s.pa, (s.A_FR + s.lidv()) & 63u), o_sr = gather(s.pa, (s.A_SR + s.lidv()) & 63u);
  if (s.lidv() < n && a.executed_len) a.executed_len[(size_t)inst * n + s.lidv()] = o_exec;
  if (a.stats) {
    unsigned long long* st = a.stats + (size_t)inst * FX_SIM_STATS;
#ifdef FX_SIMX_DIAG
    if (false) {
#else
    if (s.lidv() < NMAX) {
#endif
      const bool v = s.lidv() < n;
      st[FX_SIM_STAT_FAST + s.lidv()] = v ? o_fast : 0u;
      st[FX_SIM_STAT_SLOW + s.lidv()] = v ? o_slow : 0u;
      st[FX_SIM_STAT_STABLE + s.lidv()] = v ? o_stab : 0u;
      st[FX_SIM_STAT_FAST_READS + s.lidv()] = v ? o_fr : 0u;
      st[FX_SIM_STAT_SLOW_READS + s.lidv()] = v ? o_sr : 0u;
    }
    if (s.lidv() == 0) {
      st[FX_SIM_STAT_EVENTS] = s.events;
      st[FX_SIM_STAT_END_MS] = s.now;
      st[FX_SIM_STAT_TRACE] = s.trace;
      st[FX_SIM_STAT_SEQ] = s.seq;
      st[FX_SIM_STAT_DEPS] = s.lds64(L_DEPS);
      st[FX_SIM_STAT_LAT_SUM] = s.lds64(L_LATSUM);
      st[FX_SIM_STAT_ERR_SITE] = s.err_site;
#ifdef FX_SIM_PROFILE
      for (uint32_t i = 0; i < 24; ++i) st[i] = s.prof[i];
#endif
    }
  }
  for (uint32_t i = s.lidv(); i < HC_BINS + HD_BINS; i += 64) {
    const uint32_t c = smem[i];
    if (!c) continue;
    if (i < HC_BINS) {
      if (a.chain_hist) atomicAdd(&a.chain_hist[i], (unsigned long long)c);
    } else if (a.delay_hist) {
      atomicAdd(&a.delay_hist[i - HC_BINS], (unsigned long long)c);
    }
  }
  for (uint32_t i = s.lidv(); i < HL_SLOTS; i += 64) {
    const uint32_t k = smem[HC_BINS + HD_BINS + i];
    if (k && a.lat_hist)
      atomicAdd(&a.lat_hist[k - 1u], (unsigned long long)smem[HC_BINS + HD_BINS + HL_SLOTS + i]);
  }
  if (s.lidv() == 0) a.err[inst] = s.err;
}

}  // namespace simx

// Geometry of the large-instance simulator: ring = events in flight (rounded
// up to a multiple of 64, at most 16384), dots = live dots per instance
// (per source: the next power of two of dots / n).  Defaults: 16 events per
// client (plus the GC traffic) and 8 live dots per client per process region.
bool simx_geometry(const fx_sim_spec& sp, uint32_t ring, uint32_t dots, simx::GeoX& g) {
  g = simx::GeoX{};
  return simx::geo_build(sp.n, sp.clients_per_region * sp.num_client_regions, sp.keys_per_command, sp.pool_size,
                         ring, dots, g);
}

bool simx_table_sizes(const fx_sim_spec& sp, uint32_t ring, uint32_t dots, uint32_t* R, uint32_t* NS) {
  simx::GeoX g;
  if (!simx_geometry(sp, ring, dots, g)) return false;
  *R = g.R;
  *NS = g.NS;
  return true;
}

size_t simx_arena_bytes(const fx_sim_spec& sp, uint32_t ring, uint32_t dots) {
  simx::GeoX g;
  return simx_geometry(sp, ring, dots, g) ? (size_t)g.words * 4 : 0;
}

// The arenas of the large-instance simulator: one hipMalloc'ed block per
// stream, grown when a launch needs more (hipFree waits for the device, so a
// block is never freed under a running launch) and reused by every later
// launch on that stream, which stream order serialises.  Launches on
// different streams get different blocks.  Never freed (process lifetime, as
// the batch executor's scratch).
void* simx_arena(hipStream_t hs, size_t bytes) {
  struct Block {
    hipStream_t s;
    void* p;
    size_t cap;
  };
  static std::mutex mu;
  static std::vector<Block>* blocks = new std::vector<Block>();
  std::lock_guard<std::mutex> g(mu);
  for (Block& bl : *blocks) {
    if (bl.s != hs) continue;
    if (bl.cap >= bytes) return bl.p;
    (void)hipFree(bl.p);
    bl.p = nullptr;
    bl.cap = 0;
    const size_t grown = bytes + bytes / 8;
    if (hipMalloc(&bl.p, grown) != hipSuccess) return nullptr;
    bl.cap = grown;
    return bl.p;
  }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  blocks->push_back(Block{hs, p, bytes});
  return p;
}

// Launches the large-instance simulator (fx_sim_run validated the batch).
int simx_launch(const fx_sim_batch* b, const fx_sim_output* o, hipStream_t hs) {
  using namespace simx;
  ArgsX a{};
  if (!simx_geometry(b->host_specs[0], b->ring_entries, b->dot_slots, a.g)) return FX_ERR_UNSUPPORTED;
  const size_t bytes = (size_t)a.g.words * 4 * b->instances;
  // The arena comes from a per-stream cache of hipMalloc'ed memory
  // (simx_arena) and starts zeroed; FX_SIM_FLAG_ARENA_FILL (tests) fills it
  // with 0xA5 bytes instead: the kernel initialises every word it reads, so
  // both give the same results (tests/test_poison_all.py).
  // FX_SIMX_ARENA=async (diagnostics) restores the round-5 allocation, a
  // stream-ordered pool block per launch (hipMallocAsync / hipFreeAsync): with
  // it about 2 % of small launches saw large parts of their arena zeroed by a
  // write no kernel of ours made, part-way through the run.
  static const bool async_env = [] {
    const char* e = std::getenv("FX_SIMX_ARENA");
    return e && std::string(e) == "async";
  }();
  void* arena = nullptr;
  if (async_env) {
    if (hipMallocAsync(&arena, bytes, hs) != hipSuccess) return FX_ERR_HIP;
  } else if (!(arena = simx_arena(hs, bytes))) {
    return FX_ERR_HIP;
  }
  if (hipMemsetAsync(arena, (b->flags & FX_SIM_FLAG_ARENA_FILL) ? 0xA5 : 0, bytes, hs) != hipSuccess)
    return FX_ERR_HIP;
  a.specs = b->specs;
  a.instances = b->instances;
  a.arena = (uint32_t*)arena;
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
  a.dot_client = o->dot_client;
  a.lat_hist = (unsigned long long*)o->latency_hist;
  a.lat_bins = o->lat_bins ? o->lat_bins : 1;
  a.chain_hist = (unsigned long long*)o->chain_hist;
  a.chain_bins = o->chain_bins ? o->chain_bins : 1;
  a.delay_hist = (unsigned long long*)o->delay_hist;
  a.delay_bins = o->delay_bins ? o->delay_bins : 1;
  a.stats = (unsigned long long*)o->stats;
  a.err = o->err;
  const dim3 grid(b->instances), block(64);
  const size_t lds = (size_t)LDS_WORDS * 4u;
  // configs[3]'s geometry compiled in when the batch's equals it word for word
  // (FX_SIM_FLAG_GENERIC: the run-time build, for A/B and its parity tests)
  constexpr GeoX gc1 = geo_compiled(1);
  const bool gs1 = !(b->flags & FX_SIM_FLAG_GENERIC) && std::memcmp(&a.g, &gc1, sizeof(GeoX)) == 0;
  static_assert(gc1.R > 4096 && gc1.R <= 8192, "configs[3] ring: NG = 2");
  static_assert(FX_SIMX_WPB >= 1, "instances per workgroup");
  if (gs1) {
    hipLaunchKernelGGL((k_simx<2, 1, FX_SIMX_WPB>), dim3((b->instances + FX_SIMX_WPB - 1) / FX_SIMX_WPB),
                       dim3(64 * FX_SIMX_WPB), lds * FX_SIMX_WPB, hs, a);
  } else if (a.g.R <= 4096) {
    hipLaunchKernelGGL((k_simx<1>), grid, block, lds, hs, a);
  } else if (a.g.R <= 8192) {
    hipLaunchKernelGGL((k_simx<2>), grid, block, lds, hs, a);
  } else {
    hipLaunchKernelGGL((k_simx<4>), grid, block, lds, hs, a);
  }
  const hipError_t le = hipGetLastError();
  if (async_env) (void)hipFreeAsync(arena, hs);
  return le == hipSuccess ? FX_OK : FX_ERR_HIP;
}

}  // namespace fx
