/*
 * fantoch_amd.h — C-ABI drop-in boundary of the MI355X-native GraphExecutor.
 *
 * The reference has no FFI: its boundary is the Rust trait
 * `fantoch::executor::Executor` (fantoch/src/executor/mod.rs:27-89) implemented by
 * `GraphExecutor` (fantoch_ps/src/executor/graph/executor.rs:31-114) on top of
 * `DependencyGraph` (fantoch_ps/src/executor/graph/mod.rs:45-677).  Every entry
 * point below names the reference item it replaces.  Plain pointers and sizes
 * only; HIP streams are passed as `void*` (a `hipStream_t`); no torch types.
 *
 * Two surfaces:
 *   1. fx_graph_executor_*  — one executor handle, the `Executor` trait 1:1
 *      (handle -> to_clients -> metrics -> monitor).  Adds are buffered on the
 *      host and executed on the GPU when results are pulled.
 *   2. fx_batch_*           — thousands of independent commit streams (one per
 *      (instance, process) executor) executed by one kernel launch; the form
 *      the batched simulator and bench use.  Buffers are device pointers.
 *
 * Errors: the reference panics on invariant violations (mod.rs:220,234-237,258,
 * 263; tarjan.rs:245,255).  Here every entry point returns an `int` status
 * (FX_OK = 0); batched launches also fill a per-stream error word.
 */
#ifndef FANTOCH_AMD_H
#define FANTOCH_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status */
#define FX_OK 0
#define FX_ERR_INVALID_ARG 1   /* bad pointer/size/config                      */
#define FX_ERR_CAPACITY 2      /* per-stream pending table / clock window full:
                                  rerun the stream at a larger tier            */
#define FX_ERR_DOUBLE_INDEX 3  /* mod.rs:233-237 "tried to index already indexed" */
#define FX_ERR_DEPS_UNSORTED 4 /* deps plane not strictly ascending (canonical C1) */
#define FX_ERR_DOT_RANGE 5     /* source 0 / > n, or seq >= 2^24               */
#define FX_ERR_HIP 6           /* HIP runtime error (no device, launch failed) */
#define FX_ERR_UNSUPPORTED 7   /* shard_count > 1 request/reply path (out of scope) */
#define FX_ERR_ORDER_OVERFLOW 8/* more executions than order-plane rows        */
#define FX_ERR_TIME_RANGE 9    /* t_ms >= 2^24 relative to the stream base     */
#define FX_ERR_NO_DEVICE 10    /* no GPU visible: the product never falls back */
#define FX_ERR_LOG_FORMAT 11   /* malformed execution log (rw/mod.rs:90 `expect` panics) */
#define FX_ERR_SIM_CAPACITY 12 /* a simulated instance outgrew a table of its launch geometry
                                  (message ring, dot table, executor slots, clock window) */
#define FX_ERR_SIM_LATE 13     /* a simulated message found no state for its dot, or a
                                  reference assertion failed (runner.rs:239-241, single.rs:346-349) */
#define FX_ERR_SIM_EVENTS 14   /* a simulated instance exceeded its event budget */
#define FX_ERR_TIMEOUT 15      /* a drop-in handle's device wait passed its deadline
                                  (FX_HANDLE_TIMEOUT_MS, default 2000): the resident
                                  kernel was asked to stop; sticky for the handle */

/* ------------------------------------------------- packed stream format */
/* A dot (fantoch/src/id.rs:21-27, Id<u8>{source, sequence}, derived Ord) is
 * packed as (source << 24) | seq; the packed u32 orders exactly like the
 * reference's (source, sequence) tuple. */
#define FX_SEQ_BITS 24u
#define FX_SEQ_MASK 0x00FFFFFFu
#define FX_PACK_DOT(src, seq) ((((uint32_t)(src)) << FX_SEQ_BITS) | ((uint32_t)(seq) & FX_SEQ_MASK))
#define FX_DOT_SRC(d) ((uint32_t)(d) >> FX_SEQ_BITS)
#define FX_DOT_SEQ(d) ((uint32_t)(d) & FX_SEQ_MASK)

/* Record header word: t_ms (24 bits) | ndeps (5 bits) | kind (3 bits). */
#define FX_HDR_T(h) ((uint32_t)(h) & 0x00FFFFFFu)
#define FX_HDR_ND(h) (((uint32_t)(h) >> 24) & 31u)
#define FX_HDR_KIND(h) ((uint32_t)(h) >> 29)
#define FX_MAKE_HDR(t, nd, kind) \
  (((uint32_t)(t) & 0x00FFFFFFu) | (((uint32_t)(nd) & 31u) << 24) | (((uint32_t)(kind) & 7u) << 29))
#define FX_KIND_ADD 0u        /* GraphExecutionInfo::Add -> handle_add (mod.rs:213-275) */
#define FX_KIND_INDEX_ONLY 1u /* VertexIndex::index without a search (index.rs:33-37);
                                 the hook the reference's sccs_found_and_missing_dep test uses */
#define FX_KIND_EXECUTED 2u   /* RequestReply::Executed{dot} (mod.rs:394-402): executed-clock
                                 add + check_pending; partial replication only */

/* Order-plane word: arrival index of the executed command | SCC-start flag. */
#define FX_ORDER_SCC_START 0x80000000u
#define FX_ORDER_REC(o) ((uint32_t)(o) & 0x7FFFFFFFu)
#define FX_RELEASE_NONE 0xFFFFFFFFu

/* Batch flags */
#define FX_FLAG_INIT 1u              /* start from an empty executor (else resume from state) */
#define FX_FLAG_EXECUTE_AT_COMMIT 2u /* Config::execute_at_commit (executor.rs:72-73)    */
#define FX_FLAG_SAVE_STATE 4u        /* write the executor state back for a later resume */
#define FX_FLAG_PARTIAL 8u           /* partial replication (shard_count > 1): the first search
                                        of an Add collects every missing dep (tarjan.rs:148-166),
                                        a vertex waits on all of them; FX_TIER_WIDE_HBM only,
                                        through fx_batch_execute_partial */
/* fx_batch_run_tiered only: first tier = ((flags >> FX_FLAG_TIER_SHIFT) & 15) - 1
 * (0 = the default tier, FX_TIER_DEFAULT). */
#define FX_FLAG_TIER_SHIFT 8u
#define FX_FLAG_FIRST_TIER(t) ((((uint32_t)(t)) + 1u) << FX_FLAG_TIER_SHIFT)

/* Plane layout.  Every per-(step, stream) array ("plane") is tiled in tiles
 * of 64 streams x 4 steps (1 KiB): element (step, stream) lives at
 *   fx_index(step, stream, steps) =
 *     ((stream / 64) * ceil(steps / 4) + step / 4) * 256 + (stream % 64) * 4 + step % 4
 * so one 16-byte load per lane fetches 4 consecutive steps of that lane's
 * stream and the 64 lanes of a wavefront (= 64 streams) read 1 KiB contiguous
 * per plane per 4 steps.  A plane holds fx_plane_words(S, steps) u32 words
 * (S rounded up to 64, steps to 4).  dep j of (step, stream) lives at
 * deps[j * fx_plane_words(S, steps) + fx_index(step, stream, steps)]; the
 * deps of one record are strictly ascending by packed dot (canonical C1,
 * replacing the hash order of executor.rs:76). */
#define FX_TILE_STREAMS 64u
#define FX_TILE_STEPS 4u
#if defined(__HIPCC__)
#define FX_INLINE __host__ __device__ static inline
#else
#define FX_INLINE static inline
#endif
FX_INLINE size_t fx_plane_words(uint32_t num_streams, uint32_t steps) {
  return (size_t)((num_streams + 63u) / 64u) * 64u * (size_t)((steps + 3u) / 4u) * 4u;
}
FX_INLINE size_t fx_index(uint32_t step, uint32_t stream, uint32_t steps) {
  return ((size_t)(stream >> 6) * ((steps + 3u) >> 2) + (step >> 2)) * 256u +
         ((stream & 63u) << 2) + (step & 3u);
}
typedef struct fx_stream_batch {
  const uint32_t* dot;      /* plane: packed dot of the Add                */
  const uint32_t* hdr;      /* plane: FX_MAKE_HDR(t_ms, ndeps, kind)       */
  const uint32_t* deps;     /* dmax planes: packed dep dots, ascending     */
  const uint32_t* lengths;  /* [S] valid steps per stream, or NULL = steps */
  uint32_t num_streams;     /* S                                           */
  uint32_t steps;           /* rows per plane                              */
  uint32_t dmax;            /* number of dep planes                        */
  uint32_t n;               /* processes per instance (sources 1..n)       */
} fx_stream_batch;

typedef struct fx_order_batch {
  uint32_t* order;    /* plane, row k: k-th executed command: arrival index | SCC_START */
  uint32_t* release;  /* plane, row a: step at which arrival a was executed, or NONE;
                         rows of arrivals a stream did not process (err != 0, or
                         beyond its length) are left untouched                 */
  uint32_t* nexec;    /* [S] number of executed commands                            */
  uint32_t* err;      /* [S] FX_* status of the stream                              */
} fx_order_batch;

/* Dense histograms (fantoch/src/metrics/histogram.rs:14-59 keeps an exact
 * BTreeMap; values here are small integers so a dense array is exact as long
 * as every value < nbins; the last bin counts values >= nbins-1). */
typedef struct fx_hist_batch {
  uint64_t* chain_size;       /* ExecutorMetricsKind::ChainSize (mod.rs:492-493)      */
  uint32_t nbins_chain;
  uint64_t* execution_delay;  /* ExecutorMetricsKind::ExecutionDelay (mod.rs:514-518) */
  uint32_t nbins_delay;
} fx_hist_batch;

/* Executor tiers: capacity of the per-stream pending table and of the
 * executed-clock window above each source's frontier.  A stream that exceeds
 * its tier stops with FX_ERR_CAPACITY and is rerun at the next tier
 * (fx_batch_run_tiered escalates 0 -> 1 -> 2, 3 -> 1 -> 2, 4 -> 2, 5 -> 1 -> 2,
 * 6 -> 1 -> 2, and then 2 -> 7 -> 8). */
#define FX_TIER_GROUP 0      /* 16 lanes per stream: 16 pending, 8 cached deps, n <= 16 */
#define FX_TIER_LDS_LARGE 1  /* lane per stream, LDS-resident: 32 pending, one wave per CU */
#define FX_TIER_GLOBAL 2     /* lane per stream, HBM-resident: 64 pending, 1024-bit windows */
#define FX_TIER_LANE 3       /* lane per stream, LDS-resident: 12 pending (alternative tier 0) */
#define FX_TIER_WAVE 4       /* one wavefront per stream: 64 pending, 8 cached deps, <= 14 deps */
#define FX_TIER_LANE_REG 5   /* lane per stream, register-resident slot table, lanes progress
                                independently: 12 pending, n <= 8, <= 8 deps */
#define FX_TIER_SPLIT 6      /* per 64-stream tile: tier 5 for tiles with few deps per Add,
                                tier 0 for dense ones, both launched concurrently; whole
                                batches only (FX_FLAG_INIT, no stream_map, no saved state);
                                `state` = fx_batch_state_bytes(6, n, S) bytes of scratch */
#define FX_TIER_WIDE 7       /* one wavefront per stream, the graph as tables in LDS: 512
                                pending, 1024-bit windows (rerun tier after tier 2) */
#define FX_TIER_WIDE_HBM 8   /* the same over HBM tables: 16384 pending, 32768-bit windows;
                                `state` = fx_batch_state_bytes(8, n, lanes) bytes; the one
                                wide tier that resumes (FX_FLAG_SAVE_STATE / no FX_FLAG_INIT) */
#define FX_NUM_TIERS 9
#define FX_TIER_DEFAULT FX_TIER_SPLIT

typedef struct fx_tier_info {
  uint32_t max_sources;    /* n supported                                   */
  uint32_t pending_cap;    /* vertices pending at once                       */
  uint32_t window_bits;    /* executed-clock exceptions above the frontier  */
  uint32_t state_words;    /* 32-bit state words per stream                  */
} fx_tier_info;

/* ---------------------------------------------------- batched executor */

/* Capacity of a tier for n processes. Replaces nothing in the reference (its
 * HashMap/DashMap indexes are unbounded, index.rs:18-51,145-208). */
int fx_tier_query(uint32_t tier, uint32_t n, fx_tier_info* out);

/* Bytes of resumable executor state for num_streams streams at a tier. */
size_t fx_batch_state_bytes(uint32_t tier, uint32_t n, uint32_t num_streams);

/* Run GraphExecutor::handle(Add) (executor.rs:69-93) for steps
 * [step_begin, step_end) of every stream, i.e. DependencyGraph::handle_add
 * (mod.rs:213-275) -> find_scc (409-486) -> TarjanSCCFinder::strong_connect
 * (tarjan.rs:96-316) -> save_scc (488-523) -> index_pending/check_pending/
 * try_pending (525-642), with canonical iteration C1 (deps ascending) and C2
 * (waiters ascending).
 *   stream_map: NULL, or [num_lanes] stream indices to run (tier reruns)
 *   state:      device buffer of fx_batch_state_bytes(tier, n, num_lanes)
 *               (NULL allowed with FX_FLAG_INIT and without FX_FLAG_SAVE_STATE)
 *   init_frontier: NULL, or [num_streams][8] executed-clock frontiers to start
 *               from (AboveExSet::from_events(1..=f), mod.rs:1309-1315),
 *               indexed by stream (not lane)
 * All pointers are device pointers; the call is asynchronous on hip_stream. */
int fx_batch_execute(const fx_stream_batch* in, const fx_order_batch* out,
                     uint32_t tier, const uint32_t* stream_map, uint32_t num_lanes,
                     void* state, uint32_t step_begin, uint32_t step_end,
                     uint32_t flags, const uint32_t* init_frontier, void* hip_stream);

/* Fold the executor metrics of a finished batch into dense histograms
 * (Metrics::collect, fantoch/src/metrics/mod.rs:34-48): one ChainSize sample
 * per SCC and one ExecutionDelay = t(release) - t(add) sample per executed
 * command.  Histogram buffers are accumulated into (zero them first). */
int fx_batch_metrics(const fx_stream_batch* in, const fx_order_batch* out,
                     const fx_hist_batch* hists, void* hip_stream);

/* Synchronous convenience driver: runs every stream at the first tier
 * (FX_TIER_DEFAULT unless FX_FLAG_FIRST_TIER(t) is set) and reruns the streams
 * that report FX_ERR_CAPACITY up the escalation chain.  Device pointers.
 * Returns FX_OK when every stream finished with FX_OK. */
int fx_batch_run_tiered(const fx_stream_batch* in, const fx_order_batch* out,
                        uint32_t flags, void* hip_stream, uint32_t* tier_counts);

/* Quiescent-cut driver for huge streams (BASELINE configs[4]): every stream is
 * split after each step t whose prefix is dependency-closed (every dep of an
 * Add at a step <= t was added at a step <= t); there the reference's
 * DependencyGraph (graph/mod.rs:213-642) has executed the whole prefix and
 * holds nothing pending, so each segment runs from an empty graph with its
 * prefix deps dropped and its dots renumbered per source (order-preserving).
 * Segments longer than one Add run as one batch through fx_batch_run_tiered
 * and map back; a one-Add segment executes at its own step.
 * A stream without a usable decomposition (a dep that never arrives, a
 * segment over 4096 steps, a double index, an index-only record) or whose
 * segments do not all execute completely runs whole through
 * fx_batch_run_tiered.  Output planes are identical to fx_batch_run_tiered's.
 * Synchronous; device pointers. */
typedef struct fx_cut_stats {
  uint64_t segments;                    /* segments executed as independent streams */
  uint32_t max_segment;                 /* longest segment (steps)                  */
  uint32_t whole_streams;               /* streams run whole (all reasons)          */
  uint32_t failed_streams;              /* ... of which because a segment did not
                                           execute completely (capacity, or the cut
                                           argument failing: never seen so far)     */
  uint32_t tier_counts[16];             /* segment-batch streams run per tier       */
  uint64_t single_segments;             /* segments one Add long: executed at their
                                           own step without the batch (a singleton
                                           SCC after the executed prefix)           */
} fx_cut_stats;
int fx_batch_run_cut(const fx_stream_batch* in, const fx_order_batch* out, uint32_t flags, void* hip_stream,
                     fx_cut_stats* stats);

/* ---------------------------------------- predecessors executor (Caesar) */
/* PredecessorsExecutor (fantoch_ps/src/executor/pred/{mod,index,executor}.rs):
 * commit streams as fx_stream_batch plus each Add's Caesar clock
 * (common/pred/clocks/mod.rs:15-30: (seq, process id), lexicographic) packed
 * as (seq << 8) | id in two planes (low / high 32 bits).  Phase one waits for
 * every dep to commit, phase two for every dep with a lower clock to execute;
 * the waiters of a removed PendingIndex entry are visited ascending by dot.
 * Outputs as the batched GraphExecutor: order row k = arrival index of the
 * k-th executed command (| FX_ORDER_SCC_START: every command its own group),
 * release[arrival] = executing step; fx_batch_metrics gives ExecutionDelay. */
#define FX_PRED_MAX_DEPS 256u
typedef struct fx_pred_batch {
  fx_stream_batch base;       /* dot / hdr / deps / lengths planes, S, steps, dmax, n */
  const uint32_t* clock_lo;   /* plane: low 32 bits of (clock seq << 8 | process id) */
  const uint32_t* clock_hi;   /* plane: high 32 bits                                */
  const uint32_t* ndeps;      /* plane: deps per Add (Caesar commits carry every
                                 conflicting command: up to FX_PRED_MAX_DEPS), or
                                 NULL = FX_HDR_ND (dmax <= 31) */
} fx_pred_batch;
/* Table tiers: SMALL = LDS, 64 pending (many wavefronts per CU; at n = 5 and
 * dmax = 5 also 32 dot-index slots per source, 256-seq clock windows and a
 * 32-deep recursion, so such streams reach FX_ERR_CAPACITY sooner); LDS = LDS,
 * the most of 512 / 256 / 128 pending that fit (FX_ERR_UNSUPPORTED if none
 * does); HBM = tables in `state` (fx_pred_state_bytes), 8192 pending. */
#define FX_PRED_TIER_SMALL 0u
#define FX_PRED_TIER_LDS 1u
#define FX_PRED_TIER_HBM 2u
/* One launch over num_lanes streams (stream_map NULL = all) at one table
 * tier.  Streams that run out report FX_ERR_CAPACITY.  Whole streams, from an
 * empty executor; flags: FX_FLAG_EXECUTE_AT_COMMIT. */
int fx_pred_execute(const fx_pred_batch* in, const fx_order_batch* out, const uint32_t* stream_map,
                    uint32_t num_lanes, uint32_t tier, void* state, uint32_t flags, void* hip_stream);
size_t fx_pred_state_bytes(uint32_t n, uint32_t dmax, uint32_t lanes);
/* Synchronous driver: every stream at SMALL, then the streams that ran out of
 * capacity at LDS, then HBM; *reruns (optional) = stream reruns in total. */
int fx_pred_run(const fx_pred_batch* in, const fx_order_batch* out, uint32_t flags, void* hip_stream,
                uint32_t* reruns);

/* --------------------------------------- synthetic Atlas/EPaxos streams */
/* Commit streams of `instances` independent simulated instances; instance i
 * has n processes, each coordinating cmds_per_process commands; conflict rate
 * conflict_pct[i % num_conflicts] percent (fantoch/src/client/key_gen.rs:96-128
 * semantics with a counter-based RNG, canonical C6); delivery order per process is a
 * seeded windowed shuffle; concurrent same-key commands of the same round see
 * each other with probability cycle_pct (2-/k-cycles). */
typedef struct fx_synth_params {
  uint64_t seed;
  uint32_t instances;
  uint32_t instance_base;    /* global index of the first instance (multi-GPU) */
  uint32_t n;
  uint32_t cmds_per_process;
  uint32_t window;           /* delivery jitter window (generation units)   */
  uint32_t cycle_pct;
  uint32_t horizon;          /* rounds searched back for the latest conflict */
  uint32_t num_conflicts;
  uint32_t conflict_pct[8];
  uint32_t conflict_block;   /* 0: rate = conflict_pct[i % num_conflicts] (seed-major);
                                B: rate = conflict_pct[(i / B) % num_conflicts]
                                (conflict-major: B consecutive instances share a rate) */
  uint32_t clients;          /* closed-loop clients per process (0/1: one; C >= 2:
                                seqs form rounds of C concurrent commands per source,
                                a command sees other sources' earlier rounds only, and
                                with probability cycle_pct a random concurrent command
                                of any other source: large SCCs, BASELINE configs[3];
                                cmds_per_process must be a multiple of C)            */
  uint32_t key_pool;         /* 0: the conflict-key model above.  K >= 2 (one client
                                per process): SURVEY §8(d)'s S5 stream, per-key chains
                                over a pool of K keys: every command's key is a C6
                                draw from the pool, its deps are, per source, the
                                latest command on that key within `horizon` rounds
                                (its own source: earlier seqs only), and with
                                probability cycle_pct two commands of the same round
                                depend on each other (2-cycles; longer cycles through
                                the chains).  conflict_pct is not used.              */
} fx_synth_params;

/* Planes of the synthetic batch: S = instances * n, steps = n * cmds, dmax = n. */
int fx_synth_shape(const fx_synth_params* p, uint32_t* num_streams, uint32_t* steps, uint32_t* dmax);
/* Generate into device planes (dot/hdr/deps of `out`, caller allocated). */
int fx_synth_generate(const fx_synth_params* p, uint32_t* dot, uint32_t* hdr, uint32_t* deps, void* hip_stream);
/* Same generator on the host (identical bytes). */
int fx_synth_generate_host(const fx_synth_params* p, uint32_t* dot, uint32_t* hdr, uint32_t* deps);

/* ---------------------------------------------- single executor handle */
/* Config (fantoch/src/config.rs:5-45), the fields this path reads. */
typedef struct fx_config {
  uint32_t n;
  uint32_t f;
  uint32_t shard_count;                      /* must be 1 (partial replication out of scope) */
  uint32_t execute_at_commit;                /* config.rs execute_at_commit  */
  uint32_t executor_monitor_execution_order; /* config.rs: KVStore monitor (kvs.rs:29-39) */
} fx_config;

typedef struct fx_dot { uint32_t source; uint32_t seq; } fx_dot;       /* Dot  = Id<u8>  */
typedef struct fx_rifl { uint64_t source; uint64_t seq; } fx_rifl;     /* Rifl = Id<u64> */

/* ExecutorResult (fantoch/src/executor/mod.rs:169-174) with keys as u32 ids
 * (canonical C7) and payloads dropped. */
typedef struct fx_executor_result {
  fx_rifl rifl;
  uint32_t key;
  uint32_t read_only;
} fx_executor_result;

typedef struct fx_graph_executor fx_graph_executor;

/* Partial replication (Config::shard_count > 1, graph/mod.rs:82-406): the
 * streams run on the HBM wide tables with FX_FLAG_PARTIAL semantics.  A record
 * of kind FX_KIND_EXECUTED is RequestReply::Executed{dot}; RequestReply::Info
 * is an Add.  `req` holds per stream 1 + 2 req_cap words: word 0 = count, then
 * (step, parent dot) for every dep that went missing while no vertex waited on
 * it (the first PendingIndex::index of that dot, index.rs:180-198), the
 * candidates for out-requests (the caller keeps those its shard does not
 * replicate).  n = processes over all shards (<= 8); process ids 1..=n.
 * `state` = fx_partial_state_bytes(n, S) bytes; flags: FX_FLAG_INIT /
 * FX_FLAG_SAVE_STATE (resumable).  Device pointers, async on hip_stream. */
size_t fx_partial_state_bytes(uint32_t n, uint32_t num_streams);
int fx_batch_execute_partial(const fx_stream_batch* in, const fx_order_batch* out, void* state,
                             uint32_t step_begin, uint32_t step_end, uint32_t flags,
                             const uint32_t* init_frontier, uint32_t* req, uint32_t req_cap,
                             void* hip_stream);

/* Executor::new (executor.rs:34-51). NULL on bad config or no GPU.
 * The handle starts on tier 0 and, when its stream outgrows a tier, reruns its
 * log one tier up (0 -> 1 -> 2 -> 8): up to 16384 pending vertices, beyond
 * which the handle reports FX_ERR_CAPACITY (the reference's indexes are
 * unbounded, index.rs:18-51). */
fx_graph_executor* fx_graph_executor_new(uint8_t process_id, uint64_t shard_id, const fx_config* config);
/* Drop. */
void fx_graph_executor_free(fx_graph_executor* ex);
/* Executor::set_executor_index (executor.rs:53-56); only index 0 handles Adds. */
int fx_graph_executor_set_executor_index(fx_graph_executor* ex, uint32_t index);
/* Executor::handle(GraphExecutionInfo::Add{dot, cmd, deps}) (executor.rs:69-80).
 * keys: ids of the command's keys on this shard; deps in any order (the ABI
 * canonicalises to ascending, C1, and drops duplicates); now_ms = SysTime::millis(). */
int fx_graph_executor_handle_add(fx_graph_executor* ex, fx_dot dot, fx_rifl rifl,
                                 const uint32_t* keys, uint32_t nkeys, uint32_t read_only,
                                 const fx_dot* deps, uint32_t ndeps, uint64_t now_ms);
/* Partial replication (fx_config.shard_count > 1; n x shard_count <= 8 process
 * ids; the handle runs on the HBM wide tables, FX_FLAG_PARTIAL):
 * handle_add_sharded = handle(Add) and RequestReply::Info (mod.rs:390-393)
 * with each dep's Dependency::shards as a bitmask (deps/keys/mod.rs:19-22);
 * handle_executed = RequestReply::Executed for each dot (mod.rs:394-402);
 * requests drains DependencyGraph::requests (mod.rs:148-151) as (target
 * shard, dot) pairs, ascending; to_executors drains the dots added to the
 * executed clock (mod.rs:137-144, the Executed info of fetch_to_executors,
 * executor.rs:140-152), ascending.  Requests are served by a clone (below). */
int fx_graph_executor_handle_add_sharded(fx_graph_executor* ex, fx_dot dot, fx_rifl rifl,
                                         const uint32_t* keys, uint32_t nkeys, uint32_t read_only,
                                         const fx_dot* deps, const uint32_t* dep_shards, uint32_t ndeps,
                                         uint64_t now_ms, uint64_t cmd_shards);
/* cmd_shards: the shards the command has ops on (Command::replicated_by,
 * command.rs:90-92) as a bitmask; 0 = this handle's shard only.  An Info
 * reply's command is one this shard does not replicate, so its set (the
 * request_replies row's cmd_shards) is passed back as it is.  A Request for
 * a pending dot from a shard that replicates it is the reference's panic
 * (graph/mod.rs:308-316): FX_ERR_INVALID_ARG from handle_request / cleanup. */
int fx_graph_executor_handle_executed(fx_graph_executor* ex, const fx_dot* dots, uint32_t n, uint64_t now_ms);
int fx_graph_executor_requests(fx_graph_executor* ex, uint64_t* shards, fx_dot* dots, uint32_t cap,
                               uint32_t* n_out);
int fx_graph_executor_to_executors(fx_graph_executor* ex, fx_dot* dots, uint32_t cap, uint32_t* n_out);
/* Executor index > 0 of the same process (run mode clones the executor per
 * task and shares the VertexIndex, index.rs:21): a clone of a partial-
 * replication handle reads its main handle's vertices, keeps its own executed
 * clock (GraphExecutionInfo::Executed -> handle_executed_info, mod.rs:211-223),
 * serves Requests from other shards (handle_request / process_requests,
 * mod.rs:277-355: a vertex still pending -> RequestReply::Info with its deps,
 * an executed dot -> RequestReply::Executed, otherwise buffered) and retries
 * the buffered ones on cleanup (mod.rs:183-195).  Info replies carry the rifl
 * and deps; the command's ops stay with the caller (keyed by dot).  Free the
 * clone before its main handle.  Serving a request flushes the main handle. */
typedef struct fx_request_reply {
  uint64_t to_shard;
  uint32_t kind;      /* 1 = Info{dot, cmd, deps}, 0 = Executed{dot} */
  fx_dot dot;
  fx_rifl rifl;       /* Info: the command's rifl */
  uint32_t ndeps;     /* Info: deps at deps[first_dep, first_dep + ndeps) */
  uint32_t first_dep;
  uint64_t cmd_shards; /* Info: the command's shard set (cmd.shards(), as the reference ships the cmd) */
} fx_request_reply;
fx_graph_executor* fx_graph_executor_clone(fx_graph_executor* main);
int fx_graph_executor_handle_executed_info(fx_graph_executor* ex, const fx_dot* dots, uint32_t n);
int fx_graph_executor_handle_request(fx_graph_executor* ex, uint64_t from_shard, const fx_dot* dots, uint32_t n);
int fx_graph_executor_cleanup(fx_graph_executor* ex);
int fx_graph_executor_request_replies(fx_graph_executor* ex, fx_request_reply* out, uint32_t cap, fx_dot* deps,
                                      uint32_t* dep_shards, uint32_t deps_cap, uint32_t* n_out);
/* Test hook mirroring `queue.vertex_index.index(Vertex::new(..))` (mod.rs:1164-1306). */
int fx_graph_executor_index_only(fx_graph_executor* ex, fx_dot dot, fx_rifl rifl,
                                 const uint32_t* keys, uint32_t nkeys,
                                 const fx_dot* deps, uint32_t ndeps, uint64_t now_ms);
/* Test hook mirroring `queue.executed_clock = AEClock::from(..)` (mod.rs:1309-1315):
 * frontier[i] = highest contiguous executed seq of source i+1 (any u32). Only
 * before the first Add.  Sequences: fx_dot.seq is any u32; the device holds
 * seq - frontier (24 bits), so one handle spans 2^24 - 1 sequence numbers per
 * source above the frontier it starts from (FX_ERR_DOT_RANGE beyond). */
int fx_graph_executor_set_executed_frontier(fx_graph_executor* ex, const uint64_t* frontier, uint32_t n);
/* Executor::to_clients (executor.rs:95-97): pops up to cap results in execution order. */
int fx_graph_executor_to_clients(fx_graph_executor* ex, fx_executor_result* out, uint32_t cap, uint32_t* n_out);
/* Execution order as dots (DependencyGraph::commands_to_execute in the tests, mod.rs:158-160):
 * pops up to cap executed dots; scc_start[i] = 1 if out[i] opens a new SCC. */
int fx_graph_executor_drain_dots(fx_graph_executor* ex, fx_dot* out, uint8_t* scc_start, uint32_t cap, uint32_t* n_out);
/* Executor::metrics (executor.rs:107-109): histogram as (value, count) pairs
 * sorted by value; kind 0 = ExecutionDelay, 1 = ChainSize.  Returns pair count in *n_out. */
int fx_graph_executor_metrics(fx_graph_executor* ex, uint32_t kind, uint64_t* values,
                              uint64_t* counts, uint32_t cap, uint32_t* n_out);
/* Executor::monitor (executor.rs:111-113): the rifls executed on `key`, in order. */
int fx_graph_executor_monitor(fx_graph_executor* ex, uint32_t key, fx_rifl* out, uint32_t cap, uint32_t* n_out);
/* Pending vertices and the dot each waits on (0 source = none), ascending; debug/tests
 * (VertexIndex::monitor_pending, index.rs:53-103, reports the same information). */
int fx_graph_executor_pending(fx_graph_executor* ex, fx_dot* dots, fx_dot* waiting_on, uint32_t cap, uint32_t* n_out);
/* Executor::parallel (executor.rs:103-105). */
int fx_graph_executor_parallel(void);
/* Host<->device bytes this handle has moved so far (not in the reference; lets
 * a test check that draining after every Add moves bytes linear in the Adds). */
int fx_graph_executor_transfer_stats(const fx_graph_executor* ex, uint64_t* h2d, uint64_t* d2h);
/* Persistent-mode timing (diagnostics, tools/handle_latency): the first n of
 * FX_PERSIST_STATS counters, summed over the flushes: [0] flushes, [1] host wait
 * from doorbell to status (ns), [2] the kernel's compute, [3] its publish, [4]
 * polls, [5] poll round trips (100 MHz ticks), [6] the host's row preparation,
 * [7] order conversion (ns), [8] the compute in shader-clock cycles, [9] the
 * host's whole flush, [10] its reads after the wait, [11] its work before the
 * publish (ns), [12] executor iterations (DFS edges / frame pops, try and
 * check steps), [13] cycles in the Add's first step, [14] one-Add flushes
 * whose row the kernel took from the mailbox line (the rest read the ring). The
 * kernel's words are read only with FX_HANDLE_STATS=1 in the environment. */
#define FX_PERSIST_STATS 15
int fx_graph_executor_persist_stats(const fx_graph_executor* ex, uint64_t* out, uint32_t n);
/* Test hooks of the persistent mode (tests only; 0 = off), taking effect at
 * the kernel's next launch: skip_status_flush = k makes the k-th flush of a
 * launch publish no status, so the host's bounded wait expires; hold_ms keeps
 * the kernel resident, ignoring the stop request and its idle exit, until it
 * has been idle that long (at most 10 s: it still exits by itself), so the
 * host's stop request goes unanswered and the handle is abandoned. */
int fx_graph_executor_debug_hooks(fx_graph_executor* ex, uint32_t skip_status_flush, uint32_t hold_ms);

/* ------------------------------------------------------- quorum sizes */
#define FX_PROTOCOL_ATLAS 0u
#define FX_PROTOCOL_EPAXOS 1u
#define FX_PROTOCOL_BASIC 2u  /* fantoch/src/protocol/basic.rs (the simulator's own test protocol) */
/* Fast and write quorum sizes of the commit-stream producers:
 * Config::atlas_quorum_sizes (fantoch/src/config.rs:294-301) and
 * Config::epaxos_quorum_sizes (config.rs:303-312, f ignored).  The deps of a
 * commit are a union over the fast quorum (atlas.rs:404-475, epaxos.rs:370-428). */
int fx_quorum_sizes(uint32_t protocol, uint32_t n, uint32_t f, uint32_t* fast_quorum,
                    uint32_t* write_quorum);

/* --------------------------------------------------- batched simulator */
/* One simulated instance: Runner::new(planet, config, workload,
 * clients_per_process, process_regions, client_regions) + Runner::run
 * (fantoch/src/sim/runner.rs:64-231) with the GCP planet.  Regions are
 * indices into the planet's regions in name order (canonical C12); process i
 * (id i + 1) sits in process_regions[i]. */
#define FX_SIM_MAX_N 8u
#define FX_SIM_MAX_CLIENT_REGIONS 20u
typedef struct fx_sim_spec {
  uint64_t seed;                       /* canonical C6 RNG seed                       */
  uint64_t instance;                   /* global instance index (RNG stream)          */
  uint32_t protocol;                   /* FX_PROTOCOL_{ATLAS,EPAXOS,BASIC}            */
  uint32_t n, f;                       /* Config::new(n, f)                           */
  uint32_t gc_interval_ms;             /* Config::gc_interval (0 = None)              */
  uint32_t executed_notification_ms;   /* Config::executor_executed_notification_interval */
  uint32_t clients_per_region;         /* Runner::new clients_per_process             */
  uint32_t commands_per_client;        /* Workload::commands_per_client               */
  uint32_t keys_per_command;           /* Workload::keys_per_command (1 or 2)         */
  uint32_t conflict_rate;              /* KeyGen::ConflictPool::conflict_rate (%)     */
  uint32_t pool_size;                  /* KeyGen::ConflictPool::pool_size             */
  uint32_t read_only_pct;              /* Workload::read_only_percentage              */
  int32_t extra_sim_time_ms;           /* Runner::run(extra_sim_time): -1 = None      */
  uint32_t reorder_messages;           /* Runner::reorder_messages (C6 multiplier)    */
  uint32_t nfr;                        /* Config::nfr                                 */
  uint32_t num_client_regions;
  uint8_t process_regions[FX_SIM_MAX_N];
  uint8_t client_regions[FX_SIM_MAX_CLIENT_REGIONS];
} fx_sim_spec;

/* A batch of instances on one GPU (fx_sim_run): one wavefront per instance.
 * All instances of a batch share protocol family geometry: n, clients per
 * region, number of client regions, keys per command and pool size (the
 * conflict rate, f, seeds, regions and intervals may differ per instance).
 * The GPU path simulates Atlas and EPaxos (GraphExecutor protocols).  Two
 * kernels share the entry point: the all-on-chip one (sim_wave.hip: <= 32
 * clients per instance, no read-only commands, NFR or message reordering) and
 * the large-instance one (sim_big.hip: up to 65535 clients per instance,
 * read-only commands, NFR, message reordering; per-instance state in an HBM
 * arena of fx_sim_plan_large bytes, allocated stream-ordered by fx_sim_run).
 * fx_sim_run picks the first when the batch fits it, unless
 * FX_SIM_FLAG_LARGE is set. */
#define FX_SIM_FLAG_EXEC_NOTIFICATIONS 1u /* simulate the periodic executed notifications
                                             even when they cannot change the outcome
                                             (GraphExecutor::executed is None; they matter
                                             only for where a run with extra time stops) */
#define FX_SIM_FLAG_LARGE 2u              /* run the large-instance kernel */
#define FX_SIM_FLAG_GENERIC 4u            /* either kernel's build for run-time geometry even
                                             when the batch has one of the geometries compiled in
                                             (BASELINE configs[0]-[3]; same results, for A/B tests) */
#define FX_SIM_FLAG_ARENA_FILL 8u         /* tests: the large-instance kernel's arena starts filled
                                             with 0xA5 bytes instead of zeroed (the kernel must not
                                             read a word it did not write) */
typedef struct fx_sim_batch {
  const fx_sim_spec* specs;        /* [instances] device copy                          */
  const fx_sim_spec* host_specs;   /* [instances] host copy (validation, geometry)     */
  uint32_t instances;
  uint32_t flags;                  /* FX_SIM_FLAG_*                                     */
  const uint16_t* planet_ping;     /* device [planet_regions][planet_stride] ping (ms)  */
  const uint8_t* planet_rank;      /* device [planet_regions][planet_stride]: position of
                                      region b in region a's sorted order               */
  uint32_t planet_regions, planet_stride;
  uint32_t exec_cap;               /* executed dots kept per process (the rest counted) */
  uint32_t lat_cap;                /* latencies kept per client (0 = no latency log)    */
  uint32_t max_events;             /* per-instance event budget (0 = 2^32 - 1)          */
  uint32_t ring_entries;           /* messages in flight per instance, a pool shared by the
                                      process links (<= 65534; 0 = 16 n x clients per
                                      process region)                                   */
  uint32_t dot_slots;              /* live dots per instance, a pool shared by the
                                      coordinators (<= 256; 0 = min(64, 8 clients)); the
                                      large-instance kernel: <= 8 x 65536, direct-mapped
                                      per source (0 = 8 per client per process region) */
  uint32_t pad;
} fx_sim_batch;

/* per-instance counters (u64) */
#define FX_SIM_STAT_FAST 0u     /* [n] ProtocolMetricsKind::FastPath per process  */
#define FX_SIM_STAT_SLOW 8u     /* [n] SlowPath                                    */
#define FX_SIM_STAT_STABLE 16u  /* [n] Stable (commands garbage-collected; evaluated from the
                                   committed-frontier history at the end of the run) */
#define FX_SIM_STAT_EVENTS 24u  /* actions processed (executed notifications and GC traffic excluded) */
#define FX_SIM_STAT_END_MS 25u  /* simulation time when the run stopped            */
#define FX_SIM_STAT_TRACE 26u   /* hash of the processed action sequence, GC traffic excluded (debug) */
#define FX_SIM_STAT_SEQ 27u     /* schedule insertions                             */
#define FX_SIM_STAT_DEPS 28u    /* deps of every executor Add (sum over processes) */
#define FX_SIM_STAT_LAT_SUM 29u /* sum of every client command's latency (ms)       */
#define FX_SIM_STAT_ERR_SITE 30u /* where FX_ERR_SIM_CAPACITY was raised (source line) */
#define FX_SIM_STAT_FAST_READS 32u /* [n] FastPathReads (base.rs:229-243): read-only commands */
#define FX_SIM_STAT_SLOW_READS 40u /* [n] SlowPathReads                                   */
#define FX_SIM_STATS 48u

typedef struct fx_sim_output {  /* device buffers; NULL where not wanted */
  uint32_t* executed;           /* [instances][n][exec_cap] packed dots, execution order */
  uint32_t* executed_len;       /* [instances][n] commands executed per process     */
  uint32_t* latency_log;        /* [instances][clients][lat_cap] client latency (ms) */
  uint64_t* latency_hist;       /* [planet_regions][lat_bins] per client region, accumulated */
  uint64_t* chain_hist;         /* [chain_bins] ExecutorMetricsKind::ChainSize, accumulated */
  uint64_t* delay_hist;         /* [delay_bins] ExecutionDelay (ms), accumulated    */
  uint64_t* stats;              /* [instances][FX_SIM_STATS]                        */
  uint32_t* err;                /* [instances] FX_* status                           */
  uint32_t lat_bins, chain_bins, delay_bins, pad;
  uint32_t* dot_client;         /* [instances][n][exec_cap] client id (1-based) that submitted
                                   dot (p + 1, s) at [p][s - 1], or NULL (the rifl of an
                                   executed dot: the client's k-th dot is its command k + 1) */
} fx_sim_output;

/* LDS bytes one instance of `spec` needs at the given table sizes
 * (FX_ERR_UNSUPPORTED if it does not fit the GPU path). */
int fx_sim_plan(const fx_sim_spec* spec, uint32_t ring_entries, uint32_t dot_slots, uint32_t* lds_bytes);
/* Bytes of HBM arena one instance of `spec` takes in the large-instance kernel
 * at the given table sizes (0 = defaults); FX_ERR_UNSUPPORTED if it cannot run. */
int fx_sim_plan_large(const fx_sim_spec* spec, uint32_t ring_entries, uint32_t dot_slots, uint64_t* arena_bytes);
/* Runs every instance to completion (Runner::run, runner.rs:202-231); asynchronous. */
int fx_sim_run(const fx_sim_batch* batch, const fx_sim_output* out, void* hip_stream);
/* fx_sim_run, then (synchronously) reruns the instances that stopped with
 * FX_ERR_SIM_CAPACITY with larger tables (all-on-chip kernel: a 4x, at least
 * 256 n, message pool and 256 dot slots, then the large-instance kernel;
 * large-instance kernel: 2x the events and 4x the dots, twice), writing their
 * rows of every output in place.  Histograms stay exact: the samples the
 * failed runs added before failing are removed by replaying just those runs
 * at the first geometry (the kernel is deterministic per instance) and
 * subtracting.  An instance that fails at the larger geometry too keeps its
 * error and contributes no histogram samples.  *reruns (optional) = instances
 * rerun. */
int fx_sim_run_tiered(const fx_sim_batch* batch, const fx_sim_output* out, void* hip_stream, uint32_t* reruns);

/* Planet::from(dir) (fantoch/src/planet/mod.rs:38-54, dat.rs:20-94): regions
 * in name order; ping[a][b] (ms, `as u64` of the average) and rank[a][b] = the
 * position of b in a's (latency, name) order (Planet::sorted, mod.rs:122-140),
 * row stride `cap`.  With ping == NULL only *num_regions is filled.  names:
 * newline-separated region names (may be NULL). */
int fx_planet_load(const char* dir, uint32_t cap, uint32_t* num_regions, char* names, uint32_t names_bytes,
                   uint16_t* ping, uint8_t* rank);

/* ------------------------------------------------------- execution log */
/* Reader for the run mode's execution log: LengthDelimitedCodec frames
 * (4-byte big-endian length) of bincode-1 GraphExecutionInfo, as written by
 * execution_logger_task (fantoch/src/run/task/server/execution_logger.rs:11-55,
 * Rw::write fantoch/src/run/rw/mod.rs:66-77,93-100) and read back by
 * graph_executor_replay (fantoch_ps/src/bin/graph_executor_replay.rs:29-37,
 * Rw::recv rw/mod.rs:37-53).  Each Add becomes the arguments of
 * fx_graph_executor_handle_add: keys of `shard_id` interned to u32 ids in
 * first-seen order, deps as dots.  Request/RequestReply/Executed (partial
 * replication only) are parsed and counted in `others`, never executed. */
typedef struct fx_log_summary {
  uint64_t records;       /* frames                                          */
  uint64_t adds;          /* GraphExecutionInfo::Add frames                  */
  uint64_t others;        /* Request / RequestReply / Executed frames        */
  uint64_t keys;          /* sum of keys over the Adds (on shard_id)         */
  uint64_t deps;          /* sum of deps over the Adds                       */
  uint64_t distinct_keys; /* interned key ids                                */
} fx_log_summary;

typedef struct fx_log_add {
  fx_dot dot;
  fx_rifl rifl;
  uint64_t key_off;       /* into the keys array                             */
  uint64_t dep_off;       /* into the deps array                             */
  uint32_t nkeys;
  uint32_t ndeps;
  uint32_t read_only;     /* Command::read_only (command.rs:80-87)           */
  uint32_t pad;
} fx_log_add;

/* Validates the whole log and fills the summary (sizes for the decode call).
 * FX_ERR_LOG_FORMAT on a truncated frame, unknown tag, trailing bytes, or a
 * sequence above 2^32-1 (reference: Rw::recv's `expect`, rw/mod.rs:90). */
int fx_exec_log_scan(const uint8_t* buf, uint64_t len, uint64_t shard_id, fx_log_summary* out);
/* Decodes every Add in file order into caller-allocated arrays
 * (FX_ERR_CAPACITY if one is too small). */
int fx_exec_log_decode(const uint8_t* buf, uint64_t len, uint64_t shard_id, fx_log_add* adds,
                       uint64_t cap_adds, uint32_t* keys, uint64_t cap_keys, fx_dot* deps,
                       uint64_t cap_deps, fx_log_summary* out);

/* ------------------------------------------------- histogram statistics */
/* Histogram stats (histogram.rs:61-235) over (value, count) pairs sorted by value. */
typedef struct fx_hist_stats {
  double count, mean, stddev, cov, mdtm, min, max;
} fx_hist_stats;
int fx_hist_stats_compute(const uint64_t* values, const uint64_t* counts, uint32_t n, fx_hist_stats* out);
/* Histogram::percentile (histogram.rs:111-170). */
int fx_hist_percentile(const uint64_t* values, const uint64_t* counts, uint32_t n, double p, double* out);

/* ------------------------------------------------------------- runtime */
/* Number of visible GPUs; 0 means every compute entry point returns FX_ERR_NO_DEVICE. */
int fx_device_count(void);
/* Minimal device-memory plumbing for hosts without their own GPU runtime
 * bindings (a Rust/cgo/ctypes caller); torch callers may pass their own
 * device pointers and hipStream_t instead. */
int fx_dev_alloc(void** ptr, size_t bytes);
int fx_dev_free(void* ptr);
int fx_dev_memset(void* ptr, int value, size_t bytes, void* hip_stream);
int fx_dev_h2d(void* dst, const void* src, size_t bytes, void* hip_stream);
int fx_dev_d2h(void* dst, const void* src, size_t bytes, void* hip_stream);
int fx_dev_synchronize(void* hip_stream);
/* Elapsed milliseconds of the last fx_batch_execute launch on hip_stream,
 * measured with HIP events recorded on that stream around the kernel when
 * fx_profile_enable(1) is set (bench roofline; 0 disables the events). */
int fx_profile_enable(int on);
int fx_profile_last_exec_ms(float* ms);
/* Per-kernel duration of the last profiled launch: which = 0 the whole
 * executor launch (as fx_profile_last_exec_ms), 1 the group kernel and 2 the
 * lane kernel of FX_TIER_SPLIT (events recorded on each kernel's own stream);
 * FX_ERR_INVALID_ARG if that kernel did not run. */
int fx_profile_last_kernel_ms(uint32_t which, float* ms);
/* The last profiled launch of one kernel slot, timed by HIP events on the
 * stream it ran on: slot = an executor tier (FX_TIER_*, fx_batch_execute and
 * the tiered drivers' launches), FX_PROFILE_SLOT_PRED + FX_PRED_TIER_* (the
 * predecessors executor); FX_ERR_INVALID_ARG if it did not run since
 * fx_profile_enable(1). */
#define FX_PROFILE_SLOT_PRED 16u
#define FX_PROFILE_SLOTS 20u
int fx_profile_slot_ms(uint32_t slot, float* ms);
const char* fx_status_string(int status);
const char* fx_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FANTOCH_AMD_H */
