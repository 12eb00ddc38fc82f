// executor_host.cpp — the `Executor` trait (fantoch/src/executor/mod.rs:27-89)
// as a C-ABI handle over the HIP batch kernel, plus Histogram statistics.
//
// A handle owns one commit stream.  handle_add appends the Add to a host log
// (mirrored in the tiled plane layout); pulling results (to_clients, drain,
// metrics, monitor, pending) runs the new steps on the GPU, resuming from the
// executor state saved by the previous launch, and converts the executed order
// into ExecutorResults exactly like GraphExecutor::fetch_commands_to_execute +
// execute (executor.rs:126-138,184-188) -> Command::execute (command.rs:147-162)
// -> KVStore::execute + ExecutionOrderMonitor::add (kvs.rs:53-65, monitor.rs:21-31).
// There is no CPU execution path: without a GPU the constructor fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <emmintrin.h>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "fantoch_amd.h"
#include "fx_internal.h"

namespace {

struct Cmd {
  fx_rifl rifl;
  std::vector<uint32_t> keys;  // ascending (canonical C11)
  uint32_t read_only;
  uint64_t shards = 0;  // shards the command has ops on (partial replication)
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  bool ensure(size_t b) {
    if (bytes >= b) return true;
    release();
    if (hipMalloc(&p, b) != hipSuccess) {
      p = nullptr;
      return false;
    }
    bytes = b;
    return true;
  }
  uint32_t* u32() const { return static_cast<uint32_t*>(p); }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(bytes, o.bytes);
  }
};

// pinned host memory mapped into the device's address space: the handle's
// upload staging and the words a flush reports (written by the device)
struct HostBuf {
  void* p = nullptr;
  void* dp = nullptr;
  size_t bytes = 0;
  ~HostBuf() { release(); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = dp = nullptr;
    bytes = 0;
  }
  bool ensure(size_t b, bool coherent = false) {
    if (bytes >= b) return true;
    release();
    if (hipHostMalloc(&p, b, hipHostMallocMapped | (coherent ? hipHostMallocCoherent : 0u)) != hipSuccess) {
      p = nullptr;
      return false;
    }
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) {
      release();
      return false;
    }
    bytes = b;
    return true;
  }
  uint32_t* u32() const { return static_cast<uint32_t*>(p); }
  uint32_t* du32() const { return static_cast<uint32_t*>(dp); }
  void swap(HostBuf& o) {
    std::swap(p, o.p);
    std::swap(dp, o.dp);
    std::swap(bytes, o.bytes);
  }
};

// A persistent handle's resources: its stream (a hardware queue of its own,
// ~12 ms to make) and its mapped control words, rings and state block.  A
// freed handle leaves them in a process-wide pool for the next handle, so a
// program that makes handle after handle (a test per permutation, a simulation
// per configuration) makes the queue once.  The pool is never destroyed (its
// buffers would be freed after the HIP runtime at exit).
struct PersistRes {
  hipStream_t stream = nullptr;
  HostBuf ctl, rows, out;
  DevBuf state;
};
std::mutex g_persist_pool_mu;
std::vector<PersistRes*>* g_persist_pool = new std::vector<PersistRes*>();
constexpr size_t kPersistPoolMax = 64;

constexpr uint32_t kDmaxDev = 31;

}  // namespace

struct fx_graph_executor {
  uint8_t process_id = 0;
  uint64_t shard_id = 0;
  fx_config cfg{};
  uint32_t executor_index = 0;
  hipStream_t stream = nullptr;

  // host log (arrival order)
  std::vector<uint32_t> dots, hdrs;
  std::vector<std::vector<uint32_t>> deps;
  std::vector<Cmd> cmds;
  bool have_base = false;
  uint64_t t_base = 0;
  // per-source sequence base: the device sees seq - base[source - 1] (24-bit),
  // the boundary takes any u32 sequence.  base = the executed frontier the
  // handle starts from (fx_graph_executor_set_executed_frontier), else 0; deps
  // at or below it are executed, which handle_add skips (mod.rs find_scc), so
  // they are dropped on the way in.
  uint32_t base[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t nsrc = 0;  // process ids 1..=nsrc: n x shard_count (util::all_process_ids)

  // partial replication (shard_count > 1, graph/mod.rs:82-406)
  bool partial = false;
  std::map<uint32_t, uint32_t> dep_mask;              // device dot -> Dependency::shards bitmask
  std::set<std::pair<uint64_t, uint32_t>> requests;   // out_requests: (target shard, device dot)
  std::set<uint32_t> added;                           // added_to_executed_clock (device dots)
  DevBuf d_req;                                       // first-missing ring (fx_batch_execute_partial)
  uint32_t req_cap = 0;
  std::map<uint32_t, uint32_t> rec_of;                // device dot -> arrival index of its Add (VertexIndex)
  std::set<uint32_t> executed_set;                    // device dots executed here (left the VertexIndex)
  // executor index > 0 (fx_graph_executor_clone): the handle whose VertexIndex
  // it shares (index.rs:21), its own executed clock (per source: contiguous
  // frontier + exceptions), buffered requests and the replies
  fx_graph_executor* shared = nullptr;
  std::map<uint32_t, std::pair<uint64_t, std::set<uint64_t>>> clock;
  std::map<uint64_t, std::set<std::pair<uint32_t, uint64_t>>> buffered;
  struct Reply {
    uint64_t to;
    bool info;
    uint32_t src;
    uint64_t seq;
    fx_rifl rifl;
    std::vector<fx_dot> deps;
    std::vector<uint32_t> shards;
    uint64_t cmd_shards = 0;
  };
  std::deque<Reply> replies;

  // device mirror
  uint32_t cap = 0;      // plane rows
  uint32_t dmax = 0;     // dep planes in use
  uint32_t uploaded = 0; // rows present on the device
  DevBuf d_dot, d_hdr, d_deps, d_order, d_release, d_nexec, d_err, d_state;
  uint32_t tier = FX_TIER_GROUP;  // one resumable stream: a tier with saved state
  uint32_t processed = 0;  // steps executed by the device state
  uint32_t consumed = 0;   // order entries already converted

  // outputs
  std::deque<fx_executor_result> to_clients;
  std::deque<std::pair<uint32_t, bool>> executed;  // (packed dot, scc start)
  std::map<uint64_t, uint64_t> chain_size, execution_delay;
  std::map<uint32_t, std::vector<fx_rifl>> monitor;
  DevBuf d_gather;            // release steps of the entries of one flush
  HostBuf h_up;               // upload staging (pinned), copied to d_up and scattered into the planes
  DevBuf d_up;
  HostBuf h_out;              // nexec, err, (order word, release step) per new entry (device-written)
  uint64_t bytes_h2d = 0, bytes_d2h = 0;  // transfer accounting (fx_graph_executor_transfer_stats)
  int sticky = FX_OK;

  // Persistent mode (flush_persist): one resident wavefront runs the wave
  // tier's executor over Adds published in host-mapped memory, so draining
  // after every Add costs no launch and no stream synchronisation.  Used from
  // the first flush while every Add fits the wave tier (<= 14 deps, 64
  // pending, 32-bit clock windows); any capacity error moves the handle to
  // the batch tiers for good (the log reruns from its start there, as every
  // tier escalation does).  FX_HANDLE_PERSIST=0 turns it off.
  struct Persist {
    bool active = false;    // the log is executed by the persistent kernel
    bool launched = false;  // a launch is outstanding on `stream` (it may have exited when idle)
    bool dead = false;      // a stop request went unanswered past the deadline: the stream is abandoned
    uint64_t timeout_ns = 0;  // every host wait's deadline (FX_HANDLE_TIMEOUT_MS at creation, default 2 s)
    hipStream_t stream = nullptr;
    HostBuf ctl, rows, out;
    DevBuf state;
    uint32_t pub = 0;  // rows published
    static constexpr uint32_t ROWS = 4096, OUT = 8192;
    // fx_graph_executor_persist_stats: flushes, host wait (ns), and the
    // kernel's compute / fence ticks, polls and poll round trips (100 MHz)
    uint64_t stats[FX_PERSIST_STATS] = {};  // + host prep / convert (ns), compute shader cycles, flush total / post-wait reads / pre-publish (ns)
    bool want_stats = false;  // FX_HANDLE_STATS=1: the kernel's fence / poll / cycle words too
    uint32_t debug_skip_status = 0, debug_hold_ticks = 0;  // test hooks (fx_graph_executor_debug_hooks)
  } ps;
  bool persist_ok = true;
};

namespace {

int upload_all(fx_graph_executor* ex, uint32_t new_cap, uint32_t new_dmax) {
  const size_t plane = fx_plane_words(1, new_cap);
  if (!ex->d_dot.ensure(plane * 4) || !ex->d_hdr.ensure(plane * 4) ||
      !ex->d_deps.ensure(plane * 4 * std::max<uint32_t>(new_dmax, 1)) ||
      !ex->d_order.ensure(plane * 4) || !ex->d_release.ensure(plane * 4) ||
      !ex->d_nexec.ensure(4) || !ex->d_err.ensure(4))
    return FX_ERR_HIP;
  ex->cap = new_cap;
  ex->dmax = new_dmax;
  ex->uploaded = 0;  // the whole log again, as strided rows (upload_tail)
  return FX_OK;
}

// Copies rows [uploaded, N) of the single-stream planes to the device.  The
// plane is tiled 64 streams x 4 steps; a one-stream handle fills only the
// first 4 words of each 256-word tile, so each plane goes over as a strided
// 2-D copy of those words (16 bytes per tile) instead of whole tiles.
int upload_tail(fx_graph_executor* ex) {
  const uint32_t N = (uint32_t)ex->dots.size();
  if (ex->uploaded >= N) return FX_OK;
  const uint32_t r0 = ex->uploaded & ~3u;
  const uint32_t r1 = (N + 3) & ~3u;
  const uint32_t rows = r1 - r0, nplanes = 2 + ex->dmax;
  // one staging block, plane-major (dot, hdr, dep planes), one copy, one scatter
  const size_t words = (size_t)nplanes * rows;
  if (!ex->h_up.ensure(words * 4) || !ex->d_up.ensure(words * 4)) return FX_ERR_HIP;
  uint32_t* st = ex->h_up.u32();
  std::memset(st, 0, words * 4);
  for (uint32_t i = r0; i < N; ++i) {
    const size_t at = i - r0;
    st[at] = ex->dots[i];
    st[rows + at] = ex->hdrs[i];
    for (uint32_t j = 0; j < ex->deps[i].size(); ++j) st[(size_t)(2 + j) * rows + at] = ex->deps[i][j];
  }
  ex->bytes_h2d += (uint64_t)words * 4;
  // the staging block stays untouched until the flush's synchronisation
  if (hipMemcpyAsync(ex->d_up.p, st, words * 4, hipMemcpyHostToDevice, ex->stream)) return FX_ERR_HIP;
  if (fx::scatter_rows(ex->d_up.u32(), nplanes, r0, rows, ex->cap, ex->d_dot.u32(), ex->d_hdr.u32(),
                       ex->d_deps.u32(), ex->stream))
    return FX_ERR_HIP;
  ex->uploaded = N;
  return FX_OK;
}

// An error after upload_tail queued the staging copy: the copy may still be
// reading the pinned staging block, which a later ensure() or the destructor
// frees, so the stream is drained before the error is returned (sticky)
int fail_sync(fx_graph_executor* ex, int st) {
  (void)hipStreamSynchronize(ex->stream);
  return ex->sticky = st;
}

void convert(fx_graph_executor* ex, const std::vector<uint32_t>& order, const std::vector<uint32_t>& rel,
             uint32_t nexec);

volatile uint32_t* pctl(fx_graph_executor* ex) { return reinterpret_cast<volatile uint32_t*>(ex->ps.ctl.u32()); }

// Reads of the device-written words: fine-grained host memory is not cached
// for the host (each load is a memory round trip, ~0.25 us), so they are read
// 16 bytes per load instead of word by word.  The load is one instruction in
// inline asm: from a plain intrinsic the compiler may re-read a word from
// memory instead of taking it from the loaded register, which tears a tagged
// word pair written by the device (a new tag with an old value).
inline void ld16(const volatile uint32_t* p, uint32_t out[4]) {
  __m128i v;
  asm volatile("movdqu %1, %0" : "=x"(v) : "m"(*reinterpret_cast<const volatile __m128i*>(p)) : "memory");
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out), v);
}

// The stream of a handle's persistent kernel.  The kernel stays resident, so
// whatever else is queued on the same hardware queue waits for it (up to its
// idle exit): FX_PERSIST_QUEUE picks how the stream is made -- "plain" (a
// non-blocking stream, sharing the process's hardware queues), "prio" (a
// non-blocking high-priority stream), "cumask" (a stream with an all-CU mask,
// which gets a hardware queue of its own).
hipError_t persist_stream(hipStream_t* s) {
  const char* q = std::getenv("FX_PERSIST_QUEUE");
  const std::string kind = q ? q : "cumask";
  if (kind == "prio") {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return hipErrorUnknown;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
  }
  if (kind == "cumask") {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      return hipErrorUnknown;
    std::vector<uint32_t> mask(((uint32_t)ncu + 31u) / 32u, 0u);
    for (int c = 0; c < ncu; ++c) mask[(uint32_t)c / 32u] |= 1u << ((uint32_t)c % 32u);
    return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// The persistent mode's stream, mapped control words / rings and state block;
// made when the handle is created (fx_graph_executor_new), so an Add never
// pays for them.
int persist_alloc(fx_graph_executor* ex) {
  auto& P = ex->ps;
  if (!P.stream) {
    PersistRes* r = nullptr;
    {
      std::lock_guard<std::mutex> g(g_persist_pool_mu);
      if (!g_persist_pool->empty()) {
        r = g_persist_pool->back();
        g_persist_pool->pop_back();
      }
    }
    if (r) {
      P.stream = r->stream;
      P.ctl.swap(r->ctl);
      P.rows.swap(r->rows);
      P.out.swap(r->out);
      P.state.swap(r->state);
      delete r;
    } else if (persist_stream(&P.stream) != hipSuccess) {
      P.stream = nullptr;
      return FX_ERR_HIP;
    }
  }
  if (!P.ctl.ensure(fx::PERSIST_CTL_WORDS * 4, true) ||
      !P.rows.ensure((size_t)fx_graph_executor::Persist::ROWS * fx::PERSIST_ROW_WORDS * 4, true) ||
      !P.out.ensure((size_t)fx_graph_executor::Persist::OUT * 8, true) ||
      !P.state.ensure((size_t)fx::wave_state_words_per_stream() * 4))
    return FX_ERR_HIP;
  std::memset(P.ctl.p, 0, fx::PERSIST_CTL_WORDS * 4);
  return FX_OK;
}

// Every host wait on the resident kernel is bounded (status
// codes replace panics; the reference's Executor never blocks,
// fantoch/src/executor/mod.rs:27-89).  A Wait checks, every 1024 spins, the
// deadline (FX_HANDLE_TIMEOUT_MS, default 2000 ms from the start of the wait)
// and the stream: an error there (a faulted kernel) ends the wait with
// FX_ERR_HIP.  On expiry the handle asks the kernel to stop, waits for the
// stream at most one more deadline, and the flush returns FX_ERR_TIMEOUT,
// sticky for the handle.
uint64_t persist_timeout_ns() {
  const char* e = std::getenv("FX_HANDLE_TIMEOUT_MS");
  const long ms = e ? std::atol(e) : 0;
  return (uint64_t)(ms > 0 ? ms : 2000) * 1000000ull;
}

struct Wait {
  std::chrono::steady_clock::time_point end;
  explicit Wait(uint64_t ns)
      : end(std::chrono::steady_clock::now() + std::chrono::nanoseconds(ns)) {}
  // FX_OK: keep spinning; FX_ERR_TIMEOUT: the deadline passed; FX_ERR_HIP: the
  // stream reported an error
  int check(hipStream_t s, uint64_t spin) const {
    if ((spin & 1023u) != 1023u) return FX_OK;
    const hipError_t q = hipStreamQuery(s);
    if (q != hipSuccess && q != hipErrorNotReady) return FX_ERR_HIP;
    return std::chrono::steady_clock::now() > end ? FX_ERR_TIMEOUT : FX_OK;
  }
};

// The end of a failed wait: ask the kernel to stop and give its stream one
// more deadline to drain.  A stream that drains is reusable: an expired wait
// (a slow but healthy kernel, e.g. queued behind other work) then returns
// FX_ERR_CAPACITY, and flush() moves the log to the batch tiers as it does
// for a capacity escalation (the executor state the kernel saved is not
// needed: the batch tiers rerun the log from its start).  A stream error, or a
// kernel that did not stop, is sticky; such a stream is abandoned (never
// synchronised again, never pooled, and the handle's buffers are leaked when
// it is freed: the kernel may still write them).
int persist_abort(fx_graph_executor* ex, int st, const char* where, uint32_t hi) {
  auto& P = ex->ps;
  std::fprintf(stderr, "fantoch_amd persistent handle: %s while waiting for the %s (rows %u, consumed %u)\n",
               st == FX_ERR_TIMEOUT ? "deadline passed" : "stream error", where, hi, ex->consumed);
  pctl(ex)[fx::PERSIST_EXIT] = 1u;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const Wait w(ex->ps.timeout_ns);
  for (;;) {
    const hipError_t q = hipStreamQuery(P.stream);
    if (q == hipSuccess) {
      P.launched = false;
      pctl(ex)[fx::PERSIST_EXIT] = 0u;
      break;
    }
    if (q != hipErrorNotReady || std::chrono::steady_clock::now() > w.end) {
      P.dead = true;  // the kernel did not stop: leave its stream alone
      break;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  ex->persist_ok = false;
  if (st == FX_ERR_TIMEOUT && !P.dead) return FX_ERR_CAPACITY;
  return ex->sticky = st;
}

// Stops the persistent kernel (its executor state lands in ps.state); the
// wait for its stream is bounded like every other (persist_abort on expiry).
int persist_stop(fx_graph_executor* ex) {
  if (ex->ps.dead) return FX_ERR_TIMEOUT;
  if (!ex->ps.launched) return FX_OK;
  pctl(ex)[fx::PERSIST_EXIT] = 1u;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const Wait w(ex->ps.timeout_ns);
  for (uint64_t spin = 0;; ++spin) {
    const hipError_t q = hipStreamQuery(ex->ps.stream);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) return persist_abort(ex, FX_ERR_HIP, "stop", ex->ps.pub);
    if (std::chrono::steady_clock::now() > w.end) {
      const int r = persist_abort(ex, FX_ERR_TIMEOUT, "stop", ex->ps.pub);
      return r == FX_ERR_CAPACITY ? FX_OK : r;  // drained on the second deadline: stopped
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  ex->ps.launched = false;
  pctl(ex)[fx::PERSIST_EXIT] = 0u;
  return FX_OK;
}

int persist_launch_now(fx_graph_executor* ex, bool init) {
  fx::PersistArgs a{};
  a.ctl = ex->ps.ctl.du32();
  a.rows = ex->ps.rows.du32();
  a.out = ex->ps.out.du32();
  a.state = ex->ps.state.u32();
  a.row_slots = fx_graph_executor::Persist::ROWS;
  a.out_slots = fx_graph_executor::Persist::OUT;
  a.n = ex->nsrc;
  a.at_commit = ex->cfg.execute_at_commit ? 1u : 0u;
  a.init = init ? 1u : 0u;
  a.done0 = pctl(ex)[fx::PERSIST_DONE];
  a.debug_skip_status = ex->ps.debug_skip_status;
  a.debug_hold_ticks = ex->ps.debug_hold_ticks;
  pctl(ex)[fx::PERSIST_RUN] = 1u;  // the kernel clears it when it exits
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (fx::persist_launch(a, ex->ps.stream) != FX_OK) return FX_ERR_HIP;
  ex->ps.launched = true;
  return FX_OK;
}

// The persistent-mode flush: publish the new rows, wait for the kernel's done
// word, take the new (order word, release step) pairs from the mapped ring.
// Returns FX_ERR_CAPACITY when the log must move to the batch tiers.
int flush_persist(fx_graph_executor* ex, uint32_t& nexec_out) {
  const auto tf0 = std::chrono::steady_clock::now();
  const uint32_t N = (uint32_t)ex->dots.size();
  if (N >= (1u << 28)) return FX_ERR_CAPACITY;  // the kernel's LDS doorbell word holds row counts < 2^29
  for (uint32_t i = ex->ps.pub; i < N; ++i)
    if (ex->deps[i].size() > fx::WAVE_MAX_DEPS) return FX_ERR_CAPACITY;
  auto& P = ex->ps;
  if (!P.active) {  // the first flush of the handle
    if (ex->processed != 0) return FX_ERR_CAPACITY;
    if (!P.ctl.p) {
      const int st = persist_alloc(ex);
      if (st) return st;
    }
    P.pub = 0;
    P.active = true;
    int st = persist_launch_now(ex, true);
    if (st) return st;
  }
  uint32_t nexec = ex->consumed;  // every pair of the earlier flushes was taken
  while (P.pub < N) {
    const auto tp0 = std::chrono::steady_clock::now();
    P.stats[11] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tp0 - tf0).count();
    // a chunk the rings hold: every published row and pair was consumed
    const uint32_t hi = std::min<uint32_t>(N, P.pub + fx_graph_executor::Persist::ROWS - 128u);
    uint32_t* rows = P.rows.u32();
    for (uint32_t i = P.pub; i < hi; ++i) {
      uint32_t* r = rows + (size_t)(i & (fx_graph_executor::Persist::ROWS - 1u)) * fx::PERSIST_ROW_WORDS;
      r[0] = ex->dots[i];
      r[1] = ex->hdrs[i];
      const auto& dv = ex->deps[i];
      for (uint32_t j = 0; j < fx::PERSIST_ROW_WORDS - 2u; ++j) r[2 + j] = j < dv.size() ? dv[j] : 0u;
    }
    ex->bytes_h2d += (uint64_t)(hi - P.pub) * fx::PERSIST_ROW_WORDS * 4;
    if (hi == P.pub + 1u && ex->deps[P.pub].size() <= fx::PERSIST_MB_DEPS) {
      // a one-Add flush: the row also goes into the mailbox line, which the
      // kernel reads with the doorbell.  Its 32 lanes load the line word by
      // word, so a read can mix two flushes' words: the checksum word (the
      // tag mixed in, fx::persist_mb_mix) rejects such a line and the kernel
      // takes the row from the ring
      volatile uint32_t* mb = pctl(ex) + fx::PERSIST_MB;
      const auto& dv = ex->deps[P.pub];
      uint32_t w15[15];
      w15[0] = hi;
      w15[1] = ex->dots[P.pub];
      w15[2] = ex->hdrs[P.pub];
      for (uint32_t j = 0; j < fx::PERSIST_MB_DEPS; ++j) w15[3 + j] = j < dv.size() ? dv[j] : 0u;
      uint32_t sum = 0;
      for (uint32_t k = 0; k < 15; ++k) sum ^= fx::persist_mb_mix(w15[k], k);
      for (uint32_t k = 1; k < 15; ++k) mb[k] = w15[k];
      mb[15] = sum;
      std::atomic_thread_fence(std::memory_order_release);
      mb[0] = hi;
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);  // the rows before the doorbell
    const auto tw0 = std::chrono::steady_clock::now();
    P.stats[6] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tw0 - tp0).count();
    pctl(ex)[fx::PERSIST_PUB] = hi;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (!P.launched) {
      int st = persist_launch_now(ex, false);
      if (st) return st;
    }
    // wait for the status word {done, nexec | error bit} (read with its
    // second word {done, err} as one 16-byte load); a kernel that exited when
    // idle just before the doorbell (RUN cleared, done short of hi) is
    // relaunched from its state
    uint32_t w[4];
    const Wait wt(P.timeout_ns);
    for (uint64_t spin = 0;; ++spin) {
      ld16(pctl(ex) + fx::PERSIST_DONE, w);
      if (w[0] == hi) break;
      if (const int ws = wt.check(P.stream, spin)) return persist_abort(ex, ws, "status", hi);
      if ((spin & 1023u) == 1023u && pctl(ex)[fx::PERSIST_RUN] == 0u) {
        // the kernel left (idle exit just before the doorbell): its stream
        // drains within the deadline, then it is relaunched
        for (uint64_t s2 = 1023u;; s2 += 1024u) {
          const hipError_t q = hipStreamQuery(P.stream);
          if (q == hipSuccess) break;
          if (const int ws = q != hipErrorNotReady ? FX_ERR_HIP : wt.check(P.stream, s2))
            return persist_abort(ex, ws, "idle exit", hi);
        }
        P.launched = false;
        ld16(pctl(ex) + fx::PERSIST_DONE, w);
        if (w[0] == hi) break;
        if (w[2] == w[0] && w[3]) {  // the kernel stopped on an error before these rows
          persist_stop(ex);
          return w[3] == FX_ERR_CAPACITY || w[3] == FX_ERR_ORDER_OVERFLOW ? FX_ERR_CAPACITY : (int)w[3];
        }
        int st = persist_launch_now(ex, false);
        if (st) return st;
      }
    }
    const auto tw1 = std::chrono::steady_clock::now();
    P.stats[0] += 1;
    P.stats[1] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tw1 - tw0).count();
    if (w[1] & fx::PERSIST_ERR_BIT) {  // {done, err} is written with the status; wait for it
      const Wait we(P.timeout_ns);
      for (uint64_t spin = 0; w[2] != hi; ++spin) {
        ld16(pctl(ex) + fx::PERSIST_DONE, w);
        if (const int ws = we.check(P.stream, spin)) return persist_abort(ex, ws, "error word", hi);
      }
      const uint32_t err = w[3];
      persist_stop(ex);
      return err == FX_ERR_CAPACITY || err == FX_ERR_ORDER_OVERFLOW ? FX_ERR_CAPACITY : (int)err;
    }
    if (P.want_stats) {
      uint32_t t[4];
      ld16(pctl(ex) + fx::PERSIST_TCOMP, t);
      P.stats[2] += t[0];
      P.stats[3] += t[1];
      P.stats[4] += t[2];
      P.stats[5] += t[3];
      ld16(pctl(ex) + fx::PERSIST_TCYC, t);
      P.stats[8] += t[0];
      P.stats[12] += t[1];
      P.stats[13] += t[2];
      P.stats[14] += t[3];
    }
    nexec = w[1];
    P.pub = hi;
    // the new pairs: tagged words in the control line, or the mapped ring
    if (nexec > ex->consumed) {
      const uint32_t np = nexec - ex->consumed;
      if (np > fx_graph_executor::Persist::OUT) return FX_ERR_CAPACITY;
      std::vector<uint32_t> order(np), rel(np);
      if (np <= fx::PERSIST_INLINE) {
        const Wait wp(P.timeout_ns);
        for (uint32_t j = 0; j < np; ++j) {
          uint32_t t[4];
          for (uint64_t spin = 0;; ++spin) {
            ld16(pctl(ex) + fx::PERSIST_PAIRS + 4 * j, t);
            if (t[0] == hi && t[2] == hi) break;
            if (const int ws = wp.check(P.stream, spin)) return persist_abort(ex, ws, "pairs", hi);
          }
          order[j] = t[1];
          rel[j] = t[3];
        }
      } else {
        const volatile uint32_t* q = reinterpret_cast<volatile uint32_t*>(P.out.u32());
        constexpr uint32_t M = fx_graph_executor::Persist::OUT - 1u;
        for (uint32_t k = ex->consumed; k < nexec;) {
          if ((k & 1u) == 0 && k + 1 < nexec && ((k + 1) & M) != 0) {  // two pairs per read
            uint32_t t[4];
            ld16(q + 2 * (k & M), t);
            order[k - ex->consumed] = t[0];
            rel[k - ex->consumed] = t[1];
            order[k + 1 - ex->consumed] = t[2];
            rel[k + 1 - ex->consumed] = t[3];
            k += 2;
          } else {
            order[k - ex->consumed] = q[2 * (k & M)];
            rel[k - ex->consumed] = q[2 * (k & M) + 1];
            k += 1;
          }
        }
      }
      ex->bytes_d2h += 12 + (uint64_t)(nexec - ex->consumed) * 8;
      const auto tc0 = std::chrono::steady_clock::now();
      P.stats[10] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tc0 - tw1).count();
      convert(ex, order, rel, nexec);
      P.stats[7] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now() - tc0).count();
    }
  }
  ex->processed = N;
  nexec_out = nexec;
  P.stats[9] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tf0)
                    .count();
  return FX_OK;
}

// Runs the steps not yet executed; converts new order entries.
int flush(fx_graph_executor* ex) {
  if (ex->sticky) return ex->sticky;
  const uint32_t N = (uint32_t)ex->dots.size();
  if (ex->processed >= N) return FX_OK;
  if (!ex->partial && ex->persist_ok && (ex->ps.active || ex->processed == 0)) {
    uint32_t nexec = 0;
    const int st = flush_persist(ex, nexec);
    if (st == FX_OK) return FX_OK;
    if (st != FX_ERR_CAPACITY) return ex->sticky = st;
    // to the batch tiers, from the start of the log (the consumed prefix of
    // the deterministic order is skipped there), for the rest of the handle's
    // life.  The first tier follows the cause: an Add wider than the wave
    // tier's WAVE_MAX_DEPS goes to the LDS slot tier (31 deps), a pending set
    // or clock window the wave tier cannot hold to the HBM slot tier (64
    // pending, 1024-bit windows); both escalate on capacity from there
    if (const int s2 = persist_stop(ex)) return ex->sticky = s2;
    if (ex->sticky) return ex->sticky;
    ex->persist_ok = false;
    ex->ps.active = false;
    bool wide = false;
    for (const auto& d : ex->deps) wide = wide || d.size() > fx::WAVE_MAX_DEPS;
    ex->tier = wide ? FX_TIER_LDS_LARGE : FX_TIER_GLOBAL;
    ex->processed = 0;
    ex->uploaded = 0;
  }
  uint32_t need_dmax = ex->dmax;
  for (uint32_t i = ex->uploaded; i < N; ++i) need_dmax = std::max<uint32_t>(need_dmax, (uint32_t)ex->deps[i].size());
  if (N > ex->cap || need_dmax > ex->dmax) {
    uint32_t nc = std::max<uint32_t>(64, ex->cap);
    while (nc < N) nc *= 2;
    int st = upload_all(ex, nc, std::max<uint32_t>(need_dmax, 1));
    if (st) return ex->sticky = st;
  }
  {
    int st = upload_tail(ex);
    if (st) return fail_sync(ex, st);
  }
  fx_stream_batch in{};
  in.dot = ex->d_dot.u32();
  in.hdr = ex->d_hdr.u32();
  in.deps = ex->d_deps.u32();
  in.lengths = nullptr;
  in.num_streams = 1;
  in.steps = ex->cap;
  in.dmax = ex->dmax;
  in.n = ex->nsrc;
  fx_order_batch out{ex->d_order.u32(), ex->d_release.u32(), ex->d_nexec.u32(), ex->d_err.u32()};
  uint32_t nexec = 0, err = 0;
  while (ex->partial) {  // one resumable tier: the HBM tables with partial-replication semantics
    // the ring holds this flush's first-missing parents (<= its deps + records)
    const uint32_t want = std::max<uint32_t>(1024, (N - ex->processed) * (ex->dmax + 1) * 2);
    if (want > ex->req_cap) {
      if (!ex->d_req.ensure((size_t)(1 + 2 * (size_t)want) * 4)) return fail_sync(ex, FX_ERR_HIP);
      ex->req_cap = want;
    }
    if (!ex->d_state.ensure(fx_partial_state_bytes(ex->nsrc, 1))) return fail_sync(ex, FX_ERR_HIP);
    uint32_t flags = FX_FLAG_SAVE_STATE;
    if (ex->processed == 0) flags |= FX_FLAG_INIT;
    else if (hipMemsetAsync(ex->d_req.p, 0, 4, ex->stream)) return fail_sync(ex, FX_ERR_HIP);
    int st = fx_batch_execute_partial(&in, &out, ex->d_state.p, ex->processed, N, flags, nullptr, ex->d_req.u32(),
                                      ex->req_cap, ex->stream);
    if (st) return fail_sync(ex, st);
    uint32_t nreq = 0;
    if (hipMemcpyAsync(&nexec, ex->d_nexec.p, 4, hipMemcpyDeviceToHost, ex->stream) ||
        hipMemcpyAsync(&err, ex->d_err.p, 4, hipMemcpyDeviceToHost, ex->stream) ||
        hipMemcpyAsync(&nreq, ex->d_req.p, 4, hipMemcpyDeviceToHost, ex->stream) ||
        hipStreamSynchronize(ex->stream))
      return fail_sync(ex, FX_ERR_HIP);
    if (err) return fail_sync(ex, (int)err);
    std::vector<uint32_t> ring((size_t)2 * nreq);
    if (nreq && (hipMemcpyAsync(ring.data(), ex->d_req.u32() + 1, ring.size() * 4, hipMemcpyDeviceToHost,
                                ex->stream) ||
                 hipStreamSynchronize(ex->stream)))
      return fail_sync(ex, FX_ERR_HIP);
    ex->bytes_d2h += 4 + ring.size() * 4;
    // PendingIndex::index: a first-missing parent this shard does not
    // replicate is requested from its target shard (index.rs:187-197)
    for (uint32_t k = 0; k < nreq; ++k) {
      const uint32_t m = ring[2 * k + 1];
      auto it = ex->dep_mask.find(m);
      const uint32_t mask = it == ex->dep_mask.end() ? 0u : it->second;
      if (mask == 0) return fail_sync(ex, FX_ERR_UNSUPPORTED);  // "shards should be set if it's not a noop"
      if (!((mask >> ex->shard_id) & 1u))
        ex->requests.insert({(uint64_t)(FX_DOT_SRC(m) - 1) / ex->cfg.n, m});  // Dot::target_shard (id.rs:59-61)
    }
    break;
  }
  while (!ex->partial) {
    // wider Adds than the current tier reads start over one tier up, as
    // fx_batch_run_tiered picks its first tier (group: <= GROUP_LANES deps,
    // wave: <= WAVE_MAX_DEPS)
    if ((ex->tier == FX_TIER_WAVE && in.dmax > fx::WAVE_MAX_DEPS) ||
        (ex->tier == FX_TIER_GROUP && in.dmax > fx::GROUP_LANES)) {
      ex->tier = FX_TIER_LDS_LARGE;
      ex->processed = 0;
    }
    if (!ex->d_state.ensure(fx_batch_state_bytes(ex->tier, ex->nsrc, 1))) return fail_sync(ex, FX_ERR_HIP);
    uint32_t flags = FX_FLAG_SAVE_STATE;
    if (ex->processed == 0) flags |= FX_FLAG_INIT;
    if (ex->cfg.execute_at_commit) flags |= FX_FLAG_EXECUTE_AT_COMMIT;
    int st = fx_batch_execute(&in, &out, ex->tier, nullptr, 1, ex->d_state.p, ex->processed, N, flags,
                              nullptr, ex->stream);
    if (st) return fail_sync(ex, st);
    // nexec, err and the new entries straight into mapped host memory: one
    // synchronisation per flush
    if (!ex->h_out.ensure((size_t)(2 + 2 * (size_t)ex->cap) * 4)) return fail_sync(ex, FX_ERR_HIP);
    if (fx::flush_pack(ex->d_order.u32(), ex->d_release.u32(), ex->d_nexec.u32(), ex->d_err.u32(), ex->cap,
                       ex->consumed, ex->h_out.du32(), ex->stream) ||
        hipStreamSynchronize(ex->stream))
      return fail_sync(ex, FX_ERR_HIP);
    nexec = ex->h_out.u32()[0];
    err = ex->h_out.u32()[1];
    if (err == FX_ERR_CAPACITY && ex->tier != FX_TIER_WIDE_HBM) {
      // rerun the whole log one tier up (group -> LDS -> HBM slots -> HBM
      // tables, the last one resumable like the others); the already-consumed
      // prefix of the (deterministic) order is skipped below
      ex->tier = ex->tier == FX_TIER_GROUP ? FX_TIER_LDS_LARGE
               : ex->tier == FX_TIER_WAVE || ex->tier == FX_TIER_LDS_LARGE ? FX_TIER_GLOBAL
                                                                          : FX_TIER_WIDE_HBM;
      ex->processed = 0;
      continue;
    }
    break;
  }
  if (err) return fail_sync(ex, (int)err);
  ex->processed = N;
  if (nexec <= ex->consumed) return FX_OK;
  // the new order entries and the release steps they need: packed by the
  // flush (non-partial), else read back here
  std::vector<uint32_t> order(nexec - ex->consumed);
  const uint32_t k0 = ex->consumed;
  std::vector<uint32_t> rel(nexec - k0);
  if (!ex->partial) {
    const uint32_t* w = ex->h_out.u32() + 2;
    for (uint32_t t = 0; t < nexec - k0; ++t) {
      order[t] = w[2 * t];
      rel[t] = w[2 * t + 1];
    }
    ex->bytes_d2h += 8 + (uint64_t)(nexec - k0) * 8;
  }
  if (ex->partial) {
    const uint32_t r0 = k0 & ~3u, r1 = (nexec + 3) & ~3u;
    // the first 4 words of each tile (this stream's rows), strided
    std::vector<uint32_t> rows((size_t)(r1 - r0));
    if (hipMemcpy2DAsync(rows.data(), 4 * 4, ex->d_order.u32() + fx_index(r0, 0, ex->cap), 256 * 4, 4 * 4,
                         (r1 - r0) / 4, hipMemcpyDeviceToHost, ex->stream) ||
        hipStreamSynchronize(ex->stream))
      return fail_sync(ex, FX_ERR_HIP);
    for (uint32_t k = k0; k < nexec; ++k) order[k - k0] = rows[k - r0];
  }
  // the release steps of exactly the commands converted below, gathered on
  // the device (bytes moved per flush are linear in its new order entries)
  if (ex->partial) {
    if (!ex->d_gather.ensure((size_t)(nexec - k0) * 4)) return fail_sync(ex, FX_ERR_HIP);
    if (fx::gather_release(ex->d_order.u32(), ex->d_release.u32(), ex->cap, k0, nexec,
                           ex->d_gather.u32(), ex->stream) ||
        hipMemcpyAsync(rel.data(), ex->d_gather.p, rel.size() * 4, hipMemcpyDeviceToHost, ex->stream) ||
        hipStreamSynchronize(ex->stream))
      return fail_sync(ex, FX_ERR_HIP);
    ex->bytes_d2h += (uint64_t)(order.size() + rel.size()) * 4;
  }
  convert(ex, order, rel, nexec);
  return FX_OK;
}

// fetch_commands_to_execute -> execute for the new order entries
// [consumed, nexec) and their release steps, collecting the metrics
void convert(fx_graph_executor* ex, const std::vector<uint32_t>& order, const std::vector<uint32_t>& rel,
             uint32_t nexec) {
  for (size_t x = 0; x < order.size(); ++x) {
    const uint32_t o = order[x];
    const uint32_t rec = FX_ORDER_REC(o);
    const bool start = (o & FX_ORDER_SCC_START) != 0;
    if (start && !ex->cfg.execute_at_commit) {
      uint64_t size = 1;
      while (x + size < order.size() && !(order[x + size] & FX_ORDER_SCC_START)) ++size;
      ex->chain_size[size] += 1;  // ChainSize (mod.rs:492-493)
    }
    if (!ex->cfg.execute_at_commit) {
      const uint32_t rs = rel[x];
      const uint64_t delay = (uint64_t)FX_HDR_T(ex->hdrs[rs]) - FX_HDR_T(ex->hdrs[rec]);
      ex->execution_delay[delay] += 1;  // ExecutionDelay (mod.rs:514-518)
    }
    ex->executed.emplace_back(ex->dots[rec], start);  // device-local sequence
    if (ex->partial) {
      ex->added.insert(ex->dots[rec]);  // added_to_executed_clock (tarjan.rs:294-296)
      ex->executed_set.insert(ex->dots[rec]);
    }
    const Cmd& c = ex->cmds[rec];
    for (uint32_t key : c.keys) {
      ex->to_clients.push_back(fx_executor_result{c.rifl, key, c.read_only});
      if (ex->cfg.executor_monitor_execution_order && !c.read_only) ex->monitor[key].push_back(c.rifl);
    }
  }
  ex->consumed = nexec;
}

int append(fx_graph_executor* ex, fx_dot dot, fx_rifl rifl, const uint32_t* keys, uint32_t nkeys,
           uint32_t read_only, const fx_dot* deps, uint32_t ndeps, uint64_t now_ms, uint32_t kind,
           const uint32_t* dep_shards = nullptr, uint64_t cmd_shards = 0) {
  if (!ex) return FX_ERR_INVALID_ARG;
  if (ex->sticky) return ex->sticky;
  if (ex->executor_index != 0) return FX_ERR_INVALID_ARG;  // mod.rs:220 assert_eq!(executor_index, 0)
  if (dot.source < 1 || dot.source > ex->nsrc || dot.seq <= ex->base[dot.source - 1] ||
      dot.seq - ex->base[dot.source - 1] > FX_SEQ_MASK)
    return FX_ERR_DOT_RANGE;
  if (ndeps && !deps) return FX_ERR_INVALID_ARG;
  if (nkeys && !keys) return FX_ERR_INVALID_ARG;
  if (!ex->have_base) {
    ex->have_base = true;
    ex->t_base = now_ms;
  }
  if (now_ms < ex->t_base || now_ms - ex->t_base > 0x00FFFFFFull) return FX_ERR_TIME_RANGE;
  std::vector<uint32_t> dv;
  dv.reserve(ndeps);
  for (uint32_t j = 0; j < ndeps; ++j) {
    if (deps[j].source < 1 || deps[j].source > 255 || deps[j].seq < 1) return FX_ERR_DOT_RANGE;
    const uint32_t b = deps[j].source <= ex->nsrc ? ex->base[deps[j].source - 1] : 0;
    if (deps[j].seq <= b) continue;  // executed before the handle started
    if (deps[j].seq - b > FX_SEQ_MASK) return FX_ERR_DOT_RANGE;
    dv.push_back(FX_PACK_DOT(deps[j].source, deps[j].seq - b));
    if (ex->partial) {
      const uint32_t mask = dep_shards ? dep_shards[j] : 1u << ex->shard_id;
      auto it = ex->dep_mask.find(dv.back());
      if (it != ex->dep_mask.end() && it->second != mask) return FX_ERR_INVALID_ARG;  // one command, one shard set
      ex->dep_mask[dv.back()] = mask;
    }
  }
  std::sort(dv.begin(), dv.end());  // canonical C1 (executor.rs:76 iterates a HashSet)
  dv.erase(std::unique(dv.begin(), dv.end()), dv.end());
  if (dv.size() > kDmaxDev) return FX_ERR_INVALID_ARG;
  if (ex->dots.size() + 1 >= (1u << 26)) return FX_ERR_INVALID_ARG;
  Cmd c;
  c.rifl = rifl;
  c.keys.assign(keys, keys + nkeys);
  std::sort(c.keys.begin(), c.keys.end());
  c.keys.erase(std::unique(c.keys.begin(), c.keys.end()), c.keys.end());
  c.read_only = read_only;
  c.shards = cmd_shards ? cmd_shards : (1ull << ex->shard_id);
  ex->dots.push_back(FX_PACK_DOT(dot.source, dot.seq - ex->base[dot.source - 1]));
  if (ex->partial && kind == FX_KIND_ADD) ex->rec_of[ex->dots.back()] = (uint32_t)ex->dots.size() - 1;
  ex->hdrs.push_back(FX_MAKE_HDR((uint32_t)(now_ms - ex->t_base), (uint32_t)dv.size(), kind));
  ex->deps.push_back(std::move(dv));
  ex->cmds.push_back(std::move(c));
  return FX_OK;
}

int pending_out(fx_graph_executor* ex, const std::vector<uint32_t>& d, const std::vector<uint32_t>& w, uint32_t c,
                fx_dot* dots, fx_dot* waiting_on, uint32_t cap, uint32_t* n_out) {
  std::vector<std::pair<uint32_t, uint32_t>> pw;
  for (uint32_t i = 0; i < c && i < d.size(); ++i) pw.emplace_back(d[i], w[i]);
  std::sort(pw.begin(), pw.end());
  uint32_t m = 0;
  for (const auto& e : pw) {
    if (m < cap) {
      const uint32_t s0 = FX_DOT_SRC(e.first), s1 = FX_DOT_SRC(e.second);
      dots[m] = fx_dot{s0, FX_DOT_SEQ(e.first) + ex->base[s0 - 1]};
      waiting_on[m] = fx_dot{s1, FX_DOT_SEQ(e.second) + (s1 >= 1 && s1 <= ex->nsrc ? ex->base[s1 - 1] : 0)};
    }
    ++m;
  }
  *n_out = m;
  return FX_OK;
}

}  // namespace

extern "C" {

fx_graph_executor* fx_graph_executor_new(uint8_t process_id, uint64_t shard_id, const fx_config* config) {
  if (!config || config->n < 1 || config->shard_count < 1 || (uint64_t)config->n * config->shard_count > 8 ||
      shard_id >= config->shard_count)
    return nullptr;
  if (config->shard_count > 1 && config->execute_at_commit) return nullptr;
  if (fx_device_count() <= 0) return nullptr;  // no CPU fallback
  auto* ex = new fx_graph_executor();
  ex->process_id = process_id;
  ex->shard_id = shard_id;
  ex->cfg = *config;
  ex->nsrc = config->n * config->shard_count;
  ex->partial = config->shard_count > 1;
  if (ex->partial) ex->tier = FX_TIER_WIDE_HBM;
  const char* pe = std::getenv("FX_HANDLE_PERSIST");
  ex->persist_ok = !(pe && pe[0] == '0');
  ex->ps.timeout_ns = persist_timeout_ns();
  const char* ps = std::getenv("FX_HANDLE_STATS");
  ex->ps.want_stats = ps && ps[0] == '1';
  // the handle's own stream first: a failure here has nothing else to undo
  if (hipStreamCreateWithFlags(&ex->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ex;
    return nullptr;
  }
  // the persistent mode's buffers (if they cannot be had, the batch tiers run)
  if (ex->persist_ok && !ex->partial && persist_alloc(ex) != FX_OK) ex->persist_ok = false;
  return ex;
}

void fx_graph_executor_free(fx_graph_executor* ex) {
  if (!ex) return;
  const bool stopped = persist_stop(ex) == FX_OK;
  if (ex->ps.dead) {
    // the persistent kernel never answered the stop request: it may still
    // read and write the handle's mapped words, rings and state block, and a
    // free or stream destroy would wait for it (or free memory under it).
    // The whole handle is leaked on purpose: no HIP call touches it again.
    std::fprintf(stderr, "fantoch_amd persistent handle: freed while its kernel is unresponsive; "
                         "its buffers and streams are leaked\n");
    return;
  }
  if (ex->ps.stream) {
    bool pooled = false;
    if (stopped && ex->ps.ctl.p) {  // the kernel has exited: the resources go back to the pool
      std::lock_guard<std::mutex> g(g_persist_pool_mu);
      if (g_persist_pool->size() < kPersistPoolMax) {
        auto* r = new PersistRes();
        r->stream = ex->ps.stream;
        r->ctl.swap(ex->ps.ctl);
        r->rows.swap(ex->ps.rows);
        r->out.swap(ex->ps.out);
        r->state.swap(ex->ps.state);
        g_persist_pool->push_back(r);
        pooled = true;
      }
    }
    if (!pooled) (void)hipStreamDestroy(ex->ps.stream);
  }
  hipStream_t s = ex->stream;
  delete ex;  // DevBufs free first
  if (s) (void)hipStreamDestroy(s);
}

int fx_graph_executor_set_executor_index(fx_graph_executor* ex, uint32_t index) {
  if (!ex) return FX_ERR_INVALID_ARG;
  if (ex->shared && index == 0) return FX_ERR_INVALID_ARG;  // a clone serves requests (index > 0)
  ex->executor_index = index;
  return FX_OK;
}

int fx_graph_executor_handle_add(fx_graph_executor* ex, fx_dot dot, fx_rifl rifl, const uint32_t* keys,
                                 uint32_t nkeys, uint32_t read_only, const fx_dot* deps, uint32_t ndeps,
                                 uint64_t now_ms) {
  return append(ex, dot, rifl, keys, nkeys, read_only, deps, ndeps, now_ms, FX_KIND_ADD);
}

int fx_graph_executor_handle_add_sharded(fx_graph_executor* ex, fx_dot dot, fx_rifl rifl, const uint32_t* keys,
                                         uint32_t nkeys, uint32_t read_only, const fx_dot* deps,
                                         const uint32_t* dep_shards, uint32_t ndeps, uint64_t now_ms,
                                         uint64_t cmd_shards) {
  if (!ex || (ndeps && !dep_shards)) return FX_ERR_INVALID_ARG;
  if (!ex->partial) return FX_ERR_UNSUPPORTED;
  // cmd_shards: the command's shard set, 0 = unknown.  An Add of this shard's
  // command includes shard_id; a RequestReply::Info carries a command this
  // shard does not replicate (mod.rs:391-393: only shards outside cmd.shards()
  // are sent one), so any non-empty set is accepted
  return append(ex, dot, rifl, keys, nkeys, read_only, deps, ndeps, now_ms, FX_KIND_ADD, dep_shards, cmd_shards);
}

int fx_graph_executor_handle_executed(fx_graph_executor* ex, const fx_dot* dots, uint32_t n, uint64_t now_ms) {
  if (!ex || (n && !dots)) return FX_ERR_INVALID_ARG;
  if (!ex->partial) return FX_ERR_UNSUPPORTED;
  for (uint32_t i = 0; i < n; ++i) {
    // RequestReply::Executed{dot} (mod.rs:394-402): the dot may be at or below
    // a source's starting frontier (already executed here: a clock no-op)
    const fx_dot d = dots[i];
    if (d.source < 1 || d.source > ex->nsrc || d.seq < 1) return FX_ERR_DOT_RANGE;
    if (d.seq <= ex->base[d.source - 1]) continue;
    int st = append(ex, d, fx_rifl{0, 0}, nullptr, 0, 0, nullptr, 0, now_ms, FX_KIND_EXECUTED);
    if (st) return st;
    ex->added.insert(FX_PACK_DOT(d.source, d.seq - ex->base[d.source - 1]));
  }
  return FX_OK;
}

int fx_graph_executor_requests(fx_graph_executor* ex, uint64_t* shards, fx_dot* dots, uint32_t cap,
                               uint32_t* n_out) {
  if (!ex || !n_out || (cap && (!shards || !dots))) return FX_ERR_INVALID_ARG;
  int st = flush(ex);
  if (st) return st;
  uint32_t c = 0;
  while (c < cap && !ex->requests.empty()) {
    const auto e = *ex->requests.begin();
    ex->requests.erase(ex->requests.begin());
    const uint32_t src = FX_DOT_SRC(e.second);
    shards[c] = e.first;
    dots[c] = fx_dot{src, FX_DOT_SEQ(e.second) + ex->base[src - 1]};
    ++c;
  }
  *n_out = c;
  return FX_OK;
}

int fx_graph_executor_to_executors(fx_graph_executor* ex, fx_dot* dots, uint32_t cap, uint32_t* n_out) {
  if (!ex || !n_out || (cap && !dots)) return FX_ERR_INVALID_ARG;
  int st = flush(ex);
  if (st) return st;
  uint32_t c = 0;
  while (c < cap && !ex->added.empty()) {
    const uint32_t d = *ex->added.begin();
    ex->added.erase(ex->added.begin());
    const uint32_t src = FX_DOT_SRC(d);
    dots[c++] = fx_dot{src, FX_DOT_SEQ(d) + ex->base[src - 1]};
  }
  *n_out = c;
  return FX_OK;
}

// ---- executor index > 0 (partial replication, mod.rs:183-355)
fx_graph_executor* fx_graph_executor_clone(fx_graph_executor* main) {
  if (!main || !main->partial || main->shared) return nullptr;
  auto* c = new fx_graph_executor();
  c->process_id = main->process_id;
  c->shard_id = main->shard_id;
  c->cfg = main->cfg;
  c->nsrc = main->nsrc;
  c->partial = true;
  c->shared = main;
  c->executor_index = 1;  // set_executor_index may change it (> 0)
  return c;
}

namespace {
bool clone_clock_contains(const fx_graph_executor* c, uint32_t src, uint64_t seq) {
  auto it = c->clock.find(src);
  return it != c->clock.end() && (seq <= it->second.first || it->second.second.count(seq));
}
void clone_clock_add(fx_graph_executor* c, uint32_t src, uint64_t seq) {  // AboveExSet::add
  auto& e = c->clock[src];
  if (seq <= e.first) return;
  e.second.insert(seq);
  while (e.second.count(e.first + 1)) e.second.erase(++e.first);
}
// process_requests (mod.rs:294-355): a dot still in the shared VertexIndex is
// answered with its vertex (Info), an executed one with Executed, the rest
// are buffered for cleanup
int process_requests(fx_graph_executor* c, uint64_t from, const std::set<std::pair<uint32_t, uint64_t>>& dots) {
  fx_graph_executor* m = c->shared;
  int st = flush(m);
  if (st) return st;
  for (const auto& gd : dots) {
    const uint32_t src = gd.first;
    const uint64_t seq = gd.second;
    auto it = m->rec_of.end();
    uint32_t dd = 0;
    if (src >= 1 && src <= m->nsrc && seq > m->base[src - 1] && seq - m->base[src - 1] <= FX_SEQ_MASK) {
      dd = FX_PACK_DOT(src, (uint32_t)(seq - m->base[src - 1]));
      it = m->rec_of.find(dd);
    }
    if (it != m->rec_of.end() && !m->executed_set.count(dd)) {
      const Cmd& cmd = m->cmds[it->second];
      // the requesting shard replicates the command: the reference panics (graph/mod.rs:308-316)
      if (from < 64 && ((cmd.shards >> from) & 1u)) return FX_ERR_INVALID_ARG;
      fx_graph_executor::Reply r{from, true, src, seq, cmd.rifl, {}, {}, cmd.shards};
      for (uint32_t x : m->deps[it->second]) {
        const uint32_t s2 = FX_DOT_SRC(x);
        r.deps.push_back(fx_dot{s2, FX_DOT_SEQ(x) + (s2 >= 1 && s2 <= m->nsrc ? m->base[s2 - 1] : 0)});
        auto mk = m->dep_mask.find(x);
        r.shards.push_back(mk == m->dep_mask.end() ? 0u : mk->second);
      }
      c->replies.push_back(std::move(r));
    } else if (clone_clock_contains(c, src, seq)) {
      c->replies.push_back(fx_graph_executor::Reply{from, false, src, seq, fx_rifl{0, 0}, {}, {}});
    } else {
      c->buffered[from].insert(gd);
    }
  }
  return FX_OK;
}
}  // namespace

int fx_graph_executor_handle_executed_info(fx_graph_executor* ex, const fx_dot* dots, uint32_t n) {
  if (!ex || (n && !dots)) return FX_ERR_INVALID_ARG;
  if (ex->executor_index == 0 || !ex->shared) return FX_OK;  // handle_executed: index 0 ignores it
  for (uint32_t i = 0; i < n; ++i) clone_clock_add(ex, dots[i].source, dots[i].seq);
  return FX_OK;
}

int fx_graph_executor_handle_request(fx_graph_executor* ex, uint64_t from_shard, const fx_dot* dots, uint32_t n) {
  if (!ex || (n && !dots)) return FX_ERR_INVALID_ARG;
  if (ex->executor_index == 0 || !ex->shared) return FX_ERR_INVALID_ARG;  // mod.rs:283 assert!(executor_index > 0)
  std::set<std::pair<uint32_t, uint64_t>> ds;
  for (uint32_t i = 0; i < n; ++i) ds.insert({dots[i].source, dots[i].seq});
  return process_requests(ex, from_shard, ds);
}

int fx_graph_executor_cleanup(fx_graph_executor* ex) {
  if (!ex) return FX_ERR_INVALID_ARG;
  if (ex->executor_index == 0 || !ex->shared) return FX_OK;
  std::map<uint64_t, std::set<std::pair<uint32_t, uint64_t>>> b;
  b.swap(ex->buffered);
  for (const auto& kv : b) {
    int st = process_requests(ex, kv.first, kv.second);
    if (st) return st;
  }
  return FX_OK;
}

int fx_graph_executor_request_replies(fx_graph_executor* ex, fx_request_reply* out, uint32_t cap, fx_dot* deps,
                                      uint32_t* dep_shards, uint32_t deps_cap, uint32_t* n_out) {
  if (!ex || !n_out || (cap && !out) || (deps_cap && (!deps || !dep_shards))) return FX_ERR_INVALID_ARG;
  uint32_t c = 0, k = 0;
  while (c < cap && !ex->replies.empty()) {
    const auto& r = ex->replies.front();
    if (k + r.deps.size() > deps_cap) break;
    out[c] = fx_request_reply{r.to, r.info ? 1u : 0u, fx_dot{r.src, (uint32_t)r.seq}, r.rifl,
                              (uint32_t)r.deps.size(), k, r.info ? r.cmd_shards : 0u};
    for (size_t j = 0; j < r.deps.size(); ++j, ++k) {
      deps[k] = r.deps[j];
      dep_shards[k] = r.shards[j];
    }
    ex->replies.pop_front();
    ++c;
  }
  *n_out = c;
  return FX_OK;
}

int fx_graph_executor_index_only(fx_graph_executor* ex, fx_dot dot, fx_rifl rifl, const uint32_t* keys,
                                 uint32_t nkeys, const fx_dot* deps, uint32_t ndeps, uint64_t now_ms) {
  return append(ex, dot, rifl, keys, nkeys, 0, deps, ndeps, now_ms, FX_KIND_INDEX_ONLY);
}

int fx_graph_executor_set_executed_frontier(fx_graph_executor* ex, const uint64_t* frontier, uint32_t n) {
  if (!ex || !frontier || n > 8 || n > ex->nsrc) return FX_ERR_INVALID_ARG;
  if (!ex->dots.empty()) return FX_ERR_INVALID_ARG;
  for (uint32_t p = 0; p < n; ++p)
    if (frontier[p] > 0xFFFFFFFFull) return FX_ERR_DOT_RANGE;
  for (uint32_t p = 0; p < n; ++p) ex->base[p] = (uint32_t)frontier[p];
  return FX_OK;
}

int fx_graph_executor_to_clients(fx_graph_executor* ex, fx_executor_result* out, uint32_t cap, uint32_t* n_out) {
  if (!ex || (cap && !out) || !n_out) return FX_ERR_INVALID_ARG;
  int st = flush(ex);
  if (st) return st;
  uint32_t c = 0;
  while (c < cap && !ex->to_clients.empty()) {
    out[c++] = ex->to_clients.front();
    ex->to_clients.pop_front();
  }
  *n_out = c;
  return FX_OK;
}

int fx_graph_executor_drain_dots(fx_graph_executor* ex, fx_dot* out, uint8_t* scc_start, uint32_t cap,
                                 uint32_t* n_out) {
  if (!ex || (cap && !out) || !n_out) return FX_ERR_INVALID_ARG;
  int st = flush(ex);
  if (st) return st;
  uint32_t c = 0;
  while (c < cap && !ex->executed.empty()) {
    const auto e = ex->executed.front();
    ex->executed.pop_front();
    const uint32_t src = FX_DOT_SRC(e.first);
    out[c] = fx_dot{src, FX_DOT_SEQ(e.first) + ex->base[src - 1]};
    if (scc_start) scc_start[c] = e.second ? 1 : 0;
    ++c;
  }
  *n_out = c;
  return FX_OK;
}

int fx_graph_executor_metrics(fx_graph_executor* ex, uint32_t kind, uint64_t* values, uint64_t* counts,
                              uint32_t cap, uint32_t* n_out) {
  if (!ex || !n_out || kind > 1 || (cap && (!values || !counts))) return FX_ERR_INVALID_ARG;
  int st = flush(ex);
  if (st) return st;
  const auto& h = kind == 0 ? ex->execution_delay : ex->chain_size;
  uint32_t c = 0;
  for (const auto& kv : h) {
    if (c < cap) {
      values[c] = kv.first;
      counts[c] = kv.second;
    }
    ++c;
  }
  *n_out = c;
  return FX_OK;
}

int fx_graph_executor_monitor(fx_graph_executor* ex, uint32_t key, fx_rifl* out, uint32_t cap, uint32_t* n_out) {
  if (!ex || !n_out || (cap && !out)) return FX_ERR_INVALID_ARG;
  if (!ex->cfg.executor_monitor_execution_order) return FX_ERR_INVALID_ARG;  // monitor() = None
  int st = flush(ex);
  if (st) return st;
  auto it = ex->monitor.find(key);
  uint32_t c = 0;
  if (it != ex->monitor.end()) {
    for (const auto& r : it->second) {
      if (c < cap) out[c] = r;
      ++c;
    }
  }
  *n_out = c;
  return FX_OK;
}

int fx_graph_executor_pending(fx_graph_executor* ex, fx_dot* dots, fx_dot* waiting_on, uint32_t cap,
                              uint32_t* n_out) {
  if (!ex || !n_out || (cap && (!dots || !waiting_on))) return FX_ERR_INVALID_ARG;
  int st = flush(ex);
  if (st) return st;
  *n_out = 0;
  if (ex->processed == 0) return FX_OK;
  if (ex->ps.active) {  // the persistent kernel's state, saved when it stops
    if (const int s2 = persist_stop(ex)) return s2;
    std::vector<uint32_t> block(fx::wave_state_words_per_stream());
    // on the handle's own stream: a null-stream copy would also wait for other
    // handles' resident kernels (their streams are blocking ones)
    if (hipMemcpyAsync(block.data(), ex->ps.state.p, block.size() * 4, hipMemcpyDeviceToHost, ex->ps.stream) ||
        hipStreamSynchronize(ex->ps.stream))
      return FX_ERR_HIP;
    std::vector<uint32_t> d(64), w(64);
    const uint32_t c = fx::decode_pending(FX_TIER_WAVE, block.data(), 0, d.data(), w.data(), 64);
    return pending_out(ex, d, w, c, dots, waiting_on, cap, n_out);
  }
  std::vector<uint32_t> block((ex->partial ? fx_partial_state_bytes(ex->nsrc, 1)
                                           : fx_batch_state_bytes(ex->tier, ex->nsrc, 1)) / 4);
  if (hipMemcpyAsync(block.data(), ex->d_state.p, block.size() * 4, hipMemcpyDeviceToHost, ex->stream) ||
      hipStreamSynchronize(ex->stream))
    return FX_ERR_HIP;
  const uint32_t slots = ex->partial ? 16384 * 64 : ex->tier == FX_TIER_WIDE_HBM ? 16384 : 64;
  std::vector<uint32_t> d(slots), w(slots);
  const uint32_t c = ex->tier == FX_TIER_WIDE_HBM
                         ? fx::wide_decode_pending(block.data(), ex->nsrc, d.data(), w.data(), slots, ex->partial)
                         : fx::decode_pending(ex->tier, block.data(), 0, d.data(), w.data(), slots);
  return pending_out(ex, d, w, c, dots, waiting_on, cap, n_out);
}


int fx_graph_executor_parallel(void) { return 1; }

int fx_graph_executor_persist_stats(const fx_graph_executor* ex, uint64_t* out, uint32_t n) {
  if (!ex || (!out && n)) return FX_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < n && i < FX_PERSIST_STATS; ++i) out[i] = ex->ps.stats[i];
  return FX_OK;
}

int fx_graph_executor_debug_hooks(fx_graph_executor* ex, uint32_t skip_status_flush, uint32_t hold_ms) {
  if (!ex || hold_ms > 10000u) return FX_ERR_INVALID_ARG;
  ex->ps.debug_skip_status = skip_status_flush;
  ex->ps.debug_hold_ticks = hold_ms * 100000u;  // s_memrealtime: 100 MHz
  return FX_OK;
}

int fx_graph_executor_transfer_stats(const fx_graph_executor* ex, uint64_t* h2d, uint64_t* d2h) {
  if (!ex || !h2d || !d2h) return FX_ERR_INVALID_ARG;
  *h2d = ex->bytes_h2d;
  *d2h = ex->bytes_d2h;
  return FX_OK;
}

// ------------------------------------------------------------ histogram
// histogram.rs:172-235
int fx_hist_stats_compute(const uint64_t* values, const uint64_t* counts, uint32_t n, fx_hist_stats* out) {
  if (!out || (n && (!values || !counts))) return FX_ERR_INVALID_ARG;
  uint64_t sum = 0, cnt = 0;
  double mn = NAN, mx = NAN;
  for (uint32_t i = 0; i < n; ++i) {
    if (i && values[i] <= values[i - 1]) return FX_ERR_INVALID_ARG;
    if (!counts[i]) continue;
    sum += values[i] * counts[i];
    cnt += counts[i];
    if (std::isnan(mn)) mn = (double)values[i];
    mx = (double)values[i];
  }
  const double count = (double)cnt;
  const double mean = (double)sum / count;
  double var_acc = 0.0, dist_acc = 0.0;
  for (uint32_t i = 0; i < n; ++i) {
    if (!counts[i]) continue;
    const double x = (double)values[i], xc = (double)counts[i];
    const double diff = mean - x;
    var_acc += (diff * diff) * xc;
    dist_acc += std::fabs(diff) * xc;
  }
  const double stddev = std::sqrt(var_acc / (count - 1.0));  // corrected (n - 1)
  out->count = count;
  out->mean = mean;
  out->stddev = stddev;
  out->cov = stddev / mean;
  out->mdtm = dist_acc / count;
  out->min = mn;
  out->max = mx;
  return FX_OK;
}

// histogram.rs:111-170
int fx_hist_percentile(const uint64_t* values, const uint64_t* counts, uint32_t n, double p, double* out) {
  if (!out || p < 0.0 || p > 1.0 || (n && (!values || !counts))) return FX_ERR_INVALID_ARG;
  std::vector<std::pair<uint64_t, uint64_t>> data;
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (counts[i]) {
      data.emplace_back(values[i], counts[i]);
      total += counts[i];
    }
  if (data.empty()) {
    *out = 0.0;
    return FX_OK;
  }
  const double index = p * (double)total;
  const double index_rounded = std::round(index);  // Rust f64::round: half away from zero
  const bool whole = std::fabs(index - index_rounded) == 0.0;
  uint64_t idx = (uint64_t)index_rounded;
  size_t pos = 0;
  double left = 0.0, right = 0.0;
  bool have_right = false;
  while (true) {
    if (pos >= data.size()) return FX_ERR_INVALID_ARG;  // "there should a next histogram value"
    const uint64_t value = data[pos].first, count = data[pos].second;
    ++pos;
    if (idx == count) {
      left = (double)value;
      if (pos < data.size()) {
        right = (double)data[pos].first;
        have_right = true;
      }
      break;
    } else if (idx < count) {
      left = (double)value;
      right = left;
      have_right = true;
      break;
    }
    idx -= count;
  }
  if (whole) {
    if (!have_right) return FX_ERR_INVALID_ARG;  // "there should be a right value"
    *out = (left + right) / 2.0;
  } else {
    *out = left;
  }
  return FX_OK;
}

}  // extern "C"
