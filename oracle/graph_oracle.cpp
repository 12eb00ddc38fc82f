// oracle/graph_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of fantoch_ps's dependency-graph executor, used as the
// CHECKER of the HIP path (tests/, __graft_entry__.smoke(), bench.py's
// cpu_baseline leg).  Nothing in the product links or calls this file.
//
// It follows the reference's data structures one to one instead of the GPU
// design (slot tables, iterative DFS, windowed clocks), so the two are
// independent implementations:
//   Dot / derived Ord ............ fantoch/src/id.rs:21-56
//   AEClock / AboveExSet ......... crate threshold 0.9.1 (absent here; its
//                                  published semantics: per-actor contiguous
//                                  max + exception set above it), used at
//                                  graph/mod.rs:49,94,207,339,397 and
//                                  tarjan.rs:101,131-132,293
//   Vertex ....................... graph/tarjan.rs:319-356
//   VertexIndex .................. graph/index.rs:18-51
//   PendingIndex ................. graph/index.rs:145-208
//   TarjanSCCFinder .............. graph/tarjan.rs:25-316
//   DependencyGraph .............. graph/mod.rs:45-677 (with partial
//                                  replication: first-search collection,
//                                  out-requests, Executed replies and the
//                                  request-serving clone, graph_oracle.hpp)
//   GraphExecutor::handle ........ graph/executor.rs:69-93
//
// Canonicalisation: C1 a vertex's deps are iterated in
// ascending Dot order (replaces `Vec::from_iter(HashSet)`, executor.rs:76);
// C2 the waiters of a released dot are tried in ascending Dot order (replaces
// `for dot in pending` over a HashSet, mod.rs:601).  Everything else (LIFO
// check_pending, visited-skip rule, immediate executed-clock update) is the
// reference's own order.
//
// Parity pinning: see tests/test_oracle_kat.py — the reference's graph unit
// tests (mod.rs:714-1348) and its histogram KATs (histogram.rs:390-463).

#include "graph_oracle.hpp"
#include "../include/fantoch_amd.h"  // plane layout (fx_index) only

// ============================================================ C interface
using oracle::Dot;
using oracle::DependencyGraph;

namespace {
constexpr uint32_t SEQ_BITS = 24;
constexpr uint32_t SEQ_MASK = (1u << SEQ_BITS) - 1;
constexpr uint32_t ORDER_SCC_START = 0x80000000u;
constexpr uint32_t RELEASE_NONE = 0xFFFFFFFFu;

Dot unpack(uint32_t d) { return Dot{d >> SEQ_BITS, (uint64_t)(d & SEQ_MASK)}; }

// Runs one stream of the plane layout (include/fantoch_amd.h) through a fresh
// DependencyGraph, exactly as GraphExecutor::handle would see it.
int run_stream(const uint32_t* dot, const uint32_t* hdr, const uint32_t* deps, uint32_t S,
               uint32_t steps, uint32_t dmax, uint32_t len, uint32_t n, uint32_t flags,
               const uint32_t* init_frontier, uint32_t s, uint32_t* order, uint32_t* release,
               uint32_t* nexec, uint32_t* max_pending, uint32_t* max_window) {
  DependencyGraph g(1, n);
  if (init_frontier) {
    for (uint32_t p = 0; p < 8 && p < n; ++p) {
      uint32_t f = init_frontier[(size_t)s * 8 + p];
      if (f) g.executed_clock.clock[p + 1].max = f;  // AboveExSet::from_events(1..=f)
    }
  }
  const size_t plane = fx_plane_words(S, steps);
  for (uint32_t i = 0; i < steps; ++i) release[fx_index(i, s, steps)] = RELEASE_NONE;
  uint32_t k = 0;
  int status = 0;
  const bool at_commit = (flags & 2u) != 0;
  for (uint32_t i = 0; i < len; ++i) {
    size_t at = fx_index(i, s, steps);
    uint32_t h = hdr[at];
    uint32_t t = h & 0x00FFFFFFu;
    uint32_t nd = (h >> 24) & 31u;
    uint32_t kind = h >> 29;
    Dot d = unpack(dot[at]);
    if (at_commit) {  // executor.rs:72-73: execute immediately, no graph
      order[fx_index(k, s, steps)] = i | ORDER_SCC_START;
      release[at] = i;
      ++k;
      continue;
    }
    std::vector<Dot> dv;
    dv.reserve(nd);
    for (uint32_t j = 0; j < nd && j < dmax; ++j)
      dv.push_back(unpack(deps[j * plane + at]));
    if (kind == 1) {  // INDEX_ONLY: vertex_index.index without a search
      auto v = std::make_unique<oracle::Vertex>();
      v->dot = d;
      v->rec = i;
      std::sort(dv.begin(), dv.end());
      v->deps = dv;
      v->start_time_ms = t;
      if (!g.index(std::move(v))) { status = 3; break; }
      continue;
    }
    if (!g.handle_add(d, i, dv, t)) { status = 3; break; }
    for (const auto& e : g.to_execute) {
      if (k >= steps) { status = 8; break; }
      order[fx_index(k, s, steps)] = e.rec | (e.scc_start ? ORDER_SCC_START : 0u);
      release[fx_index(e.rec, s, steps)] = i;
      ++k;
    }
    g.to_execute.clear();
    if (max_pending && g.vertex_index.size() > max_pending[s]) max_pending[s] = (uint32_t)g.vertex_index.size();
    if (max_window) {
      for (const auto& kv : g.executed_clock.clock)
        if (!kv.second.exs.empty()) {
          uint64_t wdt = *kv.second.exs.rbegin() - kv.second.max;
          if (wdt > max_window[s]) max_window[s] = (uint32_t)wdt;
        }
    }
    if (status) break;
  }
  nexec[s] = k;
  return status;
}
}  // namespace

extern "C" {

// Batch form over the plane layout; one DependencyGraph per stream, streams
// distributed over `nthreads` std::threads (the reference's rayon par_iter over
// independent simulations, fantoch_ps/src/bin/simulation.rs:49-57,216-217).
int oracle_batch_execute(const uint32_t* dot, const uint32_t* hdr, const uint32_t* deps,
                         uint32_t S, uint32_t steps, uint32_t dmax, const uint32_t* lengths,
                         uint32_t n, uint32_t flags, const uint32_t* init_frontier,
                         uint32_t* order, uint32_t* release, uint32_t* nexec, uint32_t* err,
                         int nthreads, uint32_t* max_pending, uint32_t* max_window) {
  if (nthreads < 1) nthreads = 1;
  std::atomic<uint32_t> next{0};
  auto worker = [&]() {
    while (true) {
      uint32_t s = next.fetch_add(1);
      if (s >= S) break;
      uint32_t len = lengths ? lengths[s] : steps;
      try {
        err[s] = (uint32_t)run_stream(dot, hdr, deps, S, steps, dmax, len, n, flags,
                                      init_frontier, s, order, release, nexec, max_pending,
                                      max_window);
      } catch (const std::exception&) {
        err[s] = 99;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nthreads; ++t) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  return 0;
}

// ---- single graph handle, for the reference's unit-test shapes ----------
void* oracle_graph_new(uint32_t process_id, uint32_t n) { return new DependencyGraph(process_id, n); }
void oracle_graph_free(void* g) { delete static_cast<DependencyGraph*>(g); }

static std::vector<Dot> make_deps(const uint32_t* dep_src, const uint64_t* dep_seq, uint32_t nd) {
  std::vector<Dot> v;
  for (uint32_t j = 0; j < nd; ++j) v.push_back(Dot{dep_src[j], dep_seq[j]});
  return v;
}

// DependencyGraph::handle_add; returns 0, or 3 on double index, 99 on a
// reference assertion failure.
int oracle_graph_handle_add(void* gp, uint32_t src, uint64_t seq, const uint32_t* dep_src,
                            const uint64_t* dep_seq, uint32_t nd, uint64_t t_ms, uint32_t rec) {
  auto* g = static_cast<DependencyGraph*>(gp);
  try {
    return g->handle_add(Dot{src, seq}, rec, make_deps(dep_src, dep_seq, nd), t_ms) ? 0 : 3;
  } catch (const std::exception&) {
    return 99;
  }
}

// queue.vertex_index.index(Vertex::new(..)) (mod.rs:1164-1306).
int oracle_graph_index_only(void* gp, uint32_t src, uint64_t seq, const uint32_t* dep_src,
                            const uint64_t* dep_seq, uint32_t nd, uint64_t t_ms, uint32_t rec) {
  auto* g = static_cast<DependencyGraph*>(gp);
  auto v = std::make_unique<oracle::Vertex>();
  v->dot = Dot{src, seq};
  v->rec = rec;
  v->deps = make_deps(dep_src, dep_seq, nd);
  std::sort(v->deps.begin(), v->deps.end());
  v->start_time_ms = t_ms;
  return g->index(std::move(v)) ? 0 : 3;
}

// queue.executed_clock = AEClock::from(vclock(..)) (mod.rs:1309-1315).
void oracle_graph_set_executed(void* gp, uint32_t src, uint64_t frontier) {
  auto* g = static_cast<DependencyGraph*>(gp);
  oracle::AboveExSet s;
  s.max = frontier;
  g->executed_clock.clock[src] = s;
}

// queue.find_scc(first_find, root, ..) as called directly by the
// sccs_found_and_missing_dep test (mod.rs:1317-1321).  Returns the
// FinderInfo kind (0 Found, 1 MissingDependencies, 2 NotPending) and fills the
// missing deps (up to cap) and the ready count.
int oracle_graph_find_scc(void* gp, uint32_t src, uint64_t seq, int first_find,
                          uint32_t* missing_src, uint64_t* missing_seq, uint32_t cap,
                          uint32_t* n_missing, uint64_t* ready_commands, uint32_t* n_dots) {
  auto* g = static_cast<DependencyGraph*>(gp);
  size_t total = 0;
  std::vector<Dot> dots;
  std::set<Dot> visited;
  std::set<std::pair<Dot, uint32_t>> missing;
  oracle::FinderResult r;
  try {
    r = g->find_scc(first_find != 0, Dot{src, seq}, total, 0, dots, visited, missing);
  } catch (const std::exception&) {
    return 99;
  }
  uint32_t m = 0;
  for (const auto& dep : missing) {
    const Dot& d = dep.first;
    if (m < cap) { missing_src[m] = d.source; missing_seq[m] = d.sequence; }
    ++m;
  }
  *n_missing = m;
  *ready_commands = total;
  *n_dots = (uint32_t)dots.size();
  return r == oracle::FinderResult::Found ? 0 : r == oracle::FinderResult::MissingDependencies ? 1 : 2;
}

// ---- partial replication (shard_count > 1; mod.rs:82-406, tarjan.rs:148-166)
void* oracle_graph_new_sharded(uint32_t process_id, uint32_t n, uint32_t shard_id, uint32_t shard_count) {
  return new DependencyGraph(process_id, n, shard_id, shard_count);
}

// handle_add with each dep's Dependency::shards bitmask (RequestReply::Info
// is the same call, mod.rs:390-393)
int oracle_graph_handle_add_sharded(void* gp, uint32_t src, uint64_t seq, const uint32_t* dep_src,
                                    const uint64_t* dep_seq, const uint32_t* dep_shards, uint32_t nd,
                                    uint64_t t_ms, uint32_t rec) {
  auto* g = static_cast<DependencyGraph*>(gp);
  try {
    return g->handle_add_sharded(Dot{src, seq}, rec, make_deps(dep_src, dep_seq, nd),
                                 std::vector<uint32_t>(dep_shards, dep_shards + nd), t_ms)
               ? 0
               : 3;
  } catch (const std::exception&) {
    return 99;
  }
}

// RequestReply::Executed (mod.rs:394-402)
int oracle_graph_executed_reply(void* gp, uint32_t src, uint64_t seq, uint64_t t_ms) {
  auto* g = static_cast<DependencyGraph*>(gp);
  try {
    g->handle_executed_reply(Dot{src, seq}, t_ms);
  } catch (const std::exception&) {
    return 99;
  }
  return 0;
}

// DependencyGraph::requests (mod.rs:148-151), drained: (target shard, dot) ascending
uint32_t oracle_graph_requests(void* gp, uint32_t* shard, uint32_t* src, uint64_t* seq, uint32_t cap) {
  auto* g = static_cast<DependencyGraph*>(gp);
  uint32_t m = 0;
  for (const auto& kv : g->out_requests)
    for (const Dot& d : kv.second) {
      if (m < cap) {
        shard[m] = kv.first;
        src[m] = d.source;
        seq[m] = d.sequence;
      }
      ++m;
    }
  g->out_requests.clear();
  return m;
}

// DependencyGraph::to_executors (mod.rs:137-144), drained: dots added to the
// executed clock, ascending
uint32_t oracle_graph_to_executors(void* gp, uint32_t* src, uint64_t* seq, uint32_t cap) {
  auto* g = static_cast<DependencyGraph*>(gp);
  uint32_t m = 0;
  for (const Dot& d : g->added_to_executed_clock) {
    if (m < cap) {
      src[m] = d.source;
      seq[m] = d.sequence;
    }
    ++m;
  }
  g->added_to_executed_clock.clear();
  return m;
}

// Every PendingIndex registration (waiting vertex, missing parent), ascending.
uint32_t oracle_graph_waits(void* gp, uint32_t* vsrc, uint64_t* vseq, uint32_t* psrc, uint64_t* pseq,
                            uint32_t cap) {
  auto* g = static_cast<DependencyGraph*>(gp);
  std::set<std::pair<Dot, Dot>> all;
  for (const auto& kv : g->pending_index)
    for (const Dot& c : kv.second) all.insert({c, kv.first});
  uint32_t m = 0;
  for (const auto& e : all) {
    if (m < cap) {
      vsrc[m] = e.first.source;
      vseq[m] = e.first.sequence;
      psrc[m] = e.second.source;
      pseq[m] = e.second.sequence;
    }
    ++m;
  }
  return m;
}

// Executor index > 0 sharing `gp`'s VertexIndex (partial replication).
void* oracle_clone_new(void* gp) { return new oracle::ExecutorClone{static_cast<DependencyGraph*>(gp), {}, {}, {}}; }
void oracle_clone_free(void* c) { delete static_cast<oracle::ExecutorClone*>(c); }
void oracle_clone_handle_executed(void* c, const uint32_t* src, const uint64_t* seq, uint32_t n) {
  std::vector<Dot> dots;
  for (uint32_t i = 0; i < n; ++i) dots.push_back(Dot{src[i], seq[i]});
  static_cast<oracle::ExecutorClone*>(c)->handle_executed(dots);
}
void oracle_clone_handle_request(void* c, uint32_t from, const uint32_t* src, const uint64_t* seq, uint32_t n) {
  std::set<Dot> dots;
  for (uint32_t i = 0; i < n; ++i) dots.insert(Dot{src[i], seq[i]});
  static_cast<oracle::ExecutorClone*>(c)->handle_request(from, dots);
}
void oracle_clone_cleanup(void* c) { static_cast<oracle::ExecutorClone*>(c)->cleanup(); }
// Drains request replies: per reply (to shard, kind 1 Info / 0 Executed, dot,
// rec, ndeps) and its deps appended to dep_src / dep_seq / dep_shards.
uint32_t oracle_clone_replies(void* c, uint32_t* to_shard, uint32_t* kind, uint32_t* src, uint64_t* seq,
                              uint32_t* rec, uint32_t* ndeps, uint32_t cap, uint32_t* dep_src, uint64_t* dep_seq,
                              uint32_t* dep_shards, uint32_t dep_cap) {
  auto* cl = static_cast<oracle::ExecutorClone*>(c);
  uint32_t m = 0, k = 0;
  for (const auto& r : cl->out_request_replies) {
    if (m >= cap || k + r.deps.size() > dep_cap) break;
    to_shard[m] = r.to_shard;
    kind[m] = r.info ? 1 : 0;
    src[m] = r.dot.source;
    seq[m] = r.dot.sequence;
    rec[m] = r.rec;
    ndeps[m] = (uint32_t)r.deps.size();
    for (size_t j = 0; j < r.deps.size(); ++j, ++k) {
      dep_src[k] = r.deps[j].source;
      dep_seq[k] = r.deps[j].sequence;
      dep_shards[k] = r.dep_shards[j];
    }
    ++m;
  }
  cl->out_request_replies.erase(cl->out_request_replies.begin(), cl->out_request_replies.begin() + m);
  return m;
}

// DependencyGraph::commands_to_execute (mod.rs:158-160): drains executed dots.
uint32_t oracle_graph_drain(void* gp, uint32_t* src, uint64_t* seq, uint32_t* rec,
                            uint8_t* scc_start, uint32_t cap) {
  auto* g = static_cast<DependencyGraph*>(gp);
  uint32_t m = 0;
  for (const auto& e : g->to_execute) {
    if (m >= cap) break;
    src[m] = e.dot.source;
    seq[m] = e.dot.sequence;
    rec[m] = e.rec;
    scc_start[m] = e.scc_start ? 1 : 0;
    ++m;
  }
  g->to_execute.erase(g->to_execute.begin(), g->to_execute.begin() + m);
  return m;
}

// Pending vertices (VertexIndex) ascending, with the dot each is registered
// on in the PendingIndex (0,0 if none).
uint32_t oracle_graph_pending(void* gp, uint32_t* src, uint64_t* seq, uint32_t* wsrc,
                              uint64_t* wseq, uint32_t cap) {
  auto* g = static_cast<DependencyGraph*>(gp);
  uint32_t m = 0;
  for (const auto& kv : g->vertex_index) {
    if (m >= cap) break;
    src[m] = kv.first.source;
    seq[m] = kv.first.sequence;
    wsrc[m] = 0;
    wseq[m] = 0;
    for (const auto& pk : g->pending_index)
      if (pk.second.count(kv.first)) { wsrc[m] = pk.first.source; wseq[m] = pk.first.sequence; }
    ++m;
  }
  return m;
}

// Metrics as (value, count) pairs: kind 0 ExecutionDelay, 1 ChainSize.
uint32_t oracle_graph_metrics(void* gp, uint32_t kind, uint64_t* values, uint64_t* counts,
                              uint32_t cap) {
  auto* g = static_cast<DependencyGraph*>(gp);
  const auto& h = kind == 0 ? g->execution_delay : g->chain_size;
  uint32_t m = 0;
  for (const auto& kv : h) {
    if (m < cap) { values[m] = kv.first; counts[m] = kv.second; }
    ++m;
  }
  return m;
}

}  // extern "C"
