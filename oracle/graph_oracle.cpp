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
//   DependencyGraph .............. graph/mod.rs:45-677 (shard_count == 1)
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

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../include/fantoch_amd.h"  // plane layout (fx_index) only

namespace oracle {

// fantoch/src/id.rs:21-27 — Id<ProcessId>{source, sequence}, derived Ord.
struct Dot {
  uint32_t source = 0;
  uint64_t sequence = 0;
  bool operator<(const Dot& o) const {
    return source != o.source ? source < o.source : sequence < o.sequence;
  }
  bool operator==(const Dot& o) const { return source == o.source && sequence == o.sequence; }
  bool operator!=(const Dot& o) const { return !(*this == o); }
};

// threshold::AboveExSet — events 1..=max are all present, plus the exception
// set `exs` of events above max.
struct AboveExSet {
  uint64_t max = 0;
  std::set<uint64_t> exs;
  // AboveExSet::add: returns whether the event is new.
  bool add(uint64_t event) {
    if (event == max + 1) {
      max = event;
      // compress: absorb exceptions that are now contiguous
      while (true) {
        auto it = exs.find(max + 1);
        if (it == exs.end()) break;
        exs.erase(it);
        max += 1;
      }
      return true;
    } else if (event > max + 1) {
      return exs.insert(event).second;
    }
    return false;
  }
  bool contains(uint64_t event) const { return event <= max || exs.count(event) > 0; }
};

// threshold::AEClock<ProcessId> — one AboveExSet per actor
// (AEClock::with(ids), graph/mod.rs:90-94).
struct AEClock {
  std::map<uint32_t, AboveExSet> clock;
  bool contains(uint32_t actor, uint64_t event) const {
    auto it = clock.find(actor);
    return it != clock.end() && it->second.contains(event);
  }
  bool add(uint32_t actor, uint64_t event) { return clock[actor].add(event); }
};

// graph/tarjan.rs:319-356
struct Vertex {
  Dot dot;
  uint32_t rec = 0;              // arrival index in the stream (stands in for `cmd`)
  std::vector<Dot> deps;         // canonical C1: ascending
  uint64_t start_time_ms = 0;
  size_t id = 0;
  size_t low = 0;
  bool on_stack = false;
};

enum class FinderResult { Found, MissingDependencies, NotPending, NotFound };

// One executed command as the executor emits it (save_scc, mod.rs:488-523).
struct Executed {
  Dot dot;
  uint32_t rec;
  bool scc_start;
  uint64_t delay_ms;
};

struct DependencyGraph {
  uint32_t process_id;
  uint32_t n;
  AEClock executed_clock;
  std::map<Dot, std::unique_ptr<Vertex>> vertex_index;  // VertexIndex (index.rs:18-51)
  std::map<Dot, std::set<Dot>> pending_index;           // PendingIndex (index.rs:145-208), C2
  // TarjanSCCFinder (tarjan.rs:25-33)
  size_t finder_id = 0;
  std::vector<Dot> stack;
  std::vector<std::set<Dot>> sccs;  // SCC = BTreeSet<Dot> (tarjan.rs:15)
  // to_execute (mod.rs:59)
  std::vector<Executed> to_execute;
  // metrics (mod.rs:492-518)
  std::map<uint64_t, uint64_t> chain_size;
  std::map<uint64_t, uint64_t> execution_delay;

  DependencyGraph(uint32_t pid, uint32_t n_) : process_id(pid), n(n_) {
    // AEClock::with(all process ids) — mod.rs:90-94
    for (uint32_t p = 1; p <= n; ++p) executed_clock.clock[p];
  }

  Vertex* find(const Dot& d) {
    auto it = vertex_index.find(d);
    return it == vertex_index.end() ? nullptr : it->second.get();
  }

  // VertexIndex::index (index.rs:33-37); returns false if already indexed.
  bool index(std::unique_ptr<Vertex> v) {
    Dot d = v->dot;
    auto res = vertex_index.emplace(d, nullptr);
    if (!res.second) return false;
    res.first->second = std::move(v);
    return true;
  }

  // mod.rs:213-275; returns false on the double-index panic (mod.rs:233-237).
  bool handle_add(const Dot& dot, uint32_t rec, std::vector<Dot> deps, uint64_t time_ms) {
    auto v = std::make_unique<Vertex>();
    v->dot = dot;
    v->rec = rec;
    std::sort(deps.begin(), deps.end());  // C1
    deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
    v->deps = std::move(deps);
    v->start_time_ms = time_ms;
    if (!index(std::move(v))) return false;

    size_t initial_ready = to_execute.size();
    size_t total_scc_count = 0;
    std::vector<Dot> dots;
    std::set<Dot> visited;
    std::set<Dot> missing;
    FinderResult r = find_scc(true, dot, total_scc_count, time_ms, dots, visited, missing);
    if (r == FinderResult::Found) {
      check_pending(dots, total_scc_count, time_ms);
    } else if (r == FinderResult::MissingDependencies) {
      index_pending(dot, missing);
      check_pending(dots, total_scc_count, time_ms);
    } else {
      throw std::logic_error("just added dot must be pending");  // mod.rs:257-259
    }
    if (to_execute.size() != initial_ready + total_scc_count)  // mod.rs:263
      throw std::logic_error("newly ready commands not incorporated");
    return true;
  }

  // mod.rs:409-486.  Out-params: dots of the SCCs saved, visited, missing deps.
  FinderResult find_scc(bool first_find, const Dot& dot, size_t& total_scc_count, uint64_t time_ms,
                        std::vector<Dot>& dots, std::set<Dot>& visited, std::set<Dot>& missing) {
    size_t scc_count = 0;
    size_t missing_deps_count = 0;
    Dot result_missing;
    FinderResult fr;
    Vertex* v = find(dot);
    if (v == nullptr) {
      fr = FinderResult::NotPending;  // mod.rs:664-667
    } else {
      fr = strong_connect(first_find, dot, v, scc_count, missing_deps_count, result_missing);
    }
    total_scc_count += scc_count;
    // save new SCCs (mod.rs:438-444)
    std::vector<std::set<Dot>> found;
    found.swap(sccs);
    for (auto& scc : found) save_scc(scc, dots, time_ms);
    // finalize (tarjan.rs:60-93): reset ids of the vertices still on the stack
    finder_id = 0;
    visited.clear();
    while (!stack.empty()) {
      Dot d = stack.back();
      stack.pop_back();
      Vertex* sv = find(d);
      if (sv == nullptr) throw std::logic_error("stack member should exist");  // tarjan.rs:81-84
      sv->id = 0;
      visited.insert(d);
    }
    missing.clear();
    switch (fr) {
      case FinderResult::Found:
        return FinderResult::Found;
      case FinderResult::MissingDependencies:
        missing.insert(result_missing);
        return FinderResult::MissingDependencies;
      case FinderResult::NotPending:
        return FinderResult::NotPending;
      case FinderResult::NotFound:
      default:
        // only reachable with partial replication (missing deps collected)
        throw std::logic_error("either there's a missing dependency, or we should find an SCC");
    }
  }

  // tarjan.rs:96-316 (shard_count == 1: give up on the first missing dep).
  FinderResult strong_connect(bool first_find, const Dot& dot, Vertex* vertex, size_t& scc_count,
                              size_t& missing_deps_count, Dot& missing_out) {
    (void)first_find;
    finder_id += 1;
    vertex->id = finder_id;
    vertex->low = finder_id;
    vertex->on_stack = true;
    stack.push_back(dot);

    for (size_t i = 0; i < vertex->deps.size(); ++i) {
      Dot dep_dot = vertex->deps[i];
      // ignore self or already executed (tarjan.rs:128-145)
      if (dep_dot == dot || executed_clock.contains(dep_dot.source, dep_dot.sequence)) continue;
      Vertex* dep_vertex = find(dep_dot);
      if (dep_vertex == nullptr) {
        missing_out = dep_dot;  // tarjan.rs:148-157
        return FinderResult::MissingDependencies;
      }
      if (dep_vertex->id == 0) {
        size_t dep_missing_deps_count = 0;
        FinderResult r = strong_connect(first_find, dep_dot, dep_vertex, scc_count,
                                        dep_missing_deps_count, missing_out);
        missing_deps_count += dep_missing_deps_count;
        if (r == FinderResult::MissingDependencies) return r;  // tarjan.rs:202-204
        vertex->low = std::min(vertex->low, dep_vertex->low);   // tarjan.rs:211
      } else if (dep_vertex->on_stack) {
        vertex->low = std::min(vertex->low, dep_vertex->id);    // tarjan.rs:217-221
      }
    }

    if (missing_deps_count == 0 && vertex->id == vertex->low) {  // tarjan.rs:233
      std::set<Dot> scc;
      while (true) {
        if (stack.empty()) throw std::logic_error("there should be an SCC member on the stack");
        Dot member = stack.back();
        stack.pop_back();
        Vertex* mv = find(member);
        if (mv == nullptr) throw std::logic_error("stack member should exist");
        scc_count += 1;
        mv->on_stack = false;
        if (!scc.insert(member).second) throw std::logic_error("duplicate SCC member");
        executed_clock.add(member.source, member.sequence);  // tarjan.rs:293
        if (member == dot) break;
      }
      sccs.push_back(std::move(scc));
      return FinderResult::Found;
    }
    return FinderResult::NotFound;
  }

  // mod.rs:488-523 — members in ascending Dot order (BTreeSet iteration).
  void save_scc(const std::set<Dot>& scc, std::vector<Dot>& dots, uint64_t time_ms) {
    chain_size[scc.size()] += 1;
    bool first = true;
    for (const Dot& d : scc) {
      auto it = vertex_index.find(d);
      if (it == vertex_index.end()) throw std::logic_error("dots from an SCC should exist");
      std::unique_ptr<Vertex> v = std::move(it->second);
      vertex_index.erase(it);
      dots.push_back(d);
      uint64_t duration = time_ms - v->start_time_ms;  // Vertex::into_command
      execution_delay[duration] += 1;
      to_execute.push_back(Executed{d, v->rec, first, duration});
      first = false;
    }
  }

  // mod.rs:525-554 + PendingIndex::index (index.rs:168-202); shard_count == 1
  // means every dep is "mine", so no out-requests.
  void index_pending(const Dot& dot, const std::set<Dot>& missing) {
    for (const Dot& dep : missing) pending_index[dep].insert(dot);
  }

  // mod.rs:556-587 — LIFO over the released dots.
  void check_pending(std::vector<Dot>& dots, size_t& total_scc_count, uint64_t time_ms) {
    while (!dots.empty()) {
      Dot d = dots.back();
      dots.pop_back();
      auto it = pending_index.find(d);  // PendingIndex::remove (index.rs:205-207)
      if (it != pending_index.end()) {
        std::set<Dot> pending = std::move(it->second);
        pending_index.erase(it);
        try_pending(pending, dots, total_scc_count, time_ms);
      }
    }
  }

  // mod.rs:589-642 — waiters in ascending Dot order (C2).
  void try_pending(const std::set<Dot>& pending, std::vector<Dot>& dots, size_t& total_scc_count,
                   uint64_t time_ms) {
    std::set<Dot> visited;
    for (const Dot& d : pending) {
      if (visited.count(d)) continue;
      std::vector<Dot> new_dots;
      std::set<Dot> new_visited;
      std::set<Dot> missing;
      FinderResult r = find_scc(false, d, total_scc_count, time_ms, new_dots, new_visited, missing);
      if (r == FinderResult::Found) {
        visited.clear();
        dots.insert(dots.end(), new_dots.begin(), new_dots.end());
      } else if (r == FinderResult::MissingDependencies) {
        index_pending(d, missing);
        if (!new_dots.empty()) {
          visited.clear();
        } else {
          visited.insert(new_visited.begin(), new_visited.end());
        }
        dots.insert(dots.end(), new_dots.begin(), new_dots.end());
      }
      // NotPending: nothing (mod.rs:635-638)
    }
  }
};

}  // namespace oracle

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
  std::set<Dot> visited, missing;
  oracle::FinderResult r;
  try {
    r = g->find_scc(first_find != 0, Dot{src, seq}, total, 0, dots, visited, missing);
  } catch (const std::exception&) {
    return 99;
  }
  uint32_t m = 0;
  for (const Dot& d : missing) {
    if (m < cap) { missing_src[m] = d.source; missing_seq[m] = d.sequence; }
    ++m;
  }
  *n_missing = m;
  *ready_commands = total;
  *n_dots = (uint32_t)dots.size();
  return r == oracle::FinderResult::Found ? 0 : r == oracle::FinderResult::MissingDependencies ? 1 : 2;
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
