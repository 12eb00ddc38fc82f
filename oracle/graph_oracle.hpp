// oracle/graph_oracle.hpp — TEST INFRASTRUCTURE ONLY.
//
// The CPU restatement of fantoch_ps's DependencyGraph (see graph_oracle.cpp
// for the reference map), shared by the plane-layout batch oracle
// (graph_oracle.cpp) and the simulator oracle (sim_oracle.cpp).
#pragma once
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


// census hooks for tools/dense_census.cpp (no-ops in every other build)
#ifndef ORACLE_CENSUS
#define ORACLE_CENSUS(x)
#endif

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
  std::vector<uint32_t> dep_shards;  // Dependency::shards as a bitmask (0 = None, a noop)
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
  // partial replication (mod.rs:82-122, shard_count > 1): this executor's
  // shard, the number of shards, n processes per shard (ids 1..=n * shards)
  uint32_t shard_id = 0, shard_count = 1, n_shard = 0;
  std::set<std::pair<Dot, uint32_t>> missing_deps;  // TarjanSCCFinder::missing_deps (dep, shards)
  std::map<uint32_t, std::set<Dot>> out_requests;    // mod.rs:61 out_requests (target shard -> dots)
  std::set<Dot> added_to_executed_clock;             // mod.rs:63 (drained by to_executors)
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

  DependencyGraph(uint32_t pid, uint32_t n_) : process_id(pid), n(n_), n_shard(n_) {
    // AEClock::with(all process ids) — mod.rs:90-94
    for (uint32_t p = 1; p <= n; ++p) executed_clock.clock[p];
  }
  // Config::set_shard_count + DependencyGraph::new(process_id, shard_id, ..):
  // the executed clock spans util::all_process_ids(shard_count, n) (util.rs:135-143)
  DependencyGraph(uint32_t pid, uint32_t n_, uint32_t shard, uint32_t shards)
      : process_id(pid), n(n_ * shards), shard_id(shard), shard_count(shards), n_shard(n_) {
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
    std::vector<uint32_t> shards(deps.size(), 1u << shard_id);
    return handle_add_sharded(dot, rec, std::move(deps), std::move(shards), time_ms);
  }
  // deps with their Dependency::shards masks (partial replication)
  bool handle_add_sharded(const Dot& dot, uint32_t rec, std::vector<Dot> deps, std::vector<uint32_t> shards,
                          uint64_t time_ms) {
    auto v = std::make_unique<Vertex>();
    v->dot = dot;
    v->rec = rec;
    std::vector<std::pair<Dot, uint32_t>> ds;
    for (size_t i = 0; i < deps.size(); ++i) ds.push_back({deps[i], shards[i]});
    std::sort(ds.begin(), ds.end());  // C1
    ds.erase(std::unique(ds.begin(), ds.end(),
                         [](const std::pair<Dot, uint32_t>& a, const std::pair<Dot, uint32_t>& b) {
                           return a.first == b.first;
                         }),
             ds.end());
    for (auto& d : ds) {
      v->deps.push_back(d.first);
      v->dep_shards.push_back(d.second);
    }
    v->start_time_ms = time_ms;
    if (!index(std::move(v))) return false;

    size_t initial_ready = to_execute.size();
    size_t total_scc_count = 0;
    std::vector<Dot> dots;
    std::set<Dot> visited;
    std::set<std::pair<Dot, uint32_t>> missing;
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
                        std::vector<Dot>& dots, std::set<Dot>& visited,
                        std::set<std::pair<Dot, uint32_t>>& missing) {
    size_t scc_count = 0;
    size_t missing_deps_count = 0;
    std::pair<Dot, uint32_t> result_missing;
    FinderResult fr;
    Vertex* v = find(dot);
    if (v == nullptr) {
      fr = FinderResult::NotPending;  // mod.rs:664-667
    } else {
      fr = strong_connect(first_find, dot, v, scc_count, missing_deps_count, result_missing);
    }
    ORACLE_CENSUS(search(first_find, (int)fr, scc_count, stack, dot, result_missing.first));
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
    std::set<std::pair<Dot, uint32_t>> collected;
    collected.swap(missing_deps);  // finalize returns the collected missing deps (tarjan.rs:91-92)
    if (collected.size() > missing_deps_count) throw std::logic_error("more missing deps than the ones counted");
    switch (fr) {
      case FinderResult::Found:
        return FinderResult::Found;
      case FinderResult::MissingDependencies:
        if (!collected.empty())  // mod.rs:468-471
          throw std::logic_error("if MissingDependencies is returned, missing_deps must be empty");
        missing.insert(result_missing);
        return FinderResult::MissingDependencies;
      case FinderResult::NotPending:
        return FinderResult::NotPending;
      case FinderResult::NotFound:
      default:
        // partial replication, first search: every missing dep collected (mod.rs:478-484)
        if (collected.empty())
          throw std::logic_error("either there's a missing dependency, or we should find an SCC");
        missing = std::move(collected);
        return FinderResult::MissingDependencies;
    }
  }

  // tarjan.rs:96-316: shard_count == 1 or a retry gives up on the first
  // missing dep; the first search with partial replication collects every
  // missing dep and keeps going (tarjan.rs:148-166).
  FinderResult strong_connect(bool first_find, const Dot& dot, Vertex* vertex, size_t& scc_count,
                              size_t& missing_deps_count, std::pair<Dot, uint32_t>& missing_out) {
    ORACLE_CENSUS(recursion(first_find));
    finder_id += 1;
    vertex->id = finder_id;
    vertex->low = finder_id;
    vertex->on_stack = true;
    stack.push_back(dot);

    for (size_t i = 0; i < vertex->deps.size(); ++i) {
      Dot dep_dot = vertex->deps[i];
      ORACLE_CENSUS(edge(first_find));
      // ignore self or already executed (tarjan.rs:128-145)
      if (dep_dot == dot || executed_clock.contains(dep_dot.source, dep_dot.sequence)) continue;
      Vertex* dep_vertex = find(dep_dot);
      if (dep_vertex == nullptr) {
        // vertices indexed without shards (test hook) replicate on this shard
        const uint32_t sh = i < vertex->dep_shards.size() ? vertex->dep_shards[i] : 1u << shard_id;
        if (shard_count == 1 || !first_find) {
          missing_out = {dep_dot, sh};  // tarjan.rs:148-157
          return FinderResult::MissingDependencies;
        }
        missing_deps.insert({dep_dot, sh});  // tarjan.rs:158-166
        missing_deps_count += 1;
        continue;
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
        if (shard_count > 1) added_to_executed_clock.insert(member);  // tarjan.rs:294-296
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

  // mod.rs:525-554 + PendingIndex::index (index.rs:168-202): the first time a
  // dep is missing, a dep this shard does not replicate is requested from
  // its target shard (Dot::target_shard, id.rs:59-61); with shard_count == 1
  // every dep is "mine", so no out-requests.
  void index_pending(const Dot& dot, const std::set<std::pair<Dot, uint32_t>>& missing) {
    for (const auto& dep : missing) {
      auto it = pending_index.find(dep.first);
      if (it == pending_index.end()) {
        pending_index[dep.first].insert(dot);
        if (dep.second == 0) throw std::logic_error("shards should be set if it's not a noop");
        const bool is_mine = (dep.second >> shard_id) & 1u;
        if (!is_mine) out_requests[(dep.first.source - 1) / n_shard].insert(dep.first);
      } else {
        it->second.insert(dot);
      }
    }
  }

  // RequestReply::Executed (mod.rs:394-402): the requested dot was executed
  // at its shard
  void handle_executed_reply(const Dot& dot, uint64_t time_ms) {
    executed_clock.add(dot.source, dot.sequence);
    added_to_executed_clock.insert(dot);
    std::vector<Dot> dots{dot};
    size_t total_scc_count = 0;
    check_pending(dots, total_scc_count, time_ms);
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
      if (visited.count(d)) { ORACLE_CENSUS(skip()); continue; }
      std::vector<Dot> new_dots;
      std::set<Dot> new_visited;
      std::set<std::pair<Dot, uint32_t>> missing;
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

// An executor with index > 0 of the same process (partial replication, run
// mode): it clones the DependencyGraph but shares its VertexIndex (index.rs:21,
// an Arc), keeps its own executed clock fed by GraphExecutionInfo::Executed
// (handle_executed, mod.rs:211-223) and serves Requests from other shards
// (handle_request / process_requests, mod.rs:277-355; cleanup retries the
// buffered ones, mod.rs:183-195, 669-675).
struct RequestReply {
  uint32_t to_shard;
  bool info;  // Info{dot, cmd, deps} or Executed{dot}
  Dot dot;
  uint32_t rec;  // the vertex's arrival index (stands in for `cmd`)
  std::vector<Dot> deps;
  std::vector<uint32_t> dep_shards;
};

struct ExecutorClone {
  DependencyGraph* main;
  AEClock executed_clock;
  std::map<uint32_t, std::set<Dot>> buffered_in_requests;
  std::vector<RequestReply> out_request_replies;

  void handle_executed(const std::vector<Dot>& dots) {
    for (const Dot& d : dots) executed_clock.add(d.source, d.sequence);
  }
  void process_requests(uint32_t from, const std::set<Dot>& dots) {
    for (const Dot& dot : dots) {  // a HashSet in the reference; ascending here
      Vertex* v = main->find(dot);
      if (v != nullptr) {
        RequestReply r{from, true, dot, v->rec, v->deps, v->dep_shards};
        if (r.dep_shards.size() < r.deps.size()) r.dep_shards.resize(r.deps.size(), 1u << main->shard_id);
        out_request_replies.push_back(std::move(r));
      } else if (executed_clock.contains(dot.source, dot.sequence)) {
        out_request_replies.push_back(RequestReply{from, false, dot, 0, {}, {}});
      } else {
        buffered_in_requests[from].insert(dot);
      }
    }
  }
  void handle_request(uint32_t from, const std::set<Dot>& dots) { process_requests(from, dots); }
  void cleanup() {  // check_pending_requests
    std::map<uint32_t, std::set<Dot>> buffered;
    buffered.swap(buffered_in_requests);
    for (auto& kv : buffered) process_requests(kv.first, kv.second);
  }
};

}  // namespace oracle

