// oracle/pred_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of Caesar's PredecessorsGraph
// (fantoch_ps/src/executor/pred/mod.rs:28-384, index.rs:10-120): the checker
// of the GPU predecessors executor (fantoch_amd/csrc/pred_exec.hip).  Nothing
// in the product links or calls this file.
//
// A command is committed with its Caesar clock (seq, process id), ordered
// lexicographically (common/pred/clocks/mod.rs:15-30), and its predecessor
// set.  Phase one waits until every dep is committed (committed clock);
// phase two until every dep with a LOWER clock is executed; then the command
// executes, which may complete other commands' phase two, recursively.
// Canonicalisation: the reference iterates the HashSet a PendingIndex::remove
// returns (index.rs:117-119) — here ascending by dot, as C2 does for the
// graph executor; the order of a vertex's deps only orders index insertions,
// which nothing observes.
#include <algorithm>
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../include/fantoch_amd.h"
#include "graph_oracle.hpp"

namespace predo {

using oracle::Dot;

struct Vertex {  // index.rs:10-63
  Dot dot;
  uint32_t rec = 0;
  uint64_t clock = 0;  // (seq << 8) | process id: lexicographic (seq, id)
  std::vector<Dot> deps;
  uint64_t start_ms = 0;
  size_t missing = 0;
};

struct Executed {
  uint32_t rec;
  uint32_t step;
};

class PredecessorsGraph {  // mod.rs:28-384
 public:
  PredecessorsGraph(uint32_t n) {
    for (uint32_t p = 1; p <= n; ++p) {
      committed.clock[p];
      executed.clock[p];
    }
  }
  bool execute_at_commit = false;
  std::vector<Executed> out;
  std::map<uint64_t, uint64_t> delay;  // ExecutionDelay
  uint32_t step = 0;
  uint64_t now = 0;

  // mod.rs:104-152; false on the double-index panic (mod.rs:284-289)
  bool add(const Dot& dot, uint32_t rec, uint64_t clock, std::vector<Dot> deps) {
    // assert!(self.committed_clock.add(..)) (mod.rs:123): a dot commits once
    if (!committed.add(dot.source, dot.sequence)) return false;
    if (execute_at_commit) {
      execute(dot, rec);
      return true;
    }
    auto v = std::make_unique<Vertex>();
    v->dot = dot;
    v->rec = rec;
    v->clock = clock;
    std::sort(deps.begin(), deps.end());
    deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
    v->deps = std::move(deps);
    v->start_ms = now;
    if (!index.emplace(dot, std::move(v)).second) return false;
    try_phase_one_pending(dot);
    move_to_phase_one(dot);
    return true;
  }

 private:
  oracle::AEClock committed, executed;
  std::map<Dot, std::unique_ptr<Vertex>> index;
  std::map<Dot, std::set<Dot>> phase_one, phase_two;  // PendingIndex (index.rs:96-120)

  Vertex& find(const Dot& d) {
    auto it = index.find(d);
    if (it == index.end()) throw std::logic_error("vertex must exist");
    return *it->second;
  }
  std::set<Dot> remove(std::map<Dot, std::set<Dot>>& idx, const Dot& d) {
    auto it = idx.find(d);
    if (it == idx.end()) return {};
    std::set<Dot> s = std::move(it->second);
    idx.erase(it);
    return s;
  }

  void move_to_phase_one(const Dot& dot) {  // mod.rs:154-206
    Vertex& v = find(dot);
    size_t missing = 0;
    for (const Dot& d : v.deps)
      if (!committed.contains(d.source, d.sequence)) {
        ++missing;
        phase_one[d].insert(dot);
      }
    if (missing) {
      v.missing = missing;
    } else {
      move_to_phase_two(dot);
    }
  }

  void move_to_phase_two(const Dot& dot) {  // mod.rs:208-275
    Vertex& v = find(dot);
    size_t missing = 0;
    for (const Dot& d : v.deps)
      if (!executed.contains(d.source, d.sequence)) {
        const Vertex& dep = find(d);  // "non-executed dependency must exist"
        if (dep.clock < v.clock) {
          ++missing;
          phase_two[d].insert(dot);
        }
      }
    if (missing) {
      v.missing = missing;
    } else {
      save_to_execute(dot);
    }
  }

  void try_phase_one_pending(const Dot& dot) {  // mod.rs:295-316
    for (const Dot& p : remove(phase_one, dot)) {
      Vertex& v = find(p);
      if (v.missing == 0) throw std::logic_error("missing deps underflow");
      if (--v.missing == 0) move_to_phase_two(p);
    }
  }

  void try_phase_two_pending(const Dot& dot) {  // mod.rs:318-339
    for (const Dot& p : remove(phase_two, dot)) {
      Vertex& v = find(p);
      if (v.missing == 0) throw std::logic_error("missing deps underflow");
      if (--v.missing == 0) save_to_execute(p);
    }
  }

  void save_to_execute(const Dot& dot) {  // mod.rs:341-367
    auto it = index.find(dot);
    if (it == index.end()) throw std::logic_error("ready-to-execute command should exist");
    std::unique_ptr<Vertex> v = std::move(it->second);
    index.erase(it);
    delay[now - v->start_ms] += 1;
    execute(dot, v->rec);
    try_phase_two_pending(dot);
  }

  void execute(const Dot& dot, uint32_t rec) {  // mod.rs:369-383
    executed.add(dot.source, dot.sequence);
    out.push_back({rec, step});
  }
};

}  // namespace predo

extern "C" {

// Runs S predecessor streams (tiled planes as fx_stream_batch, plus the
// packed clock planes and an optional deps-count plane) through the restatement.  Outputs as the GPU: order
// plane (arrival index | FX_ORDER_SCC_START: every command its own group),
// release plane, nexec, status.
int oracle_pred_batch(const uint32_t* dot, const uint32_t* hdr, const uint32_t* deps, const uint32_t* clo,
                      const uint32_t* chi, const uint32_t* ndeps, const uint32_t* lengths, uint32_t S, uint32_t steps, uint32_t dmax,
                      uint32_t n, uint32_t flags, uint32_t* order, uint32_t* release, uint32_t* nexec, uint32_t* err,
                      uint32_t threads) {
  const size_t pw = fx_plane_words(S, steps);
  auto run = [&](uint32_t s) {
    predo::PredecessorsGraph g(n);
    g.execute_at_commit = (flags & FX_FLAG_EXECUTE_AT_COMMIT) != 0;
    const uint32_t L = lengths ? std::min(lengths[s], steps) : steps;
    uint32_t status = 0;
    for (uint32_t i = 0; i < steps; ++i) release[fx_index(i, s, steps)] = FX_RELEASE_NONE;
    try {
      for (uint32_t i = 0; i < L; ++i) {
        const size_t at = fx_index(i, s, steps);
        const uint32_t d = dot[at], h = hdr[at];
        std::vector<oracle::Dot> dv;
        const uint32_t nd = ndeps ? ndeps[at] : FX_HDR_ND(h);
        for (uint32_t j = 0; j < nd && j < dmax; ++j) {
          const uint32_t x = deps[j * pw + at];
          dv.push_back(oracle::Dot{FX_DOT_SRC(x), FX_DOT_SEQ(x)});
        }
        g.step = i;
        g.now = FX_HDR_T(h);
        const uint64_t clock = ((uint64_t)chi[at] << 32) | clo[at];
        if (!g.add(oracle::Dot{FX_DOT_SRC(d), FX_DOT_SEQ(d)}, i, clock, dv)) {
          status = FX_ERR_DOUBLE_INDEX;
          break;
        }
      }
    } catch (const std::exception&) {
      status = 99;
    }
    for (size_t k = 0; k < g.out.size(); ++k) {
      order[fx_index((uint32_t)k, s, steps)] = g.out[k].rec | FX_ORDER_SCC_START;
      release[fx_index(g.out[k].rec, s, steps)] = g.out[k].step;
    }
    nexec[s] = (uint32_t)g.out.size();
    err[s] = status;
  };
  threads = std::max(1u, threads);
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (uint32_t s = t; s < S; s += threads) run(s);
    });
  for (auto& th : pool) th.join();
  return 0;
}

}  // extern "C"
