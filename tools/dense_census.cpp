// tools/dense_census.cpp — work census of the reference executor on the dense
// synthetic streams of `bench.py --mode dense` (BASELINE configs[3] shape:
// n = 5, 64 clients per process, 100 % conflicts, 30 % cycles, window 320):
// searches, DFS recursions and edges per Add, split into the first search of
// an Add and the try_pending retries.  Measurement only (runs the oracle).
// build: g++ -O2 -std=c++17 -Iinclude -Ifantoch_amd/csrc -o /tmp/dense_census tools/dense_census.cpp
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <vector>

struct Census {
  uint64_t rec[2] = {0, 0}, edges[2] = {0, 0}, srch[2] = {0, 0}, found[2] = {0, 0}, miss[2] = {0, 0};
  uint64_t saved_then_miss = 0, skips = 0, scc_members = 0, stack_left = 0;
  void recursion(bool f) { rec[f]++; }
  void edge(bool f) { edges[f]++; }
  // search-result cache (sim_big.hip x_add_): root -> (missing dot, executions at the search)
  std::map<std::pair<uint32_t, uint64_t>, std::pair<std::pair<uint32_t, uint64_t>, uint64_t>> cache;
  uint64_t execs = 0, hits = 0, hit_ok = 0;
  bool predicted = false;
  std::pair<uint32_t, uint64_t> pred_m;
  // refined rule: the walk's vertices (the stack at the failure) all still pending
  std::map<std::pair<uint32_t, uint64_t>, std::pair<std::pair<uint32_t, uint64_t>, std::vector<std::pair<uint32_t, uint64_t>>>> rcache;
  uint64_t rhits = 0, rhit_ok = 0;
  bool rpredicted = false;
  std::pair<uint32_t, uint64_t> rpred_m;
  template <class D>
  void search(bool f, int fr, size_t scc, const std::vector<D>& stack, const D& root, const D& m) {
    const size_t stk = stack.size();
    if (f && rpredicted) {
      if (fr == 1 && scc == 0 && m.source == rpred_m.first && m.sequence == rpred_m.second) rhit_ok++;
      rpredicted = false;
    }
    if (fr == 1 && scc == 0) {
      auto& e = rcache[{root.source, root.sequence}];
      e.first = {m.source, m.sequence};
      e.second.clear();
      for (auto& x : stack) e.second.push_back({x.source, x.sequence});
    }
    if (f && predicted) {
      if (fr == 1 && scc == 0 && m.source == pred_m.first && m.sequence == pred_m.second) hit_ok++;
      predicted = false;
    }
    execs += scc;
    if (fr == 1 && scc == 0) cache[{root.source, root.sequence}] = {{m.source, m.sequence}, execs};
    srch[f]++;
    if (fr == 0) found[f]++;
    if (fr == 1) { miss[f]++; if (scc) saved_then_miss++; }
    scc_members += scc;
    stack_left += stk;
  }
  void skip() { skips++; }
};
static Census C;
#define ORACLE_CENSUS(x) C.x
#include "../oracle/graph_oracle.hpp"
#include "fx_synth.h"

int main(int argc, char** argv) {
  const uint32_t inst = argc > 1 ? atoi(argv[1]) : 1;
  const uint32_t cmds_per_client = argc > 2 ? atoi(argv[2]) : 20;
  fx_synth_params p{};
  p.seed = 1;
  p.instances = inst;
  p.n = 5;
  p.clients = 64;
  p.cmds_per_process = 64 * cmds_per_client;
  p.window = 5 * 64;
  p.cycle_pct = 30;
  p.horizon = 64;
  p.num_conflicts = 1;
  p.conflict_pct[0] = 100;
  const uint32_t n = p.n, N = n * p.cmds_per_process;
  uint64_t adds = 0, maxpend = 0, sumpend = 0, maxspread = 0, coll256 = 0, coll512 = 0;
  for (uint32_t i = 0; i < inst; ++i) {
    const fx::SynthInstance si = fx::synth_instance(p, i);
    for (uint32_t proc = 1; proc <= n; ++proc) {
      std::vector<std::pair<uint32_t, uint32_t>> ordr;
      for (uint32_t g = 0; g < N; ++g) ordr.push_back({fx::synth_arrival(si, proc, g), g});
      std::sort(ordr.begin(), ordr.end());
      oracle::DependencyGraph gr(proc, n);
      uint32_t r = 0;
      for (auto& [a, g] : ordr) {
        uint32_t dv[32];
        const uint32_t nd = fx::synth_deps(si, g, dv);
        std::vector<oracle::Dot> deps;
        for (uint32_t j = 0; j < nd; ++j) deps.push_back(oracle::Dot{dv[j] >> 24, dv[j] & 0xFFFFFFu});
        const oracle::Dot v{g % n + 1, g / n + 1};
        // cache rule: first dep u neither v nor executed; u pending with a cached
        // miss m stored at the current execution count; m still missing, m != v
        for (auto& u : deps) {
          if (u == v || gr.executed_clock.contains(u.source, u.sequence)) continue;
          if (gr.find(u)) {
            auto it = C.cache.find({u.source, u.sequence});
            auto rt = C.rcache.find({u.source, u.sequence});
            if (rt != C.rcache.end()) {
              const oracle::Dot m{rt->second.first.first, rt->second.first.second};
              bool ok = !(m == v) && !gr.find(m) && !gr.executed_clock.contains(m.source, m.sequence);
              for (auto& x : rt->second.second) ok = ok && gr.find(oracle::Dot{x.first, x.second}) != nullptr;
              if (ok) {
                C.rhits++;
                C.rpredicted = true;
                C.rpred_m = rt->second.first;
              }
            }
            if (it != C.cache.end() && it->second.second == C.execs) {
              const oracle::Dot m{it->second.first.first, it->second.first.second};
              if (!(m == v) && !gr.find(m) && !gr.executed_clock.contains(m.source, m.sequence)) {
                C.hits++;
                C.predicted = true;
                C.pred_m = it->second.first;
              }
            }
          }
          break;
        }
        gr.handle_add(v, r++, deps, a);
        gr.to_execute.clear();
        ++adds;
        sumpend += gr.vertex_index.size();
        {  // index-slot collisions at Q = 256 / 512 and the per-source seq spread of the pending set
          std::map<uint32_t, std::pair<uint64_t, uint64_t>> mm;
          std::set<std::pair<uint32_t, uint64_t>> s256, s512;
          bool c256 = false, c512 = false;
          for (auto& kv : gr.vertex_index) {
            auto& e = mm.emplace(kv.first.source, std::make_pair(kv.first.sequence, kv.first.sequence)).first->second;
            e.first = std::min(e.first, kv.first.sequence);
            e.second = std::max(e.second, kv.first.sequence);
            c256 |= !s256.insert({kv.first.source, kv.first.sequence % 256}).second;
            c512 |= !s512.insert({kv.first.source, kv.first.sequence % 512}).second;
          }
          for (auto& kv : mm) maxspread = std::max<uint64_t>(maxspread, kv.second.second - kv.second.first + 1);
          coll256 += c256;
          coll512 += c512;
        }
        maxpend = std::max<uint64_t>(maxpend, gr.vertex_index.size());
      }
    }
  }
  const double A = (double)adds;
  printf("adds %llu  pending avg %.1f max %llu\n", (unsigned long long)adds, sumpend / A, (unsigned long long)maxpend);
  const char* nm[2] = {"try  ", "first"};
  for (int f = 1; f >= 0; --f)
    printf("%s searches/Add %.2f (found %.2f missing %.2f)  recursions/Add %.1f  edges/Add %.1f\n", nm[f],
           C.srch[f] / A, C.found[f] / A, C.miss[f] / A, C.rec[f] / A, C.edges[f] / A);
  printf("saved-then-missing %.3f/Add  skips %.2f/Add  SCC members %.2f/Add  stack left on miss %.1f/search\n",
         C.saved_then_miss / A, C.skips / A, C.scc_members / A,
         (double)C.stack_left / (double)(C.miss[0] + C.miss[1] + 1));
  printf("max per-source pending seq spread %llu; Adds with an index collision at Q=256: %llu, Q=512: %llu\n",
         (unsigned long long)maxspread, (unsigned long long)coll256, (unsigned long long)coll512);
  printf("refined cache hits %.3f/Add, prediction held %llu of %llu\n", C.rhits / A, (unsigned long long)C.rhit_ok,
         (unsigned long long)C.rhits);
  printf("cache hits %.3f/Add, prediction held %llu of %llu\n", C.hits / A, (unsigned long long)C.hit_ok,
         (unsigned long long)C.hits);
  return 0;
}
