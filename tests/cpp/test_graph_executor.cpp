// C++ port of the reference's graph-executor unit tests
// (fantoch_ps/src/executor/graph/mod.rs:690-1348) against the C++ Executor
// mirror (include/fantoch_amd.hpp), i.e. through the C-ABI onto the GPU.
// Run by tests/test_gpu_cpp.py (needs a GPU).  Exit status 0 = all passed.
#include <algorithm>
#include <cstdio>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "fantoch_amd.hpp"

using namespace fantoch_amd;

static int g_failures = 0;
#define EXPECT(cond, msg)                                             \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
      ++g_failures;                                                   \
    }                                                                 \
  } while (0)

struct Arg {
  Dot dot;
  std::vector<Key> keys;  // empty -> the single CONF key
  std::set<Dot> deps;
};

using Sorted = std::map<Key, std::vector<Rifl>>;

static constexpr Key CONF = 100;

// check_termination (mod.rs:1045-1113)
static Sorted check_termination(uint32_t n, const std::vector<Arg>& args) {
  Config config(n, 1);
  GraphExecutor queue(1, 0, config);
  std::set<Rifl> all_rifls;
  Sorted sorted;
  uint64_t t = 0;
  for (const auto& a : args) {
    std::vector<Dependency> deps;
    for (const auto& d : a.deps) deps.push_back(Dependency{d});
    Rifl rifl(a.dot.source, a.dot.sequence);  // Rifl::new(dot.source() as ClientId, dot.sequence())
    std::vector<Key> keys = a.keys.empty() ? std::vector<Key>{CONF} : a.keys;
    Command cmd = Command::from(rifl, keys);
    EXPECT(all_rifls.insert(rifl).second, "rifl inserted twice");
    queue.handle(GraphExecutionInfo::add(a.dot, cmd, deps), t++);
    for (const auto& r : queue.to_clients_iter()) {
      all_rifls.erase(r.rifl);
      sorted[r.key].push_back(r.rifl);
    }
  }
  EXPECT(all_rifls.empty(), "the set of all rifls should be empty");
  return sorted;
}

static void shuffle_it(uint32_t n, std::vector<Arg> args) {
  const Sorted total = check_termination(n, args);
  std::vector<size_t> idx(args.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  do {
    std::vector<Arg> perm;
    for (size_t i : idx) perm.push_back(args[i]);
    EXPECT(check_termination(n, perm) == total, "per-key order differs across permutations");
  } while (std::next_permutation(idx.begin(), idx.end()));
}

// simple (mod.rs:714-752)
static void test_simple() {
  Config config(2, 1);
  GraphExecutor queue(1, 0, config);
  Dot dot_0(1, 1), dot_1(2, 1);
  Command cmd_0 = Command::from(Rifl(1, 1), {0});
  Command cmd_1 = Command::from(Rifl(2, 1), {0});
  queue.handle(GraphExecutionInfo::add(dot_0, cmd_0, {Dependency{dot_1}}), 0);
  EXPECT(queue.drain_dots().empty(), "nothing ready after cmd 0");
  queue.handle(GraphExecutionInfo::add(dot_1, cmd_1, {Dependency{dot_0}}), 0);
  auto ready = queue.drain_dots();
  EXPECT(ready.size() == 2 && ready[0].first == dot_0 && ready[1].first == dot_1,
         "expected [cmd_0, cmd_1]");
  EXPECT(ready.size() == 2 && ready[0].second && !ready[1].second, "one SCC of 2");
}

// cycle (mod.rs:896-917)
static void test_cycle() {
  Dot d1(1, 1), d2(2, 1), d3(3, 1);
  shuffle_it(3, {{d1, {}, {d3}}, {d2, {}, {d1}}, {d3, {}, {d2}}});
}

// random_adds (mod.rs:932-1031) with a seeded generator
static std::vector<Arg> random_adds(std::mt19937_64& rng, uint32_t n, uint32_t events) {
  std::vector<Dot> dots;
  for (uint32_t p = 1; p <= n; ++p)
    for (uint32_t e = 1; e <= events; ++e) dots.emplace_back((ProcessId)p, e);
  std::map<Dot, std::pair<std::vector<Key>, std::set<Dot>>> data;
  std::vector<Key> possible = {0, 1, 2, 3};  // 'A'..='D'
  for (const auto& d : dots) {
    std::shuffle(possible.begin(), possible.end(), rng);
    std::vector<Key> ks = {possible[0], possible[1]};
    std::sort(ks.begin(), ks.end());
    data[d] = {ks, {}};
  }
  for (size_t a = 0; a < dots.size(); ++a)
    for (size_t b = a + 1; b < dots.size(); ++b) {
      const Dot left = dots[a], right = dots[b];
      auto& L = data[left];
      auto& R = data[right];
      bool conflict = false;
      for (Key k : L.first)
        if (std::find(R.first.begin(), R.first.end(), k) != R.first.end()) conflict = true;
      if (!conflict) continue;
      if (left.source == right.source) {
        if (left.sequence < right.sequence) R.second.insert(left);
        else L.second.insert(right);
      } else {
        switch (rng() % 3) {
          case 0: L.second.insert(right); break;
          case 1: R.second.insert(left); break;
          default:
            L.second.insert(right);
            R.second.insert(left);
        }
      }
    }
  std::vector<Arg> args;
  for (const auto& kv : data) args.push_back(Arg{kv.first, kv.second.first, kv.second.second});
  return args;
}

// test_add_random (mod.rs:919-930)
static void test_add_random() {
  std::mt19937_64 rng(20250213);
  for (int it = 0; it < 10; ++it) shuffle_it(2, random_adds(rng, 2, 3));
}

// transitive_conflicts_assumption_regression_test_1 (mod.rs:788-824)
static void test_regression_1() {
  Dot d1(1, 1), d2(1, 2), d3(1, 3), d4(1, 4), d5(1, 5);
  auto a = check_termination(5, {{d3, {}, {d5}}, {d4, {}, {d3}}, {d5, {}, {d4}}, {d1, {}, {d4}}, {d2, {}, {d4}}});
  auto b = check_termination(5, {{d3, {}, {d5}}, {d4, {}, {d3}}, {d5, {}, {d4}}, {d2, {}, {d4}}, {d1, {}, {d4}}});
  EXPECT(a != b, "regression 1 orders must differ");
}

// transitive_conflicts_assumption_regression_test_2 (mod.rs:855-894)
static void test_regression_2() {
  Dot d11(1, 1), d12(1, 2), d21(2, 1);
  const Key A = 0, B = 1;
  auto a = check_termination(3, {{d11, {A}, {}}, {d12, {B}, {}}, {d21, {A, B}, {d12}}});
  auto b = check_termination(3, {{d12, {B}, {}}, {d21, {A, B}, {d12}}, {d11, {A}, {}}});
  EXPECT(a != b, "regression 2 orders must differ");
}

// sccs_found_and_missing_dep (mod.rs:1115-1348)
static void test_sccs_found_and_missing_dep() {
  Config config(5, 1);
  GraphExecutor queue(4, 0, config);
  const uint64_t frontier[5] = {60, 50, 50, 30, 60};
  check(fx_graph_executor_set_executed_frontier(queue.raw(), frontier, 5));
  const Key conf = 0;
  auto index_only = [&](Dot d, std::vector<Dot> deps) {
    std::vector<fx_dot> dv;
    for (auto& x : deps) dv.push_back(fx_dot{x.source, (uint32_t)x.sequence});
    check(fx_graph_executor_index_only(queue.raw(), fx_dot{d.source, (uint32_t)d.sequence}, fx_rifl{1, 1},
                                       &conf, 1, dv.data(), (uint32_t)dv.size(), 0));
  };
  for (uint64_t s = 31; s <= 40; ++s)
    index_only(Dot(4, s), {Dot(1, 60), Dot(2, 50), Dot(3, 50), Dot(4, s - 1), Dot(5, 60)});
  // find_scc(first_find = true, (5, 70)) through handle_add
  queue.handle(GraphExecutionInfo::add(Dot(5, 70), Command::from(Rifl(1, 1), {conf}),
                                       {{Dot(1, 60)}, {Dot(2, 50)}, {Dot(3, 50)}, {Dot(4, 40)}, {Dot(5, 61)}}),
               0);
  auto ready = queue.drain_dots();
  EXPECT(ready.size() == 10, "ready_commands == to_be_executed.len() == 10");
  for (size_t i = 0; i < ready.size() && i < 10; ++i)
    EXPECT(ready[i].first == Dot(4, 31 + i) && ready[i].second, "(4,31)..(4,40) as singleton SCCs");
  fx_dot pd[8], pw[8];
  uint32_t np = 0;
  check(fx_graph_executor_pending(queue.raw(), pd, pw, 8, &np));
  EXPECT(np == 1 && pd[0].source == 5 && pd[0].seq == 70, "(5,70) still pending");
  EXPECT(np == 1 && pw[0].source == 5 && pw[0].seq == 61, "single missing dependency (5,61)");
}

// execution log of the `simple` KAT, bincode-1 frames as execution_logger.rs writes
// them, replayed like graph_executor_replay (graph_executor_replay.rs:13-38)
static void put_u32be(std::vector<uint8_t>& b, uint32_t v) {
  for (int i = 3; i >= 0; --i) b.push_back((uint8_t)(v >> (8 * i)));
}
static void put_le(std::vector<uint8_t>& b, uint64_t v, int bytes) {
  for (int i = 0; i < bytes; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
static void put_str(std::vector<uint8_t>& b, const std::string& s) {
  put_le(b, s.size(), 8);
  b.insert(b.end(), s.begin(), s.end());
}
static std::vector<uint8_t> add_frame(Dot dot, Rifl rifl, const std::string& key, Dot dep) {
  std::vector<uint8_t> p;
  put_le(p, 0, 4);  // Add
  put_le(p, dot.source, 1);
  put_le(p, dot.sequence, 8);
  put_le(p, rifl.source, 8);
  put_le(p, rifl.sequence, 8);
  put_le(p, 1, 8);  // shard_to_ops: {0: {key: [Put("v")]}}
  put_le(p, 0, 8);
  put_le(p, 1, 8);
  put_str(p, key);
  put_le(p, 1, 8);
  put_le(p, 1, 4);
  put_str(p, "v");
  put_le(p, 1, 8);  // shard_to_keys: {0: [key]}
  put_le(p, 0, 8);
  put_le(p, 1, 8);
  put_str(p, key);
  put_le(p, 0, 8);  // _empty_keys
  put_le(p, 1, 8);  // deps: {Dependency{dep, None}}
  put_le(p, dep.source, 1);
  put_le(p, dep.sequence, 8);
  put_le(p, 0, 1);
  std::vector<uint8_t> f;
  put_u32be(f, (uint32_t)p.size());
  f.insert(f.end(), p.begin(), p.end());
  return f;
}

static void test_execution_log_replay() {
  std::vector<uint8_t> log = add_frame(Dot(1, 1), Rifl(1, 1), "A", Dot(2, 1));
  auto f2 = add_frame(Dot(2, 1), Rifl(2, 1), "A", Dot(1, 1));
  log.insert(log.end(), f2.begin(), f2.end());
  auto infos = read_execution_log(log);
  EXPECT(infos.size() == 2 && infos[1].dot == Dot(2, 1) && infos[1].deps.size() == 1 &&
             infos[1].deps[0].dot == Dot(1, 1) && !infos[1].cmd.read_only,
         "decoded log fields");
  Config config(2, 1);
  GraphExecutor queue(1, 0, config);
  replay_execution_log(queue, log);
  auto ready = queue.drain_dots();
  EXPECT(ready.size() == 2 && ready[0].first == Dot(1, 1) && ready[1].first == Dot(2, 1),
         "replayed log executes [cmd_0, cmd_1]");
  log.pop_back();
  bool threw = false;
  try {
    read_execution_log(log);
  } catch (const Error& e) {
    threw = e.status == FX_ERR_LOG_FORMAT;
  }
  EXPECT(threw, "truncated log is rejected");
}

int main() {
  if (fx_device_count() <= 0) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  test_simple();
  test_cycle();
  test_add_random();
  test_regression_1();
  test_regression_2();
  test_sccs_found_and_missing_dep();
  test_execution_log_replay();
  if (g_failures) {
    std::fprintf(stderr, "%d failure(s)\n", g_failures);
    return 1;
  }
  std::printf("all graph executor tests passed\n");
  return 0;
}
