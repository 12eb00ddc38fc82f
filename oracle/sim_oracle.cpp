// oracle/sim_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's discrete-event simulator driving the
// leaderless protocols whose executor is the hot path: the CHECKER of the GPU
// simulator (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg).
// Nothing in the product links or calls this file.
//
// It follows the reference's structure one to one (recursive self-delivery,
// LIFO action vectors, a priority queue on time), not the GPU design:
//   Planet / Dat ................. fantoch/src/planet/mod.rs:38-140, dat.rs:20-94
//   sort_processes_by_distance ... fantoch/src/util.rs:153-201
//   BaseProcess::discover ........ fantoch/src/protocol/base.rs:62-154
//   Schedule ..................... fantoch/src/sim/schedule.rs:6-61
//   Simulation ................... fantoch/src/sim/simulation.rs:10-188
//   Runner ....................... fantoch/src/sim/runner.rs:64-634
//   Client / Workload / KeyGen ... fantoch/src/client/{mod.rs:27-158, workload.rs:112-211,
//                                  key_gen.rs:85-128, pending.rs:7-51}
//   AggregatePending ............. fantoch/src/executor/aggregate.rs:9-88
//   Basic ........................ fantoch/src/protocol/basic.rs:29-335 + BasicExecutor
//                                  (fantoch/src/executor/basic.rs:19-65)
//   Atlas ........................ fantoch_ps/src/protocol/atlas.rs:39-475, 641-714
//   EPaxos ....................... fantoch_ps/src/protocol/epaxos.rs:36-597
//   SequentialKeyDeps ............ fantoch_ps/src/protocol/common/graph/deps/keys/sequential.rs:26-118,
//                                  keys/mod.rs:44-75
//   QuorumDeps ................... fantoch_ps/src/protocol/common/graph/deps/quorum.rs:16-103
//   Synod (single decree) ........ fantoch_ps/src/protocol/common/synod/single.rs:30-447
//   VClockGCTrack ................ fantoch/src/protocol/gc/clock.rs:21-138
//   SequentialCommandsInfo ....... fantoch/src/protocol/info/sequential.rs:17-79
//   GraphExecutor ................ fantoch_ps/src/executor/graph/executor.rs:69-188 over the
//                                  DependencyGraph restatement (graph_oracle.hpp)
//
// Canonicalisation, replacing the reference's
// unordered iteration and unseeded randomness:
//   C1/C2  inside the DependencyGraph (graph_oracle.hpp)
//   C3     Schedule ties (the BinaryHeap compares time only): protocol and client
//          actions first, FIFO by insertion; then the GC traffic (periodic GC events
//          by process id, then MGarbageCollection deliveries by (from, to))
//   C4     a message's targets are visited in ascending process id (HashSet order)
//   C5     clients start in ascending client id (HashMap order)
//   C6     every draw of rand::thread_rng is a counter-based hash of
//          (seed, instance, client, command index, draw, purpose); gen_range(0..100)
//          is `u mod 100`, gen_range(0.0..10.0) is `10 * (u >> 11) / 2^53`
//   C7     keys are u32 ids: "CONFLICT{r}" -> r, the client's own key -> pool_size + client id
//   C8     to_processes / to_executors are popped LIFO (Vec::pop), as in the reference
//   C11    a command's keys are visited in ascending id
//   C12    region r = index of the region in name order (Region derives Ord on the name)

#include <dirent.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../include/fantoch_amd.h"
#include "graph_oracle.hpp"

namespace simo {

using oracle::Dot;

// --------------------------------------------------------------- Planet
// planet/mod.rs:38-140 + dat.rs:20-94: one `<region>.dat` per region, lines
// `min/avg/max/mdev:<to-region>`; latency = avg floored to u64 (dat.rs:62-66),
// intra-region latency 0 (mod.rs:19, dat.rs:46-50); sorted = (latency, region)
// ascending (mod.rs:122-140).
struct Planet {
  std::vector<std::string> names;               // ascending by name
  std::vector<std::vector<int64_t>> lat;        // ping ms, -1 = unknown
  std::vector<std::vector<uint32_t>> sorted;    // per region: regions by (lat, name)

  int index(const std::string& name) const {
    auto it = std::lower_bound(names.begin(), names.end(), name);
    return it != names.end() && *it == name ? (int)(it - names.begin()) : -1;
  }

  bool load(const std::string& dir) {
    DIR* d = opendir(dir.c_str());
    if (!d) return false;
    std::vector<std::string> files;
    while (dirent* e = readdir(d)) {
      std::string f = e->d_name;
      if (f.size() > 4 && f.compare(f.size() - 4, 4, ".dat") == 0) files.push_back(f);
    }
    closedir(d);
    for (auto& f : files) names.push_back(f.substr(0, f.size() - 4));  // Dat::region
    std::sort(names.begin(), names.end());
    const size_t R = names.size();
    lat.assign(R, std::vector<int64_t>(R, -1));
    for (size_t a = 0; a < R; ++a) {
      std::ifstream in(dir + "/" + names[a] + ".dat");
      std::string line;
      while (std::getline(in, line)) {
        if (line.empty()) continue;
        // Dat::latency: split on '/' or ':'; the 2nd entry is the average,
        // the last entry the region
        std::vector<std::string> parts;
        std::string cur;
        for (char c : line) {
          if (c == '/' || c == ':') {
            parts.push_back(cur);
            cur.clear();
          } else {
            cur.push_back(c);
          }
        }
        parts.push_back(cur);
        if (parts.size() < 3) return false;
        const double avg = std::strtod(parts[1].c_str(), nullptr);
        int b = index(parts.back());
        if (b < 0) return false;
        lat[a][b] = (size_t)b == a ? 0 : (int64_t)avg;  // `as u64` truncates
      }
    }
    sorted.assign(R, {});
    for (size_t a = 0; a < R; ++a) {
      std::vector<std::pair<int64_t, uint32_t>> v;
      for (size_t b = 0; b < R; ++b)
        if (lat[a][b] >= 0) v.push_back({lat[a][b], (uint32_t)b});  // b ascending = name order
      std::sort(v.begin(), v.end());
      for (auto& x : v) sorted[a].push_back(x.second);
    }
    return true;
  }

  uint64_t ping(uint32_t a, uint32_t b) const {
    if (lat[a][b] < 0) throw std::logic_error("both regions should exist on the planet");
    return (uint64_t)lat[a][b];
  }
};

// util.rs:153-185: processes sorted by the position of their region in
// planet.sorted(region); same region -> by id.  Returns process ids.
std::vector<uint32_t> sort_processes_by_distance(const Planet& pl, uint32_t region,
                                                 const std::vector<std::pair<uint32_t, uint32_t>>& procs) {
  std::vector<uint32_t> pos(pl.names.size(), 0);
  for (size_t i = 0; i < pl.sorted[region].size(); ++i) pos[pl.sorted[region][i]] = (uint32_t)i;
  std::vector<std::pair<uint32_t, uint32_t>> v = procs;  // (id, region)
  std::sort(v.begin(), v.end(), [&](const auto& x, const auto& y) {
    if (x.second == y.second) return x.first < y.first;
    return pos[x.second] < pos[y.second];
  });
  std::vector<uint32_t> out;
  for (auto& x : v) out.push_back(x.first);
  return out;
}

// ------------------------------------------------------------ RNG (C6)
static inline uint64_t mix64(uint64_t x) {  // splitmix64 finalizer
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static inline uint64_t sim_rand(uint64_t seed, uint64_t inst, uint64_t client, uint64_t idx,
                                uint64_t purpose) {
  return mix64(mix64(mix64(mix64(seed ^ 0x5851F42D4C957F2Dull) + inst) + client) + ((idx << 8) | purpose));
}
enum : uint64_t { R_CONFLICT = 1, R_POOL = 2, R_READ_ONLY = 3, R_REORDER = 4 };

// -------------------------------------------------------------- types
struct Rifl {
  uint64_t source = 0, seq = 0;
  bool operator<(const Rifl& o) const { return source != o.source ? source < o.source : seq < o.seq; }
  bool operator==(const Rifl& o) const { return source == o.source && seq == o.seq; }
};
struct Cmd {
  Rifl rifl;
  std::vector<uint32_t> keys;  // C11: ascending
  bool read_only = false;
};

enum class MK : uint8_t {
  // Atlas / EPaxos (atlas.rs:816-865, epaxos.rs:667-700)
  MCollect, MCollectAck, MCommit, MConsensus, MConsensusAck, MCommitDot, MGarbageCollection, MStable,
  // Basic (basic.rs:363-385)
  MStore, MStoreAck, MCommitBasic
};

struct Msg {
  MK kind = MK::MCollect;
  Dot dot;
  Cmd cmd;
  std::vector<Dot> deps;          // HashSet<Dependency>, sorted (shards are always {0})
  std::vector<uint32_t> quorum;   // HashSet<ProcessId>, sorted
  uint64_t ballot = 0;
  std::vector<uint64_t> clock;    // VClock frontier, index = process id - 1
  std::vector<std::array<uint64_t, 3>> stable;
};

struct Action {  // protocol/mod.rs:239-248
  bool forward = false;            // ToForward
  std::vector<uint32_t> target;    // ToSend target, ascending (C4)
  Msg msg;
};

enum Status : uint8_t { START, PAYLOAD, COLLECT, COMMIT };

// quorum.rs:16-103
struct QuorumDeps {
  uint32_t fq = 0;
  std::set<uint32_t> participants;
  std::map<Dot, uint32_t> counts;
  void add(uint32_t p, const std::vector<Dot>& deps) {
    participants.insert(p);
    for (auto& d : deps) counts[d] += 1;
  }
  bool all() const { return participants.size() == fq; }
  std::vector<Dot> deps() const {
    std::vector<Dot> v;
    for (auto& kv : counts) v.push_back(kv.first);
    return v;
  }
  bool check_threshold(uint32_t t) const {
    for (auto& kv : counts)
      if (kv.second < t) return false;
    return true;
  }
  bool check_equal() const {
    std::set<uint32_t> c;
    for (auto& kv : counts) c.insert(kv.second);
    if (c.empty()) return true;
    if (c.size() == 1) return *c.begin() == fq;
    return false;
  }
};

// synod/single.rs:30-447 (the paths the simulator exercises: no recovery)
struct Synod {
  uint32_t pid = 0, n = 0, f = 0;
  uint64_t p_ballot = 0;
  std::set<uint32_t> accepts;
  uint64_t a_ballot = 0;
  uint64_t acc_ballot = 0;
  std::vector<Dot> acc_value;
  bool chosen = false;
  bool set_if_not_accepted(const std::vector<Dot>& v) {
    if (a_ballot == 0) {
      acc_ballot = 0;
      acc_value = v;
      return true;
    }
    return false;
  }
  uint64_t skip_prepare() {
    if (a_ballot != 0) throw std::logic_error("skip_prepare: acceptor ballot != 0");
    p_ballot = pid;
    return p_ballot;
  }
  void handle_chosen(const std::vector<Dot>& v) {  // MChosen
    chosen = true;
    acc_ballot = 0;
    acc_value = v;
  }
  // MAccept: 0 = nothing, 1 = MChosen(value) (out), 2 = MAccepted(b)
  int handle_accept(uint64_t b, const std::vector<Dot>& v, std::vector<Dot>& out) {
    if (chosen) {
      out = acc_value;
      return 1;
    }
    if (b >= a_ballot) {
      a_ballot = b;
      acc_ballot = b;
      acc_value = v;
      return 2;
    }
    return 0;
  }
  // MAccepted: true = MChosen(value) (out)
  bool handle_accepted(uint32_t from, uint64_t b, std::vector<Dot>& out) {
    if (p_ballot != b) return false;
    accepts.insert(from);
    if (accepts.size() == f + 1) {
      accepts.clear();
      if (acc_ballot != (uint64_t)pid)
        throw std::logic_error("there should have been proposal before a value can be chosen");
      out = acc_value;
      return true;
    }
    return false;
  }
};

struct Info {
  Status status = START;
  std::vector<uint32_t> quorum;
  Synod synod;
  bool has_cmd = false;
  Cmd cmd;
  QuorumDeps qd;
  std::set<uint32_t> acks;  // Basic
};

// gc/clock.rs:21-138 (MaxSet clocks)
struct GCTrack {
  uint32_t n = 0;
  std::vector<oracle::AboveExSet> my_clock;
  std::map<uint32_t, std::vector<uint64_t>> others;
  std::vector<uint64_t> prev_stable;
  void init(uint32_t n_) {
    n = n_;
    my_clock.assign(n, {});
    prev_stable.assign(n, 0);
  }
  void add(const Dot& d) { my_clock[d.source - 1].add(d.sequence); }
  std::vector<uint64_t> frontier() const {
    std::vector<uint64_t> v(n);
    for (uint32_t i = 0; i < n; ++i) v[i] = my_clock[i].max;
    return v;
  }
  void update(uint32_t from, const std::vector<uint64_t>& c) {
    auto it = others.find(from);
    if (it == others.end()) {
      others[from] = c;
    } else {
      for (uint32_t i = 0; i < n; ++i) it->second[i] = std::max(it->second[i], c[i]);
    }
  }
  std::vector<std::array<uint64_t, 3>> stable() {
    std::vector<uint64_t> cur(n, 0);
    if (others.size() == n - 1) {
      cur = frontier();
      for (auto& kv : others)
        for (uint32_t i = 0; i < n; ++i) cur[i] = std::min(cur[i], kv.second[i]);
    }
    std::vector<std::array<uint64_t, 3>> out;
    for (uint32_t i = 0; i < n; ++i) {
      const uint64_t start = prev_stable[i] + 1, end = cur[i];
      cur[i] = std::max(cur[i], prev_stable[i]);
      if (start <= end) out.push_back({(uint64_t)i + 1, start, end});
    }
    prev_stable = cur;
    return out;
  }
};

// deps/keys/sequential.rs:26-163 + keys/mod.rs:44-75 (the simulator never
// adds noops — no recovery — but the reference's KeyDeps tests do)
struct KeyDeps {
  bool nfr = false;
  struct RW {
    bool has_read = false, has_write = false;
    Dot read, write;
  };
  std::map<uint32_t, RW> latest;
  bool has_noop = false;
  Dot latest_noop;
  void maybe_add_deps(bool read_only, const RW& rw, std::set<Dot>& deps) const {  // keys/mod.rs:44-75
    if (rw.has_write) deps.insert(rw.write);
    if (!read_only && !nfr && rw.has_read) deps.insert(rw.read);
  }
  std::vector<Dot> add_cmd(const Dot& dot, const Cmd& cmd, const std::vector<Dot>* past) {
    std::set<Dot> deps;
    if (past) deps.insert(past->begin(), past->end());
    for (uint32_t key : cmd.keys) {
      RW& rw = latest[key];
      maybe_add_deps(cmd.read_only, rw, deps);
      if (cmd.read_only) {
        rw.has_read = true;
        rw.read = dot;
      } else {
        rw.has_write = true;
        rw.write = dot;
      }
    }
    if (has_noop) deps.insert(latest_noop);  // maybe_add_noop_latest
    return std::vector<Dot>(deps.begin(), deps.end());
  }
  std::vector<Dot> add_noop(const Dot& dot) {  // sequential.rs:120-149
    std::set<Dot> deps;
    if (has_noop) deps.insert(latest_noop);
    has_noop = true;
    latest_noop = dot;
    for (auto& kv : latest) {
      if (kv.second.has_read) deps.insert(kv.second.read);
      if (kv.second.has_write) deps.insert(kv.second.write);
    }
    return std::vector<Dot>(deps.begin(), deps.end());
  }
  std::vector<Dot> cmd_deps(const Cmd& cmd) const {  // test query (sequential.rs:46-52, 151-162)
    std::set<Dot> deps;
    if (has_noop) deps.insert(latest_noop);
    for (uint32_t key : cmd.keys) {
      auto it = latest.find(key);
      if (it != latest.end()) maybe_add_deps(cmd.read_only, it->second, deps);
    }
    return std::vector<Dot>(deps.begin(), deps.end());
  }
  std::vector<Dot> noop_deps() const {
    std::set<Dot> deps;
    if (has_noop) deps.insert(latest_noop);
    for (auto& kv : latest) {
      if (kv.second.has_read) deps.insert(kv.second.read);
      if (kv.second.has_write) deps.insert(kv.second.write);
    }
    return std::vector<Dot>(deps.begin(), deps.end());
  }
};

// An execution info: GraphExecutionInfo::Add (executor.rs:197-214) or
// BasicExecutionInfo (basic.rs:70-80).
struct ExecInfo {
  Dot dot;
  Cmd cmd;
  std::vector<Dot> deps;
  uint32_t key = 0;  // Basic: one info per key
};

struct ExecResult {  // ExecutorResult (executor/mod.rs:169-184)
  Rifl rifl;
  uint32_t key;
};

// ------------------------------------------------------------- process
struct Process {
  uint32_t protocol = FX_PROTOCOL_ATLAS;
  uint32_t id = 0, n = 0, f = 0, synod_f = 0;
  uint32_t fq_size = 0, wq_size = 0;
  bool gc_running = false;
  // BaseProcess (base.rs:62-154)
  std::vector<uint32_t> all, all_but_me, majority_q, fast_q, write_q;
  uint64_t next_seq = 0;
  // metrics (base.rs:229-249)
  uint64_t fast_paths = 0, slow_paths = 0, stable = 0, fast_reads = 0, slow_reads = 0;
  KeyDeps key_deps;
  std::map<Dot, Info> cmds;  // SequentialCommandsInfo
  std::map<Dot, std::pair<uint32_t, std::vector<Dot>>> buffered_commits;  // atlas/epaxos
  std::set<Dot> buffered_mcommits;                                       // basic
  GCTrack gc;
  std::vector<Action> to_processes;
  std::vector<ExecInfo> to_executors;
  // GraphExecutor / BasicExecutor
  std::unique_ptr<oracle::DependencyGraph> graph;
  std::map<Dot, Cmd> graph_cmds;
  uint32_t graph_rec = 0;
  std::vector<ExecResult> exec_to_clients;  // drained after each handle
  std::vector<uint32_t> executed;           // packed dots, execution order
  // optional capture of the executor's input (oracle_sim_capture): per Add
  // packed dot, time_ms, ndeps, deps ascending (C1)
  bool capture = false;
  std::vector<uint32_t> adds;
  std::map<uint32_t, std::vector<Rifl>> monitor;
  // AggregatePending (aggregate.rs:9-88)
  std::map<Rifl, uint32_t> pending;  // rifl -> results still missing

  Info& info(const Dot& d) {
    auto it = cmds.find(d);
    if (it != cmds.end()) return it->second;
    Info& in = cmds[d];
    in.synod.pid = id;
    in.synod.n = n;
    in.synod.f = synod_f;
    // EPaxosInfo::new uses fast_quorum_size - 1 (epaxos.rs:650-662)
    in.qd.fq = protocol == FX_PROTOCOL_EPAXOS ? fq_size - 1 : fq_size;
    return in;
  }

  void discover(const std::vector<uint32_t>& sorted) {
    const uint32_t maj = n / 2 + 1;
    all = sorted;
    std::sort(all.begin(), all.end());
    all_but_me.clear();
    for (uint32_t p : all)
      if (p != id) all_but_me.push_back(p);
    auto take = [&](uint32_t k) {
      std::vector<uint32_t> v(sorted.begin(), sorted.begin() + std::min<size_t>(k, sorted.size()));
      std::sort(v.begin(), v.end());
      return v;
    };
    majority_q = take(maj);
    fast_q = take(fq_size);
    write_q = take(wq_size);
  }

  void send(std::vector<uint32_t> target, Msg m) {
    Action a;
    a.target = std::move(target);
    a.msg = std::move(m);
    to_processes.push_back(std::move(a));
  }
  void forward(Msg m) {
    Action a;
    a.forward = true;
    a.msg = std::move(m);
    to_processes.push_back(std::move(a));
  }

  // Protocol::submit (atlas.rs:210-249, epaxos.rs:199-221, basic.rs:171-185)
  void submit(const Cmd& cmd) {
    const Dot dot{id, ++next_seq};
    Msg m;
    m.dot = dot;
    m.cmd = cmd;
    if (protocol == FX_PROTOCOL_BASIC) {
      m.kind = MK::MStore;
      m.quorum = fast_q;
    } else {
      m.kind = MK::MCollect;
      m.deps = key_deps.add_cmd(dot, cmd, nullptr);
      m.quorum = fast_q;  // maybe_adjust_fast_quorum: NFR only for single-key reads
      if (key_deps.nfr && cmd.read_only && cmd.keys.size() == 1) m.quorum = majority_q;
    }
    send(all, std::move(m));
  }

  void handle(uint32_t from, const Msg& m) {
    switch (m.kind) {
      case MK::MCollect: return handle_mcollect(from, m);
      case MK::MCollectAck: return handle_mcollectack(from, m);
      case MK::MCommit: return handle_mcommit(from, m.dot, m.deps);
      case MK::MConsensus: return handle_mconsensus(from, m);
      case MK::MConsensusAck: return handle_mconsensusack(from, m);
      case MK::MCommitDot:
        if (from != id) throw std::logic_error("MCommitDot from another process");
        gc.add(m.dot);
        return;
      case MK::MGarbageCollection: {
        gc.update(from, m.clock);
        auto st = gc.stable();
        if (!st.empty()) {
          Msg s;
          s.kind = MK::MStable;
          s.stable = std::move(st);
          forward(std::move(s));
        }
        return;
      }
      case MK::MStable: {
        if (from != id) throw std::logic_error("MStable from another process");
        uint64_t count = 0;
        for (auto& r : m.stable)
          for (uint64_t q = r[1]; q <= r[2]; ++q) count += cmds.erase(Dot{(uint32_t)r[0], q});
        stable += count;
        return;
      }
      case MK::MStore: return basic_mstore(from, m);
      case MK::MStoreAck: return basic_mstoreack(from, m.dot);
      case MK::MCommitBasic: return basic_mcommit(m.dot);
    }
  }

  // periodic GarbageCollection (atlas.rs:699-714, epaxos.rs:577-592, basic.rs:319-330)
  void handle_gc_event() {
    Msg m;
    m.kind = MK::MGarbageCollection;
    m.clock = gc.frontier();
    send(all_but_me, std::move(m));
  }

  // atlas.rs:251-325 / epaxos.rs:223-301
  void handle_mcollect(uint32_t from, const Msg& m) {
    Info& in = info(m.dot);
    if (in.status != START) return;
    if (!std::binary_search(m.quorum.begin(), m.quorum.end(), id)) {
      in.status = PAYLOAD;
      in.has_cmd = true;
      in.cmd = m.cmd;
      auto it = buffered_commits.find(m.dot);
      if (it != buffered_commits.end()) {
        auto b = std::move(it->second);
        buffered_commits.erase(it);
        handle_mcommit(b.first, m.dot, b.second);
      }
      return;
    }
    const bool from_self = from == id;
    std::vector<Dot> deps = from_self ? m.deps : key_deps.add_cmd(m.dot, m.cmd, &m.deps);
    in.status = COLLECT;
    in.qd.fq = protocol == FX_PROTOCOL_EPAXOS ? (uint32_t)m.quorum.size() - 1 : (uint32_t)m.quorum.size();
    in.quorum = m.quorum;
    in.has_cmd = true;
    in.cmd = m.cmd;
    if (!in.synod.set_if_not_accepted(deps)) throw std::logic_error("set_if_not_accepted");
    if (protocol == FX_PROTOCOL_EPAXOS && from_self) return;  // epaxos.rs:290-300
    Msg a;
    a.kind = MK::MCollectAck;
    a.dot = m.dot;
    a.deps = std::move(deps);
    send({from}, std::move(a));
  }

  // atlas.rs:327-402 / epaxos.rs:303-368
  void handle_mcollectack(uint32_t from, const Msg& m) {
    if (protocol == FX_PROTOCOL_EPAXOS && from == id) throw std::logic_error("epaxos ack from self");
    Info& in = info(m.dot);
    if (in.status != COLLECT) return;
    in.qd.add(from, m.deps);
    if (!in.qd.all()) return;
    bool fast;
    std::vector<Dot> deps = in.qd.deps();
    if (protocol == FX_PROTOCOL_ATLAS) {
      const uint32_t minority = (n / 2 + 1) - 1;
      const uint32_t threshold = (uint32_t)in.quorum.size() - minority;
      fast = in.qd.check_threshold(threshold);
    } else {
      fast = in.qd.check_equal();
    }
    if (fast) fast_paths += 1; else slow_paths += 1;  // BaseProcess::path (base.rs:229-243)
    if (in.cmd.read_only) {
      if (fast) fast_reads += 1; else slow_reads += 1;
    }
    if (fast) {
      Msg c;
      c.kind = MK::MCommit;
      c.dot = m.dot;
      c.deps = std::move(deps);
      send(all, std::move(c));
    } else {
      const uint64_t ballot = in.synod.skip_prepare();
      Msg c;
      c.kind = MK::MConsensus;
      c.dot = m.dot;
      c.ballot = ballot;
      c.deps = std::move(deps);
      send(write_q, std::move(c));
    }
  }

  // atlas.rs:404-475 / epaxos.rs:370-428
  void handle_mcommit(uint32_t from, const Dot& dot, const std::vector<Dot>& deps) {
    (void)from;
    Info& in = info(dot);
    if (in.status == START) {
      buffered_commits[dot] = {from, deps};
      return;
    }
    if (in.status == COMMIT) return;
    if (!in.has_cmd) throw std::logic_error("there should be a command payload");
    ExecInfo e;
    e.dot = dot;
    e.cmd = in.cmd;
    e.deps = deps;
    to_executors.push_back(std::move(e));
    in.status = COMMIT;
    in.synod.handle_chosen(deps);
    if (gc_running) {
      Msg c;
      c.kind = MK::MCommitDot;
      c.dot = dot;
      forward(std::move(c));
    } else {
      cmds.erase(dot);  // gc_single
    }
  }

  // atlas.rs:477-524 / epaxos.rs:430-477
  void handle_mconsensus(uint32_t from, const Msg& m) {
    Info& in = info(m.dot);
    std::vector<Dot> out;
    const int r = in.synod.handle_accept(m.ballot, m.deps, out);
    if (r == 0) return;
    Msg a;
    a.dot = m.dot;
    if (r == 2) {
      a.kind = MK::MConsensusAck;
      a.ballot = m.ballot;
    } else {
      a.kind = MK::MCommit;
      a.deps = std::move(out);
    }
    send({from}, std::move(a));
  }

  // atlas.rs:526-558 / epaxos.rs:479-517
  void handle_mconsensusack(uint32_t from, const Msg& m) {
    Info& in = info(m.dot);
    std::vector<Dot> out;
    if (!in.synod.handle_accepted(from, m.ballot, out)) return;
    Msg c;
    c.kind = MK::MCommit;
    c.dot = m.dot;
    c.deps = std::move(out);
    send(all, std::move(c));
  }

  // basic.rs:187-282
  void basic_mstore(uint32_t from, const Msg& m) {
    Info& in = info(m.dot);
    in.has_cmd = true;
    in.cmd = m.cmd;
    if (std::binary_search(m.quorum.begin(), m.quorum.end(), id)) {
      Msg a;
      a.kind = MK::MStoreAck;
      a.dot = m.dot;
      send({from}, std::move(a));
    }
    if (buffered_mcommits.erase(m.dot)) basic_mcommit(m.dot);
  }
  void basic_mstoreack(uint32_t from, const Dot& dot) {
    Info& in = info(dot);
    in.acks.insert(from);
    if (in.acks.size() == f + 1) {
      Msg c;
      c.kind = MK::MCommitBasic;
      c.dot = dot;
      send(all, std::move(c));
    }
  }
  void basic_mcommit(const Dot& dot) {
    Info& in = info(dot);
    if (!in.has_cmd) {
      buffered_mcommits.insert(dot);
      return;
    }
    for (uint32_t key : in.cmd.keys) {  // one BasicExecutionInfo per key (C11)
      ExecInfo e;
      e.dot = dot;
      e.cmd = in.cmd;
      e.key = key;
      to_executors.push_back(std::move(e));
    }
    if (gc_running) {
      Msg c;
      c.kind = MK::MCommitDot;
      c.dot = dot;
      forward(std::move(c));
    } else {
      cmds.erase(dot);
    }
  }

  // Executor::handle + to_clients (executor.rs:69-188, basic.rs:39-53)
  void executor_handle(const ExecInfo& e, uint64_t time_ms) {
    if (protocol == FX_PROTOCOL_BASIC) {
      executed.push_back(FX_PACK_DOT(e.dot.source, e.dot.sequence));
      exec_to_clients.push_back({e.cmd.rifl, e.key});
      return;
    }
    graph_cmds[e.dot] = e.cmd;
    if (capture) {
      std::vector<uint32_t> dv;
      for (const Dot& d : e.deps) dv.push_back(FX_PACK_DOT(d.source, d.sequence));
      std::sort(dv.begin(), dv.end());
      dv.erase(std::unique(dv.begin(), dv.end()), dv.end());
      adds.push_back(FX_PACK_DOT(e.dot.source, e.dot.sequence));
      adds.push_back((uint32_t)time_ms);
      adds.push_back((uint32_t)dv.size());
      adds.insert(adds.end(), dv.begin(), dv.end());
    }
    if (!graph->handle_add(e.dot, graph_rec++, e.deps, time_ms))
      throw std::logic_error("tried to index already indexed dot");
    for (const auto& x : graph->to_execute) {
      auto it = graph_cmds.find(x.dot);
      executed.push_back(FX_PACK_DOT(x.dot.source, x.dot.sequence));
      const Cmd& c = it->second;
      for (uint32_t key : c.keys) {  // Command::execute: one result per key (C11)
        exec_to_clients.push_back({c.rifl, key});
        if (!c.read_only) monitor[key].push_back(c.rifl);
      }
      graph_cmds.erase(it);
    }
    graph->to_execute.clear();
  }

  // AggregatePending::add_executor_result (aggregate.rs:48-87)
  bool add_executor_result(const ExecResult& r) {
    auto it = pending.find(r.rifl);
    if (it == pending.end()) return false;
    if (--it->second == 0) {
      pending.erase(it);
      return true;
    }
    return false;
  }
};

// Workload::gen_cmd (workload.rs:142-197) for command `idx` (0-based) of
// client `client`: rifl (client, idx + 1); gen_unique_keys draws
// KeyGenState::gen_conflict_rate (key_gen.rs:96-110) until keys_per_command
// distinct keys; then the read-only draw (workload.rs:158-160).
bool gen_cmd(const fx_sim_spec& spec, uint64_t client, uint64_t idx, Cmd& cmd) {
  cmd.rifl = Rifl{client, idx + 1};
  std::vector<uint32_t> keys;
  uint64_t draw = 0;
  while (keys.size() != spec.keys_per_command) {
    bool conflict;  // true_if_random_is_less_than(conflict_rate) (key_gen.rs:122-128)
    if (spec.conflict_rate == 0) conflict = false;
    else if (spec.conflict_rate >= 100) conflict = true;
    else conflict = sim_rand(spec.seed, spec.instance, client, idx * 64 + draw, R_CONFLICT) % 100 < spec.conflict_rate;
    uint32_t key;
    if (conflict) {  // "CONFLICT{gen_range(0..pool_size)}"
      key = spec.pool_size <= 1
                ? 0u
                : (uint32_t)(sim_rand(spec.seed, spec.instance, client, idx * 64 + draw, R_POOL) % spec.pool_size);
    } else {  // the client's own key
      key = spec.pool_size + (uint32_t)client;
    }
    ++draw;  // the reference draws until it has keys_per_command distinct keys
    if (draw > 65536u) return false;
    if (std::find(keys.begin(), keys.end(), key) == keys.end()) keys.push_back(key);
  }
  std::sort(keys.begin(), keys.end());  // C11
  cmd.keys = keys;
  if (spec.read_only_pct == 0) cmd.read_only = false;
  else if (spec.read_only_pct >= 100) cmd.read_only = true;
  else cmd.read_only = sim_rand(spec.seed, spec.instance, client, idx, R_READ_ONLY) % 100 < spec.read_only_pct;
  return true;
}

// --------------------------------------------------------------- client
struct Client {
  uint64_t id = 0;
  uint32_t region = 0;
  uint32_t process = 0;     // closest process (shard 0)
  uint64_t issued = 0;      // Workload::command_count
  uint64_t rifl_seq = 0;
  std::map<Rifl, uint64_t> pending;  // rifl -> start micros (client/pending.rs)
  std::vector<uint64_t> latencies_ms;
};

// --------------------------------------------------------------- runner
enum class SK : uint8_t { SubmitToProc, SendToProc, SendToClient, PeriodicProcessEvent, PeriodicExecutedNotification };

struct SchedAction {
  SK kind;
  uint32_t to = 0, from = 0;  // process ids / client id (SendToClient: to = client)
  uint64_t client = 0;
  Cmd cmd;
  Rifl rifl;
  Msg msg;
  uint64_t delay = 0;
};

struct Result {
  std::vector<std::vector<uint32_t>> executed;       // per process
  std::vector<std::vector<uint32_t>> adds;           // per process, when captured
  std::vector<std::map<uint32_t, std::vector<Rifl>>> monitors;
  std::map<uint32_t, std::map<uint64_t, uint64_t>> latency;  // region -> (ms -> count)
  std::map<uint32_t, uint64_t> issued;                       // region -> issued
  std::vector<uint64_t> fast, slow, stable, fast_reads, slow_reads;
  std::map<uint64_t, uint64_t> chain, delay;  // executor metrics summed over processes
  uint64_t end_ms = 0, events = 0, trace = 0;
};

class Runner {
 public:
  void set_capture() {
    for (auto& p : procs) p.capture = true;
  }
  Runner(const Planet& pl, const fx_sim_spec& s) : planet(pl), spec(s) {
    const uint32_t n = s.n;
    if (n < 1 || n > FX_SIM_MAX_N) throw std::logic_error("bad n");
    // Runner::new (runner.rs:64-190)
    procs.resize(n + 1);
    std::vector<std::pair<uint32_t, uint32_t>> to_discover;
    for (uint32_t i = 0; i < n; ++i) to_discover.push_back({i + 1, s.process_regions[i]});
    // Config::new panics on f > n/2 (config.rs:53-55); quorum sizes:
    // basic_quorum_size (config.rs:285-287, no write quorum, basic.rs:41-42),
    // atlas_quorum_sizes (295-301), epaxos_quorum_sizes (304-312)
    if (s.f > n / 2) throw std::logic_error("f is larger than a minority");
    uint32_t fq = 0, wq = 0;
    if (s.protocol == FX_PROTOCOL_BASIC) {
      fq = s.f + 1;
      wq = 0;
    } else if (s.protocol == FX_PROTOCOL_ATLAS) {
      fq = n / 2 + s.f;
      wq = s.f + 1;
    } else if (s.protocol == FX_PROTOCOL_EPAXOS) {
      const uint32_t fe = n / 2;
      fq = fe + (fe + 1) / 2;
      wq = fe + 1;
    } else {
      throw std::logic_error("unknown protocol");
    }
    for (uint32_t i = 0; i < n; ++i) {
      Process& p = procs[i + 1];
      p.protocol = s.protocol;
      p.id = i + 1;
      p.n = n;
      p.f = s.f;
      p.synod_f = s.protocol == FX_PROTOCOL_EPAXOS ? n / 2 : s.f;  // EPaxos::allowed_faults
      p.fq_size = fq;
      p.wq_size = wq;
      p.gc_running = s.gc_interval_ms != 0;
      p.key_deps.nfr = s.nfr != 0;
      p.gc.init(n);
      p.graph.reset(new oracle::DependencyGraph(i + 1, n));
      p.discover(sort_processes_by_distance(planet, s.process_regions[i], to_discover));
      process_region.push_back(s.process_regions[i]);
    }
    uint64_t cid = 0;
    for (uint32_t r = 0; r < s.num_client_regions; ++r) {
      for (uint32_t k = 0; k < s.clients_per_region; ++k) {
        Client c;
        c.id = ++cid;
        c.region = s.client_regions[r];
        c.process = sort_processes_by_distance(planet, c.region, to_discover)[0];
        clients.push_back(std::move(c));
      }
    }
    // periodic process events, then executed notifications (runner.rs:179-187)
    if (s.gc_interval_ms)
      for (uint32_t i = 1; i <= n; ++i) {
        SchedAction a;
        a.kind = SK::PeriodicProcessEvent;
        a.to = i;
        a.delay = s.gc_interval_ms;
        schedule(a.delay, std::move(a));
      }
    for (uint32_t i = 1; i <= n; ++i) {
      SchedAction a;
      a.kind = SK::PeriodicExecutedNotification;
      a.to = i;
      a.delay = s.executed_notification_ms;
      schedule(a.delay, std::move(a));
    }
  }

  Result run() {
    // Simulation::start_clients (simulation.rs:62-76), C5: ascending client id
    for (auto& c : clients) {
      Cmd cmd;
      if (!cmd_send(c, cmd)) throw std::logic_error("clients should submit at least one command");
      schedule_submit(c.id, c.process, std::move(cmd));
    }
    simulation_loop();
    Result r;
    const uint32_t n = spec.n;
    for (uint32_t i = 1; i <= n; ++i) {
      Process& p = procs[i];
      r.executed.push_back(p.executed);
      r.adds.push_back(std::move(p.adds));
      r.monitors.push_back(p.monitor);
      r.fast.push_back(p.fast_paths);
      r.slow.push_back(p.slow_paths);
      r.stable.push_back(p.stable);
      r.fast_reads.push_back(p.fast_reads);
      r.slow_reads.push_back(p.slow_reads);
      for (auto& kv : p.graph->chain_size) r.chain[kv.first] += kv.second;
      for (auto& kv : p.graph->execution_delay) r.delay[kv.first] += kv.second;
    }
    for (auto& c : clients) {  // clients_latencies (runner.rs:619-634)
      r.issued[c.region] += c.issued;
      auto& h = r.latency[c.region];
      for (uint64_t ms : c.latencies_ms) h[ms] += 1;
    }
    r.end_ms = now_us / 1000;
    r.events = events;
    r.trace = trace;
    return r;
  }

 private:
  const Planet& planet;
  fx_sim_spec spec;
  std::vector<Process> procs;  // index = process id
  std::vector<uint32_t> process_region;
  std::vector<Client> clients;
  // (time ms, class, seq) -> action.  C3: ties at one time go first to the
  // protocol/client actions in insertion (FIFO) order, then to the GC traffic
  // (periodic GC events by process id, then MGarbageCollection deliveries by
  // (from, to)).  GC actions touch only the GC track, which no other action
  // reads, so this is one of the reference's legal tie orders (its
  // BinaryHeap orders equal times arbitrarily), and the one that lets the GC
  // traffic be evaluated apart from the event order (sim_wave.hip).
  std::map<std::tuple<uint64_t, uint64_t, uint64_t>, SchedAction> queue;
  uint64_t seq = 0;
  uint64_t now_us = 0;
  uint64_t events = 0, trace = 0, reorder_draws = 0, exec_notifications = 0, gc_events = 0;

  uint64_t now_ms() const { return now_us / 1000; }

  void schedule(uint64_t delay_ms, SchedAction a) {  // Schedule::schedule (schedule.rs:38-49)
    uint64_t cls = 0;
    if (a.kind == SK::PeriodicProcessEvent)
      cls = (1ull << 20) | ((uint64_t)a.to << 8);
    else if (a.kind == SK::SendToProc && a.msg.kind == MK::MGarbageCollection)
      cls = (2ull << 20) | ((uint64_t)a.from << 8) | a.to;
    queue.emplace(std::make_tuple(now_ms() + delay_ms, cls, seq++), std::move(a));
  }

  uint32_t region_of_process(uint32_t p) const { return process_region[p - 1]; }
  uint32_t region_of_client(uint64_t c) const { return clients[c - 1].region; }

  // Runner::distance (runner.rs:575-595): half the ping, not symmetric
  uint64_t distance(uint32_t a, uint32_t b) const { return planet.ping(a, b) / 2; }

  // Runner::schedule_message (runner.rs:507-530)
  void schedule_message(uint32_t from_region, uint32_t to_region, SchedAction a) {
    uint64_t d = distance(from_region, to_region);
    if (spec.reorder_messages) {
      const uint64_t u = sim_rand(spec.seed, spec.instance, 0, reorder_draws++, R_REORDER);
      const double mult = (double)(u >> 11) * (1.0 / 9007199254740992.0) * 10.0;
      d = (uint64_t)((double)d * mult);
    }
    schedule(d, std::move(a));
  }

  void schedule_submit(uint64_t client, uint32_t pid, Cmd cmd) {
    SchedAction a;
    a.kind = SK::SubmitToProc;
    a.to = pid;
    a.client = client;
    a.cmd = std::move(cmd);
    schedule_message(region_of_client(client), region_of_process(pid), std::move(a));
  }

  // Client::cmd_send -> Workload::next_cmd (workload.rs:113-128)
  bool cmd_send(Client& c, Cmd& cmd) {
    if (c.issued >= spec.commands_per_client) return false;
    const uint64_t idx = c.issued;
    c.issued += 1;
    if (!gen_cmd(spec, c.id, idx, cmd)) throw std::logic_error("could not draw distinct keys");
    c.pending[cmd.rifl] = now_us;  // Pending::start
    return true;
  }

  void note(uint64_t kind, uint64_t a, uint64_t b, uint64_t c) {
    ++events;
    trace = mix64(trace ^ (now_ms() << 24) ^ (kind << 20) ^ (a << 12) ^ (b << 4)) + c;
  }

  // Runner::simulation_loop (runner.rs:233-313)
  void simulation_loop() {
    enum { RUNNING, EXTRA, DONE } status = RUNNING;
    uint64_t clients_done = 0;
    uint64_t final_ms = 0;
    const uint64_t client_count = clients.size();
    while (status != DONE) {
      if (queue.empty()) throw std::logic_error("there should be a new action");
      auto it = queue.begin();
      const uint64_t t = std::get<0>(it->first);
      SchedAction a = std::move(it->second);
      queue.erase(it);
      if (t * 1000 < now_us) throw std::logic_error("time went backwards");
      now_us = t * 1000;  // SimTime::set_millis
      switch (a.kind) {
        case SK::PeriodicProcessEvent: {
          ++gc_events;  // GC traffic is counted apart, not part of the action trace
          procs[a.to].handle_gc_event();
          send_to_processes_and_executors(a.to);
          SchedAction b;
          b.kind = SK::PeriodicProcessEvent;
          b.to = a.to;
          b.delay = a.delay;
          schedule(b.delay, std::move(b));
          break;
        }
        case SK::PeriodicExecutedNotification: {
          // GraphExecutor / BasicExecutor::executed are None (executor/mod.rs:74-79):
          // counted apart, not part of the action trace
          ++exec_notifications;
          SchedAction b;
          b.kind = SK::PeriodicExecutedNotification;
          b.to = a.to;
          b.delay = a.delay;
          schedule(b.delay, std::move(b));
          break;
        }
        case SK::SubmitToProc: {
          note(2, a.to, a.client, a.cmd.rifl.seq);
          Process& p = procs[a.to];
          p.pending[a.cmd.rifl] = (uint32_t)a.cmd.keys.size();  // AggregatePending::wait_for
          p.submit(a.cmd);
          send_to_processes_and_executors(a.to);
          break;
        }
        case SK::SendToProc: {
          if (a.msg.kind == MK::MGarbageCollection)
            ++gc_events;
          else
            note(3, a.to, a.from, (uint64_t)a.msg.kind << 32 | FX_PACK_DOT(a.msg.dot.source, a.msg.dot.sequence));
          handle_send_to_proc(a.from, a.to, a.msg);
          break;
        }
        case SK::SendToClient: {
          note(4, a.client, 0, a.rifl.seq);
          Client& c = clients[a.client - 1];
          // Client::cmd_recv (client/mod.rs:115-137, pending.rs:30-45)
          auto pit = c.pending.find(a.rifl);
          if (pit == c.pending.end()) throw std::logic_error("can't end a command not started");
          const uint64_t lat_us = now_us - pit->second;
          c.pending.erase(pit);
          c.latencies_ms.push_back(lat_us / 1000);  // Duration::as_millis
          Cmd next;
          if (cmd_send(c, next)) {
            schedule_submit(c.id, c.process, std::move(next));
          } else {
            clients_done += 1;
            if (clients_done == client_count) {
              if (spec.extra_sim_time_ms >= 0) {
                final_ms = now_ms() + (uint64_t)spec.extra_sim_time_ms;
                status = EXTRA;
              } else {
                status = DONE;
              }
            }
          }
          break;
        }
      }
      if (status == EXTRA && now_ms() > final_ms) status = DONE;
    }
  }

  void handle_send_to_proc(uint32_t from, uint32_t to, const Msg& m) {
    procs[to].handle(from, m);
    send_to_processes_and_executors(to);
  }

  // Runner::send_to_processes_and_executors (runner.rs:395-441)
  void send_to_processes_and_executors(uint32_t pid) {
    Process& p = procs[pid];
    std::vector<Action> actions;
    while (!p.to_processes.empty()) {  // Vec::pop: LIFO (C8)
      actions.push_back(std::move(p.to_processes.back()));
      p.to_processes.pop_back();
    }
    std::vector<Rifl> ready;
    while (!p.to_executors.empty()) {
      ExecInfo e = std::move(p.to_executors.back());
      p.to_executors.pop_back();
      p.executor_handle(e, now_ms());
      for (auto& r : p.exec_to_clients)
        if (p.add_executor_result(r)) ready.push_back(r.rifl);
      p.exec_to_clients.clear();
    }
    // schedule_protocol_actions (runner.rs:444-488)
    for (auto& a : actions) {
      if (a.forward) {
        handle_send_to_proc(pid, pid, a.msg);
        continue;
      }
      for (uint32_t to : a.target) {  // C4: ascending
        if (to == pid) {
          handle_send_to_proc(pid, pid, a.msg);
        } else {
          SchedAction s;
          s.kind = SK::SendToProc;
          s.from = pid;
          s.to = to;
          s.msg = a.msg;
          schedule_message(region_of_process(pid), region_of_process(to), std::move(s));
        }
      }
    }
    // schedule_to_client (runner.rs:491-504)
    for (auto& rifl : ready) {
      SchedAction s;
      s.kind = SK::SendToClient;
      s.client = rifl.source;
      s.rifl = rifl;
      schedule_message(region_of_process(pid), region_of_client(rifl.source), std::move(s));
    }
  }
};

}  // namespace simo

// ============================================================ C interface
using oracle::Dot;
extern "C" {

// ---- unit hooks for the reference's KATs of the simulator's building blocks
// (packed dots: source << 24 | seq)

// QuorumDeps (quorum.rs:16-103): `reports` deps sets from processes 1..;
// returns the union (ascending) and both fast-path checks.
int oracle_quorum_deps(uint32_t fq, uint32_t nreports, const uint32_t* report_len, const uint32_t* deps,
                       uint32_t threshold, uint32_t* out_union, uint32_t cap, uint32_t* n_union,
                       uint32_t* all, uint32_t* threshold_ok, uint32_t* equal_ok) {
  simo::QuorumDeps q;
  q.fq = fq;
  size_t off = 0;
  for (uint32_t r = 0; r < nreports; ++r) {
    std::vector<Dot> v;
    for (uint32_t j = 0; j < report_len[r]; ++j, ++off) v.push_back(Dot{deps[off] >> 24, deps[off] & 0xFFFFFFu});
    q.add(r + 1, v);
  }
  auto u = q.deps();
  *n_union = (uint32_t)u.size();
  for (size_t i = 0; i < u.size() && i < cap; ++i) out_union[i] = FX_PACK_DOT(u[i].source, u[i].sequence);
  *all = q.all();
  *threshold_ok = q.check_threshold(threshold);
  *equal_ok = q.check_equal();
  return 0;
}

// SequentialKeyDeps driven by a script of operations (keys/mod.rs:120-485):
// op kind 0 add_cmd(dot, keys, read_only), 1 add_noop(dot), 2 cmd_deps(keys,
// read_only) query, 3 noop_deps query.  For each op the resulting deps are
// written to out[op * cap ..] with their count in out_len[op].
int oracle_key_deps_script(uint32_t nfr, uint32_t nops, const uint32_t* kind, const uint32_t* dot,
                           const uint32_t* nkeys, const uint32_t* keys, const uint32_t* read_only,
                           uint32_t cap, uint32_t* out, uint32_t* out_len) {
  simo::KeyDeps kd;
  kd.nfr = nfr != 0;
  size_t koff = 0;
  for (uint32_t i = 0; i < nops; ++i) {
    simo::Cmd c;
    for (uint32_t j = 0; j < nkeys[i]; ++j) c.keys.push_back(keys[koff++]);
    std::sort(c.keys.begin(), c.keys.end());
    c.read_only = read_only[i] != 0;
    const Dot d{dot[i] >> 24, dot[i] & 0xFFFFFFu};
    std::vector<Dot> r;
    switch (kind[i]) {
      case 0: r = kd.add_cmd(d, c, nullptr); break;
      case 1: r = kd.add_noop(d); break;
      case 2: r = kd.cmd_deps(c); break;
      default: r = kd.noop_deps(); break;
    }
    out_len[i] = (uint32_t)r.size();
    for (size_t j = 0; j < r.size() && j < cap; ++j) out[(size_t)i * cap + j] = FX_PACK_DOT(r[j].source, r[j].sequence);
  }
  return 0;
}

// VClockGCTrack (gc/clock.rs:21-138) driven by a script: op 0 add_to_clock(dot),
// 1 update_clock_of(from, clock[n]), 2 stable() -> out ranges (p, start, end).
int oracle_gc_script(uint32_t n, uint32_t nops, const uint32_t* kind, const uint32_t* arg,
                     const uint64_t* clocks, uint32_t cap, uint64_t* out, uint32_t* out_len,
                     uint64_t* frontier_out) {
  simo::GCTrack g;
  g.init(n);
  for (uint32_t i = 0; i < nops; ++i) {
    out_len[i] = 0;
    if (kind[i] == 0) {
      g.add(Dot{arg[i] >> 24, arg[i] & 0xFFFFFFu});
    } else if (kind[i] == 1) {
      g.update(arg[i], std::vector<uint64_t>(clocks + (size_t)i * n, clocks + (size_t)(i + 1) * n));
    } else {
      auto st = g.stable();
      out_len[i] = (uint32_t)st.size();
      for (size_t j = 0; j < st.size() && j < cap; ++j)
        for (int k = 0; k < 3; ++k) out[((size_t)i * cap + j) * 3 + k] = st[j][k];
    }
    auto f = g.frontier();
    for (uint32_t k = 0; k < n; ++k) frontier_out[(size_t)i * n + k] = f[k];
  }
  return 0;
}

// Regions of the planet in `dir` (name order); returns the region count.
int oracle_planet_regions(const char* dir, char* names, uint32_t cap_bytes) {
  simo::Planet pl;
  if (!pl.load(dir)) return -1;
  std::string all;
  for (auto& s : pl.names) all += s + "\n";
  if (names && cap_bytes) {
    std::strncpy(names, all.c_str(), cap_bytes - 1);
    names[cap_bytes - 1] = 0;
  }
  return (int)pl.names.size();
}

// Ping latency matrix [R][R] (ms) and the per-region sorted order [R][R].
int oracle_planet_matrix(const char* dir, int64_t* lat, uint32_t* sorted, uint32_t R) {
  simo::Planet pl;
  if (!pl.load(dir) || pl.names.size() != R) return -1;
  for (uint32_t a = 0; a < R; ++a)
    for (uint32_t b = 0; b < R; ++b) {
      lat[a * R + b] = pl.lat[a][b];
      sorted[a * R + b] = pl.sorted[a][b];
    }
  return 0;
}

// util.rs:153-185 over (id, region) pairs; writes the sorted ids.
int oracle_sort_processes(const char* dir, uint32_t region, const uint32_t* ids, const uint32_t* regions,
                          uint32_t n, uint32_t* out) {
  simo::Planet pl;
  if (!pl.load(dir)) return -1;
  std::vector<std::pair<uint32_t, uint32_t>> v;
  for (uint32_t i = 0; i < n; ++i) v.push_back({ids[i], regions[i]});
  auto s = simo::sort_processes_by_distance(pl, region, v);
  for (uint32_t i = 0; i < n; ++i) out[i] = s[i];
  return 0;
}

// Output of one simulated instance (dense, caller-allocated).
typedef struct oracle_sim_out {
  uint32_t* executed;      // [n][exec_cap] packed dots in execution order
  uint64_t* executed_len;  // [n]
  uint32_t exec_cap;
  uint64_t* latency;       // [R][lat_bins] client latency ms histogram per region
  uint64_t* issued;        // [R]
  uint32_t R, lat_bins;    // latencies >= lat_bins - 1 land in the last bin
  uint64_t* fast;          // [n]
  uint64_t* slow;          // [n]
  uint64_t* stable;        // [n]
  uint64_t* chain;         // [chain_bins] executor ChainSize (summed over processes)
  uint64_t* delay;         // [delay_bins] executor ExecutionDelay
  uint32_t chain_bins, delay_bins;
  uint64_t end_ms, events, trace;
  int32_t status;          // 0 ok, 1 reference assertion, 2 capacity of this buffer
  int32_t pad;
  uint64_t* monitor_hash;  // [n] hash of the ExecutionOrderMonitor (per key, rifls in order), or NULL
  uint64_t* fast_reads;    // [n] FastPathReads (base.rs:229-243), or NULL
  uint64_t* slow_reads;    // [n] SlowPathReads, or NULL
} oracle_sim_out;

static int fill(const simo::Result& r, const fx_sim_spec& s, oracle_sim_out* o) {
  int st = 0;
  for (uint32_t p = 0; p < s.n; ++p) {
    const auto& e = r.executed[p];
    o->executed_len[p] = e.size();
    if (e.size() > o->exec_cap) st = 2;
    if (o->executed)
      for (size_t i = 0; i < e.size() && i < o->exec_cap; ++i) o->executed[(size_t)p * o->exec_cap + i] = e[i];
    o->fast[p] = r.fast[p];
    o->slow[p] = r.slow[p];
    o->stable[p] = r.stable[p];
    if (o->fast_reads) o->fast_reads[p] = r.fast_reads[p];
    if (o->slow_reads) o->slow_reads[p] = r.slow_reads[p];
  }
  for (auto& kv : r.latency)
    for (auto& h : kv.second) {
      const uint64_t b = std::min<uint64_t>(h.first, o->lat_bins - 1);
      o->latency[(size_t)kv.first * o->lat_bins + b] += h.second;
    }
  for (auto& kv : r.issued) o->issued[kv.first] += kv.second;
  for (auto& kv : r.chain) o->chain[std::min<uint64_t>(kv.first, o->chain_bins - 1)] += kv.second;
  for (auto& kv : r.delay) o->delay[std::min<uint64_t>(kv.first, o->delay_bins - 1)] += kv.second;
  if (o->monitor_hash)
    for (uint32_t p = 0; p < s.n; ++p) {
      uint64_t h = 0x1234567ull;
      for (auto& kv : r.monitors[p]) {
        h = simo::mix64(h ^ ((uint64_t)kv.first << 32));
        for (auto& rf : kv.second) h = simo::mix64(h ^ (rf.source << 40) ^ rf.seq);
      }
      o->monitor_hash[p] = h;
    }
  o->end_ms = r.end_ms;
  o->events = r.events;
  o->trace = r.trace;
  return st;
}

// Keys of the first `count` commands of client `client` (Workload::gen_cmd,
// workload.rs:142-197, with the C6 RNG), packed keys_per_command per command;
// read_only flags in ro.
int oracle_workload_keys(const fx_sim_spec* spec, uint64_t client, uint32_t count, uint32_t* keys,
                         uint32_t* ro) {
  for (uint32_t i = 0; i < count; ++i) {
    simo::Cmd c;
    if (!simo::gen_cmd(*spec, client, i, c)) return 1;
    for (uint32_t k = 0; k < spec->keys_per_command; ++k) keys[(size_t)i * spec->keys_per_command + k] = c.keys[k];
    ro[i] = c.read_only;
  }
  return 0;
}

// Runs one instance.  Histogram outputs are accumulated into (zero them first).
int oracle_sim_run(const char* planet_dir, const fx_sim_spec* spec, oracle_sim_out* out) {
  simo::Planet pl;
  if (!pl.load(planet_dir)) return -1;
  try {
    simo::Runner runner(pl, *spec);
    simo::Result r = runner.run();
    out->status = fill(r, *spec, out);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "oracle_sim_run: %s\n", e.what());
    out->status = 1;
  }
  return out->status;
}

// Runs one instance capturing each process's executor input (the commit
// stream its GraphExecutor receives, in handle order) as fixed-width rows:
// process p's Add i at [p * cap + i] of dot / t_ms / nd, its deps (ascending,
// C1) at deps[(p * cap + i) * 8 + j]; len[p] Adds.  The execution order the
// simulation produced at p: executed[p * cap + k], k < exec_len[p].
// Status 2 if a stream is longer than cap or an Add has more than 8 deps.
int oracle_sim_capture(const char* planet_dir, const fx_sim_spec* spec, uint64_t cap, uint32_t* dot,
                       uint32_t* t_ms, uint32_t* nd, uint32_t* deps, uint64_t* len, uint32_t* executed,
                       uint64_t* exec_len) {
  simo::Planet pl;
  if (!pl.load(planet_dir)) return -1;
  try {
    simo::Runner runner(pl, *spec);
    runner.set_capture();
    simo::Result r = runner.run();
    int st = 0;
    for (uint32_t p = 0; p < spec->n; ++p) {
      const auto& a = r.adds[p];
      const auto& e = r.executed[p];
      uint64_t i = 0;
      for (size_t w = 0; w < a.size(); ++i) {
        const uint32_t k = a[w + 2];
        if (i < cap && k <= 8) {
          const uint64_t at = p * cap + i;
          dot[at] = a[w];
          t_ms[at] = a[w + 1];
          nd[at] = k;
          for (uint32_t j = 0; j < 8; ++j) deps[at * 8 + j] = j < k ? a[w + 3 + j] : 0u;
        } else {
          st = 2;
        }
        w += 3 + k;
      }
      len[p] = i;
      exec_len[p] = e.size();
      if (e.size() > cap) st = 2;
      for (size_t k = 0; k < e.size() && k < cap; ++k) executed[p * cap + k] = e[k];
    }
    return st;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "oracle_sim_capture: %s\n", e.what());
    return 1;
  }
}

// Runs `count` instances on `nthreads` std::threads (the reference's rayon
// par_iter over independent simulations, simulation.rs:51-57,216-217).
// outs[i] receives instance i's results.  Returns the number of failed instances.
int oracle_sim_batch(const char* planet_dir, const fx_sim_spec* specs, uint32_t count, oracle_sim_out* outs,
                     int nthreads) {
  simo::Planet pl;
  if (!pl.load(planet_dir)) return -1;
  if (nthreads < 1) nthreads = 1;
  std::atomic<uint32_t> next{0}, failed{0};
  auto worker = [&]() {
    while (true) {
      const uint32_t i = next.fetch_add(1);
      if (i >= count) break;
      try {
        simo::Runner runner(pl, specs[i]);
        simo::Result r = runner.run();
        outs[i].status = fill(r, specs[i], &outs[i]);
      } catch (const std::exception&) {
        outs[i].status = 1;
      }
      if (outs[i].status) failed.fetch_add(1);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nthreads; ++t) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  return (int)failed.load();
}

}  // extern "C"
