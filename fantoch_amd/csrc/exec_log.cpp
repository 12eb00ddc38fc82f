// exec_log.cpp — reader for the run mode's execution log.
//
// File format, as written by execution_logger_task
// (fantoch/src/run/task/server/execution_logger.rs:11-55) through Rw::write
// (fantoch/src/run/rw/mod.rs:66-77, 93-100): a sequence of frames from
// tokio_util's LengthDelimitedCodec with its defaults (4-byte big-endian
// length, then the payload); each payload is `bincode::serialize` (bincode
// 1.3.3 default options: little-endian, fixed-width integers, u64 lengths for
// sequences/maps/strings, u32 enum variant tags, u8 Option tags) of one
// GraphExecutionInfo (fantoch_ps/src/executor/graph/executor.rs:197-214):
//
//   Add { dot: Dot, cmd: Command, deps: HashSet<Dependency> }   tag 0
//   Request { from: ShardId, dots: HashSet<Dot> }                tag 1
//   RequestReply { infos: Vec<RequestReply> }                    tag 2
//   Executed { dots: HashSet<Dot> }                              tag 3
//
//   Dot = Id<u8>  {source u8, sequence u64}     (fantoch/src/id.rs:21-27)
//   Rifl = Id<u64> {source u64, sequence u64}
//   Command { rifl, shard_to_ops: Map<u64, Map<String, Arc<Vec<KVOp>>>>,
//             shard_to_keys: Arc<Map<u64, Vec<String>>>,
//             _empty_keys: Map<String, Arc<Vec<KVOp>>> }  (fantoch/src/command.rs:13-22;
//             serde "rc": an Arc serialises as its contents)
//   KVOp = Get (tag 0) | Put(String) (tag 1) | Delete (tag 2)   (fantoch/src/kvs.rs:13-17)
//   Dependency { dot: Dot, shards: Option<BTreeSet<u64>> }
//             (fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:19-22)
//   RequestReply = Info { dot, cmd, deps: Vec<Dependency> } (tag 0) | Executed { dot } (tag 1)
//             (fantoch_ps/src/executor/graph/mod.rs:34-43)
//
// Decoding maps each Add to the C-ABI's handle_add arguments: the keys of the
// command on the reader's shard (Command::iter(shard_id), command.rs:165-173)
// interned to u32 ids in first-seen order (canonical C7 for logs), read_only as
// Command::read_only (command.rs:80-87), deps as dots.  Request / RequestReply /
// Executed only occur with shard_count > 1 (out of scope): they are parsed so
// the stream stays in sync and counted, never executed.  Host-only code: the
// replay runs the decoded Adds through the GPU executor.
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "fantoch_amd.h"

namespace {

struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;

  bool need(uint64_t n) {
    if (!ok || (uint64_t)(end - p) < n) ok = false;
    return ok;
  }
  uint8_t u8() {
    if (!need(1)) return 0;
    return *p++;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    uint32_t v;
    std::memcpy(&v, p, 4);  // bincode is little-endian, as is gfx950's host
    p += 4;
    return v;
  }
  uint64_t u64() {
    if (!need(8)) return 0;
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  // sequence length: bounded by the bytes left so a corrupt length fails fast
  uint64_t len(uint64_t min_elem_bytes) {
    uint64_t n = u64();
    if (ok && min_elem_bytes && n > (uint64_t)(end - p) / min_elem_bytes) ok = false;
    return ok ? n : 0;
  }
  std::string str() {
    uint64_t n = len(1);
    if (!need(n)) return std::string();
    std::string s(reinterpret_cast<const char*>(p), (size_t)n);
    p += n;
    return s;
  }
  void skip_str() {
    uint64_t n = len(1);
    if (need(n)) p += n;
  }
};

struct Decoded {
  fx_dot dot;
  fx_rifl rifl;
  uint32_t read_only;
  std::vector<uint32_t> keys;
  std::vector<fx_dot> deps;
};

struct Reader {
  uint64_t shard_id;
  std::unordered_map<std::string, uint32_t> key_ids;
  fx_log_summary sum{};

  uint32_t intern(const std::string& k) {
    auto it = key_ids.find(k);
    if (it != key_ids.end()) return it->second;
    uint32_t id = (uint32_t)key_ids.size();
    key_ids.emplace(k, id);
    return id;
  }

  static fx_dot dot(Cursor& c) {
    fx_dot d;
    d.source = c.u8();
    uint64_t seq = c.u64();
    d.seq = (uint32_t)seq;
    if (seq > 0xFFFFFFFFull) c.ok = false;  // fx_dot holds u32 sequences
    return d;
  }

  // Vec<KVOp>; returns whether every op is a Get
  static bool ops(Cursor& c) {
    bool all_get = true;
    uint64_t n = c.len(4);
    for (uint64_t i = 0; i < n && c.ok; i++) {
      uint32_t tag = c.u32();
      if (tag == 1) {
        c.skip_str();
        all_get = false;
      } else if (tag == 2) {
        all_get = false;
      } else if (tag != 0) {
        c.ok = false;
      }
    }
    return all_get;
  }

  // Command; keys of shard `shard_id` go to out->keys when out != nullptr
  void command(Cursor& c, Decoded* out) {
    fx_rifl r;
    r.source = c.u64();
    r.seq = c.u64();
    bool read_only = true;
    uint64_t nshards = c.len(16);
    for (uint64_t s = 0; s < nshards && c.ok; s++) {
      uint64_t shard = c.u64();
      uint64_t nkeys = c.len(16);
      for (uint64_t k = 0; k < nkeys && c.ok; k++) {
        std::string key = c.str();
        read_only = ops(c) && read_only;
        if (out && c.ok && shard == shard_id) out->keys.push_back(intern(key));
      }
    }
    uint64_t nsk = c.len(16);  // shard_to_keys (derived from shard_to_ops)
    for (uint64_t s = 0; s < nsk && c.ok; s++) {
      (void)c.u64();
      uint64_t nk = c.len(8);
      for (uint64_t k = 0; k < nk && c.ok; k++) c.skip_str();
    }
    uint64_t ne = c.len(16);  // _empty_keys (always empty when written by the reference)
    for (uint64_t k = 0; k < ne && c.ok; k++) {
      c.skip_str();
      (void)ops(c);
    }
    if (out) {
      out->rifl = r;
      out->read_only = read_only ? 1u : 0u;
    }
  }

  static void dependency(Cursor& c, std::vector<fx_dot>* out) {
    fx_dot d = dot(c);
    uint8_t some = c.u8();
    if (some == 1) {
      uint64_t n = c.len(8);
      for (uint64_t i = 0; i < n && c.ok; i++) (void)c.u64();
    } else if (some != 0) {
      c.ok = false;
    }
    if (out && c.ok) out->push_back(d);
  }

  static void dots(Cursor& c) {
    uint64_t n = c.len(9);
    for (uint64_t i = 0; i < n && c.ok; i++) (void)dot(c);
  }

  // one GraphExecutionInfo payload; returns true and fills `out` for an Add
  bool info(Cursor& c, Decoded* out) {
    uint32_t tag = c.u32();
    switch (tag) {
      case 0: {  // Add
        out->keys.clear();
        out->deps.clear();
        out->dot = dot(c);
        command(c, out);
        uint64_t nd = c.len(10);
        for (uint64_t i = 0; i < nd && c.ok; i++) dependency(c, &out->deps);
        return c.ok;
      }
      case 1:  // Request
        (void)c.u64();
        dots(c);
        return false;
      case 2: {  // RequestReply
        uint64_t n = c.len(4);
        for (uint64_t i = 0; i < n && c.ok; i++) {
          uint32_t rt = c.u32();
          if (rt == 0) {
            (void)dot(c);
            command(c, nullptr);
            uint64_t nd = c.len(10);
            for (uint64_t j = 0; j < nd && c.ok; j++) dependency(c, nullptr);
          } else if (rt == 1) {
            (void)dot(c);
          } else {
            c.ok = false;
          }
        }
        return false;
      }
      case 3:  // Executed
        dots(c);
        return false;
      default:
        c.ok = false;
        return false;
    }
  }

  // Walks every frame; `sink(const Decoded&)` sees each Add in file order.
  template <class Sink>
  int walk(const uint8_t* buf, uint64_t len, Sink&& sink) {
    const uint8_t* p = buf;
    const uint8_t* end = buf + len;
    Decoded d;
    while (p < end) {
      if (end - p < 4) return FX_ERR_LOG_FORMAT;
      uint64_t flen = ((uint64_t)p[0] << 24) | ((uint64_t)p[1] << 16) | ((uint64_t)p[2] << 8) | p[3];
      p += 4;
      if ((uint64_t)(end - p) < flen) return FX_ERR_LOG_FORMAT;
      Cursor c{p, p + flen};
      bool add = info(c, &d);
      if (!c.ok || c.p != c.end) return FX_ERR_LOG_FORMAT;  // bincode rejects trailing bytes too
      sum.records++;
      if (add) {
        sum.adds++;
        sum.keys += d.keys.size();
        sum.deps += d.deps.size();
        int st = sink(d);
        if (st != FX_OK) return st;
      } else {
        sum.others++;
      }
      p += flen;
    }
    sum.distinct_keys = key_ids.size();
    return FX_OK;
  }
};

}  // namespace

extern "C" int fx_exec_log_scan(const uint8_t* buf, uint64_t len, uint64_t shard_id, fx_log_summary* out) {
  if ((!buf && len) || !out) return FX_ERR_INVALID_ARG;
  Reader r{shard_id, {}, {}};
  int st = r.walk(buf, len, [](const Decoded&) { return FX_OK; });
  *out = r.sum;
  return st;
}

extern "C" int fx_exec_log_decode(const uint8_t* buf, uint64_t len, uint64_t shard_id, fx_log_add* adds,
                                  uint64_t cap_adds, uint32_t* keys, uint64_t cap_keys, fx_dot* deps,
                                  uint64_t cap_deps, fx_log_summary* out) {
  if ((!buf && len) || !out) return FX_ERR_INVALID_ARG;
  Reader r{shard_id, {}, {}};
  uint64_t na = 0, nk = 0, nd = 0;
  int st = r.walk(buf, len, [&](const Decoded& d) {
    if (na >= cap_adds || nk + d.keys.size() > cap_keys || nd + d.deps.size() > cap_deps)
      return FX_ERR_CAPACITY;
    if (!adds || (d.keys.size() && !keys) || (d.deps.size() && !deps)) return FX_ERR_INVALID_ARG;
    fx_log_add& a = adds[na++];
    a.dot = d.dot;
    a.rifl = d.rifl;
    a.key_off = nk;
    a.dep_off = nd;
    a.nkeys = (uint32_t)d.keys.size();
    a.ndeps = (uint32_t)d.deps.size();
    a.read_only = d.read_only;
    a.pad = 0;
    for (uint32_t k : d.keys) keys[nk++] = k;
    for (const fx_dot& x : d.deps) deps[nd++] = x;
    return FX_OK;
  });
  *out = r.sum;
  return st;
}
