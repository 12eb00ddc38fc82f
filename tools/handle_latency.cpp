// handle_latency — the drop-in handle's per-Add cost without an interpreter in
// the loop: the reference simulator's calling pattern (runner.rs:406-424:
// handle(Add) then drain to_clients, one Add at a time) as a C++ loop over the
// C-ABI.  Reads a captured commit stream written by bench_handle.py:
//   u32 n, u32 process_id, u32 count, then per Add:
//   u32 src, u32 seq, u32 t_ms, u32 ndeps, ndeps x (u32 src, u32 seq)
// With a third argument H > 1 the same stream goes to H handles, one Add to
// each in turn (the simulator's pattern: one executor per process, all driven
// from one thread), and the time is per Add per handle.
// and prints one JSON line: microseconds per Add (median of `reps` passes, each
// on a fresh handle) and the execution order as packed dots (src << 24 | seq).
// Measurement helper, not product code.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "fantoch_amd.h"
#include <cstdlib>

struct Add {
  fx_dot dot;
  uint32_t t;
  std::vector<fx_dot> deps;
};

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: handle_latency stream.bin [reps] [handles]\n");
    return 2;
  }
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  const int H = argc > 3 ? std::max(1, std::atoi(argv[3])) : 1;
  setenv("FX_HANDLE_STATS", "1", 0);  // the kernel's timing words (one more 16-byte read per flush)
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  uint32_t hdr[3];
  if (std::fread(hdr, 4, 3, f) != 3) return 2;
  std::vector<Add> adds(hdr[2]);
  for (auto& a : adds) {
    uint32_t w[4];
    if (std::fread(w, 4, 4, f) != 4) return 2;
    a.dot = fx_dot{w[0], w[1]};
    a.t = w[2];
    a.deps.resize(w[3]);
    for (auto& d : a.deps) {
      uint32_t x[2];
      if (std::fread(x, 4, 2, f) != 2) return 2;
      d = fx_dot{x[0], x[1]};
    }
  }
  std::fclose(f);
  fx_config cfg{hdr[0], 1, 1, 0, 0};
  std::vector<double> us;
  double new_us = 0;
  std::vector<uint32_t> order;
  std::vector<fx_dot> buf(256);
  std::vector<uint8_t> start(256);
  const uint32_t key = 0;
  for (int r = 0; r < reps + 1; ++r) {  // pass 0 warms up (module load, first allocations)
    std::vector<fx_graph_executor*> hs(H);
    const auto tn = std::chrono::steady_clock::now();
    for (auto& h : hs)
      if (!(h = fx_graph_executor_new((uint8_t)hdr[1], 0, &cfg))) return 3;
    new_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tn).count() / H;
    fx_graph_executor* ex = hs[0];
    order.clear();
    const auto t0 = std::chrono::steady_clock::now();
    double add_ns = 0, drain_ns = 0;
    for (const auto& a : adds) {
      fx_rifl rifl{a.dot.source, a.dot.seq};
      for (int hi = 0; hi < H; ++hi) {
        const auto ta = std::chrono::steady_clock::now();
        if (fx_graph_executor_handle_add(hs[hi], a.dot, rifl, &key, 1, 0, a.deps.data(), (uint32_t)a.deps.size(), a.t))
          return 4;
        add_ns += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - ta).count();
        uint32_t got = 0;
        const auto td = std::chrono::steady_clock::now();
        do {
          if (fx_graph_executor_drain_dots(hs[hi], buf.data(), start.data(), 256, &got)) return 5;
          if (hi == 0)
            for (uint32_t i = 0; i < got; ++i) order.push_back(FX_PACK_DOT(buf[i].source, buf[i].seq));
        } while (got == 256);
        drain_ns += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - td).count();
      }
    }
    const auto t1 = std::chrono::steady_clock::now();
    uint64_t ps[FX_PERSIST_STATS];
    fx_graph_executor_persist_stats(ex, ps, FX_PERSIST_STATS);
    if (r == reps && ps[0]) {
      const double f = (double)ps[0];
      std::printf("{\"persist\": {\"flushes\": %llu, \"host_wait_us\": %.3f, \"compute_us\": %.3f, \"fence_us\": %.3f, "
                  "\"polls_per_flush\": %.2f, \"poll_rtt_us\": %.3f, \"host_prep_us\": %.3f, \"host_convert_us\": %.3f, "
                  "\"handle_add_us\": %.3f, \"compute_mhz\": %.0f, \"flush_us\": %.3f, \"drain_call_us\": %.3f, "
                  "\"post_wait_reads_us\": %.3f, \"pre_publish_us\": %.3f, \"iters_per_flush\": %.2f, "
                  "\"step_cycles\": %.0f, \"compute_cycles\": %.0f}}\n",
                  (unsigned long long)ps[0], ps[1] / f / 1e3, ps[2] / f / 100.0, ps[3] / f / 100.0, ps[4] / f,
                  ps[5] / f / 100.0, ps[6] / f / 1e3, ps[7] / f / 1e3, add_ns / adds.size() / H / 1e3,
                  ps[2] ? 100.0 * (double)ps[8] / (double)ps[2] : 0.0, ps[9] / f / 1e3, drain_ns / adds.size() / H / 1e3,
                  ps[10] / f / 1e3, ps[11] / f / 1e3, ps[12] / f, ps[13] / f, ps[8] / f);
    }
    for (auto h : hs) fx_graph_executor_free(h);
    if (r > 0) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / adds.size() / H);
  }
  std::sort(us.begin(), us.end());
  std::printf("{\"adds\": %zu, \"reps\": %d, \"handles\": %d, \"new_us\": %.1f, \"us_per_add_median\": %.3f, "
              "\"us_per_add_min\": %.3f, \"order\": [",
              adds.size(), reps, H, new_us, us[us.size() / 2], us[0]);
  for (size_t i = 0; i < order.size(); ++i) std::printf(i ? ", %u" : "%u", order[i]);
  std::printf("]}\n");
  return 0;
}
