// fx_synth.h — seeded synthetic Atlas/EPaxos commit streams (host + device).
//
// Stands in for the commit streams the simulator's protocols hand to their
// executors (GraphExecutionInfo::Add{dot, cmd, deps}, atlas.rs:449-452,
// epaxos.rs:406-410) until the batched sim loop lands.
// Shape, per instance of n processes with one closed-loop client each
// (fantoch/src/sim/runner.rs:143-163, 1 client/region):
//   * command g = (round j, coordinator s): dot (s, j), g = (j-1)*n + (s-1)
//   * key: the shared conflict key with probability conflict_pct
//     (key_gen.rs:96-128 "CONFLICT" pool of 1), else the client's own key;
//     the draw is a counter-based RNG keyed by (seed, instance, g) — the
//     canonical C6 replacement of rand::thread_rng (key_gen.rs:104,126)
//   * deps: for every source, its latest earlier command on the same key
//     (SequentialKeyDeps latest-per-key, deps/keys/sequential.rs:74-118,
//     unioned over the quorum, quorum.rs:51-69); a concurrent same-round
//     command of a later coordinator is seen instead with probability
//     cycle_pct, which closes 2- and k-cycles (the reason the executor needs
//     Tarjan at all)
//   * delivery: process p receives command g at arrival key A = g + J(p, g),
//     J uniform in [0, window]; commands are delivered in (A, g) order and
//     t_ms = A, so dependencies can arrive after their dependents.
// Every dep refers to a command of the same instance and every command is
// delivered exactly once to each of the n processes, so a complete stream
// executes every command.
#pragma once
#include <stdint.h>

#include "fantoch_amd.h"

#if defined(__HIPCC__)
#define FX_HD __host__ __device__ __forceinline__
#else
#define FX_HD inline
#endif

namespace fx {

enum : uint64_t { PURPOSE_KEY = 1, PURPOSE_CYCLE = 2, PURPOSE_JITTER = 3 };

FX_HD uint64_t mix64(uint64_t x) {  // splitmix64 finalizer
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

FX_HD uint64_t synth_rand(uint64_t seed, uint64_t inst, uint64_t a, uint64_t b) {
  return mix64(mix64(mix64(seed ^ 0x5851F42D4C957F2Dull) + inst) + (a << 8) + b);
}

struct SynthInstance {
  uint64_t seed;
  uint32_t inst;  // global instance index
  uint32_t n, cmds, window, cycle_pct, horizon, conflict, clients, key_pool;
};

FX_HD SynthInstance synth_instance(const fx_synth_params& p, uint32_t local) {
  SynthInstance si;
  si.seed = p.seed;
  si.inst = p.instance_base + local;
  si.n = p.n;
  si.cmds = p.cmds_per_process;
  si.window = p.window;
  si.cycle_pct = p.cycle_pct;
  si.horizon = p.horizon;
  si.clients = p.clients;
  si.key_pool = p.key_pool;
  const uint32_t nc = p.num_conflicts ? p.num_conflicts : 1;
  const uint32_t ci = p.conflict_block ? (si.inst / p.conflict_block) % nc : si.inst % nc;
  si.conflict = p.conflict_pct[ci];
  return si;
}

// Does command g use the shared conflict key?
FX_HD bool synth_conflicts(const SynthInstance& si, uint32_t g) {
  if (si.conflict == 0) return false;
  if (si.conflict >= 100) return true;
  return (uint32_t)(synth_rand(si.seed, si.inst, g, PURPOSE_KEY) % 100u) < si.conflict;
}

// Key id of command g (canonical C7: conflict pool key 0, client key = source).
FX_HD uint32_t synth_key(const SynthInstance& si, uint32_t g) {
  return synth_conflicts(si, g) ? 0u : (g % si.n) + 1u;
}

// C closed-loop clients per process (C >= 2): command g = (seq - 1) n + (s - 1)
// as with one client, seqs of a source grouped in rounds of C concurrent
// commands.  A command sees, per source, the latest same-key command of an
// earlier round (its own source: the previous seq), or with probability
// cycle_pct a random concurrent command of the same round of another source
// (the dense, cyclic graph of BASELINE configs[3]).
FX_HD uint32_t synth_deps_clients(const SynthInstance& si, uint32_t g, uint32_t* out) {
  const uint32_t n = si.n, C = si.clients;
  const uint32_t s = g % n + 1;
  const uint32_t seq = g / n + 1;
  const uint32_t round0 = (seq - 1) / C * C;  // seqs of earlier rounds are <= round0
  const bool shared = synth_conflicts(si, g);
  uint32_t nd = 0;
  for (uint32_t s2 = 1; s2 <= n; ++s2) {
    if (!shared && s2 != s) continue;
    uint32_t dep = 0;
    if (shared && s2 != s && si.cycle_pct > 0 &&
        (uint32_t)(synth_rand(si.seed, si.inst, ((uint64_t)g << 4) | s2, PURPOSE_CYCLE) % 100u) < si.cycle_pct) {
      const uint32_t k2 = (uint32_t)(synth_rand(si.seed, si.inst, ((uint64_t)g << 4) | s2, PURPOSE_JITTER + 1) % C);
      const uint32_t q = round0 + k2 + 1;
      if (synth_conflicts(si, (q - 1) * n + (s2 - 1))) dep = q;
    }
    if (dep == 0) {
      const uint32_t top = s2 == s ? seq - 1 : round0;
      const uint32_t lo = top > si.horizon ? top - si.horizon : 0u;
      for (uint32_t q = top; q > lo; --q)
        if (synth_conflicts(si, (q - 1) * n + (s2 - 1)) == shared) {
          dep = q;
          break;
        }
    }
    if (dep) out[nd++] = FX_PACK_DOT(s2, dep);
  }
  return nd;
}

// S5 (BASELINE configs[4]): per-key chains over a pool of
// key_pool keys.  Command g's key is a C6 draw from the pool; per source, it
// depends on that source's latest command on the same key within `horizon`
// rounds (SequentialKeyDeps latest-per-key, sequential.rs:74-118, unioned over
// the quorum) — except that with probability cycle_pct the pair (s, s2) of
// round j depends on each other (a concurrent pair whose MCollects crossed:
// a 2-cycle; chains through such pairs close longer cycles).
FX_HD uint32_t synth_pool_key(const SynthInstance& si, uint32_t g) {
  return (uint32_t)(synth_rand(si.seed, si.inst, g, PURPOSE_KEY) % si.key_pool);
}
FX_HD bool synth_pair_cycle(const SynthInstance& si, uint32_t j, uint32_t a, uint32_t b) {
  const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
  return si.cycle_pct > 0 &&
         (uint32_t)(synth_rand(si.seed, si.inst, ((uint64_t)j << 8) | (lo << 4) | hi, PURPOSE_CYCLE + 8) % 100u) <
             si.cycle_pct;
}
FX_HD uint32_t synth_deps_pool(const SynthInstance& si, uint32_t g, uint32_t* out) {
  const uint32_t n = si.n;
  const uint32_t s = g % n + 1;
  const uint32_t j = g / n + 1;
  const uint32_t key = synth_pool_key(si, g);
  const uint32_t lo = j > si.horizon ? j - si.horizon : 1u;
  uint32_t nd = 0;
  for (uint32_t s2 = 1; s2 <= n; ++s2) {
    uint32_t dep = 0;
    if (s2 != s && synth_pair_cycle(si, j, s, s2)) {
      dep = j;
    } else {
      // rounds strictly before g in generation order
      for (uint32_t jj = s2 < s ? j : j - 1; jj >= lo && jj >= 1; --jj)
        if (synth_pool_key(si, (jj - 1) * n + (s2 - 1)) == key) {
          dep = jj;
          break;
        }
    }
    if (dep) out[nd++] = FX_PACK_DOT(s2, dep);
  }
  return nd;
}

// Deps of command g, ascending by packed dot (one per source at most).
FX_HD uint32_t synth_deps(const SynthInstance& si, uint32_t g, uint32_t* out) {
  if (si.key_pool > 1) return synth_deps_pool(si, g, out);
  if (si.clients > 1) return synth_deps_clients(si, g, out);
  const uint32_t n = si.n;
  const uint32_t s = g % n + 1;
  const uint32_t j = g / n + 1;
  const bool shared = synth_conflicts(si, g);
  const uint32_t lo = j > si.horizon ? j - si.horizon : 1u;
  uint32_t nd = 0;
  for (uint32_t s2 = 1; s2 <= n; ++s2) {
    if (!shared && s2 != s) continue;  // private key: only the own client's history
    uint32_t dep_round = 0;
    if (shared && s2 > s && si.cycle_pct > 0) {
      // concurrent command of the same round by a later coordinator
      const uint32_t g2 = (j - 1) * n + (s2 - 1);
      if (synth_conflicts(si, g2) &&
          (uint32_t)(synth_rand(si.seed, si.inst, ((uint64_t)g << 4) | s2, PURPOSE_CYCLE) % 100u) <
              si.cycle_pct)
        dep_round = j;
    }
    if (dep_round == 0) {
      uint32_t jj = (s2 < s) ? j : j - 1;  // rounds strictly before g in generation order
      for (; jj >= lo && jj >= 1; --jj) {
        const uint32_t g2 = (jj - 1) * n + (s2 - 1);
        if (synth_conflicts(si, g2) == shared) {
          dep_round = jj;
          break;
        }
        if (jj == 1) break;
      }
    }
    if (dep_round) out[nd++] = FX_PACK_DOT(s2, dep_round);
  }
  return nd;
}

// Arrival key of command g at process p.
FX_HD uint32_t synth_arrival(const SynthInstance& si, uint32_t p, uint32_t g) {
  if (si.window == 0) return g;
  return g + (uint32_t)(synth_rand(si.seed, si.inst, ((uint64_t)g << 4) | p, PURPOSE_JITTER) %
                        (uint64_t)(si.window + 1));
}

// Position of command g in process p's delivery order.
FX_HD uint32_t synth_rank(const SynthInstance& si, uint32_t p, uint32_t g) {
  const uint32_t N = si.n * si.cmds;
  const uint32_t a = synth_arrival(si, p, g);
  const uint32_t w = si.window;
  const uint32_t lo = g > w ? g - w : 0u;
  const uint32_t hi = (g + w < N - 1) ? g + w : N - 1;
  uint32_t rank = lo;
  for (uint32_t g2 = lo; g2 <= hi; ++g2) {
    if (g2 == g) continue;
    const uint32_t a2 = synth_arrival(si, p, g2);
    if (a2 < a || (a2 == a && g2 < g)) ++rank;
  }
  return rank;
}

// Writes command g of instance `local` into the delivery planes of its n
// streams (stream = local * n + p - 1).  Unused dep slots are zeroed.
FX_HD void synth_emit(const fx_synth_params& p, uint32_t local, uint32_t g, uint32_t S, uint32_t steps,
                      uint32_t* dot, uint32_t* hdr, uint32_t* deps) {
  const SynthInstance si = synth_instance(p, local);
  const uint32_t n = si.n;
  uint32_t dv[32];
  const uint32_t nd = synth_deps(si, g, dv);
  const uint32_t d = FX_PACK_DOT(g % n + 1, g / n + 1);
  for (uint32_t proc = 1; proc <= n; ++proc) {
    const uint32_t stream = local * n + (proc - 1);
    const uint32_t rank = synth_rank(si, proc, g);
    const size_t at = fx_index(rank, stream, steps);
    const size_t plane = fx_plane_words(S, steps);
    dot[at] = d;
    hdr[at] = FX_MAKE_HDR(synth_arrival(si, proc, g), nd, FX_KIND_ADD);
    for (uint32_t jd = 0; jd < n; ++jd) deps[jd * plane + at] = jd < nd ? dv[jd] : 0u;
  }
}

}  // namespace fx
