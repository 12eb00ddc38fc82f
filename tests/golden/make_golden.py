"""Writes the committed golden vectors under tests/golden/.

The reference (Rust, fantoch @ 2025-02-13) cannot be built or run here (no
cargo/rustc, no vendored crates — SURVEY.md §8c), so the vectors come from the
CPU oracle (oracle/graph_oracle.cpp) *after* it passes the reference's own
known-answer tests (tests/test_oracle_kat.py: graph/mod.rs:714-1348,
histogram.rs:354-463).  They freeze the oracle's outputs so that the GPU path
is checked against data that does not move with later oracle edits, and
tests/test_golden.py re-derives them on every CPU run.

    python tests/golden/make_golden.py      # rewrites the .npz/.json files

Contents
  synth_<name>.npz  seeded synthetic commit streams (fx_synth, host generator):
                    params, sha256 of the input planes, and the expected
                    order rows (Σnexec words, stream-major), release rows
                    (S×steps, compact), nexec, err, ChainSize/ExecutionDelay bins.
  kats.json         the reference's graph-test shapes with the per-key execution
                    orders check_termination (mod.rs:1045-1113) produces.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from fantoch_amd import _lib  # noqa: E402
from fantoch_amd import streams as fs  # noqa: E402
from oracle import oracle_lib  # noqa: E402
import kat_shapes as K  # noqa: E402

NBINS_CHAIN = 64
NBINS_DELAY = 2048

SYNTH = {
    "n5_mix": dict(seed=101, n=5, instances=20, cmds=60, window=8, cycle_pct=30),
    "n3_cycles": dict(seed=102, n=3, instances=30, cmds=50, window=6, cycle_pct=50),
    "n7": dict(seed=103, n=7, instances=10, cmds=40, window=8, cycle_pct=30),
    "deep_pending": dict(seed=104, n=5, instances=6, cmds=150, window=30, cycle_pct=70,
                         conflicts=(100,)),
    "no_pending": dict(seed=105, n=5, instances=10, cmds=40, window=0, cycle_pct=0),
    "ragged_n2": dict(seed=106, n=2, instances=33, cmds=37, window=5, cycle_pct=40),
    # SURVEY §8(d) S5's shape (configs[4]): per-key chains over a key pool plus cycles
    "s5_pool": dict(seed=107, n=5, instances=4, cmds=400, window=8, cycle_pct=30, horizon=96, key_pool=50),
}


def planes_digest(planes):
    h = hashlib.sha256()
    for a in (planes.dot, planes.hdr, planes.deps):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def compact(planes, order, release, nexec):
    """Tiled planes -> (order rows stream-major, release S×steps)."""
    S, steps = planes.S, planes.steps
    rows = [order[_lib.index(np.arange(int(nexec[s])), s, steps)] for s in range(S)]
    o = np.concatenate(rows) if rows else np.zeros(0, np.uint32)
    r = np.stack([release[_lib.index(np.arange(steps), s, steps)] for s in range(S)])
    return o.astype(np.uint32), r.astype(np.uint32)


def hists(planes, order, release, nexec, nbc=NBINS_CHAIN, nbd=NBINS_DELAY):
    """ChainSize / ExecutionDelay bins (save_scc, graph/mod.rs:488-523) from the
    order and release planes; arrival time t_ms is the low 24 header bits."""
    chain = np.zeros(nbc, np.uint64)
    delay = np.zeros(nbd, np.uint64)
    t = planes.hdr & 0xFFFFFF
    for s in range(planes.S):
        k = int(nexec[s])
        if not k:
            continue
        o = order[_lib.index(np.arange(k), s, planes.steps)]
        rec = (o & 0x7FFFFFFF).astype(np.int64)
        start = (o & _lib.FX_ORDER_SCC_START) != 0
        rel = release[_lib.index(rec, s, planes.steps)].astype(np.int64)
        d = t[_lib.index(rel, s, planes.steps)].astype(np.int64) - t[_lib.index(rec, s, planes.steps)]
        np.add.at(delay, np.minimum(d, nbd - 1), 1)
        starts = np.flatnonzero(start)
        sizes = np.diff(np.append(starts, k))
        np.add.at(chain, np.minimum(sizes, nbc - 1), 1)
    return chain, delay


def synth_params_array(case):
    conf = list(case.get("conflicts", (0, 2, 10, 50, 100)))
    keys = ["seed", "n", "instances", "cmds", "window", "cycle_pct"]
    extra = [case["horizon"], case["key_pool"]] if "key_pool" in case else []  # (older vectors: none)
    return np.array([case[k] for k in keys] + [len(conf)] + conf + extra, np.int64)


def params_from_array(a):
    seed, n, instances, cmds, window, cycle_pct, nc = (int(x) for x in a[:7])
    conf = tuple(int(x) for x in a[7:7 + nc])
    out = dict(seed=seed, n=n, instances=instances, cmds=cmds, window=window,
               cycle_pct=cycle_pct, conflicts=conf)
    if len(a) >= 9 + nc:
        out.update(horizon=int(a[7 + nc]), key_pool=int(a[8 + nc]))
    return out


def synth_expected(case):
    planes = fs.synth_host(fs.synth_params(**case))
    order, release, nexec, err = oracle_lib.batch_execute(planes, threads=8)
    o, r = compact(planes, order, release, nexec)
    chain, delay = hists(planes, order, release, nexec)
    return planes, dict(params=synth_params_array(case), order=o, release=r, nexec=nexec,
                        err=err, chain=chain, delay=delay)


class _OracleExec:
    def __init__(self, n):
        self.g = oracle_lib.Graph(1, n)

    def handle_add(self, dot, deps, t):
        self.g.handle_add(dot, sorted(deps), t)

    def drain(self):
        return [d for d, _, _ in self.g.drain()]


def _per_key(n, args):
    res = K.check_termination(_OracleExec, n, args)
    return {k: [list(d) for d in v] for k, v in sorted(res.items())}


def _args_json(args):
    return [[list(d), keys, sorted(list(x) for x in deps)] for d, keys, deps in args]


def kats():
    out = {"source": "fantoch_ps/src/executor/graph/mod.rs (tests) restated in tests/kat_shapes.py"}
    out["simple"] = {"n": K.SIMPLE["n"], "adds": [[list(d), [list(x) for x in deps]]
                                                  for d, deps in K.SIMPLE["adds"]],
                     "ready_after": [[list(x) for x in r] for r in K.SIMPLE["ready_after"]]}
    out["cycle"] = {"n": K.CYCLE["n"], "args": _args_json(K.CYCLE["args"]),
                    "per_key": _per_key(K.CYCLE["n"], K.CYCLE["args"])}
    for name, f in (("regression_1", K.REGRESSION_1), ("regression_2", K.REGRESSION_2)):
        out[name] = {"n": f["n"], "order_a": _args_json(f["order_a"]),
                     "order_b": _args_json(f["order_b"]),
                     "per_key_a": _per_key(f["n"], f["order_a"]),
                     "per_key_b": _per_key(f["n"], f["order_b"])}
    out["random"] = [{"args": _args_json(a), "per_key": _per_key(2, a)} for a in K.random_cases()]
    f = K.SCCS_MISSING
    out["sccs_found_and_missing_dep"] = {
        "n": f["n"], "process_id": f["process_id"], "executed": f["executed"],
        "root": [list(f["root"][0]), [list(x) for x in f["root"][1]]],
        "indexed": [[list(d), [list(x) for x in deps]] for d, deps in f["indexed"]],
        "missing": [list(x) for x in f["missing"]],
        "executed_after": [[4, s] for s in range(31, 41)]}
    return out


def main(only=None):
    for name, case in SYNTH.items():
        if only and name not in only:
            continue
        planes, exp = synth_expected(case)
        np.savez_compressed(os.path.join(HERE, "synth_%s.npz" % name), digest=planes_digest(planes),
                            **exp)
        print(name, planes.S, planes.steps, int(exp["nexec"].sum()))
    with open(os.path.join(HERE, "kats.json"), "w") as fh:
        json.dump(kats(), fh, indent=1, sort_keys=True)


if __name__ == "__main__":  # python make_golden.py [case ...]: only those vectors (and kats.json)
    main(sys.argv[1:] or None)
