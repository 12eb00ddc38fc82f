"""Committed golden vectors (tests/golden/, written by make_golden.py).

CPU: the oracle and the host stream generator still reproduce every vector.
GPU: the HIP path (tiered batch executor and the single-stream GraphExecutor)
reproduces them bit-exactly without consulting the oracle at all."""
import glob
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden as G  # noqa: E402
from fantoch_amd import _lib  # noqa: E402
from fantoch_amd import streams as fs  # noqa: E402

NPZ = sorted(glob.glob(os.path.join(HERE, "golden", "synth_*.npz")))
KATS = json.load(open(os.path.join(HERE, "golden", "kats.json")))


def load(path):
    with np.load(path) as z:  # allow_pickle=False (default)
        return {k: z[k] for k in z.files}


def ids(paths):
    return [os.path.basename(p)[6:-4] for p in paths]


def test_every_synth_case_has_a_vector():
    assert sorted(ids(NPZ)) == sorted(G.SYNTH)


@pytest.mark.parametrize("path", NPZ, ids=ids(NPZ))
def test_host_generator_reproduces_inputs(path):
    g = load(path)
    planes = fs.synth_host(fs.synth_params(**G.params_from_array(g["params"])))
    assert G.planes_digest(planes) == str(g["digest"])


@pytest.mark.parametrize("path", NPZ, ids=ids(NPZ))
def test_oracle_reproduces_vector(path):
    g = load(path)
    _, exp = G.synth_expected(G.params_from_array(g["params"]))
    for k in ("order", "release", "nexec", "err", "chain", "delay"):
        assert np.array_equal(exp[k], g[k]), k


def _per_key(n, args_json):
    args = [(tuple(d), keys, {tuple(x) for x in deps}) for d, keys, deps in args_json]
    return G._per_key(n, args)


def test_kats_json_matches_oracle():
    c = KATS["cycle"]
    assert _per_key(c["n"], c["args"]) == c["per_key"]
    for name in ("regression_1", "regression_2"):
        r = KATS[name]
        assert _per_key(r["n"], r["order_a"]) == r["per_key_a"]
        assert _per_key(r["n"], r["order_b"]) == r["per_key_b"]
        assert r["per_key_a"] != r["per_key_b"]  # mod.rs:822, 892
    for case in KATS["random"]:
        assert _per_key(2, case["args"]) == case["per_key"]


# ----------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("path", NPZ, ids=ids(NPZ))
def test_gpu_matches_vector(gpu, path):
    from fantoch_amd import device as fd
    g = load(path)
    planes = fs.synth_host(fs.synth_params(**G.params_from_array(g["params"])))
    res = fd.run_batch(planes, nbins_chain=G.NBINS_CHAIN, nbins_delay=G.NBINS_DELAY)
    assert res.status == _lib.FX_OK
    o, r = G.compact(planes, res.order, res.release, res.nexec)
    assert np.array_equal(res.err, g["err"])
    assert np.array_equal(res.nexec, g["nexec"])
    assert np.array_equal(o, g["order"])
    assert np.array_equal(r, g["release"])
    assert np.array_equal(res.chain, g["chain"])
    assert np.array_equal(res.delay, g["delay"])


@pytest.mark.gpu
def test_gpu_executor_matches_kats(gpu):
    from test_gpu_parity import make_gpu as Ex
    import kat_shapes as K

    def per_key(n, args_json):
        args = [(tuple(d), keys, {tuple(x) for x in deps}) for d, keys, deps in args_json]
        res = K.check_termination(Ex, n, args)
        return {k: [list(d) for d in v] for k, v in sorted(res.items())}

    c = KATS["cycle"]
    assert per_key(c["n"], c["args"]) == c["per_key"]
    for name in ("regression_1", "regression_2"):
        r = KATS[name]
        assert per_key(r["n"], r["order_a"]) == r["per_key_a"]
        assert per_key(r["n"], r["order_b"]) == r["per_key_b"]
    for case in KATS["random"]:
        assert per_key(2, case["args"]) == case["per_key"]
