"""The predecessors-executor oracle (oracle/pred_oracle.cpp) against the
reference's own PredecessorsGraph tests (pred/mod.rs:419-657), CPU only."""
import itertools

import numpy as np

import pred_shapes as P
from fantoch_amd import _lib
from fantoch_amd import streams as fs
from oracle import oracle_lib as O


def run(streams, n, **kw):
    planes, clo, chi, nd = P.pack_pred_streams(streams, n)
    return planes, O.pred_batch_execute(planes, clo, chi, threads=4, ndeps=nd, **kw)


def orders(planes, order, nexec):
    return [[int(x) & 0x7FFFFFFF for x in order[_lib.index(np.arange(int(nexec[s])), s, planes.steps)]]
            for s in range(planes.S)]


def test_simple():
    planes, (order, release, nexec, err) = run([P.SIMPLE], 2)
    assert err[0] == 0 and nexec[0] == 2
    assert orders(planes, order, nexec)[0] == P.SIMPLE_ORDER  # mod.rs:455-456
    # nothing executes until the second Add (mod.rs:448-449)
    assert list(release[_lib.index(np.arange(2), 0, planes.steps)]) == [1, 1]


def per_key_order(args, perm_order):
    """check_termination (mod.rs:593-655): key -> rifls in execution order."""
    out = {}
    for rec in perm_order:
        dot, _deps, _clock, keys = args[rec]
        for k in keys:
            out.setdefault(k, []).append(dot)
    return out


def test_add_random_permutation_invariance():
    """mod.rs:461-470 + shuffle_it (581-591): every delivery order executes
    every command and gives the same per-key order."""
    for args in P.random_cases():
        perms = list(itertools.permutations(range(len(args))))
        streams = [[(args[i][0], args[i][1], 0, (args[i][2], 1)) for i in perm] for perm in perms]
        planes, (order, release, nexec, err) = run(streams, 2)
        assert np.all(err == 0) and np.all(nexec == len(args))
        got = orders(planes, order, nexec)
        ref = None
        for perm, o in zip(perms, got):
            pk = per_key_order(args, [perm[r] for r in o])
            if ref is None:
                ref = pk
            assert pk == ref


def test_execute_at_commit_and_double_index():
    planes, (order, release, nexec, err) = run([P.SIMPLE], 2, execute_at_commit=True)
    assert orders(planes, order, nexec)[0] == [0, 1]
    dup = [((1, 1), [(2, 1)], 0, (2, 1)), ((1, 1), [], 1, (3, 1))]
    planes, (order, release, nexec, err) = run([dup], 2)
    assert err[0] == _lib.FX_ERR_DOUBLE_INDEX


def test_large_deps_delivery_order_invariance():
    """random_streams (Caesar commits with up to ~100 deps, beyond the 5-bit
    header count: the ndeps plane): 6 delivery orders of one command set all
    execute everything with the same per-key order."""
    base = P.random_streams(11, 1, 3, 30, keys=6)[0]
    rng = np.random.default_rng(5)
    streams = [base]
    for _ in range(5):
        perm = rng.permutation(len(base))
        streams.append([base[i][:2] + (t,) + base[i][3:] for t, i in enumerate(perm)])
    assert max(len(a[1]) for a in base) > 31
    planes, (order, release, nexec, err) = run(streams, 3)
    assert np.all(err == 0) and np.all(nexec == len(base))
    ref = None
    for st, o in zip(streams, orders(planes, order, nexec)):
        pk = {}
        for rec in o:
            for k in st[rec][4]:
                pk.setdefault(k, []).append(st[rec][0])
        ref = ref or pk
        assert pk == ref
