"""The reference's graph-executor unit-test shapes (fantoch_ps/src/executor/graph/mod.rs:690-1348),
restated as data + a driver that works with any executor exposing
`handle_add(dot, deps, t)` and `drain()` -> executed dots.  Shared by the
oracle KATs (CPU) and the GPU parity tests."""
import itertools
import random

CONF = "CONF"


def random_adds(rng, n, events_per_process):
    """random_adds (mod.rs:932-1031) with a seeded `random.Random` instead of thread_rng."""
    possible = ["A", "B", "C", "D"]
    dots = [(p, e) for p in range(1, n + 1) for e in range(1, events_per_process + 1)]
    data = {}
    for d in dots:
        rng.shuffle(possible)
        data[d] = (sorted(possible[:2]), set())
    for left, right in itertools.combinations(dots, 2):
        lk, ld = data[left]
        rk, rd = data[right]
        if not set(lk) & set(rk):
            continue
        if left[0] == right[0]:
            if left[1] < right[1]:
                rd.add(left)
            else:
                ld.add(right)
        else:
            r = rng.randrange(3)
            if r == 0:
                ld.add(right)
            elif r == 1:
                rd.add(left)
            else:
                ld.add(right)
                rd.add(left)
    return [(d, data[d][0], data[d][1]) for d in dots]


def check_termination(make_executor, n, args):
    """check_termination (mod.rs:1045-1113): per-key rifl order.  `args` is a
    list of (dot, keys or None, deps); rifl = (dot.source, dot.seq)."""
    ex = make_executor(n)
    keys_of = {}
    all_rifls = set()
    sorted_ = {}
    for t, (dot, keys, deps) in enumerate(args):
        keys = keys if keys else [CONF]
        keys_of[dot] = keys
        assert dot not in all_rifls
        all_rifls.add(dot)
        ex.handle_add(dot, deps, t)
        for d in ex.drain():
            all_rifls.remove(d)
            for k in keys_of[d]:
                sorted_.setdefault(k, []).append(d)
    assert not all_rifls, "the set of all rifls should be empty"
    return sorted_


def shuffle_it(make_executor, n, args):
    total = check_termination(make_executor, n, args)
    for perm in itertools.permutations(args):
        assert check_termination(make_executor, n, list(perm)) == total


SIMPLE = {"n": 2, "adds": [((1, 1), [(2, 1)]), ((2, 1), [(1, 1)])],
          "ready_after": [[], [(1, 1), (2, 1)]]}

CYCLE = {"n": 3, "args": [((1, 1), None, {(3, 1)}), ((2, 1), None, {(1, 1)}),
                          ((3, 1), None, {(2, 1)})]}

REGRESSION_1 = {
    "n": 5,
    "order_a": [((1, 3), None, {(1, 5)}), ((1, 4), None, {(1, 3)}), ((1, 5), None, {(1, 4)}),
                ((1, 1), None, {(1, 4)}), ((1, 2), None, {(1, 4)})],
    "order_b": [((1, 3), None, {(1, 5)}), ((1, 4), None, {(1, 3)}), ((1, 5), None, {(1, 4)}),
                ((1, 2), None, {(1, 4)}), ((1, 1), None, {(1, 4)})],
}

REGRESSION_2 = {
    "n": 3,
    "order_a": [((1, 1), ["A"], set()), ((1, 2), ["B"], set()), ((2, 1), ["A", "B"], {(1, 2)})],
    "order_b": [((1, 2), ["B"], set()), ((2, 1), ["A", "B"], {(1, 2)}), ((1, 1), ["A"], set())],
}

# sccs_found_and_missing_dep (mod.rs:1115-1348)
SCCS_MISSING = {
    "n": 5,
    "process_id": 4,
    "executed": [60, 50, 50, 30, 60],
    "root": ((5, 70), [(1, 60), (2, 50), (3, 50), (4, 40), (5, 61)]),
    "indexed": [((4, s), [(1, 60), (2, 50), (3, 50), (4, s - 1), (5, 60)]) for s in range(31, 41)],
    "missing": [(5, 61)],
}


def random_cases(seed=20250213, iterations=10):
    rng = random.Random(seed)
    return [random_adds(rng, 2, 3) for _ in range(iterations)]
