"""Predecessors-executor stream shapes (test infrastructure): the reference's
PredecessorsGraph unit-test fixtures (fantoch_ps/src/executor/pred/mod.rs:
419-657) restated as data with a seeded RNG, and a packer that adds the
packed Caesar clock planes ((seq << 8) | process id, split in two u32
planes) to the ordinary stream planes."""
import itertools
import random

import numpy as np

from fantoch_amd import _lib
from fantoch_amd import streams as fs


def pack_clock(seq, pid):
    return (int(seq) << 8) | int(pid)


def pack_pred_streams(streams, n):
    """streams: lists of (dot, deps, t_ms, (clock_seq, clock_pid)).  Returns
    (planes, clock_lo, clock_hi, ndeps): the header's 5-bit deps count cannot
    hold a Caesar commit's deps, the ndeps plane does."""
    planes = fs.pack_streams([[(a[0], a[1], a[2]) for a in st] for st in streams], n)
    clo = np.zeros(planes.plane, np.uint32)
    chi = np.zeros(planes.plane, np.uint32)
    nd = np.zeros(planes.plane, np.uint32)
    for s, st in enumerate(streams):
        for i, a in enumerate(st):
            c = pack_clock(*a[3])
            at = _lib.index(np.array([i]), s, planes.steps)[0]
            clo[at] = c & 0xFFFFFFFF
            chi[at] = c >> 32
            nd[at] = len(set(a[1]))
    return planes, clo, chi, nd


# mod.rs:419-459 `simple`: n = 2; (1,1) clock (2, 1) deps {(2,1)}; (2,1) clock (1, 2) deps {(1,1)}
SIMPLE = [((1, 1), [(2, 1)], 0, (2, 1)), ((2, 1), [(1, 1)], 0, (1, 2))]
SIMPLE_ORDER = [1, 0]  # cmd_1 then cmd_0


def random_adds(rng, n, events_per_process):
    """mod.rs:472-579: every pair of commands with intersecting keys (2 of
    A..D each) puts the lower-clock one in the other's deps, and the reverse
    with probability 1/2; clocks are a random permutation of 1..N (id 1)."""
    dots = [(p, e) for p in range(1, n + 1) for e in range(1, events_per_process + 1)]
    clocks = list(range(1, len(dots) + 1))
    rng.shuffle(clocks)
    data = {}
    for d in dots:
        keys = ["A", "B", "C", "D"]
        rng.shuffle(keys)
        data[d] = (set(keys[:2]), clocks.pop(), set())
    for left, right in itertools.combinations(dots, 2):
        lk, lc, ld = data[left]
        rk, rc, rd = data[right]
        if lk & rk:
            if lc < rc:
                add_lr, add_rl = True, rng.random() < 0.5
            else:
                add_lr, add_rl = rng.random() < 0.5, True
            if add_lr:
                rd.add(left)
            if add_rl:
                ld.add(right)
    return [(d, sorted(data[d][2]), data[d][1], sorted(data[d][0])) for d in dots]


def random_cases(seed=20250213, iterations=10, n=2, events=3):
    rng = random.Random(seed)
    return [random_adds(rng, n, events) for _ in range(iterations)]


def random_streams(seed, n_streams, n, events, keys=8, window=0, reverse_pct=50):
    """Larger random predecessor streams in the reference's test model
    (random_adds): every conflicting pair (sharing one of 2-of-`keys` keys)
    puts the lower-clock command in the other's deps, the reverse with
    probability reverse_pct; each stream is one random delivery order
    (window > 0: a windowed shuffle of the clock order instead)."""
    rng = random.Random(seed)
    out = []
    for _ in range(n_streams):
        dots = [(p, e) for p in range(1, n + 1) for e in range(1, events + 1)]
        N = len(dots)
        clocks = list(range(1, N + 1))
        rng.shuffle(clocks)
        ks = [set(rng.sample(range(keys), 2)) for _ in dots]
        deps = [set() for _ in dots]
        for a in range(N):
            for b in range(a + 1, N):
                if ks[a] & ks[b]:
                    lo, hi = (a, b) if clocks[a] < clocks[b] else (b, a)
                    deps[hi].add(dots[lo])
                    if rng.random() * 100 < reverse_pct:
                        deps[lo].add(dots[hi])
        if window:
            by_clock = sorted(range(N), key=lambda i: clocks[i])
            key = {i: pos + rng.random() * window for pos, i in enumerate(by_clock)}
            order = sorted(range(N), key=lambda i: key[i])
        else:
            order = list(range(N))
            rng.shuffle(order)
        out.append([(dots[i], sorted(deps[i]), t, (clocks[i], 1), sorted(ks[i])) for t, i in enumerate(order)])
    return out
