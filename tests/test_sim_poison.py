"""The all-on-chip simulator must not read register state it never wrote.

Before every launch the register file of every SIMD is filled with known
garbage (tests/poison/poison.hip): tagged values (VGPR / AGPR r of lane l
holds tag << 24 | r << 6 | l) under two tags, and zeros.  A read of a register
the kernel never wrote (or read too early: round 3's k_sim read the VGPR
holding its parameters one wait state too soon, so it saw the register's
previous contents) then returns that garbage instead of whatever an earlier
kernel happened to leave there.  The big tagged values and the zeros push such
a read to opposite sides of every count and bound: the round-3 failure read
the per-client command count, which zero turns into "no commands" (a client
never starts).  The cases are the simulator parity cases of test_sim_gpu.py
whose results once changed with the compiler's instruction schedule
(test_region_subsets_n7, test_no_gc) plus the configs[0] / configs[1] shapes;
each must stay bit-exact vs the oracle under every fill.  Run it on another
build of the library with FX_LIB=... (e.g. the iterative-ILP k_sim variant,
`make variant`)."""
import ctypes
import itertools
import os

import numpy as np
import pytest

from fantoch_amd import _lib
from fantoch_amd import sim as S
from oracle import oracle_lib as O
from test_sim_gpu import assert_instance_parity, planet, to_oracle

pytestmark = pytest.mark.gpu

POISON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "poison", "build", "libpoison.so")
FILLS = ((1, 0x5A), (1, 0xC3), (4, 0))  # (mode, tag): tagged vector registers twice, zeroed
_LIB = None


def poison_lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(POISON)
        _LIB.fx_dbg_poison_mode.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    return _LIB


def poisoner(mode, tag):
    def before(stream):
        # 4,096 single-wave workgroups of 512 registers: every SIMD of the
        # 256 CUs runs at least one, so every register line is overwritten
        assert poison_lib().fx_dbg_poison_mode(tag, 4096, mode, stream) == 0
    return before


def n7_specs():
    pl = planet()
    subsets = list(itertools.combinations(range(pl.R), 7))[::9973][:12]
    return [S.spec(S.ATLAS, 7, 1 + (i % 2), list(sub), list(sub), commands_per_client=60,
                   conflict_rate=10, seed=5, instance=i) for i, sub in enumerate(subsets)]


def no_gc_specs():
    regs = planet().ids(S.GCP5[:5])
    return [S.spec(S.EPAXOS, 5, 2, regs, regs, commands_per_client=80, conflict_rate=50,
                   gc_interval_ms=0, seed=4, instance=i) for i in range(4)]


def sweep_specs():
    regs = planet().ids(S.GCP5[:5])
    return [S.spec(S.EPAXOS, 5, 2, regs, regs, commands_per_client=100, conflict_rate=c,
                   seed=77, instance=i) for i, c in enumerate([0, 2, 10, 50, 100] * 4)]


def config0_specs():
    regs = planet().ids(S.GCP5[:3])
    return [S.spec(S.ATLAS, 3, 1, regs, regs, commands_per_client=300, conflict_rate=c, seed=1, instance=i)
            for i, c in enumerate((2, 50))]


CASES = {"n7": n7_specs, "no_gc": no_gc_specs, "sweep_n5": sweep_specs, "config0": config0_specs}


def describe(res, specs, tag):
    """Where a failed instance stopped, and any tagged garbage in its outputs."""
    out = []
    for i in range(len(specs)):
        if int(res.err[i]):
            out.append("instance %d err %d site %d events %d end %d" % (
                i, int(res.err[i]), int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE]), res.events(i), res.end_ms(i)))
        for p, e in enumerate(res.executed(i)):
            g = e[(e >> 24) == tag]
            if len(g):
                out.append("instance %d process %d: poisoned values %s (register %s lane %s)" % (
                    i, p, [hex(int(x)) for x in g[:4]], [int(x >> 6) & 0x1FF for x in g[:4]],
                    [int(x) & 63 for x in g[:4]]))
    return "; ".join(out)


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("generic", [False, True])
def test_poisoned_registers_do_not_change_results(case, generic):
    specs = CASES[case]()
    orc = O.sim_batch([to_oracle(s) for s in specs], threads=8)
    for mode, tag in FILLS:
        res = S.run(specs, planet(), generic=generic, before_launch=poisoner(mode, tag))
        bad = [(i, int(e)) for i, e in enumerate(res.err) if e]
        assert not bad, "tag %#x: %s" % (tag, describe(res, specs, tag))
        for i, (s, o) in enumerate(zip(specs, orc)):
            try:
                assert_instance_parity(res, i, s, o)
            except AssertionError as e:
                raise AssertionError("tag %#x instance %d: %s; %s" % (tag, i, e, describe(res, specs, tag)))
        assert np.array_equal(res.chain, sum(o["chain"] for o in orc)[:res.chain.shape[0]])
