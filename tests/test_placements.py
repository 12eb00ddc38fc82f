"""configs[2] placement enumeration and sharding (host logic, CPU)."""
import math

import bench_placements as BP


def test_enumeration_is_the_full_sweep_in_canonical_order():
    allp = BP.enumerate_placements(20)
    assert len(allp) == 2 * math.comb(20, 5) + 2 * math.comb(20, 7) == 186_048
    assert allp[0] == (5, 1, (0, 1, 2, 3, 4))
    assert allp[math.comb(20, 5)] == (5, 2, (0, 1, 2, 3, 4))
    assert allp[-1] == (7, 2, tuple(range(13, 20)))
    # lexicographic subsets inside a group (C12: regions in name order)
    g = [p[2] for p in allp if p[0] == 7 and p[1] == 1]
    assert g == sorted(g) and len(set(g)) == len(g)


def test_contiguous_shards_cover_every_placement_once():
    P = 186_048
    for world in (1, 2, 3, 8):
        seen = []
        for r in range(world):
            seen.extend(range(r * P // world, (r + 1) * P // world))
        assert seen == list(range(P))


def test_limit():
    assert len(BP.enumerate_placements(20, limit=1000)) == 1000
