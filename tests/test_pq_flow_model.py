"""lg_pq_flow's queue and bookkeeping, modelled tile by tile on the CPU (tests/pqf_model.py):
entries, look-back, range words, inline and deferred swaps, the children's slots, the
records-in-leaves count and the leaf list, under random interleavings of the workgroups' steps
and small grids (ranges with more tiles than workgroups take the deferred path). The result must be libstdc++'s std::sort
permutation (pb_model.std_sort) and the launch must drain with every ticket served."""
import random

import pytest

from pb_model import std_sort
from pqf_model import flow_sort


def _records(n, keys, seed):
    rng = random.Random(seed)
    return [(rng.randrange(keys) << 32) | i for i in range(n)]


@pytest.mark.parametrize("n,keys,grid,seed", [
    (3000, 400, 4, 1),        # one cut: two leaves
    (9000, 2000, 6, 2),       # children ranges, one of them cut again
    (20000, 50, 5, 3),        # tie-heavy: long equal runs, uneven cuts
    (20000, 20000, 3, 4),     # ranges of more tiles than workgroups: deferred swaps
    (40000, 5000, 16, 5),
    (49128, 5400, 12, 6),     # C5's index_vector length
])
def test_flow_model_equals_std_sort(n, keys, grid, seed):
    recs = _records(n, keys, seed)
    got, st = flow_sort(recs, grid=grid, seed=seed)
    assert got == std_sort(recs)
    assert st["ranges"] >= 1


def test_flow_model_sorted_and_reversed_inputs():
    for recs in ([(i << 32) | i for i in range(12000)], [((12000 - i) << 32) | i for i in range(12000)],
                 [(7 << 32) | i for i in range(6000)]):
        got, _ = flow_sort(recs, grid=4, seed=9)
        assert got == std_sort(recs)


def test_flow_model_depth_cap_route5():
    """Route 5's cap: the children of range 0 go to the leaf list whatever their length."""
    recs = _records(30000, 3000, 11)
    got, st = flow_sort(recs, grid=8, seed=11, depth_cap=1)
    assert got == std_sort(recs) and st["ranges"] == 1
