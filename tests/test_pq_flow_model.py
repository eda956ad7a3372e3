"""lg_pq_flow's queue and bookkeeping, modelled tile by tile on the CPU (tests/pqf_model.py):
entries, look-back, range words, inline and deferred swaps, the children's slots, `pend` and
the leaf tasks, under random interleavings of the workgroups' steps and small grids (ranges with
more tiles than workgroups take the deferred path). The result must be libstdc++'s std::sort
permutation (pb_model.std_sort) and the launch must drain with every ticket served."""
import random

import pytest

from pb_model import std_sort
from pqf_model import flow_sort


def _records(n, keys, seed):
    rng = random.Random(seed)
    return [(rng.randrange(keys) << 32) | i for i in range(n)]


@pytest.mark.parametrize("n,keys,grid,leaves,seed", [
    (3000, 400, 4, False, 1),        # one cut: two leaves
    (9000, 2000, 6, False, 2),       # children ranges, one of them cut again
    (20000, 50, 5, False, 3),        # tie-heavy: long equal runs, uneven cuts
    (20000, 20000, 3, True, 4),      # leaves as tasks; ranges of more tiles than workgroups
    (40000, 5000, 16, True, 5),
    (49128, 5400, 12, False, 6),     # C5's index_vector length
])
def test_flow_model_equals_std_sort(n, keys, grid, leaves, seed):
    recs = _records(n, keys, seed)
    got, st = flow_sort(recs, grid=grid, seed=seed, leaves_in_flow=leaves)
    assert got == std_sort(recs)
    assert st["pend"] == 1 and st["ranges"] >= 1


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


@pytest.mark.parametrize("n,keys,seed", [(6000, 900, 21), (14000, 1500, 22)])
def test_flow_model_leaf_and_mid_tasks(n, keys, seed):
    """LG_PQ_MODE 2: leaves sorted inside the launch (pb_model's thread model of the LDS sort),
    their 65-512-record ranges queued as mid tasks with the records handed back through the
    buffer; every output written once, the launch drains with pend at 1."""
    recs = _records(n, keys, seed)
    got, st = flow_sort(recs, grid=6, seed=seed, leaves_in_flow=True, model_mids=True)
    assert got == std_sort(recs) and st["pend"] == 1
