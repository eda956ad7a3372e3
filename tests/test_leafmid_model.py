"""The queue of cg_large.hip lg_pcl_leafmid (the leaves and their mid ranges in one launch),
modelled on the CPU: workgroups take leaf tickets, and a leaf publishes its mid ranges one by one
(slot reservation on the shared count, then the entry) and counts itself done after its last
reservation returned; workgroups without a leaf take mid tickets and poll their entry, leaving
when every leaf is done and no slot at or past their ticket was reserved. A random scheduler
interleaves the workgroups' steps, with fewer workgroups than tickets and workgroups that start
late. Every published mid range must be processed exactly once, no workgroup may leave while a
range at its ticket can still appear, and the launch must drain."""
import random

import pytest


def leafmid(n_leaves, mids_per_leaf, grid, seed, late=0.3):
    rng = random.Random(seed)
    leaf_tk = [0]
    mid_tk = [0]
    leaves_done = [0]
    count = [0]                     # S.pq[PQ_MIDS]: slots reserved
    mq = {}                         # slot -> entry (absent: not yet published)
    processed = []
    exits = []

    def workgroup(wid):
        while True:                                  # leaves, by ticket
            b = leaf_tk[0]
            leaf_tk[0] += 1
            yield
            if b >= n_leaves:
                break
            for j in range(mids_per_leaf[b]):        # the leaf's levels, then PqfMid per range
                yield
                q = count[0]                         # atomicAdd: the slot
                count[0] += 1
                yield                                # (the entry store lands later)
                mq[q] = (b, j)
            yield
            leaves_done[0] += 1                      # after every reservation of the leaf returned
        while True:                                  # mid ranges, by ticket
            m = mid_tk[0]
            mid_tk[0] += 1
            while True:
                yield
                if m in mq:
                    processed.append(mq[m])
                    break
                if leaves_done[0] >= n_leaves and count[0] <= m:
                    # nothing can be published at m any more
                    assert all(k < m for k in mq), "left while a range at its ticket existed"
                    exits.append(wid)
                    return
        # (unreachable)

    gens = {}
    pending = list(range(grid))
    rng.shuffle(pending)
    steps = 0
    while pending or gens:
        if pending and (not gens or rng.random() < late):
            w = pending.pop()
            gens[w] = workgroup(w)
        w = rng.choice(list(gens))
        try:
            next(gens[w])
        except StopIteration:
            del gens[w]
        steps += 1
        assert steps < 5_000_000, "no progress"
    return processed, exits, count[0]


@pytest.mark.parametrize("n_leaves,grid,seed", [(0, 4, 1), (1, 1, 2), (5, 3, 3), (40, 16, 4), (40, 64, 5),
                                                (200, 8, 6)])
def test_leafmid_queue_drains_and_serves_every_range(n_leaves, grid, seed):
    rng = random.Random(seed)
    mids = [rng.choice([0, 0, 1, 2, 5, 9]) for _ in range(n_leaves)]
    processed, exits, reserved = leafmid(n_leaves, mids, grid, seed)
    want = sorted((b, j) for b in range(n_leaves) for j in range(mids[b]))
    assert sorted(processed) == want and reserved == len(want)
    assert len(processed) == len(set(processed))
    assert len(exits) == grid


def test_leafmid_many_interleavings():
    for seed in range(60):
        rng = random.Random(seed)
        n = rng.randint(0, 30)
        mids = [rng.randint(0, 6) for _ in range(n)]
        processed, exits, _ = leafmid(n, mids, rng.randint(1, 24), seed, late=rng.random())
        assert sorted(processed) == sorted((b, j) for b in range(n) for j in range(mids[b]))
