"""Full-size C3 (10k nodes x 100k pods, the bench's device-generated cluster)
checked through size-independent properties of the sequential greedy
(the oracle's extended-mode semantics):
  * capacity conservation: final free = initial free - requests of the pods
    placed on each node, every resource >= 0;
  * sampled pods are exactly sequential-greedy: recompute the capacity at the
    pod's own turn from the placements before it, then the pod's node must be
    the (cost, node)-smallest fitting node of its oracle cost row, with the
    same integer score (unschedulable iff nothing fits);
  * a second pass returns identical placements."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
N, P, SEED = 10000, 100000, 0x4E4153


@pytest.mark.parametrize("profile", [0, 1])
def test_c3_fullsize_properties(engine, profile):
    # profile 1: SURVEY.md §8(d)'s full-range operands (configs.C3_fullrange)
    engine.synth_cluster(SEED, N, P, "i8", peers=8, profile=profile)
    engine.reset_capacity()
    node, _, score = engine.place()
    _, L, cap0, req = engine.read_inputs(0, 0, want_L=True)
    free = engine.get_capacity()

    placed = node >= 0
    used = np.zeros((N, 3), np.int64)
    np.add.at(used, node[placed], req[placed].astype(np.int64))
    assert (cap0.astype(np.int64) - used == free).all()
    assert (free >= 0).all()
    assert (node >= -1).all() and (node < N).all()

    L32 = L.astype(np.int32)
    rng = np.random.default_rng(7)
    pods = np.concatenate([[0, P - 1], rng.choice(P, 10, replace=False)])
    for p in pods.tolist():
        before = placed.copy()
        before[p:] = False
        u = np.zeros((N, 3), np.int64)
        np.add.at(u, node[before], req[before].astype(np.int64))
        turn = cap0.astype(np.int64) - u                      # capacity at p's turn
        WA, _, _, _ = engine.read_inputs(p, 1, want_L=False)
        cost = WA.astype(np.int32) @ L32                        # (1, N), exact in int32
        fits = (req[p].astype(np.int64) <= turn).all(axis=1)
        if not fits.any():
            assert node[p] == oracle.EMPTY, p
            continue
        cand = np.where(fits, cost[0].astype(np.int64), np.iinfo(np.int64).max)
        want = int(np.argmin(cand))                             # lowest node among ties
        assert node[p] == want, (p, node[p], want)
        assert score[p] == cost[0, want], p

    t1 = engine.timings()
    engine.reset_capacity()
    again, _, score2 = engine.place()
    t2 = engine.timings()
    diff = np.nonzero((again != node) | (score2 != score))[0]
    assert len(diff) == 0, (len(diff), diff[:8].tolist(), node[diff[:4]].tolist(),
                            again[diff[:4]].tolist(), t1, t2)
