"""CPU tests of the oracle itself: pinned against the reference's known answers
(SURVEY.md Appendix A), the literal loop against its closed form over every Go
map order at N = 5, and the extended-mode oracle against brute force."""
import json
import os

import numpy as np
import pytest

import oracle
from util import all_perms, cluster, random_snapshot

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("case", load("vote_kat.json")["cases"], ids=lambda c: c["name"])
def test_vote_known_answers(case):
    best, win, scores = oracle.vote(case["metrics"], case["order1"], case["order2"])
    assert best == case["best"]
    assert list(scores) == case["scores"]
    assert list(win) == case["winners"]
    # bestNetBandwith is never assigned (scheduler.go:351-354, :364)
    assert win[4] == oracle.NONE


def test_vote_random_golden():
    for c in load("vote_random.json")["cases"]:
        best, win, scores = oracle.vote(c["metrics"], c["order1"], c["order2"])
        assert best == c["best"] and list(win) == c["winners"] and list(scores) == c["scores"]


@pytest.mark.parametrize("ties", [False, True])
def test_literal_equals_closed_form_every_order(ties):
    """Appendix B restatement == literal loop for all 120 x 720 Go map orders."""
    rng = np.random.default_rng(11 + ties)
    p1, p2 = all_perms(5), all_perms(6)
    for _ in range(2):
        m = random_snapshot(rng, 5, ties)
        for o1 in p1:
            for o2 in p2[rng.choice(len(p2), 48, replace=False)]:
                a = oracle.vote(m, o1, o2)
                b = oracle.vote(m, o1, o2, closed=True)
                assert a[0] == b[0] and list(a[1]) == list(b[1])


def test_vote_nan_and_signed_zero():
    # NaN never wins a strict comparison (Go semantics); -0.0 == +0.0 ties to the first in order
    m = {"cpu": [np.nan, -0.0, 0.0], "mem": [np.nan, np.nan, np.nan], "rx": [3, 3, 3],
         "tx": [99999999999, 99999999999, 5], "bw": [np.nan, -0.0, 1.0], "disk": [0, 999, 998]}
    for o1 in all_perms(3):
        for o2 in all_perms(4)[:6]:
            a = oracle.vote(m, o1, o2)
            b = oracle.vote(m, o1, o2, closed=True)
            assert a[0] == b[0] and list(a[1]) == list(b[1])
            assert a[1][1] == oracle.NONE           # all-NaN memory: no winner
            assert a[1][0] == [x for x in o1 if x in (1, 2)][0]  # first of the signed zeros


def test_vote_rejects_non_permutation():
    m = random_snapshot(np.random.default_rng(0), 5)
    with pytest.raises(ValueError):
        oracle.vote(m, [0, 1, 2, 3, 3], [0, 1, 2, 3, 4, 5], closed=True)


def test_place_golden():
    g = load("place_small.json")
    node, cost, free_after = oracle.place(np.array(g["WA"], np.int8), np.array(g["L"], np.int8),
                                          np.array(g["req"]), np.array(g["free"]), "i8")
    assert node.tolist() == g["node"] and cost.tolist() == g["cost"]
    assert free_after.tolist() == g["free_after"]


def brute_place(WA, L, req, free):
    cost = WA.astype(np.int64) @ L.astype(np.int64)
    free = free.copy()
    out = []
    for p in range(WA.shape[0]):
        fits = np.all(req[p][None, :] <= free, axis=1)
        if not fits.any():
            out.append(-1)
            continue
        c = np.where(fits, cost[p], np.iinfo(np.int64).max)
        n = int(np.argmin(c))  # first minimum = lowest node index
        free[n] -= req[p]
        out.append(n)
    return np.array(out), free


@pytest.mark.parametrize("seed", range(4))
def test_place_matches_brute_force(seed):
    rng = np.random.default_rng(seed)
    WA, L, free, req = cluster(rng, 120, 17, lo=-5, hi=20, cap_scale=0.15)
    node, cost, free_after = oracle.place(WA, L, req, free, "i8")
    bn, bfree = brute_place(WA, L, req, free)
    assert node.tolist() == bn.tolist()
    assert (free_after == bfree).all()
    assert (node == -1).any() and (node >= 0).any()  # both branches exercised


def test_topk_and_commit_reproduce_place():
    """Top-k lists + commit-with-rescore == sequential greedy (the GPU algorithm)."""
    rng = np.random.default_rng(5)
    WA, L, free, req = cluster(rng, 200, 23, cap_scale=0.2)
    want, _, want_free = oracle.place(WA, L, req, free, "i8")
    cost = oracle.cost(WA, L, "i8")
    cur = free.copy()
    got = np.full(len(req), -3, np.int32)
    p = 0
    rounds = 0
    while p < len(req):
        mask = oracle.fit_mask(req[p:], cur)
        nodes, _, cnt = oracle.topk(cost[p:], mask, 4)
        node, _, cur, stop = oracle.commit(nodes, cnt, req[p:], cur)
        got[p:p + stop] = node[:stop]
        p += stop
        rounds += 1
    assert rounds > 1  # the rescore path ran
    assert got.tolist() == want.tolist()
    assert (cur == want_free).all()


def test_topk_matches_sort():
    rng = np.random.default_rng(3)
    WA, L, free, req = cluster(rng, 50, 40, cap_scale=0.1)
    cost = oracle.cost(WA, L, "i8")
    mask = oracle.fit_mask(req, free)
    nodes, cc, cnt = oracle.topk(cost, mask, 4)
    for p in range(50):
        fit = [n for n in range(40) if mask[p, n // 32] >> (n % 32) & 1]
        order = sorted(fit, key=lambda n: (cost[p, n], n))[:4]
        assert cnt[p] == len(order)
        assert nodes[p, :cnt[p]].tolist() == order


def test_gomap_loop_equals_literal_on_its_orders():
    """The Go-map restatement (bench's reference-mode CPU baseline) returns the
    map orders it walked; the literal loop on those orders gives the same
    decision for every pod."""
    rng = np.random.default_rng(5)
    snaps = [random_snapshot(rng, 40, ties=bool(i % 2)) for i in range(30)]
    batch = {k: np.stack([s[k] for s in snaps]) for k in snaps[0]}
    best, o1, o2, (fill, loop) = oracle.vote_gomap(batch)
    assert fill > 0 and loop > 0
    for p, s in enumerate(snaps):
        assert sorted(o1[p].tolist()) == list(range(40))
        assert sorted(o2[p].tolist()) == list(range(41))
        b, _, _ = oracle.vote(s, o1[p], o2[p])
        assert b == best[p], p
