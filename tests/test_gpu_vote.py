"""GPU parity of the reference-mode vote kernel (k_vote.hip) against the oracle
restatement of scheduler/scheduler.go:248-394.  Bit-exact: best node and all
six winners per pod."""
import json
import os

import numpy as np
import pytest

import oracle
from util import all_perms, random_snapshot, stack_snapshots

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_known_answers(engine):
    for c in load("vote_kat.json")["cases"]:
        engine.upload_snapshot({k: np.array(v) for k, v in c["metrics"].items()})
        best, win = engine.score_reference(1, c["order1"], c["order2"])
        assert best[0] == c["best"], c["name"]
        assert win[0].tolist() == c["winners"], c["name"]


def test_random_golden(engine):
    for c in load("vote_random.json")["cases"]:
        engine.upload_snapshot({k: np.array(v) for k, v in c["metrics"].items()})
        best, win = engine.score_reference(1, c["order1"], c["order2"])
        assert best[0] == c["best"] and win[0].tolist() == c["winners"]


@pytest.mark.parametrize("ties", [False, True])
def test_every_go_map_order_n5(engine, ties):
    """All 120 x 720 (order1, order2) pairs at N = 5 -- every behaviour the Go
    binary could show for one metrics snapshot -- as 86,400 snapshots with
    per-snapshot orders."""
    rng = np.random.default_rng(21 + ties)
    m = random_snapshot(rng, 5, ties)
    p1, p2 = all_perms(5), all_perms(6)
    o1 = np.repeat(p1, len(p2), axis=0)
    o2 = np.tile(p2, (len(p1), 1))
    S = len(o1)
    snap = {k: np.tile(np.asarray(v), (S, 1)) for k, v in m.items()}
    engine.upload_snapshot(snap)
    engine.upload_orders(o1, o2)
    best, win = engine.score_reference(S)
    want_best, want_win = oracle.vote_batch(snap, o1, o2)
    assert (best == want_best).all()
    assert (win == want_win).all()


@pytest.mark.parametrize("n,S", [(1, 64), (2, 64), (10, 500), (333, 300), (1000, 200), (10000, 24)])
def test_random_sizes_shared_order(engine, n, S):
    rng = np.random.default_rng(n)
    snap = stack_snapshots([random_snapshot(rng, n, ties=(s % 3 == 0)) for s in range(S)])
    o1 = rng.permutation(n).astype(np.int32)
    o2 = rng.permutation(n + 1).astype(np.int32)
    engine.upload_snapshot(snap)
    best, win = engine.score_reference(S, o1, o2)
    want_best, want_win = oracle.vote_batch(snap, o1, o2)
    assert (best == want_best).all() and (win == want_win).all()


def test_pod_snapshot_gather_and_orders_per_snapshot(engine):
    rng = np.random.default_rng(99)
    n, S, P = 61, 40, 257
    snap = stack_snapshots([random_snapshot(rng, n, ties=True) for _ in range(S)])
    o1 = np.stack([rng.permutation(n) for _ in range(S)]).astype(np.int32)
    o2 = np.stack([rng.permutation(n + 1) for _ in range(S)]).astype(np.int32)
    ps = rng.integers(0, S, P).astype(np.int32)
    engine.upload_snapshot(snap)
    engine.upload_orders(o1, o2)
    best, win = engine.score_reference(P, pod_snapshot=ps)
    want_best, want_win = oracle.vote_batch(snap, o1, o2, ps)
    assert (best == want_best).all() and (win == want_win).all()


@pytest.mark.parametrize("S", [1, 7])
def test_orders_per_pod(engine, S):
    """nas_upload_pod_orders: every pod of a batch carries its own map orders
    over a shared snapshot (host scheduler.cpp vote(): ONE scrape, P pods)."""
    rng = np.random.default_rng(50 + S)
    n, P = 83, 300
    snaps = [random_snapshot(rng, n, ties=True) for _ in range(S)]
    o1 = np.stack([rng.permutation(n) for _ in range(P)]).astype(np.int32)
    o2 = np.stack([rng.permutation(n + 1) for _ in range(P)]).astype(np.int32)
    ps = rng.integers(0, S, P).astype(np.int32)
    engine.upload_snapshot(stack_snapshots(snaps))
    engine.upload_pod_orders(o1, o2)
    best, win = engine.score_reference(P, pod_snapshot=ps)
    for p in range(P):
        b, w, _ = oracle.vote(snaps[ps[p]], o1[p], o2[p])
        assert best[p] == b and win[p].tolist() == list(w), p
    from kubernetesnetawarescheduler_amd import NasError
    with pytest.raises(NasError):  # the sets belong to exactly P pods
        engine.score_reference(P - 1, pod_snapshot=ps[:-1])
    if S == 1:  # per-snapshot sets again replace them
        engine.upload_orders(o1[0], o2[0])
        best, _ = engine.score_reference(P, pod_snapshot=ps)
        assert (best == oracle.vote(snaps[0], o1[0], o2[0])[0]).all()


def test_edge_values(engine):
    """NaN metrics, signed zeros, sentinel-equal values, all-zero (Atoi failure) rows."""
    n = 7
    base = {"cpu": [np.nan, -0.0, 0.0, 99999999999.0, 1e9, 1e9, np.nan],
            "mem": [np.nan] * n,
            "rx": [99999999999, 0, 0, 5, 5, 99999999998, 0],
            "tx": [99999999999] * n,
            "bw": [np.nan, -0.0, 0.0, 1e300, 1e300, np.inf, -1.0],
            "disk": [0, 999, 998, 0, 1, 1, 0]}
    rng = np.random.default_rng(1)
    S = 200
    snap = {k: np.tile(np.asarray(v), (S, 1)) for k, v in base.items()}
    o1 = np.stack([rng.permutation(n) for _ in range(S)]).astype(np.int32)
    o2 = np.stack([rng.permutation(n + 1) for _ in range(S)]).astype(np.int32)
    engine.upload_snapshot(snap)
    engine.upload_orders(o1, o2)
    best, win = engine.score_reference(S)
    want_best, want_win = oracle.vote_batch(snap, o1, o2)
    assert (best == want_best).all() and (win == want_win).all()


def test_bad_orders_rejected(engine):
    from kubernetesnetawarescheduler_amd import NasError
    engine.upload_snapshot(random_snapshot(np.random.default_rng(0), 5))
    with pytest.raises(NasError):
        engine.score_reference(1, [0, 1, 2, 3, 3], [0, 1, 2, 3, 4, 5])
    with pytest.raises(NasError):
        engine.score_reference(1, [0, 1, 2, 3, 4], [0, 1, 2, 3, 4, 4])


def test_synthetic_full_width_sampled(engine):
    """Device-generated 10k-node snapshots (the bench workload shape), sampled
    pods checked against the oracle on the bytes read back from HBM."""
    n, S = 10000, 512
    engine.synth_snapshots(0x4E4153, n, S)
    rng = np.random.default_rng(3)
    o1 = rng.permutation(n).astype(np.int32)
    o2 = rng.permutation(n + 1).astype(np.int32)
    best, win = engine.score_reference(S, o1, o2)
    for s in rng.choice(S, 24, replace=False):
        snap = engine.read_snapshot(int(s))
        b, w, _ = oracle.vote(snap, o1, o2)
        assert best[s] == b and win[s].tolist() == list(w)
