"""Node-sharded reference mode on CPU (vote row).

The six loops of scheduler.go:334-359 are first-occurrence arg-extrema in
order1, so a snapshot splits over node slices: each slice reduces to a
partial record (include/nas.h nas_vote_partial), and the records merge into
the decision of the literal loop.  Checked here with the oracle's
restatement against the literal Go loop (every slicing of the KATs, random
and tie-heavy snapshots, edge values), and over gloo world_size 2 -- the
all-gather nas_score_reference runs over RCCL on a node-sharded snapshot."""
import json
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from util import random_snapshot, rdv_url

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIELDS = ("cpu", "mem", "rx", "tx", "bw", "disk")


def sliced(m, lo, hi):
    return {f: np.asarray(m[f])[lo:hi] for f in FIELDS}


def sharded_vote(m, order1, order2, cuts):
    """Partials of the slices [cuts[i], cuts[i+1]), merged."""
    parts = [oracle.vote_partial(sliced(m, a, b), a, order1) for a, b in zip(cuts[:-1], cuts[1:])]
    return oracle.vote_from_partials(parts, order1, order2)


def all_cuts(n):
    """Every split of [0, n) into contiguous non-empty slices (n <= 6)."""
    out = []
    for mask in range(1 << (n - 1)):
        cuts = [0] + [i + 1 for i in range(n - 1) if mask >> i & 1] + [n]
        out.append(cuts)
    return out


def edge_snapshot(rng, n):
    """Values the guards and ties care about: NaN, +-0.0, sentinel-equal
    values (never win), disk 0 (excluded) and 999 (= sentinel), duplicates."""
    m = random_snapshot(rng, n, ties=True)
    pick = rng.random((6, n))
    m["cpu"] = np.where(pick[0] < 0.15, np.nan, m["cpu"])
    m["cpu"] = np.where(pick[1] < 0.1, 99999999999.0, m["cpu"])
    m["mem"] = np.where(pick[2] < 0.2, rng.choice([0.0, -0.0], n), m["mem"])
    m["bw"] = np.where(pick[3] < 0.2, rng.choice([np.nan, -0.0, 9e7], n), m["bw"])
    m["rx"] = np.where(pick[4] < 0.15, 99999999999, m["rx"]).astype(np.int64)
    m["disk"] = np.where(pick[5] < 0.15, 999, m["disk"]).astype(np.int64)
    return m


def check(m, o1, o2, cuts):
    want_best, want_win, _ = oracle.vote(m, o1, o2)
    best, win = sharded_vote(m, o1, o2, cuts)
    assert best == want_best and list(win) == list(want_win), (cuts, best, want_best)


def test_kats_every_slicing():
    with open(os.path.join(GOLD, "vote_kat.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        m = {k: np.asarray(v) for k, v in c["metrics"].items()}
        for cuts in all_cuts(len(c["order1"])):
            check(m, c["order1"], c["order2"], cuts)


@pytest.mark.parametrize("kind", ["random", "ties", "edges"])
def test_random_snapshots_random_slicings(kind):
    rng = np.random.default_rng({"random": 1, "ties": 2, "edges": 3}[kind])
    for trial in range(150):
        n = int(rng.integers(1, 40))
        m = (edge_snapshot(rng, n) if kind == "edges"
             else random_snapshot(rng, n, ties=(kind == "ties")))
        o1 = rng.permutation(n).astype(np.int32)
        o2 = rng.permutation(n + 1).astype(np.int32)
        g = int(rng.integers(1, min(n, 8) + 1))
        inner = sorted(rng.choice(np.arange(1, n), g - 1, replace=False).tolist()) if g > 1 else []
        check(m, o1, o2, [0] + inner + [n])


def test_partial_record_of_empty_qualifying_slice():
    # all sentinel / NaN / zero-disk: nothing beats a sentinel -> NOPOS, value 0
    m = {"cpu": np.array([np.nan, 99999999999.0]), "mem": np.array([np.nan, np.nan]),
         "rx": np.array([99999999999, 99999999999]), "tx": np.array([99999999999, 10**12]),
         "bw": np.array([0.0, -1.0]), "disk": np.array([0, 999])}
    rec = oracle.vote_partial(m, 0, [1, 0])
    assert rec == [(0, oracle.NOPOS)] * 6
    best, win = oracle.vote_from_partials([rec], [1, 0], [2, 0, 1])
    # every winner is "none": 3+2+1+1+3+1 = 11 on the none key
    assert best == oracle.NONE and win == [oracle.NONE] * 6


def test_record_merge_is_order_free():
    rng = np.random.default_rng(9)
    for _ in range(50):
        n = 24
        m = random_snapshot(rng, n, ties=True)
        o1 = rng.permutation(n).astype(np.int32)
        o2 = rng.permutation(n + 1).astype(np.int32)
        cuts = [0, 5, 11, 17, n]
        parts = [oracle.vote_partial(sliced(m, a, b), a, o1) for a, b in zip(cuts[:-1], cuts[1:])]
        a = oracle.vote_from_partials(parts, o1, o2)
        b = oracle.vote_from_partials(parts[::-1], o1, o2)
        assert a == b


# ---- gloo world_size 2: the exchange nas_score_reference runs over RCCL ----
WORLD, NODES, SNAPS = 2, 57, 40


def _inputs():
    rng = np.random.default_rng(77)
    snaps = [edge_snapshot(rng, NODES) if s % 3 == 0 else random_snapshot(rng, NODES, s % 2 == 1)
             for s in range(SNAPS)]
    o1 = [rng.permutation(NODES).astype(np.int32) for _ in range(SNAPS)]
    o2 = [rng.permutation(NODES + 1).astype(np.int32) for _ in range(SNAPS)]
    return snaps, o1, o2


def _worker(rank, url, out):
    dist.init_process_group("gloo", init_method=url, rank=rank, world_size=WORLD)
    snaps, o1, o2 = _inputs()  # identical on every rank; each keeps its slice
    lo, hi = rank * NODES // WORLD, (rank + 1) * NODES // WORLD
    mine = np.array([[v for rec in [oracle.vote_partial(sliced(m, lo, hi), lo, o1[s])]
                      for pair in rec for v in pair] for s, m in enumerate(snaps)], np.int64)
    got = [torch.empty(mine.shape, dtype=torch.int64) for _ in range(WORLD)]
    dist.all_gather(got, torch.from_numpy(mine))
    res = []
    for s in range(SNAPS):
        parts = [[(int(g[s, 2 * f]), int(g[s, 2 * f + 1])) for f in range(6)] for g in got]
        best, win = oracle.vote_from_partials(parts, o1[s], o2[s])
        res.append([best] + list(win))
    np.save(out + f".{rank}.npy", np.array(res, np.int64))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_node_sharded_vote(tmp_path):
    out = str(tmp_path / "vote")
    mp.spawn(_worker, args=(rdv_url(tmp_path), out), nprocs=WORLD, join=True)
    r0, r1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert (r0 == r1).all()  # every rank returns the full result
    snaps, o1, o2 = _inputs()
    for s, m in enumerate(snaps):
        best, win, _ = oracle.vote(m, o1[s], o2[s])
        assert r0[s].tolist() == [best] + list(win)
