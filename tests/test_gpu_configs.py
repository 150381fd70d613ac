"""BASELINE configs C4 and C5 at their full shapes on one GPU.

C4 -- 50k nodes x 500k pods (the node-sharded config, here at world 1: the
shard is the whole cluster): checked through size-independent properties of
the sequential greedy, as test_gpu_fullsize.py does for C3 -- capacity
conservation, sampled pods exactly sequential-greedy at their own turn
(cost rows from the oracle on the traffic read back exactly), and a repeat
pass identical.

C5 -- 64 independent 5k-node clusters x 5k pods in one batched nas_place:
per-cluster capacity conservation, and every cluster's first 256 pods equal
the sequential oracle on that cluster's own inputs (the oracle over a prefix
depends only on that prefix).
"""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine

pytestmark = pytest.mark.gpu
SEED = 0x4E4153


def conservation(node, req, cap0, free):
    N = cap0.shape[0]
    placed = node >= 0
    used = np.zeros((N, 3), np.int64)
    np.add.at(used, node[placed], req[placed].astype(np.int64))
    assert (cap0.astype(np.int64) - used == free).all()
    assert (free >= 0).all()
    assert (node >= -1).all() and (node < N).all()


def test_c4_fullsize_properties():
    N, P = 50000, 500000
    with Engine(0) as e:
        e.synth_cluster(SEED, N, P, "i8", peers=8)
        node, _, score = e.place()
        free = e.get_capacity()
        _, L, cap0, req = e.read_inputs(0, 0, want_L=True)
        conservation(node, req, cap0, free)
        rng = np.random.default_rng(4)
        pods = np.sort(np.concatenate([[0, 1, P - 1], rng.choice(P, 9, replace=False)]))
        rows = np.concatenate([e.read_inputs(int(p), 1, want_L=False)[0] for p in pods])
        cost = oracle.cost(rows, L, "i8")  # exact int64 rows of the sampled pods
        placed = node >= 0
        for i, p in enumerate(pods.tolist()):
            before = placed.copy()
            before[p:] = False
            u = np.zeros((N, 3), np.int64)
            np.add.at(u, node[before], req[before].astype(np.int64))
            fits = (req[p].astype(np.int64) <= cap0.astype(np.int64) - u).all(axis=1)
            if not fits.any():
                assert node[p] == oracle.EMPTY, p
                continue
            want = int(np.argmin(np.where(fits, cost[i], np.iinfo(np.int64).max)))
            assert node[p] == want, (p, node[p], want)
            assert score[p] == cost[i, want], p
        e.reset_capacity()
        again, _, score2 = e.place()
        assert (again == node).all() and (score2 == score).all()


def test_c5_fullsize_batch():
    B, N, P, S = 64, 5000, 5000, 256
    with Engine(0) as e:
        e.synth_batch(SEED, B, N, P, "i8", peers=8)
        node, _, score = e.place()
        free = e.get_capacity()
    assert node.shape == (B, P) and free.shape == (B, N, 3)
    for b in range(B):
        with Engine(0) as s:  # cluster b of the batch is the single cluster of seed + b
            s.synth_cluster(SEED + b, N, P, "i8", peers=8)
            WA, L, cap0, req = s.read_inputs(0, S, want_L=True)
        conservation(node[b], req, cap0, free[b])
        want, wcost, _ = oracle.place(WA, L, req[:S], cap0, "i8")
        assert node[b, :S].tolist() == want.tolist(), b
        assert score[b, :S].tolist() == wcost.tolist(), b
