"""Exact network cost on the int8 path with traffic beyond int8.

The north star's cost is cost[p, n] = sum_q W[p, q] * L[node(q), n]: the
aggregated traffic WA[p, m] = sum of W[p, q] over peers q bound on node m is
never saturated.  The engine keeps an int8 plane (entries clamped to
[-128, 127]) as the MFMA operand and adds each pod's few entries outside it
exactly in the cost kernel's epilogue (include/nas.h NAS_DT_I32,
nas_internal.h nas::Ovf).  Every check here is against the oracle on the
UNCLIPPED int64 traffic: candidate lists, integer costs, placements and the
remaining capacity bit-identical.
"""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import NasError, _lib, workloads
from util import cluster

pytestmark = pytest.mark.gpu


def upload(e, WA, L, free, req):
    e.upload_latency(L, "i8")
    e.upload_capacity(free)
    e.upload_pods(req)
    e.upload_traffic(WA, "i8")


def colliding_csr(rng, P, N, peers=8, wmax=127, hot=16):
    """Pods whose peers sit on few nodes: several peers per node, so the
    aggregates exceed int8 (the C3 generator's home-rack collisions)."""
    deg = rng.integers(1, peers + 1, P)
    row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    home = rng.integers(0, max(1, N // hot), P)
    nnz = int(row_ptr[-1])
    rows = np.repeat(np.arange(P), deg)
    node = np.minimum(home[rows] * hot + rng.integers(0, 4, nnz), N - 1).astype(np.int32)
    node[rng.random(nnz) < 0.1] = -1  # unbound peers are skipped
    w = rng.integers(16, wmax + 1, nnz).astype(np.int8)
    return row_ptr, node, w


@pytest.mark.parametrize("P,N,cap", [(2000, 300, 0.2), (5000, 1000, 0.05), (1500, 4096, 1.0)])
def test_csr_colliding_peers_exact(engine, P, N, cap):
    rng = np.random.default_rng(P + N)
    _, L, free, req = cluster(rng, P, N, lo=1, hi=100, cap_scale=cap)
    row_ptr, peer, w = colliding_csr(rng, P, N)
    WA = workloads.csr_to_dense(row_ptr, peer, w, N)
    assert WA.max() > 127 and (WA > 127).sum() > P // 4
    engine.upload_latency(L, "i8")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic_csr(row_ptr, peer, w, "i8", N)
    node, _, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist()
    assert ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()
    # the candidate lists of the last pass equal the oracle's exact ranking
    engine.reset_capacity()
    engine.score()
    cn, cc, _, cnt, _ = engine.candidates()
    wn, wc, wcnt = oracle.topk(oracle.cost(WA, L, "i8"), oracle.fit_mask(req, free), 8)
    for p in range(0, P, 7):
        c = cnt[p]
        assert c >= min(4, wcnt[p])
        assert cn[p, :c].tolist() == wn[p, :c].tolist(), p
        assert cc[p, :c].tolist() == wc[p, :c].tolist(), p


def test_csr_int32_weights_exact(engine):
    """int32 peer weights (NAS_DT_I32): MB-scale volumes, negative entries too."""
    rng = np.random.default_rng(3)
    P, N = 1200, 500
    _, L, free, req = cluster(rng, P, N, lo=-60, hi=100, cap_scale=0.1)
    row_ptr, peer, _ = colliding_csr(rng, P, N)
    w = rng.integers(-3000, 50000, row_ptr[-1]).astype(np.int32)
    WA = workloads.csr_to_dense(row_ptr, peer, w, N)
    engine.upload_latency(L, "i8")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic_csr(row_ptr, peer, w, "i8", N)
    node, _, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert np.abs(oracle.cost(WA, L, "i8")).max() > 2**24  # far beyond int8 traffic's costs
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()
    rows, _, _, _ = engine.read_inputs(0, P, want_L=False)
    assert (rows == WA).all()  # read-back is the exact traffic


@pytest.mark.parametrize("P,N", [(700, 130), (2048, 2000)])
def test_dense_int32_traffic_exact(engine, P, N):
    rng = np.random.default_rng(P * N)
    WA8, L, free, req = cluster(rng, P, N, lo=-20, hi=60, cap_scale=0.08)
    WA = WA8.astype(np.int32)
    hot = rng.random((P, N)) < 0.01
    WA[hot] = rng.integers(-100000, 100000, int(hot.sum()))
    upload(engine, WA, L, free, req)
    node, _, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()


def test_overflow_through_gathered_rescores(engine):
    """Crowded preferences (commit stops, gathered rescore views whose rows map
    back to pods) with most of the preference carried by overflow entries."""
    rng = np.random.default_rng(17)
    P, N = 12000, 256
    WA8, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.5)
    WA = WA8.astype(np.int32)
    WA[:, :24] += rng.integers(200, 5000, (P, 24))  # everyone wants nodes 0..23, beyond int8
    upload(engine, WA, L, free, req)
    node, _, ci = engine.place()
    t = engine.timings()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert t["rescore_rounds"] > 0
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()


def test_synthetic_cluster_has_exact_collisions(engine):
    """The bench generator (C3 shape, scaled down): home-rack peer collisions
    give aggregates past int8; read-back returns them exactly and the first
    pods' placements equal the sequential oracle on the unclipped traffic."""
    N, P, S = 2048, 4096, 1024
    engine.synth_cluster(0x4E4153, N, P, "i8", peers=8)
    WA, L, cap, req = engine.read_inputs(0, S, want_L=True)
    assert WA.dtype == np.int32 and WA.max() > 127
    assert ((WA > 127).sum(axis=1) > 0).mean() > 0.1  # many pods' peers collide
    node, _, ci = engine.place()
    want, wcost, _ = oracle.place(WA, L, req[:S], cap, "i8")
    assert node[:S].tolist() == want.tolist() and ci[:S].tolist() == wcost.tolist()


def test_batch_synthetic_overflow(engine):
    """A batch of synthetic clusters: each cluster's overflow lists and Lr are
    its own (cluster-offset indexing in the epilogue)."""
    from kubernetesnetawarescheduler_amd import Engine
    B, N, P, S = 4, 1024, 2048, 512
    with Engine(0) as e:
        e.synth_batch(99, B, N, P, "i8", peers=8)
        node, _, ci = e.place()
    for b in range(B):
        with Engine(0) as e1:
            e1.synth_cluster(99 + b, N, P, "i8", peers=8)
            WA, L, cap, req = e1.read_inputs(0, S, want_L=True)
        assert WA.max() > 127
        want, wcost, _ = oracle.place(WA, L, req[:S], cap, "i8")
        assert node[b, :S].tolist() == want.tolist() and ci[b, :S].tolist() == wcost.tolist()


def test_int32_cost_range_refused(engine):
    """sum_m |WA[p,m]| * max|L| beyond int32 cannot be scored exactly: refused."""
    rng = np.random.default_rng(1)
    P, N = 64, 64
    WA8, L, free, req = cluster(rng, P, N, lo=0, hi=10)
    WA = WA8.astype(np.int32)
    L[0, 0] = 127
    WA[5, 0] = 2**31 // 100  # * 127 > INT32_MAX
    upload(engine, WA, L, free, req)
    with pytest.raises(NasError) as ei:
        engine.place()
    assert ei.value.code == _lib.NAS_ERR_UNSUPPORTED
    WA[5, 0] = 2**31 // 200  # * 127 < INT32_MAX with the rest of the row
    upload(engine, WA, L, free, req)
    node, _, ci = engine.place()
    want, wcost, _ = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()


def test_reupload_larger_pods_resets_lists(engine):
    """after a pass, re-uploading more pods must not let the commit
    or the candidate getters use lists sized for the old pod count."""
    rng = np.random.default_rng(5)
    WA, L, free, req = cluster(rng, 300, 100, cap_scale=0.3)
    upload(engine, WA, L, free, req)
    engine.place()
    WA2, _, _, req2 = cluster(rng, 5000, 100, cap_scale=0.3)
    engine.upload_pods(req2)
    engine.upload_traffic(WA2, "i8")
    with pytest.raises(NasError) as ei:
        engine.commit(0, np.zeros(5000, np.int32))
    assert ei.value.code == _lib.NAS_ERR_STATE
    with pytest.raises(NasError):
        engine.candidates()
    engine.reset_capacity()  # the first pass consumed capacity
    node, _, ci = engine.place()
    want, wcost, _ = oracle.place(WA2, L, req2, free, "i8")
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
