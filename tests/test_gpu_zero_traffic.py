"""Zero-traffic pods (k_commit.hip): a pod with no traffic to any bound peer
costs exactly 0 on every node, so its sequential choice is the lowest-index
node that fits.  When its candidate list runs out, the commit scans the
capacity above the list's bound instead of halting for a rescore.  Every case
must equal the sequential oracle (placements, integer scores, remaining
capacity); the scan's own effect is checked through the rescore counter."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine, workloads
from util import cluster

pytestmark = pytest.mark.gpu


def upload(e, WA, L, free, req, dtype="i8"):
    e.upload_latency(L, dtype)
    e.upload_capacity(free)
    e.upload_pods(req)
    e.upload_traffic(WA, dtype)


def first_fit(req, free):
    """Sequential greedy for all-zero traffic: every pod takes the lowest-index
    node that fits (the oracle's (cost, node) order with every cost 0)."""
    free = free.astype(np.int64).copy()
    node = np.full(len(req), -1, np.int64)
    for p, r in enumerate(req.astype(np.int64)):
        fits = np.flatnonzero((free >= r).all(1))
        if len(fits):
            node[p] = fits[0]
            free[fits[0]] -= r
    return node, free


def check(e, WA, L, req, free, dtype="i8"):
    node, _, ci = e.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, dtype)
    assert node.tolist() == want.tolist()
    assert ci.tolist() == wcost.tolist()
    assert (e.get_capacity() == wfree).all()
    return e.timings()


@pytest.mark.parametrize("P,N,frac", [(3000, 300, 1.0), (3000, 300, 0.4), (4096, 640, 0.7)])
def test_zero_traffic_herd_exact(engine, P, N, frac):
    """A herd of zero-traffic pods (all, or mixed with ordinary pods) at
    tight capacity: exact, and all-zero herds need no rescore at all."""
    rng = np.random.default_rng(P + N + int(frac * 10))
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.05)
    zero = rng.random(P) < frac
    WA[zero] = 0
    upload(engine, WA, L, free, req)
    t = check(engine, WA, L, req, free)
    if frac == 1.0:
        assert t["rescore_rounds"] == 0
    assert int((WA == 0).all(1).sum()) == int(zero.sum())


def test_zero_traffic_unschedulable_without_rescore(engine):
    """More zero-traffic pods than the cluster holds: the scan reaches the
    last node and the pod gets NAS_EMPTY (no rescore)."""
    rng = np.random.default_rng(5)
    P, N = 700, 100
    WA, L, free, req = cluster(rng, P, N, cap_scale=0.02)
    WA[:] = 0
    upload(engine, WA, L, free, req)
    t = check(engine, WA, L, req, free)
    assert t["rescore_rounds"] == 0
    assert t["unschedulable"] > 0


def test_zero_traffic_scan_limit_falls_back_to_rescore(engine):
    """A herd deeper than the scan limit (1,024 nodes past the list): one pod
    per node, 2,600 pods march through 2,600 nodes, so the later pods' scans
    run out and they are rescored -- still exact."""
    P, N = 2600, 3000
    rng = np.random.default_rng(6)
    WA, L, free, req = cluster(rng, P, N)
    WA[:] = 0
    free[:, 2] = 1  # one pod slot per node
    upload(engine, WA, L, free, req)
    node, _, ci = engine.place()
    want, wfree = first_fit(req, free)
    assert node.tolist() == want.tolist()
    assert (ci == 0).all()
    assert (engine.get_capacity() == wfree).all()
    assert engine.timings()["rescore_rounds"] > 0


def test_zero_traffic_l2_commit(engine):
    """N > 11,541: the capacity lives in L2 (short scans, rescore beyond)."""
    P, N = 17000, 14000  # > 16,384 pods: the 1024-thread commit, capacity in L2
    rng = np.random.default_rng(7)
    req = np.stack([rng.integers(1, 540, P), rng.integers(7_464, 303_749, P),
                    np.ones(P, np.int64)], 1).astype(np.int32)
    free = np.stack([np.full(N, 1200), np.full(N, 2_000_000), np.full(N, 110)], 1).astype(np.int32)
    L = rng.integers(0, 100, (N, N), dtype=np.int8)
    row_ptr = np.zeros(P + 1, np.int32)  # no traffic at all
    engine.upload_latency(L, "i8")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic_csr(row_ptr, np.zeros(0, np.int32), np.zeros(0, np.int8), "i8", N)
    node, _, ci = engine.place()
    want, wfree = first_fit(req, free)
    assert node.tolist() == want.tolist()
    assert (ci == 0).all()
    assert (engine.get_capacity() == wfree).all()


def test_zero_traffic_multi_chunk(engine):
    """Enough pods for several scoring chunks (the first is 8,192 pods)."""
    P, N = 20000, 500
    rng = np.random.default_rng(8)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.3)
    WA[rng.random(P) < 0.5] = 0
    upload(engine, WA, L, free, req)
    check(engine, WA, L, req, free)


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_zero_traffic_float(engine, dtype):
    P, N = 2000, 256
    rng = np.random.default_rng(9)
    _, _, free, req = cluster(rng, P, N, cap_scale=0.05)
    # integer-valued operands: every product and partial sum is exact in the
    # fp32 accumulation, so the placements must be identical (no near ties)
    L = rng.integers(50, 251, (N, N)).astype(np.float32)
    WA = rng.integers(0, 101, (P, N)).astype(np.float32)
    WA[rng.random(P) < 0.6] = 0.0
    if dtype == "bf16":
        to16 = lambda a: (a.view(np.uint32) >> 16).astype(np.uint16)  # noqa: E731
        L, WA = to16(L), to16(WA)
    upload(engine, WA, L, free, req, dtype)
    node, _, _ = engine.place()
    want, _, wfree = oracle.place(WA, L, req, free, dtype)
    assert node.tolist() == want.tolist()
    assert (engine.get_capacity() == wfree).all()


def test_zero_traffic_batch():
    B, P, N = 3, 1500, 300
    rng = np.random.default_rng(10)
    cs = []
    for b in range(B):
        WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.05)
        WA[rng.random(P) < 0.3 * (b + 1)] = 0
        cs.append((WA, L, free, req))
    with Engine(0) as e:
        e.set_batch(B)
        e.upload_latency(np.stack([c[1] for c in cs]), "i8")
        e.upload_capacity(np.stack([c[2] for c in cs]))
        e.upload_pods(np.stack([c[3] for c in cs]))
        e.upload_traffic(np.stack([c[0] for c in cs]), "i8")
        node, _, score = e.place()
        cap = e.get_capacity()
    for b, (WA, L, free, req) in enumerate(cs):
        want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
        assert node[b].tolist() == want.tolist(), b
        assert score[b].tolist() == wcost.tolist(), b
        assert (cap[b] == wfree).all(), b


def test_c2_needs_no_rescore():
    """C2's rescores all came from its 1,654 pods without a bound peer."""
    c = workloads.c2_cluster(0x4E4153, 1000, 10000)
    with Engine(0) as e:
        e.upload_latency(c["L"], "i8")
        e.upload_capacity(c["free"])
        e.upload_pods(c["req"])
        e.upload_traffic_csr(c["row_ptr"], c["peer_node"], c["weight"], "i8", 1000)
        node, _, score = e.place()
        t = e.timings()
    WA = workloads.csr_to_dense(c["row_ptr"], c["peer_node"], c["weight"], 1000)
    want, wcost, _ = oracle.place(WA, c["L"], c["req"], c["free"], "i8")
    assert node.tolist() == want.tolist() and score.tolist() == wcost.tolist()
    assert t["rescore_rounds"] == 0


@pytest.mark.parametrize("G", [2, 3])
def test_zero_traffic_node_shards(G):
    """Node shards (host exchange, replicated commit): every shard holds the
    whole WA, so every shard flags the same zero-traffic pods and scans the
    same replicated capacity -- equal to the oracle and on every shard."""
    from kubernetesnetawarescheduler_amd.sharded import place_local_shards
    P, N = 3000, 400
    rng = np.random.default_rng(11 + G)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.05)
    WA[rng.random(P) < 0.5] = 0
    engines = []
    try:
        for r in range(G):
            e = Engine(0)
            engines.append(e)
            e.set_shard(r, G)
            upload(e, WA, L, free, req)
        node, score, _ = place_local_shards(engines, P)
        caps = [e.get_capacity() for e in engines]
    finally:
        for e in engines:
            e.close()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist()
    assert score.tolist() == wcost.tolist()
    for c in caps:
        assert (c == wfree).all()
