"""GPU parity of the extended mode: fit filter (k_fit), MFMA cost + fused top-k
(k_cost), merge, and greedy commit (k_commit) against the CPU oracle.

int8 inputs: exact -- masks, candidate lists, integer costs, placements and
the remaining capacity are bit-identical.  bf16 inputs: integer-valued bf16
is exact too (products and fp32 sums stay below 2^24); general bf16 costs
must be within REL_TOL of the fp64 oracle (the north star's 1e-5)."""
import json
import os

import numpy as np
import pytest

import oracle
from util import bf16_bits_to_f64, cluster

pytestmark = pytest.mark.gpu
REL_TOL = 1e-5
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def upload(engine, WA, L, free, req, dtype):
    engine.upload_latency(L, dtype)
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic(WA, dtype)


def test_place_golden(engine):
    with open(os.path.join(GOLD, "place_small.json")) as f:
        g = json.load(f)
    upload(engine, np.array(g["WA"], np.int8), np.array(g["L"], np.int8), np.array(g["free"]),
           np.array(g["req"]), "i8")
    node, cf, ci = engine.place()
    assert node.tolist() == g["node"]
    assert ci.tolist() == g["cost"]
    assert engine.get_capacity().tolist() == g["free_after"]


@pytest.mark.parametrize("P,N,cap", [(1, 1, 0.05), (3, 5, 0.05), (300, 70, 0.05), (257, 129, 0.05),
                                     (1000, 300, 0.05), (513, 1000, 0.05), (700, 300, 20.0),
                                     (1100, 1000, 0.3)])
def test_fit_mask(engine, P, N, cap):
    """Bit-exact fit words: mostly failing (0.05), every pod fitting every
    node (20: k_fit's scalar fast path for whole chunks), and a mix (0.3)."""
    rng = np.random.default_rng(P * 7 + N)
    WA, L, free, req = cluster(rng, P, N, cap_scale=cap)
    upload(engine, WA, L, free, req, "i8")
    got = engine.filter()  # [ceil(N/64)][P] uint64, bit j <-> node 64c + j
    want = oracle.fit_mask(req, free)  # [P][ceil(N/32)] uint32
    for c in range(got.shape[0]):
        lo = want[:, 2 * c].astype(np.uint64)
        hi = want[:, 2 * c + 1].astype(np.uint64) if 2 * c + 1 < want.shape[1] else 0
        assert (got[c] == (lo | (np.uint64(hi) << np.uint64(32)))).all()


@pytest.mark.parametrize("P,N,lo,hi", [(256, 256, 0, 20), (300, 70, -20, 20), (1000, 1000, 0, 127),
                                       (700, 1500, -128, 127), (2048, 4096, 0, 8)])
def test_candidates_i8_exact(engine, P, N, lo, hi):
    """The usable prefix of each list (count entries) is exactly the oracle's
    ranking of fitting nodes by (cost, node), with exact integer costs; it
    holds at least min(4, #fitting) entries; complete lists hold them all."""
    rng = np.random.default_rng(P + N)
    WA, L, free, req = cluster(rng, P, N, lo=lo, hi=hi, cap_scale=0.1)
    upload(engine, WA, L, free, req, "i8")
    engine.score()
    node, ci, cf, cnt, complete = engine.candidates()
    cost = oracle.cost(WA, L, "i8")
    mask = oracle.fit_mask(req, free)
    wn, wc, wcnt = oracle.topk(cost, mask, 8)
    assert (cnt >= np.minimum(4, wcnt)).all()
    for p in range(P):
        c = cnt[p]
        assert node[p, :c].tolist() == wn[p, :c].tolist(), p
        assert ci[p, :c].tolist() == wc[p, :c].tolist(), p
        assert (node[p, c:] == -1).all()
        if complete[p]:  # nothing dropped: the list is every fitting node
            assert c == wcnt[p] < 8


@pytest.mark.parametrize("P,N,cap", [(500, 200, 0.3), (1200, 333, 0.05), (3000, 1000, 0.02),
                                     (4096, 640, 0.01)])
def test_place_i8_exact(engine, P, N, cap):
    """Placements, integer scores and remaining capacity identical to the
    sequential oracle -- including commit conflicts, rescore rounds and
    unschedulable pods at tight capacity."""
    rng = np.random.default_rng(P ^ N)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=60, cap_scale=cap)
    # make locality strong so many pods want the same few nodes
    WA[:, : N // 10] = np.minimum(WA[:, : N // 10].astype(np.int32) + 60, 127).astype(np.int8)
    upload(engine, WA, L, free, req, "i8")
    node, cf, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist()
    assert ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()
    t = engine.timings()
    assert t["unschedulable"] == int((want < 0).sum())


def test_rescore_path_runs(engine):
    rng = np.random.default_rng(77)
    P, N = 2000, 256
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.02)
    WA[:, :8] = 127  # everyone wants nodes 0..7
    upload(engine, WA, L, free, req, "i8")
    node, _, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert engine.timings()["rescore_rounds"] > 0
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()


def test_repeat_passes_with_speculative_slots(engine):
    """A pass that needed gathered rescore slots makes the next pass of the
    same shape enqueue that many slots before its first status round trip
    (nas_place slot_hint).  Every pass -- first, speculative repeats, a
    different shape, and a shape that needs no slot after one that did --
    equals the sequential oracle."""
    rng = np.random.default_rng(78)
    P, N = 2000, 256
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.02)
    WA[:, :8] = 127
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    upload(engine, WA, L, free, req, "i8")
    for it in range(3):
        engine.reset_capacity()
        node, _, ci = engine.place()
        assert engine.timings()["rescore_rounds"] > 0, it
        assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist(), it
        assert (engine.get_capacity() == wfree).all(), it
    # the same shape with roomy capacity: the speculative slots find nothing halted
    roomy = np.minimum(free.astype(np.int64) * 5000, 2**31 - 1).astype(np.int32)
    upload(engine, WA, L, roomy, req, "i8")
    node, _, ci = engine.place()
    w2, c2, f2 = oracle.place(WA, L, req, roomy, "i8")
    assert engine.timings()["rescore_rounds"] == 0
    assert node.tolist() == w2.tolist() and ci.tolist() == c2.tolist()
    assert (engine.get_capacity() == f2).all()
    # tight again: the hint is now 0, the host loop finds the stops itself
    upload(engine, WA, L, free, req, "i8")
    node, _, ci = engine.place()
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()


@pytest.mark.parametrize("P,N", [(300, 200), (1000, 700)])
def test_place_bf16_integer_valued_exact(engine, P, N):
    rng = np.random.default_rng(P + 3 * N)
    WA, L, free, req = cluster(rng, P, N, dtype="bf16", lo=0, hi=16, cap_scale=0.05)
    upload(engine, WA, L, free, req, "bf16")
    node, cf, _ = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "bf16")
    assert node.tolist() == want.tolist()
    assert np.array_equal(cf.astype(np.float64), wcost)
    assert (engine.get_capacity() == wfree).all()


def test_cost_bf16_random_within_tolerance(engine):
    """General bf16 operands, fp32 MFMA accumulation: candidate costs within
    1e-5 relative of the fp64 oracle's cost for the same node, and each
    candidate's fp64 cost within tolerance of the oracle's k-th best."""
    rng = np.random.default_rng(5)
    P, N = 512, 2048
    WA, L, free, req = cluster(rng, P, N, dtype="bf16", int_valued=False, cap_scale=1.0)
    upload(engine, WA, L, free, req, "bf16")
    engine.score()
    node, _, cf, cnt, _ = engine.candidates()
    cost = oracle.cost(WA, L, "bf16")
    mask = oracle.fit_mask(req, free)
    wn, wc, wcnt = oracle.topk(cost, mask, 8)
    assert (cnt >= np.minimum(4, wcnt)).all()
    rows = np.arange(P)[:, None]
    usable = node >= 0
    exact = cost[rows, np.maximum(node, 0)]
    rel = np.abs(cf.astype(np.float64) - exact) / np.abs(exact)
    assert rel[usable].max() <= REL_TOL
    # the GPU's j-th candidate is a true j-th best up to the tolerance
    assert (np.abs(exact - wc) <= REL_TOL * np.abs(wc))[usable].all()


def test_csr_traffic_matches_dense(engine):
    rng = np.random.default_rng(8)
    P, N = 600, 300
    _, L, free, req = cluster(rng, P, N, cap_scale=0.2)
    deg = rng.integers(0, 12, P)
    row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    peer = rng.integers(-1, N, row_ptr[-1]).astype(np.int32)  # -1 = unbound peer
    peer[rng.random(len(peer)) < 0.3] = rng.integers(0, 4, 1)[0]  # repeated nodes
    w = rng.integers(1, 40, row_ptr[-1]).astype(np.int8)
    dense = np.zeros((P, N), np.int32)
    for p in range(P):
        for x in range(row_ptr[p], row_ptr[p + 1]):
            if peer[x] >= 0:
                dense[p, peer[x]] += w[x]
    assert dense.max() > 127  # repeated nodes aggregate past int8: exact, never saturated
    engine.upload_latency(L, "i8")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic_csr(row_ptr, peer, w, "i8", N)
    node_csr, _, c_csr = engine.place()
    want, wcost, _ = oracle.place(dense, L, req, free, "i8")
    assert node_csr.tolist() == want.tolist() and c_csr.tolist() == wcost.tolist()


def test_deterministic_repeat(engine):
    rng = np.random.default_rng(12)
    WA, L, free, req = cluster(rng, 1500, 900, cap_scale=0.03)
    upload(engine, WA, L, free, req, "i8")
    a, _, ca = engine.place()
    engine.reset_capacity()
    b, _, cb = engine.place()
    assert (a == b).all() and (ca == cb).all()


def test_reset_is_stream_ordered(engine):
    """nas_reset_capacity returns without waiting: a host read right after it,
    a place right after it and an upload right after it all see the reset
    (everything is ordered on the context's stream)."""
    rng = np.random.default_rng(13)
    WA, L, free, req = cluster(rng, 1200, 700, cap_scale=0.03)
    upload(engine, WA, L, free, req, "i8")
    want = engine.place()[0].copy()
    for _ in range(3):
        engine.reset_capacity()
        assert (engine.get_capacity() == free).all()
        engine.reset_capacity()
        got, _, _ = engine.place()
        assert got.tolist() == want.tolist()
    # reset, then a new upload at once: the upload wins
    engine.reset_capacity()
    engine.upload_capacity(free // 2)
    assert (engine.get_capacity() == free // 2).all()
    w2, _, _ = oracle.place(WA, L, req, free // 2, "i8")
    got, _, _ = engine.place()
    assert got.tolist() == w2.tolist()


def test_synthetic_cluster_sampled(engine):
    """The bench's device-generated cluster (scaled down): candidate lists of
    sampled pods equal the oracle top-4 on the inputs read back from HBM, and
    the commit equals the sequential oracle replayed on the GPU's lists."""
    N, P = 2048, 8192
    engine.synth_cluster(0x4E4153, N, P, "i8", peers=8)
    engine.score()
    node, ci, _, cnt, complete = engine.candidates()
    rng = np.random.default_rng(0)
    pods = np.sort(rng.choice(P, 64, replace=False))
    _, L, cap, req = engine.read_inputs(0, 0, want_L=True)
    for p in pods:
        WA, _, _, _ = engine.read_inputs(int(p), 1, want_L=False)
        cost = oracle.cost(WA, L, "i8")
        mask = oracle.fit_mask(req[p:p + 1], cap)
        wn, wc, wcnt = oracle.topk(cost, mask, 8)
        c = cnt[p]
        assert c >= min(4, wcnt[0])
        assert node[p, :c].tolist() == wn[0, :c].tolist()
        assert ci[p, :c].tolist() == wc[0, :c].tolist()
    engine.reset_capacity()
    placed, _, _ = engine.place()
    rounds = engine.timings()["rescore_rounds"]
    want, _, wfree, stop = oracle.commit(node, cnt, req, cap, complete)
    if rounds == 0:
        assert stop == P
        assert placed.tolist() == want.tolist()
        assert (engine.get_capacity() == wfree).all()
    else:  # the GPU rescored from `stop` on: the prefix before it must agree
        assert placed[:stop].tolist() == want[:stop].tolist()


@pytest.mark.parametrize("P,N,seed", [(6000, 64, 1), (10000, 300, 2), (3000, 1000, 3)])
def test_commit_conflicts_exact(engine, P, N, seed):
    """Crowded commit windows: most pods of a 1024-pod window want the same
    few nodes, which fill up mid-window (reservation failures, releases,
    re-picks) -- placements and remaining capacity equal the sequential oracle."""
    rng = np.random.default_rng(seed)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.2)
    hot = rng.choice(N, max(2, N // 32), replace=False)
    WA[:, hot] = 127
    L[hot[:, None], hot[None, :]] = 0
    upload(engine, WA, L, free, req, "i8")
    node, _, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist()
    assert ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()


def test_commit_huge_requests_no_overflow(engine):
    """Requests near 2^30 against capacities near 2^31: a window's combined
    reservations would overflow int32; the commit never takes a resource
    below zero, so placements stay exact."""
    rng = np.random.default_rng(4)
    P, N = 3000, 40
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=20)
    free[:, 0] = rng.integers(2**31 - 2**28, 2**31 - 1, N)
    free[:, 1] = 2**31 - 1
    free[:, 2] = 2**31 - 1
    req[:, 0] = rng.integers(2**29, 2**30, P)
    req[:, 1] = rng.integers(2**29, 2**30, P)
    upload(engine, WA, L, free, req, "i8")
    node, _, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist()
    assert ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()
    assert (want < 0).sum() > 0  # the cluster overflows: unschedulable pods exist


def test_rescore_slots_across_chunks(engine):
    """Many commit stops spread over several 8192-pod scoring chunks: the
    device-side rescore slots behind each chunk's commit, and the host loop
    for stops beyond them, reproduce the sequential oracle exactly."""
    rng = np.random.default_rng(21)
    P, N = 20000, 256
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.6)
    WA[:, :24] = 127  # everyone prefers nodes 0..23, which fill up early
    upload(engine, WA, L, free, req, "i8")
    node, _, ci = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert engine.timings()["rescore_rounds"] > 0
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()


@pytest.mark.parametrize("P", [20000, 6000])
def test_l2_commit_published_capacity(engine, P):
    """More nodes than the LDS commit holds (N > 13,610): the commit works on
    the capacity in L2 with speculative reservations, and the pipelined
    scoring chunks read the published capacity it maintains (start minus
    committed pods).  Crowded preferences and 2 pod slots per node make many
    lists run dry; every placement must still equal the sequential oracle.
    P = 20000 walks in 1024-pod windows (k_commit), P = 6000 in one wave
    (k_commit_w, walks of up to 16,384 pods)."""
    rng = np.random.default_rng(31)
    N = 14000
    L = rng.integers(1, 100, (N, N)).astype(np.int8)
    a = rng.integers(0, 64, P)
    b = (a + 1 + rng.integers(0, 63, P)) % 64
    row_ptr = np.arange(0, 2 * P + 1, 2).astype(np.int32)
    peer = np.stack([a, b], 1).reshape(-1).astype(np.int32)
    w = rng.integers(1, 100, 2 * P).astype(np.int8)
    WA = np.zeros((P, N), np.int8)
    WA[np.arange(P), a] = w[0::2]
    WA[np.arange(P), b] = w[1::2]
    free = np.stack([np.full(N, 4000), np.full(N, 4 << 20), np.full(N, 2)], 1).astype(np.int32)
    req = np.stack([rng.integers(1, 540, P), rng.integers(7_464, 303_749, P),
                    np.ones(P, np.int64)], 1).astype(np.int32)
    engine.upload_latency(L, "i8")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic_csr(row_ptr, peer, w, "i8", N)
    node, _, ci = engine.place()
    t = engine.timings()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()
    assert t["rescore_rounds"] > 0
