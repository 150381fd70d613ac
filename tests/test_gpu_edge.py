"""Edge cases of the network-aware placement through the C ABI, each against
the sequential oracle: degenerate sizes, all-tie costs (lowest node index
wins), zero requests and zero capacities, negative traffic, every pod
unschedulable, and a context re-used across uploads of different sizes."""
import numpy as np
import pytest

import oracle
from util import cluster

pytestmark = pytest.mark.gpu


def run(engine, WA, L, free, req, dtype="i8"):
    engine.upload_latency(L, dtype)
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic(WA, dtype)
    node, _, score = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, dtype)
    assert node.tolist() == want.tolist()
    assert score.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()
    return node


def test_one_pod_one_node(engine):
    WA = np.array([[5]], np.int8)
    L = np.array([[0]], np.int8)
    fits = run(engine, WA, L, np.array([[100, 100, 1]], np.int32), np.array([[1, 1, 1]], np.int32))
    assert fits.tolist() == [0]
    no = run(engine, WA, L, np.array([[100, 100, 1]], np.int32), np.array([[101, 1, 1]], np.int32))
    assert no.tolist() == [-1]


def test_all_ties_fill_lowest_index_first(engine):
    P, N = 700, 130
    WA = np.zeros((P, N), np.int8)
    L = np.zeros((N, N), np.int8)
    free = np.tile(np.array([[1000, 10**6, 3]], np.int32), (N, 1))
    req = np.tile(np.array([[1, 1, 1]], np.int32), (P, 1))
    node = run(engine, WA, L, free, req)
    # three pods per node, in node order; the rest do not fit
    assert node[:3 * N].tolist() == sorted(list(range(N)) * 3)
    assert (node[3 * N:] == -1).all()


def test_zero_requests_and_zero_capacity(engine):
    rng = np.random.default_rng(4)
    P, N = 400, 90
    WA, L, free, req = cluster(rng, P, N, lo=-10, hi=30)
    free[::3] = 0                      # a third of the nodes have nothing left
    req[::5] = 0                       # every fifth pod asks for nothing: fits anywhere
    node = run(engine, WA, L, free, req)
    assert (node[::5] >= 0).all()


def test_negative_traffic(engine):
    rng = np.random.default_rng(5)
    P, N = 600, 257
    WA = rng.integers(-128, 128, (P, N)).astype(np.int8)
    L = rng.integers(-128, 128, (N, N)).astype(np.int8)
    free = np.stack([rng.integers(200, 800, N), rng.integers(10**5, 10**6, N),
                     np.full(N, 4)], 1).astype(np.int32)
    req = np.stack([rng.integers(1, 100, P), rng.integers(1000, 50000, P), np.ones(P)], 1).astype(np.int32)
    run(engine, WA, L, free, req)


def test_everything_unschedulable(engine):
    rng = np.random.default_rng(6)
    P, N = 300, 64
    WA, L, free, req = cluster(rng, P, N)
    req[:, 0] = free[:, 0].max() + 1
    node = run(engine, WA, L, free, req)
    assert (node == -1).all()
    assert engine.timings()["unschedulable"] == P


def test_context_reuse_across_sizes(engine):
    """Bigger, then smaller, then bigger problems on one context: buffers are
    reused, nothing from an earlier upload leaks into a later placement."""
    rng = np.random.default_rng(7)
    for P, N in [(2000, 500), (300, 64), (1, 3), (1500, 700)]:
        WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.1)
        run(engine, WA, L, free, req)


def test_bf16_negative_and_zero(engine):
    from util import f32_to_bf16_bits
    rng = np.random.default_rng(8)
    P, N = 500, 200
    WA = f32_to_bf16_bits(rng.integers(-50, 50, (P, N)).astype(np.float32))
    L = f32_to_bf16_bits(rng.integers(-20, 20, (N, N)).astype(np.float32))
    WA[::7] = f32_to_bf16_bits(np.full(N, -0.0, np.float32))  # -0 traffic rows: every cost 0
    _, _, free, req = cluster(rng, P, N, cap_scale=0.2)
    engine.upload_latency(L, "bf16")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic(WA, "bf16")
    node, cost, _ = engine.place()
    want, wcost, _ = oracle.place(WA, L, req, free, "bf16")
    assert node.tolist() == want.tolist()
    assert np.allclose(cost, wcost, rtol=1e-5, atol=0)


def test_wide_cost_range_exact_select_path(engine):
    """The cost epilogue keeps a lane's top-4 as packed u32 keys (cost offset
    << 6 | node slot) only when every lane's 64 costs span < 2^26 - 1, and
    falls back to the exact (cost, node) select network otherwise.  Here
    extreme int8 traffic and latency of both signs give costs of +-7e7 next
    to pods with near-zero traffic (small spans), so waves of both kinds and
    mixed ties all occur; placements, scores and capacity must equal the
    oracle exactly, and the candidate lists the oracle's ranking."""
    rng = np.random.default_rng(77)
    P, N = 512, 4608
    sign = np.where(np.arange(N) % 2 == 0, 1, -1)
    L = (sign[None, :] * rng.integers(120, 128, (N, N))).clip(-128, 127).astype(np.int8)
    WA = rng.integers(120, 128, (P, N)).astype(np.int8)
    WA[P // 2:] = rng.integers(-1, 2, (P - P // 2, N)).astype(np.int8)  # small spans
    WA[3 * P // 4:, 7] = 127  # mixes: one heavy peer on top of the small background
    free = np.stack([rng.integers(800, 3000, N), rng.integers(800_000, 3_000_000, N),
                     np.full(N, 3)], 1).astype(np.int32)
    req = np.stack([rng.integers(1, 540, P), rng.integers(7_464, 303_749, P),
                    np.ones(P)], 1).astype(np.int32)
    cost = oracle.cost(WA, L, "i8")
    assert np.ptp(cost[: P // 2], axis=1).min() > 2**26  # the wide rows really are wide
    engine.upload_latency(L, "i8")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic(WA, "i8")
    engine.score()
    node, ci, _, cnt, _ = engine.candidates()
    wn, wc, wcnt = oracle.topk(cost, oracle.fit_mask(req, free), 8)
    assert (cnt >= np.minimum(4, wcnt)).all()
    for p in range(P):
        assert node[p, :cnt[p]].tolist() == wn[p, :cnt[p]].tolist(), p
        assert ci[p, :cnt[p]].tolist() == wc[p, :cnt[p]].tolist(), p
    run(engine, WA, L, free, req)
