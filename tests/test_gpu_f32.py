"""The fp32 network-cost path (include/nas.h NAS_DT_F32): measured, unquantised
latency (microseconds) and traffic (MB) as fp32; each operand split into three
bf16 planes and contracted on the bf16 MFMA over a six-fold K (products to
2^-24 relative) with fp32 accumulation.  The north star's bar for raw
floating-point costs is 1e-5 relative to an fp64 sum (REL_TOL below); the
chosen nodes must equal the fp64 sequential oracle's wherever the cost gap at
a pod's turn exceeds that tolerance."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import workloads

pytestmark = pytest.mark.gpu
REL_TOL = 1e-5


def float_cluster(rng, P, N, cap_scale=0.1):
    u = rng.uniform(50.0, 500.0, (N, N))
    L = np.triu(u, 1)
    L = (L + L.T).astype(np.float32)  # latency in us, symmetric, zero diagonal
    WA = (rng.random((P, N)) * 0.5).astype(np.float32)  # background MB to every node
    hot = rng.random((P, N)) < 0.01
    WA[hot] += rng.uniform(10.0, 100.0, int(hot.sum())).astype(np.float32)  # heavy peers
    free = np.stack([rng.integers(int(2000 * cap_scale), int(8000 * cap_scale) + 1, N),
                     rng.integers(int(2e6 * cap_scale), int(8e6 * cap_scale) + 1, N),
                     np.full(N, max(1, int(110 * cap_scale)))], 1).astype(np.int32)
    req = np.stack([rng.integers(1, 540, P), rng.integers(7_464, 303_749, P),
                    np.ones(P, np.int64)], 1).astype(np.int32)
    return WA, L, free, req


def upload(e, WA, L, free, req):
    e.upload_latency(L, "f32")
    e.upload_capacity(free)
    e.upload_pods(req)
    e.upload_traffic(WA, "f32")


@pytest.mark.parametrize("P,N", [(300, 257), (1024, 1000), (512, 3000)])
def test_f32_candidates_within_tolerance(engine, P, N):
    rng = np.random.default_rng(P + N)
    WA, L, free, req = float_cluster(rng, P, N, cap_scale=1.0)
    upload(engine, WA, L, free, req)
    engine.score()
    node, _, cf, cnt, _ = engine.candidates()
    cost = oracle.cost(WA, L, "f32")
    wn, wc, wcnt = oracle.topk(cost, oracle.fit_mask(req, free), 8)
    assert (cnt >= np.minimum(4, wcnt)).all()
    rows = np.arange(P)[:, None]
    use = node >= 0
    exact = cost[rows, np.maximum(node, 0)]
    rel = np.abs(cf.astype(np.float64) - exact) / np.abs(exact)
    assert rel[use].max() <= REL_TOL, rel[use].max()
    # the GPU's j-th candidate is a true j-th best up to the tolerance
    assert (np.abs(exact - wc) <= REL_TOL * np.abs(wc))[use].all()


def _greedy_within_tol(node, cf, cost, req, free):
    """Every pod, on the GPU's own capacity trajectory: its node fits and its
    cost is within REL_TOL of the best fitting node's (or no node fits)."""
    cap = free.astype(np.int64).copy()
    for p in range(len(node)):
        fits = (req[p].astype(np.int64) <= cap).all(axis=1)
        if not fits.any():
            assert node[p] == -1, p
            continue
        n = node[p]
        assert n >= 0 and fits[n], p
        best = cost[p][fits].min()
        assert cost[p, n] - best <= 2 * REL_TOL * abs(best), p
        assert abs(cf[p] - cost[p, n]) <= REL_TOL * abs(cost[p, n]), p
        cap[n] -= req[p]


def _gaps_at_turn(node, cost, req, free):
    """Relative gap between the best and second-best fitting node of every pod
    at its own turn of the (oracle's) sequential walk."""
    cap = free.astype(np.int64).copy()
    gaps = np.full(len(node), np.inf)
    for p in range(len(node)):
        fits = (req[p].astype(np.int64) <= cap).all(axis=1)
        c = np.where(fits, cost[p], np.inf)
        if np.isfinite(c).sum() >= 2:
            a, b = np.partition(c, 1)[:2]
            # relative to the larger magnitude, so a zero best cost divides
            # nothing by zero; two exact zeros (a pod with no traffic: every
            # product is 0 on the GPU too) are no rounding ambiguity -- the
            # node index decides them on both sides -- so they are not a tie
            scale = max(abs(a), abs(b))
            gaps[p] = (b - a) / scale if scale > 0 else np.inf
        if node[p] >= 0:
            cap[node[p]] -= req[p]
    return gaps


@pytest.mark.parametrize("P,N,cap", [(2000, 500, 0.05), (4096, 1200, 0.02)])
def test_f32_place_matches_fp64_oracle(engine, P, N, cap):
    rng = np.random.default_rng(7 * P + N)
    WA, L, free, req = float_cluster(rng, P, N, cap_scale=cap)
    upload(engine, WA, L, free, req)
    node, cf, _ = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, free, "f32")
    cost = oracle.cost(WA, L, "f32")
    gaps = _gaps_at_turn(want, cost, req, free)
    tie = np.nonzero(gaps <= 2 * REL_TOL)[0]
    upto = tie[0] if len(tie) else P  # identical up to the first near-tie
    assert upto > 0.5 * P
    assert node[:upto].tolist() == want[:upto].tolist()
    _greedy_within_tol(node, cf, cost, req, free)  # and past it, on its own trajectory
    ok = want[:upto] >= 0
    rel = np.abs(cf[:upto][ok].astype(np.float64) - wcost[:upto][ok]) / np.abs(wcost[:upto][ok])
    assert rel.max() <= REL_TOL
    if upto == P:
        assert (engine.get_capacity() == wfree).all()


def test_f32_csr_traffic(engine):
    """Float peer weights aggregated in fp64 on the host, rounded once."""
    rng = np.random.default_rng(3)
    P, N = 1500, 400
    _, L, free, req = float_cluster(rng, P, N, cap_scale=0.2)
    deg = rng.integers(1, 9, P)
    row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    peer = np.minimum(rng.integers(0, N // 16, P).repeat(deg) * 16 + rng.integers(0, 4, deg.sum()),
                      N - 1).astype(np.int32)
    peer[rng.random(len(peer)) < 0.1] = -1
    w = rng.uniform(0.5, 120.0, len(peer)).astype(np.float32)
    WA = workloads.csr_to_dense(row_ptr, peer, w.astype(np.float64), N).astype(np.float32)
    engine.upload_latency(L, "f32")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic_csr(row_ptr, peer, w, "f32", N)
    rows, _, _, _ = engine.read_inputs(0, P, want_L=False)
    assert np.array_equal(rows, WA)
    node, cf, _ = engine.place()
    want, wcost, _ = oracle.place(WA, L, req, free, "f32")
    gaps = _gaps_at_turn(want, oracle.cost(WA, L, "f32"), req, free)
    tie = np.nonzero(gaps <= 2 * REL_TOL)[0]
    upto = tie[0] if len(tie) else P
    assert upto > 0.5 * P and node[:upto].tolist() == want[:upto].tolist()
    _greedy_within_tol(node, cf, oracle.cost(WA, L, "f32"), req, free)


def test_f32_synthetic_cluster(engine):
    """The bench generator in fp32: candidate costs of sampled pods vs fp64."""
    N, P = 1024, 2048
    engine.synth_cluster(0x4E4153, N, P, "f32", peers=8)
    engine.score()
    node, _, cf, cnt, _ = engine.candidates()
    _, L, cap, req = engine.read_inputs(0, 0, want_L=True)
    for p in (0, 17, 1000, P - 1):
        WA, _, _, _ = engine.read_inputs(p, 1, want_L=False)
        cost = oracle.cost(WA, L, "f32")[0]
        c = cnt[p]
        exact = cost[node[p, :c]]
        assert (np.abs(cf[p, :c] - exact) <= REL_TOL * np.abs(exact)).all()
