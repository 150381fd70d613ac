"""The wide cost tile (k_cost.hip: 256 nodes x 384 pods per 12-wave
workgroup) scores the main pass of one cluster with >= 32,768 padded pods at
world 1 (nas_api.hip wide_ok).  Its pod tiles straddle the 256-pod units the
rest of the pipeline counts in: chunks are whole wide tiles, and a launch's
last tile reads rows past its end (the next chunk's or the padding) without
writing their lists.  Pod counts here are chosen so the last chunk ends with
a partial tile (overshoot 128 or 256 rows); every case must equal the
sequential oracle exactly (placements, integer scores, remaining capacity)."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine
from util import cluster, f32_to_bf16_bits

pytestmark = pytest.mark.gpu


def upload(e, WA, L, free, req, dtype):
    e.upload_latency(L, dtype)
    e.upload_capacity(free)
    e.upload_pods(req)
    e.upload_traffic(WA, dtype)


@pytest.mark.parametrize("P,N", [(40000, 600), (33000, 257), (45500, 300)])
def test_wide_int8_exact(P, N):
    rng = np.random.default_rng(P + N)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.6)
    WA[:, rng.choice(N, max(2, N // 25), replace=False)] = 127  # herds: commit stops, rescores
    WA[rng.random(P) < 0.1] = 0
    with Engine(0) as e:
        upload(e, WA, L, free, req, "i8")
        node, _, ci = e.place()
        cap = e.get_capacity()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist()
    assert ci.tolist() == wcost.tolist()
    assert (cap == wfree).all()


def test_wide_int32_traffic_exact():
    """Exact traffic beyond int8 (the per-pod overflow lists seed the
    accumulators; past a launch's end they must not be read)."""
    P, N = 34000, 400
    rng = np.random.default_rng(12)
    WA8, L, free, req = cluster(rng, P, N, lo=-20, hi=60, cap_scale=0.5)
    WA = WA8.astype(np.int32)
    hot = rng.random((P, N)) < 0.01
    WA[hot] = rng.integers(-100000, 100000, int(hot.sum()))
    with Engine(0) as e:
        upload(e, WA, L, free, req, "i8")
        node, _, ci = e.place()
        cap = e.get_capacity()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
    assert (cap == wfree).all()


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_wide_float_exact(dtype):
    """Integer-valued float operands: every product and partial sum is exact
    in fp32, so placements equal the fp64 oracle's."""
    P, N = 35000, 256
    rng = np.random.default_rng(13)
    _, _, free, req = cluster(rng, P, N, cap_scale=0.5)
    L = rng.integers(50, 251, (N, N)).astype(np.float32)
    WA = rng.integers(0, 101, (P, N)).astype(np.float32)
    WA[rng.random(P) < 0.2] = 0.0
    if dtype == "bf16":
        L, WA = f32_to_bf16_bits(L), f32_to_bf16_bits(WA)
    with Engine(0) as e:
        upload(e, WA, L, free, req, dtype)
        node, _, _ = e.place()
        cap = e.get_capacity()
    want, _, wfree = oracle.place(WA, L, req, free, dtype)
    assert node.tolist() == want.tolist()
    assert (cap == wfree).all()


def test_wide_score_lists_head_and_tail():
    """nas_score over all pods (one wide launch, whose last tile is partial):
    every sampled pod's first candidate is its (cost, node)-smallest node,
    at both ends of the pod range."""
    P, N = 33000, 512
    rng = np.random.default_rng(14)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=60, cap_scale=0.8)
    with Engine(0) as e:
        upload(e, WA, L, free, req, "i8")
        e.score()
        keys, _ = e.candidate_keys()
    pods = np.concatenate([np.arange(500), np.arange(P - 500, P)])
    cost = oracle.cost(WA[pods], L, "i8")
    fits = (req[pods][:, None, :].astype(np.int64) <= free[None, :, :].astype(np.int64)).all(2)
    cost = np.where(fits, cost, np.iinfo(np.int64).max)
    best = cost.argmin(1)
    k0 = keys[pods, 0]
    assert ((k0 & np.uint64(0xFFFFFFFF)).astype(np.int64) == best).all()
    got_cost = ((k0 >> np.uint64(32)).astype(np.int64) ^ 0x80000000) - 0
    want_cost = cost[np.arange(len(pods)), best]
    assert (np.where(got_cost >= 2**31, got_cost - 2**32, got_cost) == want_cost).all()
