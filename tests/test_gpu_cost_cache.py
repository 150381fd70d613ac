"""The herd plan (NAS_OPT_HERD_PLAN: chunk after chunk -- fit + cost, merge,
commit -- on one stream, so every chunk's fit sees its predecessors'
commits) and the cost-row cache (NAS_OPT_COST_CACHE, k_rescore_cached): a pass's main
cost launches also store every (pod, node) cost, and its gathered rescore
slots build a dry pod's new 8-list from the pod's cached row against the
capacity now instead of re-running fit + contraction + merge.  The lists --
and so every placement, integer score and the capacity left -- must be the
sequential oracle's exactly, with the cache forced on, forced off, and in
auto mode (on from the second pass of a shape whose first pass needed >= 4
rescore rounds); through the node-shard exchange too."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine, LocalGroup, local_ranks
from util import cluster

pytestmark = pytest.mark.gpu


def _herd(seed, P, N, crowd, dtype="i8"):
    rng = np.random.default_rng(seed)
    WA, L, free, req = cluster(rng, P, N, dtype=dtype, lo=0, hi=30, cap_scale=0.6)
    if crowd:
        WA[:, :crowd] = 127 if dtype == "i8" else WA[:, :crowd].max()
    return WA, L, free, req


def _upload(e, WA, L, free, req, dtype="i8"):
    e.upload_latency(L, dtype)
    e.upload_capacity(free)
    e.upload_pods(req)
    e.upload_traffic(WA, dtype)


@pytest.mark.parametrize("P,N,crowd", [(12000, 1500, 40), (20000, 700, 24), (40000, 3000, 0)])
@pytest.mark.parametrize("mode,herd", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_cache_on_off_equal_oracle(engine, P, N, crowd, mode, herd):
    WA, L, free, req = _herd(P + N + crowd, P, N, crowd)
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    engine.set_option("COST_CACHE", mode)
    engine.set_option("HERD_PLAN", herd)
    try:
        _upload(engine, WA, L, free, req)
        for _ in range(2):
            engine.reset_capacity()
            node, _, score = engine.place()
            bad = np.nonzero(node != want)[0]
            assert len(bad) == 0, (mode, bad[:8], node[bad[:8]], want[bad[:8]])
            assert (score == wcost).all() and (engine.get_capacity() == wfree).all()
        if crowd and not herd:
            assert engine.timings()["rescore_rounds"] > 0
    finally:
        engine.set_option("COST_CACHE", 2)
        engine.set_option("HERD_PLAN", 2)


def test_auto_herd_plan_and_cache_keep_results():
    """Full-range operands: a global herd.  The first pass
    (pipelined plan, no cache) rescores in many rounds; from the second on
    (auto: its shape needed >= 8 rounds) the herd plan and the cache --
    identical placements, far fewer rescore rounds."""
    with Engine(0) as e:
        e.synth_cluster(0x4E4153, 3000, 60000, "i8", peers=8, profile=1)
        e.reset_capacity()
        n1, _, s1 = e.place()
        t1 = e.timings()
        assert t1["rescore_rounds"] >= 8, t1
        res = []
        for _ in range(2):
            e.reset_capacity()
            n2, _, s2 = e.place()
            res.append(e.timings())
            assert (n1 == n2).all() and (s1 == s2).all()
        WA, L, cap, req = e.read_inputs(0, 60000, want_L=True)
        want, wcost, _ = oracle.place(WA, L, req, cap, "i8")
        assert (n1 == want).all() and (s1 == wcost).all()
        # (the herd plan's chunks differ from the pipelined plan's)
        assert res[-1]["cost_launches"] != t1["cost_launches"], (t1, res)


def test_cache_bf16_herd_equals_oracle(engine):
    rng = np.random.default_rng(77)
    WA, L, free, req = cluster(rng, 12000, 1500, dtype="bf16", lo=0, hi=30, cap_scale=0.6)
    WA[:, :40] = WA[:, :40].max()
    want, _, _ = oracle.place(WA, L, req, free, "bf16")
    for mode in (1, 0):
        engine.set_option("COST_CACHE", mode)
        _upload(engine, WA, L, free, req, "bf16")
        engine.reset_capacity()
        node, _, _ = engine.place()
        assert (node == want).all(), mode
    engine.set_option("COST_CACHE", 2)


@pytest.mark.parametrize("G", [2, 4])
def test_cache_through_the_shard_exchange(G):
    """Node shards: each rank rescores its columns from its own cached rows
    into the view, the view is all-gathered and merged across ranks."""
    WA, L, free, req = _herd(G * 7, 12000, 1500, 40)
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    group = LocalGroup(G)
    engines = [Engine(0) for _ in range(G)]
    try:
        def run(r, e):
            e.set_option("COMM_TIMEOUT_MS", 60000)
            e.set_option("COST_CACHE", 1)
            e.comm_init_local(group, r)
            _upload(e, WA, L, free, req)
            e.reset_capacity()
            node, _, score = e.place()
            return node, score, e.get_capacity(), e.timings()
        res = local_ranks(engines, run)
    finally:
        for e in engines:
            e.close()
        group.close()
    for r, (node, score, cap, t) in enumerate(res):
        assert (node == want).all() and (score == wcost).all() and (cap == wfree).all(), r
        assert t["rescore_rounds"] > 0
