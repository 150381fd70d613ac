"""Node-axis sharding on one GPU: G contexts each score node columns
[r*N/G, (r+1)*N/G) (nas_set_shard, no communicator), their candidate lists
are merged on the host with the rule the RCCL path applies on device, and the
merged exact prefix must equal the oracle's unsharded ranking.  This is the
multi-GPU scoring path minus the all-gather (covered by test_dist_cpu)."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine
from util import KEY_INVALID, cluster, merge_lists, usable

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("G,P,N,dtype", [(2, 700, 1500, "i8"), (3, 1000, 1000, "i8"),
                                         (4, 300, 70, "i8"), (2, 512, 700, "bf16")])
def test_shards_merge_to_global_ranking(G, P, N, dtype):
    rng = np.random.default_rng(G * 1000 + N)
    WA, L, free, req = cluster(rng, P, N, dtype=dtype, lo=-20 if dtype == "i8" else 0, hi=40,
                               cap_scale=0.1)
    parts = []
    for r in range(G):
        with Engine(0) as e:
            e.set_shard(r, G)
            e.upload_latency(L, dtype)
            e.upload_capacity(free)
            e.upload_pods(req)
            e.upload_traffic(WA, dtype)
            e.score()
            parts.append(e.candidate_keys())
            nodes = (parts[-1][0] & np.uint64(0xFFFFFFFF)).astype(np.int64)
            valid = parts[-1][0] != KEY_INVALID
            lo, hi = r * N // G, (r + 1) * N // G
            assert ((nodes[valid] >= lo) & (nodes[valid] < hi)).all()
    mk, mb = merge_lists(parts)
    node, cnt = usable(mk, mb)
    cost = oracle.cost(WA, L, dtype)
    wn, wc, wcnt = oracle.topk(cost, oracle.fit_mask(req, free), 8)
    assert (cnt >= np.minimum(4, wcnt)).all()
    for p in range(P):
        assert node[p, :cnt[p]].tolist() == wn[p, :cnt[p]].tolist(), p
    complete = mb == KEY_INVALID
    assert (cnt[complete] == wcnt[complete]).all()
    got, _, _, stop = oracle.commit(node, cnt, req, free, complete)
    want, _, _ = oracle.place(WA, L, req, free, dtype)
    assert got[:stop].tolist() == want[:stop].tolist()


def test_shard_rejects_place_and_late_set(engine):
    with Engine(0) as e:
        e.set_shard(0, 2)
        rng = np.random.default_rng(1)
        WA, L, free, req = cluster(rng, 10, 10)
        e.upload_latency(L, "i8")
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, "i8")
        with pytest.raises(Exception):
            e.place()
        with pytest.raises(Exception):
            e.set_shard(1, 2)


@pytest.mark.parametrize("G,P,N", [(2, 3000, 500), (3, 5000, 700), (4, 2500, 257)])
def test_host_exchange_place_equals_single_context(G, P, N):
    """The whole sharded placement (score -> host exchange + merge -> replicated
    commit -> rescore windows) over G node-shard contexts equals one context's
    nas_place and the sequential oracle -- placements, scores, capacity."""
    from kubernetesnetawarescheduler_amd.sharded import place_local_shards
    rng = np.random.default_rng(G * 7 + P)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.15)
    WA[:, : N // 16] = 127  # crowding: commit conflicts and rescore windows
    engines = []
    try:
        for r in range(G):
            e = Engine(0)
            engines.append(e)
            e.set_shard(r, G)
            e.upload_latency(L, "i8")
            e.upload_capacity(free)
            e.upload_pods(req)
            e.upload_traffic(WA, "i8")
        node, score, rounds = place_local_shards(engines, P)
        caps = [e.get_capacity() for e in engines]
    finally:
        for e in engines:
            e.close()
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert rounds > 0
    assert node.tolist() == want.tolist()
    assert score.tolist() == wcost.tolist()
    for c in caps:
        assert (c == wfree).all()
    with Engine(0) as e:
        e.upload_latency(L, "i8")
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, "i8")
        n1, _, s1 = e.place()
    assert n1.tolist() == node.tolist() and s1.tolist() == score.tolist()


def test_commit_api_stops_and_resumes(engine):
    """nas_commit on one context: stop pods, rescore windows, resume --
    equals nas_place."""
    rng = np.random.default_rng(9)
    P, N = 4000, 300
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.1)
    WA[:, :10] = 127
    engine.upload_latency(L, "i8")
    engine.upload_capacity(free)
    engine.upload_pods(req)
    engine.upload_traffic(WA, "i8")
    engine.score_range(0, P)
    node = np.full(P, -9, np.int32)
    score = np.zeros(P, np.int64)
    stop, stops = 0, []
    while True:
        stop = engine.commit(stop, node, score)
        if stop >= P:
            break
        stops.append(stop)
        assert (node[:stop] != -9).all()
        engine.score_range(stop, min(P, stop + 1024))
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert stops and stops == sorted(stops)
    assert node.tolist() == want.tolist() and score.tolist() == wcost.tolist()
    assert (engine.get_capacity() == wfree).all()


@pytest.mark.parametrize("P,N,crowd", [(20000, 256, 24), (3000, 1200, 0)])
def test_rccl_world1_place_equals_oracle(P, N, crowd):
    """nas_comm_init with world 1 builds real RCCL communicators (one per
    stream), so every scoring chunk, device-side rescore slot and host-loop
    rescore goes through ncclAllGather + the cross-rank merge on this GPU.
    Placements, scores and the capacity left must equal the sequential
    oracle exactly (the multi-rank collectives themselves run on the driver's
    8-GPU node; their merge rule is covered by test_shards_merge_*)."""
    rng = np.random.default_rng(P + N)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.6)
    if crowd:
        WA[:, :crowd] = 127  # herds on the first nodes: commit stops, rescores
    with Engine(0) as e:
        e.comm_init(Engine.comm_unique_id(), 0, 1)
        e.upload_latency(L, "i8")
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, "i8")
        for _ in range(2):  # a second pass reuses the communicators
            e.reset_capacity()
            node, _, ci = e.place()
            want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
            assert node.tolist() == want.tolist() and ci.tolist() == wcost.tolist()
            assert (e.get_capacity() == wfree).all()
        if crowd:
            assert e.timings()["rescore_rounds"] > 0


@pytest.mark.parametrize("G", [2, 8])
def test_rehearsal_pass_is_well_formed(G, monkeypatch):
    """bench.py --rehearse-world: rank 0 of a G-GPU pass on one GPU (shifted
    copies stand in for the other ranks' lists, so placements are not the
    oracle's).  The commit is real, so capacity is still conserved and every
    placement is a node index that fitted."""
    rng = np.random.default_rng(G)
    P, N = 6000, 800
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=4.0)
    monkeypatch.setenv("NAS_REHEARSE_WORLD", str(G))
    with Engine(0) as e:
        e.comm_init(Engine.comm_unique_id(), 0, 1)
        monkeypatch.delenv("NAS_REHEARSE_WORLD")
        e.upload_latency(L, "i8")
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, "i8")
        node, _, _ = e.place()
        left = e.get_capacity()
    assert ((node >= 0) & (node < N) | (node == -1)).all()
    placed = node >= 0
    used = np.zeros((N, 3), np.int64)
    np.add.at(used, node[placed], req[placed].astype(np.int64))
    assert (free.astype(np.int64) - used == left).all() and (left >= 0).all()
    assert placed.sum() > P // 2
