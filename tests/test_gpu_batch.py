"""Multi-tenant batches (BASELINE config C5): independent clusters of one
shape placed by one nas_place -- one fit / cost / merge launch with the
cluster as a grid dimension, one commit workgroup per cluster, batched rescore
slots.  Every cluster's placements must equal the sequential oracle on its own
inputs (and a single-cluster context on the same inputs)."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine
from util import cluster

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,P,N", [(2, 300, 200), (5, 1500, 700), (3, 3000, 256)])
def test_batch_equals_oracle_per_cluster(B, P, N):
    rng = np.random.default_rng(B * 100 + N)
    cs = []
    for b in range(B):
        WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.1 + 0.05 * b)
        WA[:, rng.choice(N, max(2, N // 20), replace=False)] = 127  # crowding: stops, rescores
        cs.append((WA, L, free, req))
    with Engine(0) as e:
        e.set_batch(B)
        e.upload_latency(np.stack([c[1] for c in cs]), "i8")
        e.upload_capacity(np.stack([c[2] for c in cs]))
        e.upload_pods(np.stack([c[3] for c in cs]))
        e.upload_traffic(np.stack([c[0] for c in cs]), "i8")
        node, _, score = e.place()
        cap = e.get_capacity()
        t = e.timings()
    assert node.shape == (B, P)
    unsched = 0
    for b, (WA, L, free, req) in enumerate(cs):
        want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
        assert node[b].tolist() == want.tolist(), b
        assert score[b].tolist() == wcost.tolist(), b
        assert (cap[b] == wfree).all(), b
        unsched += int((want < 0).sum())
    assert t["unschedulable"] == unsched


def test_synth_batch_matches_single_clusters():
    B, N, P = 4, 1024, 3000
    with Engine(0) as e:
        e.synth_batch(0x4E4153, B, N, P, "i8", peers=8)
        nb, _, sb = e.place()
    for b in range(B):
        with Engine(0) as s:
            s.synth_cluster(0x4E4153 + b, N, P, "i8", peers=8)
            n1, _, s1 = s.place()
        assert nb[b].tolist() == n1.tolist() and sb[b].tolist() == s1.tolist(), b


def test_batch_rejects_shards():
    with Engine(0) as e:
        e.set_batch(2)
        with pytest.raises(Exception):
            e.set_shard(0, 2)


def test_c2_workload_equals_oracle():
    """BASELINE config C2 at full size (1k nodes x 10k pods, CSR traffic)."""
    from kubernetesnetawarescheduler_amd import workloads
    c = workloads.c2_cluster(0x4E4153, 1000, 10000)
    with Engine(0) as e:
        e.upload_latency(c["L"], "i8")
        e.upload_capacity(c["free"])
        e.upload_pods(c["req"])
        e.upload_traffic_csr(c["row_ptr"], c["peer_node"], c["weight"], "i8", 1000)
        node, _, score = e.place()
        cap = e.get_capacity()
    WA = workloads.csr_to_dense(c["row_ptr"], c["peer_node"], c["weight"], 1000)
    want, wcost, wfree = oracle.place(WA, c["L"], c["req"], c["free"], "i8")
    assert node.tolist() == want.tolist() and score.tolist() == wcost.tolist()
    assert (cap == wfree).all()


@pytest.mark.parametrize("B", [300, 1100])
def test_large_batch_of_tiny_clusters(B):
    """More clusters than the first pinned page of status words holds
    (4096 B / 16 B = 256): the staged placements must not be overwritten by
    the status round trip."""
    rng = np.random.default_rng(B)
    P, N = 40, 64
    cs = []
    for b in range(B):
        WA, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.05 + 0.002 * (b % 50))
        if b % 3 == 0:
            WA[:, rng.choice(N, 3, replace=False)] = 127  # crowding: stops, rescores
        cs.append((WA, L, free, req))
    with Engine(0) as e:
        e.set_batch(B)
        e.upload_latency(np.stack([c[1] for c in cs]), "i8")
        e.upload_capacity(np.stack([c[2] for c in cs]))
        e.upload_pods(np.stack([c[3] for c in cs]))
        e.upload_traffic(np.stack([c[0] for c in cs]), "i8")
        node, cost, score = e.place()
        cap = e.get_capacity()
    for b, (WA, L, free, req) in enumerate(cs):
        want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
        assert node[b].tolist() == want.tolist(), b
        assert score[b].tolist() == wcost.tolist(), b
        assert cost[b].tolist() == [float(x) for x in wcost], b
        assert (cap[b] == wfree).all(), b
