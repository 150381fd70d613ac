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
