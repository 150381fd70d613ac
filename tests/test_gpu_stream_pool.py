"""CU-masked streams come from a process-wide pool.

A node-shard context reserves CUs for its commit stream with CU-masked
streams (hipExtStreamCreateWithCUMask; each is a hardware queue with the mask
programmed into it).  Round 5's world-1 variant that made such streams for
EVERY context hung in the ~50th context's stream creation; contexts now
borrow masked streams from a pool and return them on nas_destroy, so
creating and destroying shard contexts again and again does not grow the
number of masked streams (nas_debug_counters), and the pooled streams still
run correct passes."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine, LocalGroup, local_ranks
from kubernetesnetawarescheduler_amd.engine import debug_counters
from util import cluster

pytestmark = pytest.mark.gpu


def _group_pass(G, WA, L, free, req):
    group = LocalGroup(G)
    engines = [Engine(0) for _ in range(G)]
    try:
        def run(r, e):
            e.set_option("COMM_TIMEOUT_MS", 60000)
            e.comm_init_local(group, r)  # node shard: masked streams from the pool
            e.upload_latency(L, "i8")
            e.upload_capacity(free)
            e.upload_pods(req)
            e.upload_traffic(WA, "i8")
            e.reset_capacity()
            node, _, score = e.place()
            return node, score, debug_counters()
        return local_ranks(engines, run)
    finally:
        for e in engines:
            e.close()
        group.close()


def test_shard_contexts_reuse_pooled_masked_streams():
    rng = np.random.default_rng(5)
    WA, L, free, req = cluster(rng, 9000, 1200)
    want, wcost, _ = oracle.place(WA, L, req, free, "i8")
    before = debug_counters()
    created = []
    for it in range(12):  # 12 x 4 shard contexts, one after another
        out = _group_pass(4, WA, L, free, req)
        for node, score, during in out:
            assert (node == want).all() and (score == wcost).all(), it
            # 4 ranks x (2 scoring + 1 commit + 1 exchange stream) lent at most
            assert during["masked_streams_lent"] <= before["masked_streams_lent"] + 16
        after = debug_counters()
        assert after["masked_streams_lent"] == before["masked_streams_lent"], after
        assert after["live_contexts"] == before["live_contexts"], after
        created.append(after["masked_streams_created"])
    # the first group created what it needed; every later one borrowed them
    assert created[0] - before["masked_streams_created"] <= 16
    assert all(c == created[0] for c in created), created
    assert debug_counters()["masked_streams_idle"] >= created[0] - before["masked_streams_created"]


def test_world1_contexts_make_no_masked_streams():
    before = debug_counters()
    for _ in range(20):
        with Engine(0) as e:
            e.synth_cluster(3, 500, 1024, "i8", peers=8)
            e.place()
    after = debug_counters()
    assert after["masked_streams_created"] == before["masked_streams_created"]
    assert after["live_contexts"] == before["live_contexts"]
