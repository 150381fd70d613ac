"""BASELINE config C4 (50k nodes x 500k pods, node axis split over 2/4/8
GPUs) at its own size, split into G = 2, 4 and 8 VIRTUAL node shards on one
GPU (G = 8, the 6,250-column shard geometry, VERDICT r5
item 7: eight contexts each holding the replicated 25 GB traffic matrix,
~27 GB per context of the 288 GB).

Each shard is its own context (nas_set_shard(r, G) before the uploads) that
scores only node columns [r*N/G, (r+1)*N/G) over the full 50k-deep K; the
candidate lists are merged on the host with the device rule (klist.h) and
every shard replays the same commit (sharded.place_local_shards).  This is
the multi-GPU pass minus the all-gather transport: the 25k / 12.5k-column
shard geometry, the Mp / Kp padding at 50k nodes, the L2-resident commit
(N > 11,541) and the 500k-pod windows all meet here before the first 8-GPU
run.  Placements, integer scores and the capacity left must equal the
world-1 nas_place on the same seed (the decision every rank reproduces:
scheduler.go:239-246 findNodesThatFit, extended mode), and capacity is
conserved.
"""
import numpy as np
import pytest

from kubernetesnetawarescheduler_amd import Engine
from kubernetesnetawarescheduler_amd.sharded import place_local_shards

pytestmark = pytest.mark.gpu
SEED = 0x4E4153
N, P = 50000, 500000


@pytest.fixture(scope="module")
def world1():
    with Engine(0) as e:
        e.synth_cluster(SEED, N, P, "i8", peers=8)
        node, _, score = e.place()
        free = e.get_capacity()
        _, _, cap0, req = e.read_inputs(0, 0, want_L=False)
    return node, score, free, cap0, req


@pytest.mark.parametrize("G", [2, 4, 8])
def test_c4_virtual_shards_equal_world1(world1, G):
    node1, score1, free1, cap0, req = world1
    engines = []
    try:
        for r in range(G):
            e = Engine(0)
            engines.append(e)
            e.set_shard(r, G)
            e.synth_cluster(SEED, N, P, "i8", peers=8)
        node, score, rounds = place_local_shards(engines, P)
        caps = [e.get_capacity() for e in engines]
    finally:
        for e in engines:
            e.close()
    assert node.dtype == node1.dtype and node.shape == (P,)
    bad = np.nonzero(node != node1)[0]
    assert len(bad) == 0, (G, rounds, bad[:8], node[bad[:8]], node1[bad[:8]])
    assert (score == score1).all()
    for c in caps:  # every shard's replicated commit leaves the same capacity
        assert (c == free1).all()
    placed = node >= 0
    used = np.zeros((N, 3), np.int64)
    np.add.at(used, node[placed], req[placed].astype(np.int64))
    assert (cap0.astype(np.int64) - used == free1).all() and (free1 >= 0).all()


def test_c4_local_group_g2_equals_world1(world1):
    """C4 as 2 in-process ranks (nas_comm_init_local): the
    device exchange path of nas_place -- per-chunk all-gather of distinct
    rank lists into [2][np][8 + 1], the cross-rank k_merge, the replicated L2
    commit -- at the full 50k x 500k size, equal to world 1."""
    from kubernetesnetawarescheduler_amd import LocalGroup, local_ranks
    node1, score1, free1, _, _ = world1
    group = LocalGroup(2)
    engines = [Engine(0) for _ in range(2)]
    try:
        def run(r, e):
            e.comm_init_local(group, r)
            e.synth_cluster(SEED, N, P, "i8", peers=8)
            node, _, score = e.place()
            return node, score, e.get_capacity()
        res = local_ranks(engines, run)
    finally:
        for e in engines:
            e.close()
        group.close()
    for r, (node, score, cap) in enumerate(res):
        bad = np.nonzero(node != node1)[0]
        assert len(bad) == 0, (r, bad[:8], node[bad[:8]], node1[bad[:8]])
        assert (score == score1).all() and (cap == free1).all(), r
