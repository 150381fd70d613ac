"""The node-shard path of nas_place with G DISTINCT ranks on one GPU
(VERDICT r3 item 1): G contexts joined to an in-process group
(nas_comm_init_local), each driven by its own host thread, run the real
RCCL-path code -- per-chunk local merge into the send buffer, the all-gather
(here a device-to-device pull behind host barriers instead of ncclAllGather),
the cross-rank k_merge over the rank-major [world][np][8 + 1] buffer with its
pr0 / seg strides, the replicated commit, the device rescore slots and the
gathered rescores with their own exchanges -- on genuinely different per-rank
candidate lists (rank r scores node columns [r*N/G, (r+1)*N/G) only).

Placements, integer scores and the capacity left on EVERY rank must equal the
sequential oracle (the decision each rank reproduces: scheduler.go:239-246
findNodesThatFit, extended mode) -- at oracle-sized crowded clusters in full,
at the C3 shape (10k x 100k) against the world-1 pass plus an oracle prefix.
"""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine, LocalGroup, NasError, local_ranks
from util import cluster

pytestmark = pytest.mark.gpu


def run_group(G, setup, passes=1, timeout_ms=60000):
    """G ranks of one in-process group: setup(rank, engine) uploads, then
    `passes` nas_place calls (capacity reset between them).  Returns per rank
    [(node, score, capacity, timings), ...] of every pass."""
    group = LocalGroup(G)
    engines = [Engine(0) for _ in range(G)]
    try:
        def run(r, e):
            e.set_option("COMM_TIMEOUT_MS", timeout_ms)
            e.comm_init_local(group, r)
            setup(r, e)
            out = []
            for _ in range(passes):
                e.reset_capacity()
                node, _, score = e.place()
                out.append((node, score, e.get_capacity(), e.timings()))
            return out
        return local_ranks(engines, run)
    finally:
        for e in engines:
            e.close()
        group.close()


def upload(WA, L, free, req, dtype="i8"):
    def setup(r, e):
        e.upload_latency(L, dtype)
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, dtype)
    return setup


@pytest.mark.parametrize("G,P,N,crowd", [(2, 12000, 1500, 40), (3, 12000, 1500, 40),
                                         (4, 20000, 700, 24), (8, 12000, 2100, 64),
                                         (8, 3000, 300, 0)])
def test_local_group_place_equals_oracle(G, P, N, crowd):
    """Crowded clusters: herds on the first nodes drain 8-key lists, so the
    commit halts and the device rescore slots / gathered rescores (each with
    its own all-gather + cross-rank merge) fire on every rank."""
    rng = np.random.default_rng(G * 100 + P + N)
    WA, L, free, req = cluster(rng, P, N, lo=0, hi=30, cap_scale=0.6)
    if crowd:
        WA[:, :crowd] = 127
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    res = run_group(G, upload(WA, L, free, req), passes=2)
    for r, passes in enumerate(res):
        for node, score, cap, t in passes:
            bad = np.nonzero(node != want)[0]
            assert len(bad) == 0, (G, r, bad[:8], node[bad[:8]], want[bad[:8]])
            assert score.tolist() == wcost.tolist(), (G, r)
            assert (cap == wfree).all(), (G, r)
            if crowd:
                assert t["rescore_rounds"] > 0, (G, r, t)
    # (commit_rounds may differ between ranks and runs: which reservation of a
    # window fails first depends on the order its atomics land -- the
    # placements do not, as checked above)


def test_local_group_bf16_equals_oracle():
    """bf16 (integer-valued, so exact) through the same exchange."""
    G, P, N = 3, 6000, 900
    rng = np.random.default_rng(77)
    WA, L, free, req = cluster(rng, P, N, dtype="bf16", lo=0, hi=30, cap_scale=0.5)
    want, _, wfree = oracle.place(WA, L, req, free, "bf16")
    for node, _, cap, _ in (p[0] for p in run_group(G, upload(WA, L, free, req, "bf16"))):
        assert node.tolist() == want.tolist()
        assert (cap == wfree).all()


C3_N, C3_P, C3_SEED = 10000, 100000, 0xC3C3


@pytest.fixture(scope="module")
def c3_world1():
    """World-1 passes of C3 (synthetic, seeded) at its own capacity and at a
    crowded one (capacity / 6: lists run dry, rescore slots fire), plus the
    inputs for an oracle prefix."""
    out = {}
    with Engine(0) as e:
        e.synth_cluster(C3_SEED, C3_N, C3_P, "i8", peers=8)
        WA, L, cap0, req = e.read_inputs(0, 4096, want_L=True)
        for name, cap in (("default", cap0), ("crowded", cap0 // 6)):
            e.upload_capacity(cap)
            node, _, score = e.place()
            # the first 4096 placements against the sequential oracle (a
            # prefix of a sequential greedy depends on nothing after it)
            want = oracle.place(WA, L, req[:4096], cap, "i8")
            out[name] = (cap, node, score, e.get_capacity(), e.timings(), want)
    return out


@pytest.mark.parametrize("variant", ["default", "crowded"])
@pytest.mark.parametrize("G", [2, 4, 8])
def test_local_group_c3_equals_world1(c3_world1, G, variant):
    cap, node1, score1, free1, t1, (want, wcost, _) = c3_world1[variant]
    assert node1[:4096].tolist() == want.tolist() and score1[:4096].tolist() == wcost.tolist()

    def setup(r, e):
        e.synth_cluster(C3_SEED, C3_N, C3_P, "i8", peers=8)
        e.upload_capacity(cap)

    res = run_group(G, setup)
    for r, ((node, score, left, t),) in enumerate(res):
        bad = np.nonzero(node != node1)[0]
        assert len(bad) == 0, (G, variant, r, bad[:8], node[bad[:8]], node1[bad[:8]])
        assert (score == score1).all(), (G, variant, r)
        assert (left == free1).all(), (G, variant, r)
        if variant == "crowded":
            assert t["rescore_rounds"] > 0, t


def test_local_group_vote_node_shard_equals_oracle():
    """Reference mode, node axis (nas_upload_snapshot_shard + the all-gather of
    partial records inside nas_score_reference) over 3 in-process ranks."""
    from util import random_snapshot
    G, N, S = 3, 257, 40
    rng = np.random.default_rng(5)
    snaps = [random_snapshot(rng, N) for _ in range(S)]
    o1 = rng.permutation(N).astype(np.int32)
    o2 = rng.permutation(N + 1).astype(np.int32)
    want = [oracle.vote(s, o1, o2)[0] for s in snaps]
    full = {k: np.stack([s[k] for s in snaps]) for k in snaps[0]}
    group = LocalGroup(G)
    engines = [Engine(0) for _ in range(G)]
    try:
        def run(r, e):
            e.comm_init_local(group, r)
            lo, hi = r * N // G, (r + 1) * N // G
            e.upload_snapshot_shard({k: v[:, lo:hi] for k, v in full.items()}, N, lo)
            return e.score_reference(S, o1, o2)[0]
        for best in local_ranks(engines, run):
            assert best.tolist() == want
    finally:
        for e in engines:
            e.close()
        group.close()


def test_local_group_missing_rank_fails_with_deadline():
    """A rank that never calls: the others' first exchange misses
    NAS_OPT_COMM_TIMEOUT_MS, the group breaks, every context is poisoned and
    returns NAS_ERR_COMM (no hang)."""
    rng = np.random.default_rng(3)
    WA, L, free, req = cluster(rng, 2000, 300)
    group = LocalGroup(2)
    engines = [Engine(0) for _ in range(2)]
    try:
        def run(r, e):
            e.set_option("COMM_TIMEOUT_MS", 1500)
            e.comm_init_local(group, r)
            upload(WA, L, free, req)(r, e)
            if r == 1:
                return None
            with pytest.raises(NasError) as ex:
                e.place()
            assert ex.value.code == -5  # NAS_ERR_COMM
            with pytest.raises(NasError):
                e.place()  # poisoned
            return True
        assert local_ranks(engines, run)[0] is True
        with pytest.raises(NasError):  # the group is broken for rank 1 too
            engines[1].place()
    finally:
        for e in engines:
            e.close()
        group.close()


def test_local_group_rejects_bad_joins():
    group = LocalGroup(2)
    with Engine(0) as a, Engine(0) as b:
        a.comm_init_local(group, 0)
        with pytest.raises(NasError):
            b.comm_init_local(group, 0)  # rank taken
        with pytest.raises(NasError):
            b.comm_init_local(group, 2)  # out of range
    group.close()
    with pytest.raises(NasError):
        LocalGroup(0)
