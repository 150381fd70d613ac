"""GPU parity of the node-sharded reference mode (vote row):
k_vote_partial's records bit-equal to the oracle's restatement, k_vote_merge's
decisions equal to the literal Go loop, and nas_score_reference over a
one-rank RCCL communicator (partial -> ncclAllGather -> merge) equal to the
unsharded kernel.  Bit-exact: best node and all six winners per snapshot."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine, NasError
from kubernetesnetawarescheduler_amd.engine import VOTE_PARTIAL_DTYPE
from test_vote_shard_cpu import edge_snapshot, sliced
from util import random_snapshot, stack_snapshots

pytestmark = pytest.mark.gpu
PF = ("cpu", "mem", "bw", "rx", "tx", "disk")


def snapshots(rng, n, S):
    return [edge_snapshot(rng, n) if s % 3 == 0 else random_snapshot(rng, n, s % 3 == 1)
            for s in range(S)]


def cuts_for(rng, n, G):
    inner = sorted(rng.choice(np.arange(1, n), G - 1, replace=False).tolist()) if G > 1 else []
    return [0] + inner + [n]


def gpu_partials(e, snaps, lo, hi, o1, o2):
    e.upload_snapshot_shard(stack_snapshots([sliced(m, lo, hi) for m in snaps]),
                            len(o1[0]) if np.ndim(o1) == 2 else len(o1), lo)
    if np.ndim(o1) == 2:
        e.upload_orders(o1, o2)
        return e.vote_partials()
    return e.vote_partials(None, o1, o2)


@pytest.mark.parametrize("n,S,G", [(5, 40, 2), (37, 60, 3), (300, 50, 7), (1001, 20, 8)])
def test_partials_bit_equal_oracle(engine, n, S, G):
    rng = np.random.default_rng(n * 7 + G)
    snaps = snapshots(rng, n, S)
    o1 = np.stack([rng.permutation(n) for _ in range(S)]).astype(np.int32)
    o2 = np.stack([rng.permutation(n + 1) for _ in range(S)]).astype(np.int32)
    cuts = cuts_for(rng, n, G)
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        got = gpu_partials(engine, snaps, lo, hi, o1, o2)
        for s, m in enumerate(snaps):
            want = oracle.vote_partial(sliced(m, lo, hi), lo, o1[s])
            assert [(int(r["value"]), int(r["pos1"])) for r in got[s]] == want, (lo, hi, s)
            assert (got[s]["reserved"] == 0).all()


@pytest.mark.parametrize("n,S,G,per_snapshot", [(5, 64, 5, True), (64, 200, 4, False),
                                                (999, 100, 8, True), (4097, 16, 3, False)])
def test_merge_equals_literal_loop(engine, n, S, G, per_snapshot):
    rng = np.random.default_rng(n + S + G)
    snaps = snapshots(rng, n, S)
    if per_snapshot:
        o1 = np.stack([rng.permutation(n) for _ in range(S)]).astype(np.int32)
        o2 = np.stack([rng.permutation(n + 1) for _ in range(S)]).astype(np.int32)
    else:
        o1 = rng.permutation(n).astype(np.int32)
        o2 = rng.permutation(n + 1).astype(np.int32)
    cuts = cuts_for(rng, n, G)
    parts = np.stack([gpu_partials(engine, snaps, a, b, o1, o2)
                      for a, b in zip(cuts[:-1], cuts[1:])])
    # the merging context holds the last shard and the same orders
    best, win = engine.vote_merge(parts)
    rbest, rwin = engine.vote_merge(parts[::-1].copy())  # slice order is free
    assert (best == rbest).all() and (win == rwin).all()
    for s, m in enumerate(snaps):
        a = o1[s] if per_snapshot else o1
        b = o2[s] if per_snapshot else o2
        wb, ww, _ = oracle.vote(m, a, b)
        assert best[s] == wb and win[s].tolist() == list(ww), s


def test_synth_shards_merge_to_full_kernel(engine):
    """10k nodes x 64 synthetic snapshots (the bench generator), 8 node
    slices: merged slices == the unsharded k_vote, and each synthesised slice
    == the same nodes of the full synthesis."""
    n, S, G, seed = 10000, 64, 8, 0x4E4153
    rng = np.random.default_rng(5)
    o1 = rng.permutation(n).astype(np.int32)
    o2 = rng.permutation(n + 1).astype(np.int32)
    engine.synth_snapshots(seed, n, S)
    full = [engine.read_snapshot(s) for s in (0, S - 1)]
    want_best, want_win = engine.score_reference(S, o1, o2)
    parts = []
    for r in range(G):
        lo, hi = r * n // G, (r + 1) * n // G
        engine.synth_snapshots_shard(seed, n, lo, hi - lo, S)
        for s, f in zip((0, S - 1), full):
            got = engine.read_snapshot(s)
            for k in got:
                np.testing.assert_array_equal(got[k], f[k][lo:hi])
        parts.append(engine.vote_partials(None, o1, o2))
    best, win = engine.vote_merge(np.stack(parts))
    assert (best == want_best).all() and (win == want_win).all()


@pytest.mark.parametrize("n,S", [(7, 30), (2500, 40)])
def test_rccl_world1_score_reference_on_a_shard(n, S):
    """nas_score_reference on a node-sharded snapshot with a one-rank
    communicator: partial -> ncclAllGather -> merge, incl. pod_snapshot."""
    rng = np.random.default_rng(n)
    snaps = snapshots(rng, n, S)
    snap = stack_snapshots(snaps)
    o1 = rng.permutation(n).astype(np.int32)
    o2 = rng.permutation(n + 1).astype(np.int32)
    pods = rng.integers(0, S, 3 * S).astype(np.int32)
    with Engine(0) as e:
        e.upload_snapshot_shard(snap, n, 0)
        with pytest.raises(NasError, match="nas_comm_init"):
            e.score_reference(S, o1, o2)
        e.comm_init(Engine.comm_unique_id(), 0, 1)
        for _ in range(2):
            best, win = e.score_reference(None, o1, o2, pod_snapshot=pods)
            wb, ww = oracle.vote_batch(snap, o1, o2, pods)
            assert (best == wb).all() and (win == ww).all()
        best, win = e.score_reference(S, o1, o2)
        wb, ww = oracle.vote_batch(snap, o1, o2)
        assert (best == wb).all() and (win == ww).all()


def test_shard_argument_errors(engine):
    rng = np.random.default_rng(3)
    m = random_snapshot(rng, 10)
    with pytest.raises(NasError):
        engine.upload_snapshot_shard(sliced(m, 0, 6), 5, 0)  # slice past n_nodes
    with pytest.raises(NasError):
        engine.upload_snapshot_shard(sliced(m, 0, 6), 10, 5)
    engine.upload_snapshot_shard(sliced(m, 4, 10), 10, 4)
    o1 = rng.permutation(10).astype(np.int32)
    o2 = rng.permutation(11).astype(np.int32)
    parts = engine.vote_partials(None, o1, o2)[None]
    bad = parts.copy()
    bad[0, 0, 0]["pos1"] = 10  # outside [0, n_nodes)
    with pytest.raises(NasError):
        engine.vote_merge(bad)
    with pytest.raises(NasError):
        engine.vote_partials(2)  # S > n_snapshots
    best, _ = engine.vote_merge(parts)
    assert best.shape == (1,)
    assert np.dtype(VOTE_PARTIAL_DTYPE).itemsize * 6 == 96
