"""Replay files on the GPU: a problem captured from an engine (or written by
the caller) and replayed into a fresh context gives the same decisions,
digest for digest -- dense int8 / exact int32 traffic, bf16, fp32, the
synthetic-cluster form, and reference-mode vote problems."""
import numpy as np
import pytest

import oracle
from kubernetesnetawarescheduler_amd import Engine
from kubernetesnetawarescheduler_amd import snapshot as S
from util import cluster

pytestmark = pytest.mark.gpu


def test_capture_and_replay_synthetic_cluster(tmp_path):
    with Engine(0) as e:
        e.synth_cluster(0x4E4153, 1500, 4000, "i8", peers=8)
        S.capture_place(e, tmp_path / "c.npz", rows_per_read=1000)
        node, _, score = e.place()
    with Engine(0) as e2:
        n2, _, s2 = S.replay_place(e2, tmp_path / "c.npz")
    assert S.digest(node, score) == S.digest(n2, s2)
    f = S.load(tmp_path / "c.npz")
    want, wcost, _ = oracle.place(f["WA"], f["L"], f["req"], f["free"], "i8")
    assert node.tolist() == want.tolist() and score.tolist() == wcost.tolist()
    S.save_place_synth(tmp_path / "s.npz", 0x4E4153, 1500, 4000, "i8", peers=8)
    with Engine(0) as e3:
        n3, _, s3 = S.replay_place(e3, tmp_path / "s.npz")
    assert S.digest(n3, s3) == S.digest(node, score)


@pytest.mark.parametrize("dtype", ["i8", "bf16", "f32"])
def test_dense_replay(tmp_path, dtype):
    rng = np.random.default_rng(7)
    P, N = 1200, 300
    _, _, free, req = cluster(rng, P, N, cap_scale=0.05)
    if dtype == "i8":
        L = rng.integers(0, 100, (N, N), dtype=np.int8)
        WA = rng.integers(0, 400, (P, N)).astype(np.int32)  # beyond int8: overflow lists
    else:
        L = rng.integers(50, 251, (N, N)).astype(np.float32)
        WA = rng.integers(0, 101, (P, N)).astype(np.float32)
        if dtype == "bf16":
            L, WA = ((a.view(np.uint32) >> 16).astype(np.uint16) for a in (L, WA))
    S.save_place(tmp_path / "d.npz", L, free, req, WA, dtype)
    with Engine(0) as e:
        e.upload_latency(L, dtype)
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, dtype)
        node, cf, _ = e.place()
        S.capture_place(e, tmp_path / "c.npz")
    for f in ("d.npz", "c.npz"):
        with Engine(0) as e2:
            n2, c2, _ = S.replay_place(e2, tmp_path / f)
        assert S.digest(node, cf) == S.digest(n2, c2), f


def test_vote_replay(tmp_path):
    rng = np.random.default_rng(8)
    S_, N = 50, 40
    snap = {"cpu": rng.choice([6e8, 1.2e9, 1.5e9], (S_, N)), "mem": rng.random((S_, N)) * 100,
            "bw": rng.random((S_, N)) * 9e7, "rx": rng.integers(0, 1e6, (S_, N)),
            "tx": rng.integers(0, 1e6, (S_, N)), "disk": rng.integers(0, 5, (S_, N))}
    o1, o2 = rng.permutation(N), rng.permutation(N + 1)
    S.save_vote(tmp_path / "v.npz", snap, o1, o2)
    with Engine(0) as e:
        e.upload_snapshot(snap)
        best, win = e.score_reference(order1=o1, order2=o2)
    with Engine(0) as e2:
        b2, w2 = S.replay_vote(e2, tmp_path / "v.npz")
    assert S.digest(best, win) == S.digest(b2, w2)
