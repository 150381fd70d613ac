"""Replay files (kubernetesnetawarescheduler_amd/snapshot.py, SURVEY.md §5
checkpoint / resume): layout round trips and the refusal of anything that is
not a replay file or would need unpickling.  CPU only."""
import numpy as np
import pytest

from kubernetesnetawarescheduler_amd import snapshot as S


def test_place_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    L = rng.integers(0, 100, (40, 40), dtype=np.int8)
    free = rng.integers(100, 4000, (40, 3)).astype(np.int32)
    req = rng.integers(1, 100, (70, 3)).astype(np.int32)
    WA = rng.integers(-300, 300, (70, 40)).astype(np.int32)
    p = tmp_path / "p.npz"
    S.save_place(p, L, free, req, WA, "i8", meta={"why": "test"})
    f = S.load(p)
    assert f["format"] == S.PLACE_FORMAT and f["kind"] == "dense" and f["dtype"] == "i8"
    for k, a in (("L", L), ("free", free), ("req", req), ("WA", WA)):
        assert f[k].dtype == a.dtype and np.array_equal(f[k], a)
    assert f["meta"] == {"why": "test"}


def test_synth_and_vote_roundtrip(tmp_path):
    S.save_place_synth(tmp_path / "s.npz", 0x4E4153, 10000, 100000, "bf16", peers=8)
    f = S.load(tmp_path / "s.npz")
    assert f["kind"] == "synth" and f["dtype"] == "bf16"
    assert f["synth"].tolist() == [0x4E4153, 10000, 100000, 8]
    rng = np.random.default_rng(2)
    snap = {"cpu": rng.random((3, 5)), "mem": rng.random((3, 5)), "bw": rng.random((3, 5)),
            "rx": rng.integers(0, 9, (3, 5)), "tx": rng.integers(0, 9, (3, 5)),
            "disk": rng.integers(0, 9, (3, 5))}
    S.save_vote(tmp_path / "v.npz", snap, rng.permutation(5), rng.permutation(6),
                pod_snapshot=[0, 2, 1, 1])
    v = S.load(tmp_path / "v.npz")
    assert v["format"] == S.VOTE_FORMAT
    for k in snap:
        assert np.array_equal(v[k], snap[k])
    assert v["pod_snapshot"].tolist() == [0, 2, 1, 1]


def test_refuses_foreign_and_pickled_files(tmp_path):
    np.savez(tmp_path / "x.npz", a=np.arange(3))
    with pytest.raises(ValueError):
        S.load(tmp_path / "x.npz")
    np.savez(tmp_path / "o.npz", format=np.array(S.PLACE_FORMAT),
             meta=np.array([{"evil": 1}], dtype=object))
    with pytest.raises(ValueError):  # object arrays need pickle: never loaded
        S.load(tmp_path / "o.npz")


def test_digest_sensitive_to_values_and_dtype():
    a = np.arange(10, dtype=np.int32)
    assert S.digest(a) == S.digest(a.copy())
    b = a.copy()
    b[3] = 99
    assert S.digest(a) != S.digest(b)
    assert S.digest(a) != S.digest(a.astype(np.int64))
