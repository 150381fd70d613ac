"""Generate the committed golden fixtures under tests/golden/.

The reference (scheduler/scheduler.go, Go) ships no tests, fixtures or golden
vectors and cannot be built here (no Go toolchain; the file also fails to
compile as shipped, :214/:235).  So:

  vote_kat.json     Known-answer vectors of SURVEY.md Appendix A, derived by
                    hand from scheduler.go:258-394.  The expected values are
                    WRITTEN HERE LITERALLY (not computed) and this script
                    asserts that the oracle reproduces them -- this is what
                    pins the oracle.
  vote_random.json  Seeded random snapshots (N = 5 with the reference's node
                    names, N = 10, N = 37) with random Go-map orders; expected
                    outputs from the literal oracle loop (regression fixtures).
  place_small.json  A small extended-mode case (int8 WA, L, capacities,
                    requests) with the sequential-greedy oracle's placements.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = ["ubuntu", "raspiworker0", "raspiworker1", "raspiworker2", "raspiworker3"]
NONE = -2

# SURVEY.md Appendix A; tuples (cpu, mem, rx, tx, bw, disk) per scheduler.go:24-32
M = {"cpu": [1.2e9, 6e8, 1.5e9, 1.8e9, 1.5e9], "mem": [40.0, 30.0, 20.0, 50.0, 60.0],
     "rx": [10, 20, 5, 30, 40], "tx": [5, 9, 7, 8, 6], "bw": [0.0, 9.4e7, 9.1e7, 9.0e7, 0.0],
     "disk": [3, 1, 2, 0, 5]}
M3 = dict(M, cpu=[6e8, 1.2e9, 1.5e9, 1.8e9, 1.5e9])
M4 = {"cpu": [1.5e9] * 5, "mem": [50.0] * 5, "rx": [0] * 5, "tx": [0] * 5, "bw": [0.0] * 5,
      "disk": [0] * 5}

KATS = [
    # name, metrics, order1, order2 (5 = "none"), expected scores (U, r0..r3, none), best
    ("KAT1", M, [0, 1, 2, 3, 4], [0, 1, 2, 3, 4, 5], [0, 5, 3, 0, 0, 3], 1),
    ("KAT2", M, [4, 3, 2, 1, 0], [5, 4, 3, 2, 1, 0], [1, 4, 3, 0, 0, 3], 1),
    ("KAT3", M3, [0, 1, 2, 3, 4], [5, 0, 1, 2, 3, 4], [3, 2, 3, 0, 0, 3], NONE),
    ("KAT4", M4, [0, 1, 2, 3, 4], [0, 1, 2, 3, 4, 5], [7, 0, 0, 0, 0, 4], 0),
]


def kat_fixture():
    out = []
    for name, m, o1, o2, scores, best in KATS:
        b, win, sc = oracle.vote(m, o1, o2)
        assert b == best, (name, b, best)
        assert list(sc) == scores, (name, list(sc), scores)
        out.append({"name": name, "metrics": m, "order1": o1, "order2": o2,
                    "scores": scores, "best": best, "winners": [int(x) for x in win]})
    return {"source": "SURVEY.md Appendix A (hand-derived from scheduler.go:258-394)",
            "node_names": NAMES, "none_key": 5, "cases": out}


def random_snapshot(rng, n, ties=False):
    """Metric values shaped like the reference's inputs (see oracle/synth)."""
    if ties:
        cpu = rng.choice([6e8, 1.2e9, 1.5e9], n).astype(np.float64)
        mem = rng.choice([10.0, 20.0], n)
        rx = rng.choice([0, 5, 7], n)
        tx = rng.choice([0, 5, 7], n)
        bw = rng.choice([0.0, 9e7], n)
        disk = rng.choice([0, 1, 2], n)
    else:
        freqs = np.array([6e8, 1.2e9, 1.5e9, 1.8e9], np.float32).astype(np.float64)
        cpu = freqs[rng.integers(0, 4, (n, 4))].sum(1) / 4
        total = np.float32(1 << 30) * rng.integers(1, 9, n)
        avail = (rng.random(n) * total).astype(np.float32).astype(np.float64)
        mem = 100.0 - ((avail * 100.0) / total.astype(np.float64))
        rx = np.where(rng.random(n) < 0.1, 0, rng.integers(0, 1_000_000, n))
        tx = np.where(rng.random(n) < 0.1, 0, rng.integers(0, 1_000_000, n))
        bw = np.where(rng.random(n) < 0.2, 0.0, 8e7 + rng.random(n) * 1.5e7)
        bw[0] = 0.0  # "ubuntu" (scheduler.go:287)
        disk = np.where(rng.random(n) < 0.3, 0, rng.integers(1, 1001, n))
    return {"cpu": cpu, "mem": mem, "rx": rx.astype(np.int64), "tx": tx.astype(np.int64),
            "bw": bw, "disk": disk.astype(np.int64)}


def random_fixture():
    rng = np.random.default_rng(0x4E4153)
    cases = []
    for n, count, ties in [(5, 40, False), (5, 40, True), (10, 30, False), (37, 20, True)]:
        for _ in range(count):
            m = random_snapshot(rng, n, ties)
            o1 = rng.permutation(n).astype(np.int32)
            o2 = rng.permutation(n + 1).astype(np.int32)
            b, win, sc = oracle.vote(m, o1, o2)
            cases.append({"n": n, "metrics": {k: v.tolist() for k, v in m.items()},
                          "order1": o1.tolist(), "order2": o2.tolist(), "best": b,
                          "winners": [int(x) for x in win], "scores": [int(x) for x in sc]})
    return {"source": "oracle.or_vote_literal (restatement of scheduler.go:248-394), seed 0x4E4153",
            "cases": cases}


def place_fixture():
    rng = np.random.default_rng(7)
    P, N = 48, 13
    WA = rng.integers(0, 20, (P, N)).astype(np.int8)
    L = rng.integers(0, 30, (N, N)).astype(np.int8)
    free = np.stack([rng.integers(200, 900, N), rng.integers(100_000, 400_000, N),
                     rng.integers(2, 6, N)], 1).astype(np.int32)
    req = np.stack([rng.integers(50, 300, P), rng.integers(20_000, 90_000, P),
                    np.ones(P, np.int64)], 1).astype(np.int32)
    node, cost, free_after = oracle.place(WA, L, req, free, "i8")
    return {"source": "oracle.or_place (build-defined extended mode: fit, cost = WA x L, "
                      "argmin (cost, node), sequential greedy commit)",
            "WA": WA.tolist(), "L": L.tolist(), "free": free.tolist(), "req": req.tolist(),
            "node": node.tolist(), "cost": cost.tolist(), "free_after": free_after.tolist()}


def main():
    for name, fn in [("vote_kat.json", kat_fixture), ("vote_random.json", random_fixture),
                     ("place_small.json", place_fixture)]:
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fn(), f, separators=(",", ":"))
        print("wrote", name)


if __name__ == "__main__":
    main()
