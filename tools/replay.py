"""Replay a captured scheduling problem (kubernetesnetawarescheduler_amd/
snapshot.py) on this box's GPU and print the decisions' digest, so two runs
(two boxes, two builds) can be compared.

  python tools/replay.py FILE.npz [--repeat K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubernetesnetawarescheduler_amd import Engine  # noqa: E402
from kubernetesnetawarescheduler_amd import snapshot as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    f = S.load(a.file)
    digests, ms = set(), []
    with Engine(0) as e:
        for _ in range(a.repeat):
            t0 = time.perf_counter()
            if f["format"] == S.PLACE_FORMAT:
                node, cost, _ = S.replay_place(e, a.file)
                digests.add(S.digest(node, cost))
            else:
                best, win = S.replay_vote(e, a.file)
                digests.add(S.digest(best, win))
            ms.append((time.perf_counter() - t0) * 1e3)
            if f["format"] == S.PLACE_FORMAT:
                e.reset_capacity()
    print(json.dumps({"file": a.file, "format": f["format"], "digests": sorted(digests),
                      "deterministic": len(digests) == 1, "ms_per_replay": ms, "meta": f["meta"]}))


if __name__ == "__main__":
    main()
