"""k_commit alone (nas_commit on a scored C3 context): device time for the
last n pods of the pass, to split the kernel into its fixed cost (capacity
into LDS and back, results to the host stage) and the walk, with the walk's
rounds; then the whole pass's 100k pods in one walk (as a world-1 pass of
one chunk would: herds fill nodes, so its later windows see real conflicts).
usage (GPU box, repo root): python tools/commit_probe.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetesnetawarescheduler_amd import Engine  # noqa: E402

N, P = 10000, 100000
out = {}
with Engine(0) as e:
    e.synth_cluster(0xC3, N, P, "i8", peers=8)
    e.score_range(0, P)
    node = np.zeros(P, np.int32)
    rounds = {}
    for n in (256, 1024, 4096, 16384, 23000, 50000, 100000):
        ts = []
        for _ in range(5):
            e.reset_capacity()
            e.commit(P - n, node)
            t = e.timings()
            ts.append(t["commit_ms"])
        out[n] = round(float(np.median(ts)) * 1e3, 1)
        rounds[n] = t["commit_rounds"]
    full = []
    for _ in range(5):
        e.reset_capacity()
        stop = e.commit(0, node)
        t = e.timings()
        full.append((t["commit_ms"] * 1e3, t["commit_rounds"], stop))
print(json.dumps({"commit_us_by_pods": out, "rounds_by_pods": rounds,
                  "full_walk": {"us": round(float(np.median([f[0] for f in full])), 1),
                                "rounds": full[-1][1], "stop": full[-1][2]}}))
