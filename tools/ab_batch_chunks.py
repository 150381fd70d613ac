"""A/B of the batched nas_place (BASELINE config C5: 64 clusters x 5k nodes x
5k pods) with pipelined chunks (NAS_OPT_BATCH_CHUNK_TILES = 0, auto) against
one unchunked pass (score everything, then commit), alternating on one
context so both see the same box.  Prints ms per pass and the stage sums."""
import argparse
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from kubernetesnetawarescheduler_amd import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--tiles", default="0,1048576")
a = ap.parse_args()
B, N, P = 64, 5000, 5000
variants = [int(x) for x in a.tiles.split(",")]
with Engine(0) as e:
    e.synth_batch(0x4E4153, B, N, P, "i8", peers=8)
    ref = None
    res = {v: [] for v in variants}
    for rep in range(a.reps):
        for v in variants:
            e.set_option("BATCH_CHUNK_TILES", v)
            e.reset_capacity()
            node, _, score = e.place()  # warm + check
            if ref is None:
                ref = (node, score)
            assert (node == ref[0]).all() and (score == ref[1]).all(), v
            t0 = time.perf_counter()
            for _ in range(a.steps):
                e.reset_capacity()
                e.place()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            t = e.timings()
            res[v].append(ms)
            print(f"rep {rep} tiles {v}: {ms:.3f} ms/pass  fit {t['fit_ms']:.3f} cost {t['cost_ms']:.3f} "
                  f"merge {t['merge_ms']:.3f} commit {t['commit_ms']:.3f} launches {t['cost_launches']} "
                  f"rescores {t['rescore_rounds']}", flush=True)
    for v in variants:
        print(f"tiles {v}: median {np.median(res[v]):.3f} ms, min {min(res[v]):.3f} ms")
