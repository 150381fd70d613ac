"""Diagnostic: where the host time of one bench step goes (C3 by default).

Times reset_capacity, place (wall), the device-side total of the pass
(nas_timings.total_ms) and timings() per step, with and without the cost
outputs, so the host share of ms_per_step is visible.  Run on the GPU box:
    python tools/host_overhead.py [--nodes N --pods P --rehearse-world G]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetesnetawarescheduler_amd import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--pods", type=int, default=100000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rehearse-world", type=int, default=0)
    a = ap.parse_args()
    e = Engine(0)
    if a.rehearse_world > 1:
        e.set_option("REHEARSE_WORLD", a.rehearse_world)
        e.comm_init(Engine.comm_unique_id(), 0, 1)
    e.synth_cluster(0x4E4153, a.nodes, a.pods, "i8")
    if a.rehearse_world > 1:
        e.upload_capacity(np.minimum(e.get_capacity().astype(np.int64) * 64, 2**31 - 1)
                          .astype(np.int32))
    for want_cost in (True, False):
        rows = []
        for i in range(a.steps + 2):
            t0 = time.perf_counter()
            e.reset_capacity()
            t1 = time.perf_counter()
            e.place(want_cost=want_cost)
            t2 = time.perf_counter()
            t = e.timings()
            t3 = time.perf_counter()
            if i >= 2:
                rows.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, t["total_ms"], (t3 - t2) * 1e3))
        r = np.median(np.array(rows), axis=0)
        print(f"want_cost={want_cost}: reset {r[0]:.3f} ms, place wall {r[1]:.3f} ms, "
              f"device total {r[2]:.3f} ms, host share {r[1] - r[2]:.3f} ms, timings() {r[3]:.3f} ms",
              flush=True)
    e.close()


if __name__ == "__main__":
    main()
