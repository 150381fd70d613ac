"""Run bench.py config_c1's extended-mode placement (10 nodes x 100 pods) a
few times and time each nas_place call, for a kernel trace:
rocprofv3 --kernel-trace -d DIR -- python3 tools/c1_trace.py
then python tools/pass_timeline.py DIR."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubernetesnetawarescheduler_amd import Engine  # noqa: E402


def main():
    rng = np.random.default_rng(0x4E4153)
    N, P = 10, 100
    rng.permutation(N), rng.permutation(N + 1)  # bench.py draws the vote orders first
    L = rng.integers(1, 100, (N, N)).astype(np.int8)
    L = np.triu(L, 1) + np.triu(L, 1).T
    WA = np.zeros((P, N), np.int8)
    WA[:, int(rng.integers(0, N))] = 100
    free = np.tile(np.array([[4000, 4 << 20, 110]], np.int32), (N, 1))
    req = np.stack([rng.integers(1, 540, P), rng.integers(7_464, 303_749, P), np.ones(P)],
                   1).astype(np.int32)
    with Engine(0) as e:
        e.upload_latency(L, "i8")
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, "i8")
        ms = []
        for _ in range(int(os.environ.get("C1_STEPS", "20"))):
            e.reset_capacity()
            t0 = time.perf_counter()
            e.place(want_cost=True)
            ms.append((time.perf_counter() - t0) * 1e3)
        ms.sort()
        print(f"median {ms[len(ms) // 2]:.3f} ms, min {ms[0]:.3f} ms", e.timings())


if __name__ == "__main__":
    main()
