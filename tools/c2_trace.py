"""Run the C2 placement (bench.py config_c2's inputs) a few times, for a
kernel trace: rocprofv3 --kernel-trace -d DIR -- python3 tools/c2_trace.py
then python tools/pass_timeline.py DIR."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubernetesnetawarescheduler_amd import Engine, workloads  # noqa: E402

SEED = 0x4E4153


def main():
    c = workloads.c2_cluster(SEED, 1000, 10000)
    with Engine(0) as e:
        e.upload_latency(c["L"], "i8")
        e.upload_capacity(c["free"])
        e.upload_pods(c["req"])
        e.upload_traffic_csr(c["row_ptr"], c["peer_node"], c["weight"], "i8", 1000)
        import time
        import zlib
        ms, dev = [], []
        for _ in range(int(os.environ.get("C2_STEPS", "5"))):
            e.reset_capacity()
            t0 = time.perf_counter()
            node, _, score = e.place(want_cost=True)
            ms.append((time.perf_counter() - t0) * 1e3)
            dev.append(e.timings()["total_ms"])
        ms.sort()
        dev.sort()
        print(e.timings())
        print(f"median {ms[len(ms) // 2]:.3f} ms, min {ms[0]:.3f} ms, device median "
              f"{dev[len(dev) // 2]:.3f} ms, placements crc "
              f"{zlib.crc32(node.tobytes()) ^ zlib.crc32(score.tobytes()):08x}")


if __name__ == "__main__":
    main()
