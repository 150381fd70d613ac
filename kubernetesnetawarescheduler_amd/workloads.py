"""Host-side workload generators for the BASELINE configs that are not
generated on the device.

C2 -- "clusterloader2-derived trace: 1k nodes x 10k pods, sparse
pod-communication graph": pod requests are drawn from the 408 (cpu, memory)
rows of the reference's clusterloader2 resource summaries
(data/clusterloader2_requests.json, extracted by tools/make_clusterloader2.py
from datasets/clusterloader2/*/*.json); every pod talks to k peers with
weights 1..100 (MB, the customNetworkBenchmark transfer size is 100 MB per
pod), a fraction of the pods is already bound, and a pending pod's traffic to
its bound peers lands on their nodes -- a CSR traffic matrix with <= k
entries per row (nas_upload_traffic_csr).  Latency is U[50, 500] us,
symmetric, zero diagonal, in 4-us int8 steps.
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def clusterloader2_requests():
    """(cpu millicores, memory KiB) of the 408 clusterloader2 rows."""
    with open(os.path.join(HERE, "data", "clusterloader2_requests.json")) as f:
        rows = json.load(f)["rows"]
    cpu = np.array([max(1, int(np.ceil(r["cpu_cores"] * 1000))) for r in rows], np.int32)
    mem = np.array([int(np.ceil(r["mem_bytes"] / 1024)) for r in rows], np.int32)
    return cpu, mem


def latency_us_i8(rng, N, lo=50, hi=500, unit=4):
    """Symmetric latency U[lo, hi] us with a zero diagonal,
    quantised to int8 in `unit`-us steps (50..500 us -> 12..125)."""
    u = rng.integers(lo, hi + 1, (N, N))
    u = np.triu(u, 1)
    u = u + u.T
    return np.rint(u / unit).astype(np.int8)


def c2_cluster(seed=0x4E4153, N=1000, P=10000, peers=8, bound_frac=0.2):
    """Returns dict(L (N,N) i8, free (N,3), req (P,3), row_ptr, peer_node, weight i8)."""
    rng = np.random.default_rng(seed)
    cpu, mem = clusterloader2_requests()
    pick = rng.integers(0, len(cpu), P)
    req = np.stack([cpu[pick], mem[pick], np.ones(P, np.int32)], 1).astype(np.int32)
    free = np.stack([np.full(N, 4000), np.full(N, 4 * 1048576), np.full(N, 110)], 1).astype(np.int32)
    # the communication graph: peers among all pods (pending and the 20%
    # already bound); a bound peer sits in the pending pod's home group of 32
    # nodes with probability 3/4, anywhere otherwise
    total = P + int(P * bound_frac / (1 - bound_frac))
    home = rng.integers(0, (N + 31) // 32, P)
    peer = rng.integers(0, total, (P, peers))
    is_bound = peer >= P
    local = rng.random((P, peers)) < 0.75
    node = np.where(local, np.minimum(home[:, None] * 32 + rng.integers(0, 32, (P, peers)), N - 1),
                    rng.integers(0, N, (P, peers)))
    node = np.where(is_bound, node, -1)  # pending peers have no node yet
    w = rng.integers(1, 101, (P, peers)).astype(np.int8)
    keep = node >= 0
    row_ptr = np.concatenate([[0], np.cumsum(keep.sum(1))]).astype(np.int32)
    return {"L": latency_us_i8(rng, N), "free": free, "req": req, "row_ptr": row_ptr,
            "peer_node": node[keep].astype(np.int32), "weight": w[keep]}


def csr_to_dense(row_ptr, peer_node, weight, N):
    """The dense traffic WA[p, m] = sum of p's weights to peers bound on node m,
    exact (int64 sums, no saturation; unbound peers, node -1, are skipped) --
    for oracle checks."""
    P = len(row_ptr) - 1
    w = np.asarray(weight)
    dt = np.float64 if w.dtype.kind == "f" else np.int64  # float weights: fp64 sums
    WA = np.zeros((P, N), dt)
    rows = np.repeat(np.arange(P), np.diff(row_ptr))
    keep = (peer_node >= 0) & (peer_node < N)
    np.add.at(WA, (rows[keep], peer_node[keep]), w[keep].astype(dt))
    return WA
