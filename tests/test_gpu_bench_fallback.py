"""bench.py at world size 2 with both ranks on GPU 0 (tools/bench_one_gpu_ranks.py
forces LOCAL_RANK=0): RCCL refuses two ranks on one GPU, so every rank must
agree to fall back to the host exchange (sharded.place_dist_shard over gloo)
and still print one JSON line that says so -- the insurance for a multi-GPU
node whose RCCL cannot initialise."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_rccl_failure_falls_back_to_host_exchange():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tools", "bench_one_gpu_ranks.py"), "--gpus", "2", "--nodes", "1500",
           "--pods", "4096", "--steps", "2", "--warmup", "1", "--no-configs", "--no-reference-mode",
           "--no-cpu-baseline", "--no-pmc"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["exchange"].startswith("host gloo all-gather")
    assert out["value"] > 0 and out["unschedulable"] == 0
