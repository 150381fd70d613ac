"""bench.py at world size 2 with both ranks on GPU 0 (tools/bench_one_gpu_ranks.py
forces LOCAL_RANK=0): RCCL refuses two ranks on one GPU, so every rank must
agree to fall back to the host exchange (sharded.place_dist_shard over gloo)
and still print one JSON line that says so -- the insurance for a multi-GPU
node whose RCCL cannot initialise.  The two ranks are started the way torchrun
would (RANK / LOCAL_RANK / WORLD_SIZE in the env) but rendezvous through a file
(NAS_DIST_INIT), so no probed TCP port can collide; a rank that fails takes its
peer down at once (tests/util.run_children)."""
import json
import os
import sys

import pytest

from util import rdv_url, run_children

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_rccl_failure_falls_back_to_host_exchange(tmp_path):
    args = [sys.executable, os.path.join(ROOT, "tools", "bench_one_gpu_ranks.py"), "--gpus", "2",
            "--nodes", "1500", "--pods", "4096", "--steps", "2", "--warmup", "1", "--no-configs",
            "--no-reference-mode", "--no-cpu-baseline", "--no-pmc"]
    url = rdv_url(tmp_path)
    envs = [dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", NAS_DIST_INIT=url,
                 MASTER_ADDR="127.0.0.1") for r in range(2)]
    logs = [str(tmp_path / f"rank{r}.log") for r in range(2)]
    rcs = run_children([args, args], timeout=140, env=envs, logs=logs, cwd=ROOT)
    out0 = open(logs[0]).read()
    assert rcs == [0, 0], out0[-2000:] + open(logs[1]).read()[-2000:]
    lines = [ln for ln in out0.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out0[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["exchange"].startswith("host gloo all-gather")
    assert out["value"] > 0 and out["unschedulable"] == 0


def test_bench_self_launch_two_ranks_on_one_gpu(tmp_path):
    """`python bench.py --gpus 2` with no launcher: bench.py
    starts both rank processes itself (file:// rendezvous, LOCAL_RANK wrapped
    over the visible GPUs), both land on GPU 0 here, RCCL refuses, the ranks
    agree on the host exchange, and the parent relays rank 0's one line."""
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
            "--nodes", "1500", "--pods", "4096", "--steps", "2", "--warmup", "1", "--no-configs",
            "--no-reference-mode", "--no-cpu-baseline", "--no-pmc"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NAS_DIST_INIT")}
    out_f, err_f = tmp_path / "stdout", tmp_path / "stderr"
    import subprocess
    with open(out_f, "w") as fo, open(err_f, "w") as fe:
        r = subprocess.run(args, env=env, cwd=ROOT, stdout=fo, stderr=fe, timeout=160)
    out_txt, err_txt = out_f.read_text(), err_f.read_text()
    assert r.returncode == 0, err_txt[-3000:]
    lines = [ln for ln in out_txt.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out_txt[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert "self-launch" in out["config"]["launcher"]
    assert out["config"]["exchange"].startswith("host gloo all-gather")
    assert out["value"] > 0 and out["unschedulable"] == 0
