"""bench.py's self-launch: `bench.py --gpus N` with no
launcher starts N rank processes itself (bench.launch_ranks) -- RANK /
LOCAL_RANK / WORLD_SIZE and a file:// gloo rendezvous per child --, relays
rank 0's output, and takes every rank down as soon as one fails.  CPU only:
the children here are small scripts that do what bench.py's Dist does with
the environment (gloo init from NAS_DIST_INIT, a barrier, an all-reduce)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

RANK_SCRIPT = r"""
import json, os, sys, time
import torch, torch.distributed as dist
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method=os.environ["NAS_DIST_INIT"], rank=r, world_size=w)
t = torch.tensor([r + 1], dtype=torch.int64)
dist.all_reduce(t)
dist.barrier()
if r == 0:
    print("banner line that is not the result")
    print(json.dumps({"world": w, "sum": int(t.item()), "local": int(os.environ["LOCAL_RANK"]),
                      "argv": sys.argv[1:]}))
dist.destroy_process_group()
"""


def test_launch_ranks_relays_rank0_line():
    rc, text = bench.launch_ranks([sys.executable, "-c", RANK_SCRIPT, "--gpus", "3"], 3, 2,
                                  timeout_s=120)
    assert rc == 0, text
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out == {"world": 3, "sum": 6, "local": 0, "argv": ["--gpus", "3"]}


def test_launch_ranks_local_rank_wraps_over_devices():
    script = ("import os, time\n"
              "r = int(os.environ['RANK'])\n"
              "assert int(os.environ['LOCAL_RANK']) == r % 2, os.environ['LOCAL_RANK']\n"
              "assert os.environ['WORLD_SIZE'] == '4'\n"
              "assert os.environ['NAS_DIST_INIT'].startswith('file://')\n"
              "print('{\"ok\": true}') if r == 0 else None\n")
    rc, text = bench.launch_ranks([sys.executable, "-c", script], 4, 2, timeout_s=60)
    assert rc == 0 and '{"ok": true}' in text


def test_launch_ranks_fails_fast_and_reaps():
    # rank 1 fails at once; rank 0 would wait 60 s for it: the launcher must
    # kill rank 0 right away and report rank 1's exit code
    script = ("import os, sys, time\n"
              "if os.environ['RANK'] == '1': sys.exit(3)\n"
              "time.sleep(60)\n")
    t0 = time.monotonic()
    rc, _ = bench.launch_ranks([sys.executable, "-c", script], 2, 1, timeout_s=120)
    assert rc == 3
    assert time.monotonic() - t0 < 30


def test_launch_ranks_signal_and_deadline():
    rc, _ = bench.launch_ranks([sys.executable, "-c", "import os, signal; "
                                "os.kill(os.getpid(), signal.SIGTERM)"], 2, 1, timeout_s=60)
    assert rc == 128 + 15
    t0 = time.monotonic()
    rc, _ = bench.launch_ranks([sys.executable, "-c", "import time; time.sleep(60)"], 2, 1,
                               timeout_s=2)
    assert rc == 124 and time.monotonic() - t0 < 30


def test_main_self_launches_without_world_size(monkeypatch, capsys):
    # main() with --gpus 2 and no WORLD_SIZE goes to self_launch before any
    # GPU work; the relay adds config.launcher and exits with the ranks' rc
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    def fake_launch(argv, n, ndev, timeout_s=None, extra_env=None):
        seen.update(argv=argv, n=n)
        return 0, 'noise\n{"n_gpus": 2, "config": {"workload": "C3"}}\n'

    monkeypatch.setattr(bench, "launch_ranks", fake_launch)
    monkeypatch.setattr(bench, "visible_gpus", lambda: 1)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    try:
        bench.main()
        raise AssertionError("main() must exit after relaying")
    except SystemExit as e:
        assert e.code == 0
    assert seen["n"] == 2 and seen["argv"][-4:] == ["--gpus", "2", "--steps", "1"]
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["n_gpus"] == 2 and "self-launch" in out["config"]["launcher"]


def test_ranks_die_with_the_launcher(tmp_path):
    """A driver that kills the launcher on a deadline must not leave its rank
    processes running (PR_SET_PDEATHSIG)."""
    import signal
    import subprocess
    pids = tmp_path / "pids"
    child = ("import os, time\n"
             f"open({str(pids)!r} + '.' + os.environ['RANK'], 'w').write(str(os.getpid()))\n"
             "time.sleep(120)\n")
    launcher = ("import sys\n"
                f"sys.path.insert(0, {ROOT!r})\n"
                "import bench\n"
                f"bench.launch_ranks([sys.executable, '-c', {child!r}], 2, 1)\n")
    p = subprocess.Popen([sys.executable, "-c", launcher])
    files = [tmp_path / f"pids.{r}" for r in range(2)]
    t0 = time.monotonic()
    while not all(f.exists() and f.read_text() for f in files):
        assert time.monotonic() - t0 < 60, "ranks did not start"
        time.sleep(0.05)
    ranks = [int(f.read_text()) for f in files]
    p.send_signal(signal.SIGKILL)
    p.wait()
    t0 = time.monotonic()
    alive = ranks
    while alive and time.monotonic() - t0 < 20:
        alive = []
        for pid in ranks:
            try:
                os.kill(pid, 0)
                with open(f"/proc/{pid}/stat") as f:
                    if f.read().split()[2] != "Z":
                        alive.append(pid)
            except (ProcessLookupError, FileNotFoundError):
                pass
        time.sleep(0.1)
    for pid in alive:  # (never leave them behind, even when the test fails)
        os.kill(pid, signal.SIGKILL)
    assert not alive
