"""bench.py's rank logic under torch.distributed gloo at world size 2 on CPU:
Dist (RANK / WORLD_SIZE from the env, barrier, max over ranks, broadcast of
the RCCL unique id) and time_steps (barrier-bracketed timed region, max over
ranks) -- what the driver's torchrun launch exercises on the GPU node."""
import os
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, url, out):
    # NAS_DIST_INIT: a file rendezvous instead of torchrun's MASTER_PORT
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE="2", NAS_DIST_INIT=url)
    sys.path.insert(0, ROOT)
    import bench
    d = bench.Dist(2)
    assert (d.rank, d.world) == (rank, 2)
    uid = d.bcast_bytes(b"unique-id-of-rank-0" if rank == 0 else None)
    assert uid == b"unique-id-of-rank-0"
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.05 if rank == 1 else 0.0)  # rank 1 is the slow one

    el = bench.time_steps(d, step, 4, 2)
    assert len(calls) == 6
    assert el >= 0.2  # every rank reports the slowest rank's time
    with open(f"{out}.{rank}", "w") as f:
        f.write(repr(el))
    d.barrier_sync()


def test_bench_dist_world2(tmp_path):
    from util import rdv_url
    out = str(tmp_path / "el")
    mp.spawn(_worker, args=(rdv_url(tmp_path), out), nprocs=2, join=True)
    a, b = (float(open(f"{out}.{r}").read()) for r in range(2))
    assert a == b
