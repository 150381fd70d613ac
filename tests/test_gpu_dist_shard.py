"""Two processes, one GPU, engine in the loop: each rank is an Engine(0) that
owns half the node columns (nas_set_shard(r, 2)); per-pod candidate lists
travel over torch.distributed gloo (sharded.place_dist_shard: score range ->
all-gather -> merge -> set keys -> replicated commit -> rescore windows).
Both ranks must return the sequential oracle's placements, integer scores and
remaining capacity -- the exchange logic nas_place runs over RCCL, exercised
across real process boundaries (RCCL itself refuses two ranks on one GPU)."""
import os
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_two_process_node_shards_match_oracle(tmp_path):
    sys.path.insert(0, HERE)
    from dist_gpu_worker import make_inputs
    from util import rdv_url, run_children
    seed, world = 11, 2
    out = str(tmp_path / "shard")
    url = rdv_url(tmp_path)  # file rendezvous: no TCP port to collide with
    rcs = run_children([[sys.executable, os.path.join(HERE, "dist_gpu_worker.py"), str(r),
                         str(world), url, out, str(seed)] for r in range(world)], timeout=100)
    assert rcs == [0] * world
    res = [np.load(f"{out}.{r}.npz") for r in range(world)]
    WA, L, free, req = make_inputs(seed)
    want, wcost, wfree = oracle.place(WA, L, req, free, "i8")
    assert int(res[0]["rounds"]) > 0  # the rescore windows ran across the process boundary
    for r in res:
        assert r["node"].tolist() == want.tolist()
        assert r["score"].tolist() == wcost.tolist()
        assert (r["cap"] == wfree).all()
