"""One rank of the two-process node-shard test (tests/test_gpu_dist_shard.py):
an Engine on cuda:0 holding node shard `rank` of `world` (nas_set_shard),
candidate lists exchanged over torch.distributed gloo by
sharded.place_dist_shard.  Run as a child process (never imported by pytest).

  python tests/dist_gpu_worker.py RANK WORLD INIT_URL OUT_PREFIX SEED

INIT_URL is a file:// rendezvous (no TCP port).
"""
import datetime
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from kubernetesnetawarescheduler_amd import Engine, sharded  # noqa: E402
from util import cluster  # noqa: E402

P, N = 4000, 700


def make_inputs(seed):
    rng = np.random.default_rng(seed)
    WA8, L, free, req = cluster(rng, P, N, lo=0, hi=40, cap_scale=0.03)
    WA = WA8.astype(np.int32)
    hot = rng.choice(N, 24, replace=False)
    WA[:, hot] += rng.integers(100, 400, (P, 24))  # crowding beyond int8: stops, rescores
    return WA, L, free, req


def main():
    rank, world, url, out, seed = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                   int(sys.argv[5]))
    dist.init_process_group("gloo", init_method=url, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    WA, L, free, req = make_inputs(seed)

    def all_gather(keys, bounds):
        kt = torch.from_numpy(np.ascontiguousarray(keys).view(np.int64).copy())
        bt = torch.from_numpy(np.ascontiguousarray(bounds).view(np.int64).copy())
        ks = [torch.empty_like(kt) for _ in range(world)]
        bs = [torch.empty_like(bt) for _ in range(world)]
        dist.all_gather(ks, kt)
        dist.all_gather(bs, bt)
        return [(k.numpy().view(np.uint64), b.numpy().view(np.uint64)) for k, b in zip(ks, bs)]

    with Engine(0) as e:
        e.set_shard(rank, world)
        e.upload_latency(L, "i8")
        e.upload_capacity(free)
        e.upload_pods(req)
        e.upload_traffic(WA, "i8")
        node, score, rounds = sharded.place_dist_shard(e, P, all_gather)
        cap = e.get_capacity()
    np.savez(f"{out}.{rank}.npz", node=node, score=score, rounds=rounds, cap=cap)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
