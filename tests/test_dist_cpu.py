"""Node-axis sharding on CPU (gloo, world_size 2): each rank ranks only its
node columns with the oracle, the per-pod lists (8 keys + exactness bound)
are all-gathered and merged with the engine's rule, and the merged exact
prefix must equal the unsharded ranking -- the exchange step nas_place runs
over RCCL, with torch.distributed gloo standing in for it."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from util import KEY_INVALID, cluster, keys_from_costs, merge_lists, rdv_url, usable

P, N, WORLD = 300, 77, 2


def shard_lists(WA, L, req, free, n0, n1, K=8):
    cost = oracle.cost(WA, L, "i8")[:, n0:n1]
    mask = oracle.fit_mask(req, free[n0:n1])
    nodes, cc, cnt = oracle.topk(np.ascontiguousarray(cost), mask, K)
    nodes = np.where(nodes >= 0, nodes + n0, -1)
    keys = keys_from_costs(nodes, cc)
    bound = np.where(cnt == K, keys[:, K - 1], KEY_INVALID)  # a full list may have dropped keys
    return keys, bound


def _worker(rank, url, out):
    dist.init_process_group("gloo", init_method=url, rank=rank, world_size=WORLD)
    rng = np.random.default_rng(42)  # identical inputs on every rank
    WA, L, free, req = cluster(rng, P, N, cap_scale=0.05)
    n0, n1 = rank * N // WORLD, (rank + 1) * N // WORLD
    keys, bound = shard_lists(WA, L, req, free, n0, n1)
    kt = torch.from_numpy(keys.view(np.int64).copy())
    bt = torch.from_numpy(bound.view(np.int64).copy())
    ks = [torch.empty_like(kt) for _ in range(WORLD)]
    bs = [torch.empty_like(bt) for _ in range(WORLD)]
    dist.all_gather(ks, kt)
    dist.all_gather(bs, bt)
    parts = [(k.numpy().view(np.uint64), b.numpy().view(np.uint64)) for k, b in zip(ks, bs)]
    mk, mb = merge_lists(parts)
    if rank == 0:
        np.save(out + ".keys.npy", mk)
        np.save(out + ".bound.npy", mb)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_lists_merge_to_global_ranking(tmp_path):
    out = str(tmp_path / "merged")
    mp.spawn(_worker, args=(rdv_url(tmp_path), out), nprocs=WORLD, join=True)
    mk, mb = np.load(out + ".keys.npy"), np.load(out + ".bound.npy")
    rng = np.random.default_rng(42)
    WA, L, free, req = cluster(rng, P, N, cap_scale=0.05)
    cost = oracle.cost(WA, L, "i8")
    wn, wc, wcnt = oracle.topk(cost, oracle.fit_mask(req, free), 8)
    nodes, cnt = usable(mk, mb)
    assert (cnt >= np.minimum(4, wcnt)).all()
    for p in range(P):
        assert nodes[p, :cnt[p]].tolist() == wn[p, :cnt[p]].tolist()
    # committing from the merged lists reproduces the sequential oracle up to
    # the first pod that would need a rescore
    complete = mb == KEY_INVALID
    got, _, _, stop = oracle.commit(nodes, cnt, req, free, complete)
    want, _, _ = oracle.place(WA, L, req, free, "i8")
    assert got[:stop].tolist() == want[:stop].tolist()
    assert stop > 0
