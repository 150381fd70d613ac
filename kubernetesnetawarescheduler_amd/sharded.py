"""Host-exchange placement for node shards.

nas_place runs its loop (score -> exchange -> merge -> commit -> rescore) on
the device and exchanges candidate lists over RCCL (nas_comm_init).  Hosts
that own the transport instead -- several contexts on one device, or ranks
talking over torch.distributed / the Go host's own channel -- run the same
loop here over the host-driven C-ABI steps of include/nas.h
(nas_score_range, nas_get/set_candidate_keys, nas_commit).  Every shard
scores its node columns (nas_set_shard), the lists are merged with the
device rule (klist.h: keep the 8 smallest keys, bound = min(bounds,
kept[7])), and every shard replays the same commit, so all return the same
placements -- identical to one context placing the whole cluster.
"""
import numpy as np

from . import _lib

KEY_INVALID = np.uint64(0xFFFFFFFFFFFFFFFF)
RESCORE_PODS = 1024  # pods rescored per commit stop (nas_api.hip's window)


def merge_lists(parts, K=_lib.K_CANDIDATES):
    """Merge per-shard lists [(keys (n,K) uint64, bounds (n,) uint64), ...]."""
    keys = np.sort(np.concatenate([k for k, _ in parts], axis=1), axis=1)[:, :K]
    bound = np.minimum.reduce([b for _, b in parts] + [keys[:, K - 1]])
    return np.ascontiguousarray(keys), bound


def _loop(P, sync, commit, window):
    sync(0, P)
    stop, rounds = 0, 0
    while True:
        stop = commit(stop)
        if stop >= P:
            return rounds
        rounds += 1
        sync(stop, min(P, stop + window))


def place_local_shards(engines, P, window=RESCORE_PODS):
    """Node shards held by several contexts of this process (engines[r] was
    set_shard(r, len(engines)) before its uploads).  Returns (node, int score,
    rescore rounds); raises if the replicated commits ever disagree."""
    out = [(np.full(P, _lib.NAS_EMPTY, np.int32), np.zeros(P, np.int64)) for _ in engines]

    def sync(lo, hi):
        parts = []
        for e in engines:
            e.score_range(lo, hi)
            parts.append(e.candidate_keys_range(lo, hi - lo))
        mk, mb = merge_lists(parts)
        for e in engines:
            e.set_candidate_keys(lo, mk, mb)

    def commit(p):
        stops = {e.commit(p, node, score) for e, (node, score) in zip(engines, out)}
        if len(stops) != 1:
            raise RuntimeError(f"replicated commits stopped at different pods: {stops}")
        return stops.pop()

    rounds = _loop(P, sync, commit, window)
    for node, score in out[1:]:
        if not (np.array_equal(node, out[0][0]) and np.array_equal(score, out[0][1])):
            raise RuntimeError("replicated commits placed pods differently")
    return out[0][0], out[0][1], rounds


def place_dist_shard(engine, P, all_gather, window=RESCORE_PODS):
    """This rank's shard; all_gather(keys, bounds) returns every rank's
    (keys, bounds) in rank order (e.g. over torch.distributed).  Every rank
    must call this together; all return the same placements."""
    node = np.full(P, _lib.NAS_EMPTY, np.int32)
    score = np.zeros(P, np.int64)

    def sync(lo, hi):
        engine.score_range(lo, hi)
        mk, mb = merge_lists(all_gather(*engine.candidate_keys_range(lo, hi - lo)))
        engine.set_candidate_keys(lo, mk, mb)

    rounds = _loop(P, sync, lambda p: engine.commit(p, node, score), window)
    return node, score, rounds
