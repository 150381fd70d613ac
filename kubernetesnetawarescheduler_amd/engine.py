"""Engine: a numpy-facing handle on one nas_ctx (one HIP device).

Thin plumbing over the C ABI for tests and bench.py.  Names follow the
reference: snapshots are PrometheusNodeMetrics records
(scheduler/scheduler.go:24-32), `score_reference` is prioritize +
findBestNode (:248-394), `place` is the network-aware filter/score/commit.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import NasError, as_c, ptr

FIELDS = ("cpu", "mem", "rx", "tx", "bw", "disk")
# one nas_vote_extremum (include/nas.h); a record is 6 of them (NAS_VP_* order)
VOTE_PARTIAL_DTYPE = np.dtype([("value", "<i8"), ("pos1", "<i4"), ("reserved", "<i4")])
_FDT = {"cpu": np.float64, "mem": np.float64, "rx": np.int64, "tx": np.int64,
        "bw": np.float64, "disk": np.int64}


def debug_counters():
    """nas_debug_counters: process-wide {masked_streams_created, _lent, _idle,
    live_contexts} (include/nas.h NAS_DBG_*)."""
    out = np.zeros(_lib.NAS_DBG_COUNT, np.int64)
    rc = _lib.lib().nas_debug_counters(ptr(out), _lib.NAS_DBG_COUNT)
    if rc != 0:
        raise NasError(rc, "nas_debug_counters")
    return {"masked_streams_created": int(out[_lib.NAS_DBG_MASKED_STREAMS_CREATED]),
            "masked_streams_lent": int(out[_lib.NAS_DBG_MASKED_STREAMS_LENT]),
            "masked_streams_idle": int(out[_lib.NAS_DBG_MASKED_STREAMS_IDLE]),
            "live_contexts": int(out[_lib.NAS_DBG_LIVE_CONTEXTS])}


class LocalGroup:
    """nas_local_group: `world` Engines of this process that exchange like
    RCCL ranks.  Each rank's calls must run on their own thread (ctypes
    releases the GIL inside them); see local_ranks()."""

    def __init__(self, world):
        self._L = _lib.lib()
        h = ctypes.c_void_p()
        rc = self._L.nas_local_group_create(world, ctypes.byref(h))
        if rc != 0:
            raise NasError(rc, "nas_local_group_create: world out of range")
        self.handle = h
        self.world = world

    def close(self):
        if getattr(self, "handle", None):
            self._L.nas_local_group_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


def local_ranks(engines, fn):
    """Run fn(rank, engine) for every rank of an in-process group concurrently
    (one thread each, as the group's barriers require); returns the results in
    rank order and re-raises the first rank's exception."""
    import threading

    out = [None] * len(engines)
    err = [None] * len(engines)

    def run(r):
        try:
            out[r] = fn(r, engines[r])
        except BaseException as ex:  # noqa: BLE001 -- re-raised below
            err[r] = ex

    ts = [threading.Thread(target=run, args=(r,)) for r in range(len(engines))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for ex in err:
        if ex is not None:
            raise ex
    return out


class Engine:
    def __init__(self, device=0):
        self._L = _lib.lib()
        cfg = _lib.NasConfig(device=device)
        h = ctypes.c_void_p()
        rc = self._L.nas_create(ctypes.byref(h), ctypes.byref(cfg))
        if rc != 0:
            raise NasError(rc, "nas_create failed (no GPU visible or bad device ordinal)")
        self._h = h
        self.n_nodes = 0
        self.n_pods = 0
        self.dtype = 0
        self.n_clusters = 1  # nas_set_batch: arrays carry a leading cluster axis when > 1
        self.has_comm = False

    # ------------------------------------------------------------ plumbing
    def _ck(self, rc):
        if rc != 0:
            raise NasError(rc, self._L.nas_last_error(self._h).decode())

    def close(self):
        if getattr(self, "_h", None):
            self._L.nas_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_option(self, key, value):
        """nas_set_option: key is an NAS_OPT_* constant of _lib (or its name
        without the prefix, e.g. "STAGE_TIMINGS")."""
        if isinstance(key, str):
            key = getattr(_lib, "NAS_OPT_" + key)
        self._ck(self._L.nas_set_option(self._h, key, int(value)))

    def timings(self):
        t = _lib.NasTimings()
        self._ck(self._L.nas_get_timings(self._h, ctypes.byref(t)))
        return t.as_dict()

    # ------------------------------------------------------ reference mode
    def upload_snapshot(self, snap):
        """snap: dict of FIELDS -> (n_snapshots, n_nodes) or (n_nodes,) arrays."""
        arrs = {f: as_c(snap[f], _FDT[f]) for f in FIELDS}
        a0 = arrs["cpu"]
        if a0.ndim == 1:
            arrs = {f: a.reshape(1, -1) for f, a in arrs.items()}
        S, n = arrs["cpu"].shape
        for a in arrs.values():
            if a.shape != (S, n):
                raise ValueError("snapshot fields must share one shape")
        self._ck(self._L.nas_upload_snapshot(self._h, ptr(arrs["cpu"]), ptr(arrs["mem"]),
                                             ptr(arrs["rx"]), ptr(arrs["tx"]), ptr(arrs["bw"]),
                                             ptr(arrs["disk"]), n, S))
        self.snap_nodes, self.snap_count = n, S

    def upload_snapshot_shard(self, snap, n_nodes, node_lo):
        """Node shard of a snapshot set (include/nas.h nas_upload_snapshot_shard):
        snap fields are (n_snapshots, n_local) arrays of nodes [node_lo, node_lo+n_local)."""
        arrs = {f: as_c(snap[f], _FDT[f]) for f in FIELDS}
        if arrs["cpu"].ndim == 1:
            arrs = {f: a.reshape(1, -1) for f, a in arrs.items()}
        S, nl = arrs["cpu"].shape
        for a in arrs.values():
            if a.shape != (S, nl):
                raise ValueError("snapshot fields must share one shape")
        self._ck(self._L.nas_upload_snapshot_shard(
            self._h, ptr(arrs["cpu"]), ptr(arrs["mem"]), ptr(arrs["rx"]), ptr(arrs["tx"]),
            ptr(arrs["bw"]), ptr(arrs["disk"]), n_nodes, node_lo, nl, S))
        self.snap_nodes, self.snap_count = nl, S

    def synth_snapshots_shard(self, seed, n_nodes, node_lo, n_local, n_snapshots):
        self._ck(self._L.nas_synth_snapshots_shard(self._h, seed, n_nodes, node_lo, n_local,
                                                   n_snapshots))
        self.snap_nodes, self.snap_count = n_local, n_snapshots

    def vote_partials(self, S=None, order1=None, order2=None):
        """Partial records of this context's node slice: (S, 6) VOTE_PARTIAL_DTYPE."""
        S = self.snap_count if S is None else S
        o1 = None if order1 is None else as_c(order1, np.int32)
        o2 = None if order2 is None else as_c(order2, np.int32)
        out = np.zeros((S, 6), VOTE_PARTIAL_DTYPE)
        self._ck(self._L.nas_vote_partials(self._h, ptr(o1), ptr(o2), S, ptr(out)))
        return out

    def vote_merge(self, parts, winners=True):
        """parts: (n_parts, S, 6) VOTE_PARTIAL_DTYPE -> best[S], winners[S, 6]."""
        parts = np.ascontiguousarray(parts, VOTE_PARTIAL_DTYPE)
        if parts.ndim == 2:
            parts = parts[None]
        K, S, six = parts.shape
        if six != 6:
            raise ValueError("parts must be (n_parts, S, 6)")
        best = np.empty(S, np.int32)
        win = np.empty((S, 6), np.int32) if winners else None
        self._ck(self._L.nas_vote_merge(self._h, ptr(parts), K, S, ptr(best), ptr(win)))
        return best, win

    def upload_orders(self, order1, order2):
        o1 = as_c(order1, np.int32)
        o2 = as_c(order2, np.int32)
        n_orders = 1 if o1.ndim == 1 else o1.shape[0]
        self._ck(self._L.nas_upload_orders(self._h, ptr(o1), ptr(o2), n_orders))

    def upload_pod_orders(self, order1, order2):
        """One order set per pod of the next score_reference (include/nas.h)."""
        o1 = np.atleast_2d(as_c(order1, np.int32))
        o2 = np.atleast_2d(as_c(order2, np.int32))
        self._ck(self._L.nas_upload_pod_orders(self._h, ptr(o1), ptr(o2), o1.shape[0]))

    def score_reference(self, P=None, order1=None, order2=None, pod_snapshot=None, winners=True):
        ps = None if pod_snapshot is None else as_c(pod_snapshot, np.int32)
        if P is None:
            P = self.snap_count if ps is None else ps.shape[0]
        o1 = None if order1 is None else as_c(order1, np.int32)
        o2 = None if order2 is None else as_c(order2, np.int32)
        best = np.empty(P, np.int32)
        win = np.empty((P, 6), np.int32) if winners else None
        self._ck(self._L.nas_score_reference(self._h, ptr(o1), ptr(o2), ptr(ps), P, ptr(best),
                                             ptr(win)))
        return best, win

    def synth_snapshots(self, seed, n_nodes, n_snapshots):
        self._ck(self._L.nas_synth_snapshots(self._h, seed, n_nodes, n_snapshots))
        self.snap_nodes, self.snap_count = n_nodes, n_snapshots

    def read_snapshot(self, s):
        n = self.snap_nodes
        out = {f: np.empty(n, _FDT[f]) for f in FIELDS}
        self._ck(self._L.nas_read_snapshot(self._h, s, ptr(out["cpu"]), ptr(out["mem"]),
                                           ptr(out["rx"]), ptr(out["tx"]), ptr(out["bw"]),
                                           ptr(out["disk"])))
        return out

    # -------------------------------------------------------- extended mode
    def comm_init(self, uid, rank, world):
        b = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._ck(self._L.nas_comm_init(self._h, b, rank, world))
        self.has_comm = True

    def comm_init_local(self, group, rank):
        """Join an in-process group (LocalGroup) as `rank` (include/nas.h
        nas_comm_init_local): node shard of group.world ranks whose
        exchanges run device to device instead of over RCCL."""
        self._ck(self._L.nas_comm_init_local(self._h, group.handle, rank))
        self.has_comm = True

    def set_shard(self, rank, world):
        self._ck(self._L.nas_set_shard(self._h, rank, world))

    def candidate_keys(self):
        keys = np.empty((self.n_pods, _lib.K_CANDIDATES), np.uint64)
        bounds = np.empty(self.n_pods, np.uint64)
        self._ck(self._L.nas_get_candidate_keys(self._h, ptr(keys), ptr(bounds)))
        return keys, bounds

    # host-driven steps (include/nas.h): score a range, move lists, commit
    def score_range(self, p_lo, p_hi):
        self._ck(self._L.nas_score_range(self._h, p_lo, p_hi))

    def candidate_keys_range(self, p_lo, n):
        keys = np.empty((n, _lib.K_CANDIDATES), np.uint64)
        bounds = np.empty(n, np.uint64)
        self._ck(self._L.nas_get_candidate_keys_range(self._h, p_lo, n, ptr(keys), ptr(bounds)))
        return keys, bounds

    def set_candidate_keys(self, p_lo, keys, bounds):
        keys = as_c(keys, np.uint64)
        bounds = as_c(bounds, np.uint64)
        self._ck(self._L.nas_set_candidate_keys(self._h, p_lo, bounds.shape[0], ptr(keys),
                                                ptr(bounds)))

    def commit(self, p_begin, node, score=None):
        """Commit pods [p_begin, P) into node (and score); returns the stop pod."""
        stop = ctypes.c_int32(0)
        self._ck(self._L.nas_commit(self._h, p_begin, ptr(node), None, ptr(score),
                                    ctypes.byref(stop)))
        return stop.value

    @staticmethod
    def comm_unique_id():
        b = (ctypes.c_uint8 * 128)()
        rc = _lib.lib().nas_comm_unique_id(b)
        if rc != 0:
            raise NasError(rc, "ncclGetUniqueId failed")
        return bytes(b)

    @staticmethod
    def _dt(dtype):
        return {"i8": _lib.NAS_DT_I8, "bf16": _lib.NAS_DT_BF16, "f32": _lib.NAS_DT_F32}[dtype]

    @staticmethod
    def _np(dtype):
        return {"i8": np.int8, "bf16": np.uint16, "f32": np.float32}[dtype]

    # A batch (set_batch / synth_batch) passes every extended-mode array with a
    # leading cluster axis: L (B, n, n), free (B, n, 3), req (B, P, 3), WA (B, P, n).
    def set_batch(self, n_clusters):
        self._ck(self._L.nas_set_batch(self._h, n_clusters))
        self.n_clusters = n_clusters

    def synth_batch(self, seed, n_clusters, n_nodes, P, dtype="i8", peers=8, profile=0):
        self.set_option("SYNTH_PROFILE", profile)
        self._ck(self._L.nas_synth_batch(self._h, seed, n_clusters, n_nodes, P, self._dt(dtype),
                                         peers))
        self.n_clusters, self.n_nodes, self.n_pods, self.dtype = n_clusters, n_nodes, P, dtype

    @staticmethod
    def _cols(a, last):
        """(..., last) array -> `last` contiguous columns over every cluster."""
        return [np.ascontiguousarray(a[..., i]).reshape(-1) for i in range(last)]

    def upload_latency(self, L, dtype):
        L = as_c(L, self._np(dtype))
        n = L.shape[-1]
        self._ck(self._L.nas_upload_latency(self._h, ptr(L), self._dt(dtype), n))
        self.n_nodes, self.dtype = n, dtype

    def upload_capacity(self, free):
        free = as_c(free, np.int32)
        cols = self._cols(free, 3)
        self._ck(self._L.nas_upload_capacity(self._h, *[ptr(c) for c in cols], free.shape[-2]))
        self.n_nodes = free.shape[-2]

    def reset_capacity(self):
        self._ck(self._L.nas_reset_capacity(self._h))

    def get_capacity(self):
        n, B = self.n_nodes, self.n_clusters
        cols = [np.empty(B * n, np.int32) for _ in range(3)]
        self._ck(self._L.nas_get_capacity(self._h, *[ptr(c) for c in cols], n))
        out = np.stack(cols, axis=1)
        return out if B == 1 else out.reshape(B, n, 3)

    def upload_pods(self, req):
        req = as_c(req, np.int32)
        cols = self._cols(req, 3)
        self._ck(self._L.nas_upload_pods(self._h, *[ptr(c) for c in cols], req.shape[-2]))
        self.n_pods = req.shape[-2]

    @staticmethod
    def _int_traffic(a):
        """Integer traffic for int8 scoring: an int8 array as is (NAS_DT_I8),
        any other integer array as exact int32 (NAS_DT_I32; never saturated)."""
        a = np.asarray(a)
        if a.dtype == np.int8:
            return as_c(a, np.int8), _lib.NAS_DT_I8
        if a.dtype.kind not in "iu":
            raise TypeError("int8 scoring takes integer traffic")
        if a.size and (a.min() < -2**31 or a.max() > 2**31 - 1):
            raise ValueError("traffic outside int32")
        return as_c(a, np.int32), _lib.NAS_DT_I32

    def upload_traffic(self, WA, dtype):
        """dtype "i8": integer traffic (int8 arrays as int8, wider ones as exact
        int32) against int8 latency; "bf16": bf16 bits; "f32": float32."""
        if dtype in ("i8", "i32"):
            WA, dt = self._int_traffic(WA)
        else:
            WA, dt = as_c(WA, self._np(dtype)), self._dt(dtype)
        P, n = WA.shape[-2:]
        self._ck(self._L.nas_upload_traffic_dense(self._h, ptr(WA), dt, P, n))
        self.n_pods, self.n_nodes, self.dtype = P, n, "i8" if dtype in ("i8", "i32") else dtype

    def upload_traffic_csr(self, row_ptr, peer_node, weight, dtype, n):
        rp = as_c(row_ptr, np.int32)
        pn = as_c(peer_node, np.int32)
        if dtype in ("i8", "i32"):
            w, dt = self._int_traffic(weight)
        else:
            w, dt = as_c(weight, self._np(dtype)), self._dt(dtype)
        P = rp.shape[0] - 1
        self._ck(self._L.nas_upload_traffic_csr(self._h, ptr(rp), ptr(pn), ptr(w), dt,
                                                P, n, pn.shape[0]))
        self.n_pods, self.n_nodes, self.dtype = P, n, "i8" if dtype in ("i8", "i32") else dtype

    def filter(self, want_mask=True):
        """nas_filter: the fit mask [chunk][pod] (bit j of word (c, p) = pod p
        fits node 64c + j); want_mask=False runs the kernel alone (timing)."""
        if not want_mask:
            self._ck(self._L.nas_filter(self._h, None))
            return None
        chunks = (self.n_nodes + 63) // 64
        mask = np.zeros((chunks, self.n_pods), np.uint64)
        self._ck(self._L.nas_filter(self._h, ptr(mask)))
        return mask

    def score(self):
        self._ck(self._L.nas_score(self._h))

    def candidates(self):
        P, K = self.n_pods * self.n_clusters, _lib.K_CANDIDATES
        node = np.empty((P, K), np.int32)
        ci = np.empty((P, K), np.int64)
        cf = np.empty((P, K), np.float32)
        cnt = np.empty(P, np.int32)
        complete = np.empty(P, np.int32)
        self._ck(self._L.nas_get_candidates(self._h, ptr(node), ptr(ci), ptr(cf), ptr(cnt),
                                            ptr(complete)))
        return node, ci, cf, cnt, complete.astype(bool)

    def place(self, want_cost=True, out=None):
        """-> (node, float cost, integer score) per pod.  out: optional
        (node int32, cost float32 or None, score int64 or None) arrays of
        length B*P to fill instead of fresh ones (repeated calls then touch no
        new pages)."""
        B, P = self.n_clusters, self.n_pods
        if out is not None:
            node, cf, ci = out
            for a, dt in ((node, np.int32), (cf, np.float32), (ci, np.int64)):
                if a is not None and (a.dtype != dt or a.size != B * P or not a.flags.c_contiguous):
                    raise ValueError("place(out=...): wrong dtype, size or layout")
        else:
            node = np.empty(B * P, np.int32)
            cf = np.empty(B * P, np.float32) if want_cost else None
            ci = np.empty(B * P, np.int64) if want_cost else None
        self._ck(self._L.nas_place(self._h, ptr(node), ptr(cf), ptr(ci)))
        if B > 1:
            node = node.reshape(B, P)
            cf = None if cf is None else cf.reshape(B, P)
            ci = None if ci is None else ci.reshape(B, P)
        return node, cf, ci

    def synth_cluster(self, seed, n_nodes, P, dtype="i8", peers=8, profile=0):
        """nas_synth_cluster; profile (NAS_OPT_SYNTH_PROFILE): 0 racks / zones
        with bound peers, 1 uniform over the full int8 range."""
        self.set_option("SYNTH_PROFILE", profile)
        self._ck(self._L.nas_synth_cluster(self._h, seed, n_nodes, P, self._dt(dtype), peers))
        self.n_nodes, self.n_pods, self.dtype = n_nodes, P, dtype

    def read_inputs(self, p0=0, np_=0, want_L=True):
        """-> (WA rows [p0, p0+np_) -- exact int32 traffic for int8 scoring,
        bf16 bits otherwise --, L, capacity (n, 3), requests (P, 3))."""
        n, P = self.n_nodes, self.n_pods
        dt = self._np(self.dtype)
        WA = np.empty((np_, n), np.int32 if self.dtype == "i8" else dt) if np_ else None
        L = np.empty((n, n), dt) if want_L else None
        cap = [np.empty(n, np.int32) for _ in range(3)]
        req = [np.empty(P, np.int32) for _ in range(3)]
        self._ck(self._L.nas_read_inputs(self._h, p0, np_, ptr(WA), ptr(L), *[ptr(c) for c in cap],
                                         *[ptr(r) for r in req]))
        return WA, L, np.stack(cap, axis=1), np.stack(req, axis=1)
