"""ctypes/numpy front-end of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Restates scheduler/scheduler.go:248-394 (reference mode) and the
build-defined extended mode (fit / cost / top-k / sequential greedy).
Function-level citations live in oracle.c.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

NONE = -2   # the "none" pseudo-node (scheduler.go:267-272, :364)
EMPTY = -1  # "" from findBestNode (scheduler.go:386) / unschedulable

_P = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        _LIB = ctypes.CDLL(path)
        _LIB.or_vote_literal.restype = ctypes.c_int
        _LIB.or_vote_closed.restype = ctypes.c_int
        _LIB.or_vote_batch.restype = ctypes.c_int
        _LIB.or_place.restype = ctypes.c_int
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(_P) if a is not None else None


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def vote(metrics, order1, order2, closed=False):
    """One snapshot. metrics = dict(cpu, mem, rx, tx, bw, disk) arrays of n.
    Returns (best, winners[6], scores[n+1] or None)."""
    cpu = _c(metrics["cpu"], np.float64)
    n = cpu.shape[0]
    mem = _c(metrics["mem"], np.float64)
    rx = _c(metrics["rx"], np.int64)
    tx = _c(metrics["tx"], np.int64)
    bw = _c(metrics["bw"], np.float64)
    disk = _c(metrics["disk"], np.int64)
    o1 = _c(order1, np.int32)
    o2 = _c(order2, np.int32)
    best = np.zeros(1, np.int32)
    win = np.zeros(6, np.int32)
    if closed:
        rc = lib().or_vote_closed(n, _ptr(cpu), _ptr(mem), _ptr(rx), _ptr(tx), _ptr(bw),
                                  _ptr(disk), _ptr(o1), _ptr(o2), _ptr(best), _ptr(win))
        scores = None
    else:
        scores = np.zeros(n + 1, np.int64)
        rc = lib().or_vote_literal(n, _ptr(cpu), _ptr(mem), _ptr(rx), _ptr(tx), _ptr(bw),
                                   _ptr(disk), _ptr(o1), _ptr(o2), _ptr(best), _ptr(win),
                                   _ptr(scores))
    if rc:
        raise ValueError("order is not a permutation")
    return int(best[0]), win, scores


def vote_batch(snap, order1, order2, pod_snapshot=None):
    """snap = dict of (n_snapshots, n) arrays; order1 (n_orders, n); order2 (n_orders, n+1).
    Returns best[P], winners[P, 6]."""
    cpu = _c(snap["cpu"], np.float64)
    S, n = cpu.shape
    arrs = [cpu, _c(snap["mem"], np.float64), _c(snap["rx"], np.int64),
            _c(snap["tx"], np.int64), _c(snap["bw"], np.float64), _c(snap["disk"], np.int64)]
    o1 = _c(order1, np.int32).reshape(-1, n)
    o2 = _c(order2, np.int32).reshape(-1, n + 1)
    ps = None if pod_snapshot is None else _c(pod_snapshot, np.int32)
    P = S if ps is None else ps.shape[0]
    best = np.zeros(P, np.int32)
    win = np.zeros((P, 6), np.int32)
    rc = lib().or_vote_batch(n, S, *[_ptr(a) for a in arrs], _ptr(o1), _ptr(o2), o1.shape[0],
                             _ptr(ps), P, _ptr(best), _ptr(win))
    if rc:
        raise ValueError("bad order or snapshot index")
    return best, win


def vote_gomap(snap):
    """The reference loop over Go-style maps (gomap.cpp): snap = dict of
    (P, n) arrays, one snapshot per pod.  Returns best[P], order1 (P, n) and
    order2 (P, n+1) -- the map orders walked -- and (fill_ns, loop_ns)."""
    cpu = _c(snap["cpu"], np.float64)
    P, n = cpu.shape
    arrs = [cpu, _c(snap["mem"], np.float64), _c(snap["rx"], np.int64),
            _c(snap["tx"], np.int64), _c(snap["bw"], np.float64), _c(snap["disk"], np.int64)]
    best = np.zeros(P, np.int32)
    o1 = np.zeros((P, n), np.int32)
    o2 = np.zeros((P, n + 1), np.int32)
    fill, loop = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = lib().or_vote_gomap(n, P, *[_ptr(a) for a in arrs], _ptr(best), _ptr(o1), _ptr(o2),
                             ctypes.byref(fill), ctypes.byref(loop))
    if rc:
        raise ValueError("gomap: priorities map lacks the none key")
    return best, o1, o2, (fill.value, loop.value)


def fit_mask(req, free):
    """req: (P,3) int32 [cpu_milli, mem_kib, pods]; free: (N,3). Returns uint32 (P, ceil(N/32))."""
    req = _c(req, np.int32)
    free = _c(free, np.int32)
    P, N = req.shape[0], free.shape[0]
    cols = [np.ascontiguousarray(req[:, i]) for i in range(3)]
    fcols = [np.ascontiguousarray(free[:, i]) for i in range(3)]
    W = (N + 31) // 32
    mask = np.zeros((P, W), np.uint32)
    lib().or_fit(P, N, *[_ptr(a) for a in cols], *[_ptr(a) for a in fcols], _ptr(mask))
    return mask


def _i32(WA):
    """Exact integer traffic as int32 (refuses values outside int32)."""
    a = np.asarray(WA)
    if a.dtype.kind in "iu" and a.size and (a.min() < -2**31 or a.max() > 2**31 - 1):
        raise ValueError("traffic outside int32")
    return _c(a, np.int32)


def cost(WA, L, dtype):
    """dtype 'i8': integer traffic (any int32, never saturated) x int8 latency
    -> exact int64; 'bf16': uint16 bf16 bits -> float64; 'f32': float32 ->
    float64 (exact products, fp64 sums)."""
    P, N = WA.shape
    if dtype == "i8":
        out = np.zeros((P, N), np.int64)
        lib().or_cost_i8(P, N, _ptr(_i32(WA)), _ptr(_c(L, np.int8)), _ptr(out))
    elif dtype == "f32":
        out = np.zeros((P, N), np.float64)
        lib().or_cost_f32(P, N, _ptr(_c(WA, np.float32)), _ptr(_c(L, np.float32)), _ptr(out))
    else:
        out = np.zeros((P, N), np.float64)
        lib().or_cost_bf16(P, N, _ptr(_c(WA, np.uint16)), _ptr(_c(L, np.uint16)), _ptr(out))
    return out


def topk(cost_mat, mask, k):
    cost_mat = np.ascontiguousarray(cost_mat)
    P, N = cost_mat.shape
    node = np.zeros((P, k), np.int32)
    cnt = np.zeros(P, np.int32)
    m = _c(mask, np.uint32)
    if cost_mat.dtype == np.int64:
        cc = np.zeros((P, k), np.int64)
        lib().or_topk(P, N, k, _ptr(cost_mat), None, _ptr(m), _ptr(node), _ptr(cc), None, _ptr(cnt))
    else:
        cm = _c(cost_mat, np.float64)
        cc = np.zeros((P, k), np.float64)
        lib().or_topk(P, N, k, None, _ptr(cm), _ptr(m), _ptr(node), None, _ptr(cc), _ptr(cnt))
    return node, cc, cnt


def place(WA, L, req, free, dtype):
    """Sequential greedy placement. Returns (node[P], cost[P], free_after (N,3))."""
    P, N = WA.shape
    req = _c(req, np.int32)
    free = _c(free, np.int32).copy()
    rcols = [np.ascontiguousarray(req[:, i]) for i in range(3)]
    fcols = [np.ascontiguousarray(free[:, i]) for i in range(3)]
    node = np.zeros(P, np.int32)
    if dtype == "i8":
        dt, wa, ll = 1, _i32(WA), _c(L, np.int8)
        ci = np.zeros(P, np.int64)
        cd = None
    elif dtype == "f32":
        dt, wa, ll = 3, _c(WA, np.float32), _c(L, np.float32)
        ci = None
        cd = np.zeros(P, np.float64)
    else:
        dt, wa, ll = 2, _c(WA, np.uint16), _c(L, np.uint16)
        ci = None
        cd = np.zeros(P, np.float64)
    rc = lib().or_place(P, N, dt, _ptr(wa), _ptr(ll), *[_ptr(a) for a in rcols],
                        *[_ptr(a) for a in fcols], _ptr(node), _ptr(ci), _ptr(cd))
    if rc:
        raise ValueError("bad dtype")
    return node, (ci if ci is not None else cd), np.stack(fcols, axis=1)


def commit(cand_node, count, req, free, complete=None):
    """Commit from candidate lists. Returns (node[P], slot[P], free_after, stop).
    complete[p]: list holds every fitting node (default: count < k)."""
    cand_node = _c(cand_node, np.int32)
    P, k = cand_node.shape
    req = _c(req, np.int32)
    free = _c(free, np.int32).copy()
    rcols = [np.ascontiguousarray(req[:, i]) for i in range(3)]
    fcols = [np.ascontiguousarray(free[:, i]) for i in range(3)]
    node = np.full(P, -3, np.int32)
    slot = np.full(P, -1, np.int32)
    stop = ctypes.c_int(0)
    comp = None if complete is None else _c(complete, np.int32)
    lib().or_commit(P, k, _ptr(cand_node), _ptr(_c(count, np.int32)), _ptr(comp),
                    *[_ptr(a) for a in rcols],
                    *[_ptr(a) for a in fcols], _ptr(node), _ptr(slot), ctypes.byref(stop))
    return node, slot, np.stack(fcols, axis=1), stop.value


# ---- node-sharded reference mode (SURVEY.md §8(e) vote row, Appendix B) ----
# Pure-Python/numpy restatement for small cases; records follow include/nas.h
# nas_vote_partial: six (value bits, pos1) extrema in the order
# cpu, mem, bw, rx, tx, disk; pos1 = NOPOS when no node of the slice beats
# the sentinel (value then 0).
NOPOS = 0x7FFFFFFF
PART_FIELDS = ("cpu", "mem", "bw", "rx", "tx", "disk")
# sentinels scheduler.go:258-265 (bw omitted -> 0.0); guards of :335-355
_SENT = {"cpu": 99999999999.0, "mem": 99999999999.0, "rx": 99999999999,
         "tx": 99999999999, "disk": 999, "bw": 0.0}
_IS_MAX = {"bw"}
_IS_F64 = {"cpu", "mem", "bw"}


def _bits(x, f):
    if f in _IS_F64:
        return int(np.array([x], np.float64).view(np.int64)[0])
    return int(x)


def _unbits(v, f):
    if f in _IS_F64:
        return float(np.array([v], np.int64).view(np.float64)[0])
    return int(v)


def _qualifies(x, f):
    # scheduler.go:335 / :339 / :343 / :347 (<), :351 (> 0.0), :355 (< 999 && != 0)
    if f == "bw":
        return x > _SENT[f]
    if f == "disk":
        return x != 0 and x < _SENT[f]
    return x < _SENT[f]


def _better(x, q, v, p, f):
    """(x, q) beats the kept (v, p): strictly better value, or a value that is
    neither better nor worse (equal; -0.0 == +0.0) at an earlier pos1."""
    if p == NOPOS:
        return True
    if f in _IS_MAX:
        return x > v or (not (v > x) and q < p)
    return x < v or (not (v < x) and q < p)


def vote_partial(metrics, node_lo, order1):
    """Partial record of nodes [node_lo, node_lo + len) of one snapshot:
    list of six (value_bits, pos1).  metrics: dict of the slice's arrays."""
    n_all = len(order1)
    pos1 = np.empty(n_all, np.int64)
    pos1[np.asarray(order1, np.int64)] = np.arange(n_all)
    rec = []
    for f in PART_FIELDS:
        vals = np.asarray(metrics[f], np.float64 if f in _IS_F64 else np.int64)
        v, p = 0, NOPOS
        for i in range(vals.shape[0]):
            x = vals[i].item()
            q = int(pos1[node_lo + i])
            if _qualifies(x, f) and _better(x, q, v, p, f):
                v, p = x, q
        rec.append((_bits(v, f) if p != NOPOS else 0, p))
    return rec


def vote_from_partials(parts, order1, order2):
    """Merge the records of every slice of one snapshot, then net-sent
    (scheduler.go:347-354), votes (:360-365) and findBestNode (:384-394).
    Returns (best, winners[6])."""
    n = len(order1)
    keep = {}
    for f_i, f in enumerate(PART_FIELDS):
        v, p = 0, NOPOS
        for rec in parts:
            bits, q = rec[f_i]
            if q == NOPOS:
                continue
            x = _unbits(bits, f)
            if _better(x, q, v, p, f):
                v, p = x, q
        keep[f] = p
    ps = keep["tx"]
    if keep["bw"] != NOPOS and (ps == NOPOS or keep["bw"] > ps):
        ps = keep["bw"]

    def node_at(q):
        return n if q == NOPOS else int(order1[q])

    key = [node_at(keep["cpu"]), node_at(keep["mem"]), node_at(ps), node_at(keep["rx"]),
           n, node_at(keep["disk"])]
    weight = [3, 2, 1, 1, 3, 1]
    scores = {}
    for k, w in zip(key, weight):
        scores[k] = scores.get(k, 0) + w
    maxp, best = 0, EMPTY
    for k in order2:
        sc = scores.get(int(k), 0)
        if sc > maxp:
            maxp, best = sc, (NONE if k == n else int(k))
    return best, [NONE if k == n else k for k in key]
