"""Replay files (checkpoint / resume): one placement problem or
one reference-mode scoring problem as a single .npz of plain arrays, so a
run can be replayed deterministically on another box and its decisions
compared by digest.

The reference is stateless (its only state is the informer cache); these
files capture what a scheduling pass consumed:

* network-aware mode (`nas_place`): latency L (N x N), capacity (N, 3),
  requests (P, 3), traffic WA (P x N: exact int32 for int8 scoring, bf16
  bits, or float32) -- or, for the seeded synthetic clusters of bench.py,
  only the generator's parameters (`synth`), since C3's dense traffic alone
  is 1 GB;
* reference mode (`nas_score_reference`): the six SoA metric arrays of
  `PrometheusNodeMetrics` (scheduler.go:24-32, one row per snapshot) and the
  two Go map iteration orders (:334, :387).

Files are written with numpy's savez and read with allow_pickle=False: they
carry no code.  Every file has a `format` entry naming the layout.
"""
import hashlib
import json

import numpy as np

PLACE_FORMAT = "nas-place-problem/1"
VOTE_FORMAT = "nas-vote-problem/1"
DTYPES = ("i8", "bf16", "f32")


def _meta(d):
    return np.frombuffer(json.dumps(d, sort_keys=True).encode(), np.uint8)


def _unmeta(a):
    return json.loads(bytes(np.asarray(a, np.uint8)).decode())


def save_place(path, L, free, req, WA, dtype="i8", meta=None):
    """Dense network-aware problem.  WA: integer traffic (int8 scoring, any
    int32), uint16 bf16 bits, or float32, as `Engine.upload_traffic` takes."""
    if dtype not in DTYPES:
        raise ValueError(f"dtype {dtype!r}")
    np.savez(path, format=np.array(PLACE_FORMAT), kind=np.array("dense"), dtype=np.array(dtype),
             L=np.ascontiguousarray(L), free=np.ascontiguousarray(free, np.int32),
             req=np.ascontiguousarray(req, np.int32), WA=np.ascontiguousarray(WA),
             meta=_meta(meta or {}))


def save_place_synth(path, seed, n_nodes, P, dtype="i8", peers=8, meta=None):
    """A bench.py synthetic cluster (`nas_synth_cluster`): its parameters."""
    np.savez(path, format=np.array(PLACE_FORMAT), kind=np.array("synth"), dtype=np.array(dtype),
             synth=np.array([seed, n_nodes, P, peers], np.uint64), meta=_meta(meta or {}))


def save_vote(path, snap, order1, order2, pod_snapshot=None, meta=None):
    """Reference mode: snap = dict of cpu/mem/bw (float64) and rx/tx/disk
    (int64), each (S, N) or (N,); Go map orders order1 (N,), order2 (N+1,)."""
    arrays = {k: np.atleast_2d(np.asarray(snap[k], np.float64 if k in ("cpu", "mem", "bw")
                                          else np.int64)) for k in ("cpu", "mem", "rx", "tx", "bw", "disk")}
    extra = {} if pod_snapshot is None else {"pod_snapshot": np.asarray(pod_snapshot, np.int32)}
    np.savez(path, format=np.array(VOTE_FORMAT), order1=np.asarray(order1, np.int32),
             order2=np.asarray(order2, np.int32), meta=_meta(meta or {}), **arrays, **extra)


def load(path):
    """-> dict of the file's arrays (+ 'meta' decoded); never unpickles."""
    with np.load(path, allow_pickle=False) as z:
        out = {k: z[k] for k in z.files}
    fmt = str(out.get("format", ""))
    if fmt not in (PLACE_FORMAT, VOTE_FORMAT):
        raise ValueError(f"{path}: not a replay file (format {fmt!r})")
    out["format"] = fmt
    out["meta"] = _unmeta(out["meta"]) if "meta" in out else {}
    for k in ("kind", "dtype"):
        if k in out:
            out[k] = str(out[k])
    return out


def capture_place(engine, path, rows_per_read=4096, meta=None):
    """The engine's uploaded network-aware inputs (one cluster, before a
    pass moves its capacity) into a dense replay file."""
    P, N = engine.n_pods, engine.n_nodes
    _, L, free, req = engine.read_inputs(0, 0, want_L=True)
    parts = []
    for p0 in range(0, P, rows_per_read):
        WA, _, _, _ = engine.read_inputs(p0, min(rows_per_read, P - p0), want_L=False)
        parts.append(WA)
    save_place(path, L, free, req, np.concatenate(parts, 0), engine.dtype, meta)


def replay_place(engine, path, want_cost=True):
    """Upload a replay file's problem into `engine` and run nas_place."""
    f = load(path)
    if f["format"] != PLACE_FORMAT:
        raise ValueError("not a placement problem")
    dt = f["dtype"]
    if f["kind"] == "synth":
        seed, n, P, peers = (int(x) for x in f["synth"])
        engine.synth_cluster(seed, n, P, dt, peers=peers)
    else:
        engine.upload_latency(f["L"], dt)
        engine.upload_capacity(f["free"])
        engine.upload_pods(f["req"])
        engine.upload_traffic(f["WA"], dt)
    return engine.place(want_cost=want_cost)


def replay_vote(engine, path):
    """Upload a reference-mode replay file and run nas_score_reference."""
    f = load(path)
    if f["format"] != VOTE_FORMAT:
        raise ValueError("not a vote problem")
    snap = {k: f[k] for k in ("cpu", "mem", "rx", "tx", "bw", "disk")}
    engine.upload_snapshot(snap)
    return engine.score_reference(order1=f["order1"], order2=f["order2"],
                                  pod_snapshot=f.get("pod_snapshot"))


def digest(*arrays):
    """sha256 over the arrays' bytes: compare two runs' decisions."""
    h = hashlib.sha256()
    for a in arrays:
        if a is not None:
            a = np.ascontiguousarray(a)
            h.update(str(a.dtype).encode() + str(a.shape).encode())
            h.update(a.tobytes())
    return h.hexdigest()
