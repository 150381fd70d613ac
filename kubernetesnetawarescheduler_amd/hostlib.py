"""ctypes binding of libnas_host.so (include/nas_host.h), the C++ mirror of
the reference's Go host: Go-semantics ingest, iperf3 report decode, pairwise
latency, and the CustomScheduler loop (scheduler/scheduler.go:119-549) driving
an Engine.  Used by the tests; the cluster side is Python callbacks.
"""
import ctypes
import os

import numpy as np

from ._lib import NasError

HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.path.join(HERE, "libnas_host.so")

NAS_HOST_PANIC = -10
GO_OK, GO_ERR_SYNTAX, GO_ERR_RANGE = 0, 1, 2
OUTCOMES = ("BOUND", "NO_POD", "LIST_ERROR", "BIND_ERROR", "EVENT_ERROR", "PANICKED",
            "UNSCHEDULABLE")

_c = ctypes
_P = _c.c_void_p
_CS = _c.c_char_p
_BUF = _c.c_void_p  # nas_host_buf *

HTTP_GET = _c.CFUNCTYPE(_c.c_int, _P, _CS, _BUF)
READ_FILE = _c.CFUNCTYPE(_c.c_int, _P, _CS, _BUF)
LIST_NODES = _c.CFUNCTYPE(_c.c_int, _P, _BUF, _BUF)
BIND = _c.CFUNCTYPE(_c.c_int, _P, _CS, _CS, _CS, _BUF)
EVENT = _c.CFUNCTYPE(_c.c_int, _P, _CS, _CS, _CS, _CS, _BUF)
NODE_CAP = _c.CFUNCTYPE(_c.c_int, _P, _CS, _c.POINTER(_c.c_int32), _c.POINTER(_c.c_int32),
                        _c.POINTER(_c.c_int32))
POD_NODE = _c.CFUNCTYPE(_c.c_int, _P, _CS, _BUF)
MAP_ORDER = _c.CFUNCTYPE(None, _P, _c.c_int32, _c.POINTER(_c.c_int32), _c.POINTER(_c.c_int32))


class HostIO(_c.Structure):
    _fields_ = [("user", _P), ("http_get", HTTP_GET), ("read_file", READ_FILE),
                ("list_nodes", LIST_NODES), ("bind", BIND), ("create_event", EVENT),
                ("node_capacity", NODE_CAP), ("pod_node", POD_NODE), ("map_order", MAP_ORDER)]


class HostPod(_c.Structure):
    _fields_ = [("ns", _CS), ("name", _CS), ("uid", _CS), ("scheduler_name", _CS),
                ("node_name", _CS), ("cpu_milli", _c.c_int32), ("mem_kib", _c.c_int32),
                ("n_peers", _c.c_int32), ("peers", _c.POINTER(_CS)),
                ("peer_weight", _c.POINTER(_c.c_int32))]


class HostOutcome(_c.Structure):
    _fields_ = [("kind", _c.c_int32), ("pod", _c.c_char * 128), ("node", _c.c_char * 128),
                ("message", _c.c_char * 256)]

    def as_tuple(self):
        return (OUTCOMES[self.kind], self.pod.decode(), self.node.decode(), self.message.decode())


_I32P, _I64P, _F64P = _c.POINTER(_c.c_int32), _c.POINTER(_c.c_int64), _c.POINTER(_c.c_double)
SIGNATURES = {
    "nas_host_buf_append": (None, [_BUF, _c.c_char_p, _c.c_size_t]),
    "nas_host_parse_float": (_c.c_int, [_c.c_char_p, _c.c_size_t, _c.c_int32, _F64P, _I32P]),
    "nas_host_atoi": (_c.c_int, [_c.c_char_p, _c.c_size_t, _I64P, _I32P]),
    "nas_host_node_metrics": (_c.c_int, [_c.c_char_p, _c.c_size_t, _c.c_char_p, _F64P, _F64P,
                                         _I64P, _I64P, _I64P, _c.c_char_p, _c.c_size_t]),
    "nas_host_iperf_receiver": (_c.c_int, [_c.c_char_p, _c.c_size_t, _F64P, _F64P, _I32P, _I32P]),
    "nas_host_snapshot_from_bodies": (_c.c_int, [_c.c_int32, _c.POINTER(_c.c_char_p),
                                                 _c.POINTER(_c.c_size_t), _c.POINTER(_c.c_char_p),
                                                 _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                                 _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int32]),
    "nas_host_latency_matrix": (_c.c_int, [_c.c_int32, _c.POINTER(_c.c_char_p),
                                           _c.POINTER(_c.c_size_t), _c.c_void_p]),
    "nas_host_latency_from_bps": (_c.c_int32, [_c.c_double]),
    "nas_host_latency_matrix_us": (_c.c_int, [_c.c_int32, _c.POINTER(_c.c_char_p),
                                              _c.POINTER(_c.c_size_t), _c.c_void_p]),
    "nas_host_latency_us_from_bps": (_c.c_float, [_c.c_double]),
    "nas_host_create": (_c.c_int, [_c.POINTER(_P), _P, _c.POINTER(HostIO)]),
    "nas_host_destroy": (None, [_P]),
    "nas_host_last_error": (_c.c_char_p, [_P]),
    "nas_host_set_topology": (_c.c_int, [_P, _c.POINTER(_CS), _c.POINTER(_CS), _c.c_int32]),
    "nas_host_set_iperf_path": (_c.c_int, [_P, _CS, _CS]),
    "nas_host_set_latency": (_c.c_int, [_P, _c.POINTER(_CS), _c.c_void_p, _c.c_int32]),
    "nas_host_set_latency_f32": (_c.c_int, [_P, _c.POINTER(_CS), _c.c_void_p, _c.c_int32]),
    "nas_host_enqueue": (_c.c_int, [_P, _c.POINTER(HostPod)]),
    "nas_host_queued": (_c.c_int32, [_P]),
    "nas_host_schedule_one": (_c.c_int, [_P, _c.POINTER(HostOutcome)]),
    "nas_host_schedule_batch": (_c.c_int, [_P, _c.c_int32, _c.POINTER(HostOutcome), _I32P]),
    "nas_host_place_pending": (_c.c_int, [_P, _c.POINTER(HostOutcome), _I32P]),
}

_HL = None


def hostlib():
    """Load libnas_host.so (raises if it was not built)."""
    global _HL
    if _HL is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise NasError(-2, f"{HOST_LIB_PATH} not built: run __graft_entry__.build()")
        L = _c.CDLL(HOST_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _HL = L
    return _HL


def _b(s):
    return s if isinstance(s, bytes) else str(s).encode()


# ------------------------------------------------------------ stateless ingest
def parse_float(s, bits=32):
    v, e = _c.c_double(), _c.c_int32()
    b = _b(s)
    hostlib().nas_host_parse_float(b, len(b), bits, _c.byref(v), _c.byref(e))
    return v.value, e.value


def atoi(s):
    v, e = _c.c_int64(), _c.c_int32()
    b = _b(s)
    hostlib().nas_host_atoi(b, len(b), _c.byref(v), _c.byref(e))
    return v.value, e.value


def node_metrics(body, node):
    """(cpu, mem, rx, tx, disk) or raises GoPanicError."""
    b = _b(body)
    cpu, mem = _c.c_double(), _c.c_double()
    rx, tx, disk = _c.c_int64(), _c.c_int64(), _c.c_int64()
    msg = _c.create_string_buffer(256)
    rc = hostlib().nas_host_node_metrics(b, len(b), _b(node), _c.byref(cpu), _c.byref(mem),
                                         _c.byref(rx), _c.byref(tx), _c.byref(disk), msg, 256)
    if rc == NAS_HOST_PANIC:
        raise GoPanicError(msg.value.decode())
    return cpu.value, mem.value, rx.value, tx.value, disk.value


def snapshot_from_bodies(bodies, names, threads=1):
    """n node-exporter bodies -> dict of SoA arrays (cpu, mem, rx, tx, disk)
    and status (0 or NAS_HOST_PANIC per node), parsed by `threads` workers."""
    n = len(bodies)
    bs = [_b(x) for x in bodies]
    arr = (_c.c_char_p * n)(*bs)
    lens = (_c.c_size_t * n)(*[len(x) for x in bs])
    nm = (_c.c_char_p * n)(*[_b(x) for x in names])
    out = {k: np.zeros(n, np.float64) for k in ("cpu", "mem")}
    out.update({k: np.zeros(n, np.int64) for k in ("rx", "tx", "disk")})
    out["status"] = np.zeros(n, np.int32)
    rc = hostlib().nas_host_snapshot_from_bodies(
        n, arr, lens, nm, *[out[k].ctypes.data_as(_c.c_void_p)
                            for k in ("cpu", "mem", "rx", "tx", "disk", "status")], threads)
    if rc != 0:
        raise NasError(rc, "nas_host_snapshot_from_bodies")
    return out


def iperf_receiver(data):
    """(receiver_bps, sender_bps, n_streams, valid_json)."""
    b = _b(data)
    r, s, n, v = _c.c_double(), _c.c_double(), _c.c_int32(), _c.c_int32()
    hostlib().nas_host_iperf_receiver(b, len(b), _c.byref(r), _c.byref(s), _c.byref(n), _c.byref(v))
    return r.value, s.value, n.value, bool(v.value)


def latency_from_bps(bps):
    return hostlib().nas_host_latency_from_bps(float(bps))


def latency_us_from_bps(bps):
    return hostlib().nas_host_latency_us_from_bps(float(bps))


def latency_matrix(reports, us=False):
    """reports: n x n list of bytes/None (client i -> server j).  int8 ms, or
    (us=True) float32 microseconds per MB for the fp32 path."""
    n = len(reports)
    flat = [None if reports[i][j] is None else _b(reports[i][j]) for i in range(n) for j in range(n)]
    arr = (_c.c_char_p * (n * n))(*flat)
    lens = (_c.c_size_t * (n * n))(*[0 if x is None else len(x) for x in flat])
    L = np.zeros((n, n), np.float32 if us else np.int8)
    fn = hostlib().nas_host_latency_matrix_us if us else hostlib().nas_host_latency_matrix
    rc = fn(n, arr, lens, L.ctypes.data_as(_c.c_void_p))
    if rc != 0:
        raise NasError(rc, "nas_host_latency_matrix")
    return L


class GoPanicError(RuntimeError):
    """The reference would have crashed with this Go runtime panic."""


# ---------------------------------------------------------- scheduler loop
class FakeCluster:
    """In-memory cluster for the host loop: node-exporter bodies by URL,
    iperf reports by path, bindings and events recorded, Go map orders from
    a callable (default: insertion order)."""

    def __init__(self, nodes=(), bodies=None, files=None, capacity=None, bound=None,
                 order=None):
        self.nodes = list(nodes)
        self.bodies = dict(bodies or {})
        self.files = dict(files or {})
        self.capacity = dict(capacity or {})
        self.bound = dict(bound or {})  # "ns/name" -> node
        self.order = order
        self.bindings, self.events = [], []
        self.list_error = None
        self.bind_error = None

    def io(self, append):
        def put(buf, s):
            b = _b(s)
            append(buf, b, len(b))

        def http_get(_u, url, buf):
            body = self.bodies.get(url.decode())
            if body is None:
                return 1
            put(buf, body)
            return 0

        def read_file(_u, path, buf):
            data = self.files.get(path.decode())
            if data is None:
                return 1
            put(buf, data)
            return 0

        def list_nodes(_u, names, err):
            if self.list_error:
                put(err, self.list_error)
                return 1
            put(names, "\n".join(self.nodes))
            return 0

        def bind(_u, ns, pod, node, err):
            if self.bind_error:
                put(err, self.bind_error)
                return 1
            self.bindings.append((ns.decode(), pod.decode(), node.decode()))
            self.bound[f"{ns.decode()}/{pod.decode()}"] = node.decode()
            return 0

        def event(_u, ns, pod, uid, msg, err):
            self.events.append((ns.decode(), pod.decode(), uid.decode(), msg.decode()))
            return 0

        def node_cap(_u, node, c, m, p):
            cap = self.capacity.get(node.decode())
            if cap is None:
                return 1
            c[0], m[0], p[0] = cap
            return 0

        def pod_node(_u, name, buf):
            put(buf, self.bound.get(name.decode(), ""))
            return 0

        def map_order(_u, n, o1, o2):
            if self.order is None:
                return
            a, b = self.order(n)
            for i in range(n):
                o1[i] = int(a[i])
            for i in range(n + 1):
                o2[i] = int(b[i])

        return (HTTP_GET(http_get), READ_FILE(read_file), LIST_NODES(list_nodes), BIND(bind),
                EVENT(event), NODE_CAP(node_cap), POD_NODE(pod_node), MAP_ORDER(map_order))


class HostScheduler:
    """CustomScheduler (scheduler.go:119-237) over an Engine's context."""

    def __init__(self, engine, cluster):
        L = hostlib()
        self._L = L
        self.engine = engine
        self.cluster = cluster
        self._cbs = cluster.io(L.nas_host_buf_append)  # keep the thunks alive
        self._io = HostIO(None, *self._cbs)
        h = _c.c_void_p()
        rc = L.nas_host_create(_c.byref(h), engine._h, _c.byref(self._io))
        if rc != 0:
            raise NasError(rc, "nas_host_create")
        self._h = h
        self._keep = []

    def close(self):
        if getattr(self, "_h", None):
            self._L.nas_host_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _ck(self, rc):
        if rc == NAS_HOST_PANIC:
            raise GoPanicError(self._L.nas_host_last_error(self._h).decode())
        if rc < 0:
            raise NasError(rc, self._L.nas_host_last_error(self._h).decode())
        return rc

    def set_topology(self, names, urls):
        n = len(names)
        a = (_CS * n)(*[_b(x) for x in names])
        u = (_CS * n)(*[_b(x) for x in urls])
        self._ck(self._L.nas_host_set_topology(self._h, a, u, n))

    def set_iperf_path(self, node, path):
        self._ck(self._L.nas_host_set_iperf_path(self._h, _b(node), _b(path)))

    def set_latency(self, names, L):
        """int8 ms (exact integer scores) or float32 us (fp32 costs): the
        dtype of L picks the path of place_pending."""
        f32 = np.asarray(L).dtype == np.float32
        L = np.ascontiguousarray(L, np.float32 if f32 else np.int8)
        n = len(names)
        a = (_CS * n)(*[_b(x) for x in names])
        fn = self._L.nas_host_set_latency_f32 if f32 else self._L.nas_host_set_latency
        self._ck(fn(self._h, a, L.ctypes.data_as(_c.c_void_p), n))

    def enqueue(self, ns, name, uid="", scheduler_name="netAwareScheduler", node_name="",
                cpu_milli=0, mem_kib=0, peers=()):
        names = [_b(p) for p, _ in peers]
        arr = (_CS * max(1, len(names)))(*names)
        w = (_c.c_int32 * max(1, len(names)))(*[int(x) for _, x in peers])
        self._keep.append((arr, w))
        pod = HostPod(_b(ns), _b(name), _b(uid), _b(scheduler_name), _b(node_name), cpu_milli,
                      mem_kib, len(names), arr, w)
        return self._ck(self._L.nas_host_enqueue(self._h, _c.byref(pod))) == 1

    def queued(self):
        return self._L.nas_host_queued(self._h)

    def schedule_one(self):
        o = HostOutcome()
        self._ck(self._L.nas_host_schedule_one(self._h, _c.byref(o)))
        return o.as_tuple()

    def schedule_batch(self, max_pods):
        out = (HostOutcome * max_pods)()
        n = _c.c_int32()
        self._ck(self._L.nas_host_schedule_batch(self._h, max_pods, out, _c.byref(n)))
        return [out[i].as_tuple() for i in range(n.value)]

    def place_pending(self):
        q = max(1, self.queued())
        out = (HostOutcome * q)()
        n = _c.c_int32()
        self._ck(self._L.nas_host_place_pending(self._h, out, _c.byref(n)))
        return [out[i].as_tuple() for i in range(n.value)]
