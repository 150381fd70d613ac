"""ctypes binding of libnas.so (include/nas.h).

Loads the in-tree HIP library and declares every exported symbol.  There is
no fallback: if the library is missing or a call fails, NasError is raised.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnas.so")

NAS_OK = 0
NAS_ERR_ARG = -1
NAS_ERR_HIP = -2
NAS_ERR_STATE = -3
NAS_ERR_NOMEM = -4
NAS_ERR_COMM = -5
NAS_ERR_UNSUPPORTED = -6
NAS_NONE = -2
NAS_EMPTY = -1
NAS_DT_I8 = 1
NAS_DT_BF16 = 2
NAS_DT_I32 = 3  # traffic only (int8 latency): exact int32 traffic
NAS_DT_F32 = 4  # fp32 latency and traffic, fp32 MFMA
NAS_OPT_STAGE_TIMINGS = 1
NAS_OPT_COMM_TIMEOUT_MS = 2
NAS_OPT_REHEARSE_WORLD = 3
NAS_OPT_INJECT_STALL_MS = 4
NAS_OPT_COMMIT_WAIT_MS = 5
NAS_OPT_INJECT_COMMIT_STALL_MS = 6
NAS_OPT_SYNTH_PROFILE = 7
NAS_OPT_COMMIT_CUS = 8
NAS_OPT_COST_CACHE = 9
NAS_OPT_HERD_PLAN = 10
NAS_DBG_MASKED_STREAMS_CREATED = 0
NAS_DBG_MASKED_STREAMS_LENT = 1
NAS_DBG_MASKED_STREAMS_IDLE = 2
NAS_DBG_LIVE_CONTEXTS = 3
NAS_DBG_COUNT = 4
K_CANDIDATES = 8
VOTE_NOPOS = 0x7FFFFFFF
# include/nas.h nas_vote_partial: six (value, pos1, reserved) extrema, NAS_VP_* order
VOTE_FIELDS = ("cpu", "mem", "bw", "rx", "tx", "disk")

_ERRNAMES = {
    NAS_ERR_ARG: "NAS_ERR_ARG", NAS_ERR_HIP: "NAS_ERR_HIP", NAS_ERR_STATE: "NAS_ERR_STATE",
    NAS_ERR_NOMEM: "NAS_ERR_NOMEM", NAS_ERR_COMM: "NAS_ERR_COMM",
    NAS_ERR_UNSUPPORTED: "NAS_ERR_UNSUPPORTED",
}


class NasError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class NasConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("reserved0", ctypes.c_int32), ("reserved1", ctypes.c_int32)]


class NasTimings(ctypes.Structure):
    _fields_ = [("fit_ms", ctypes.c_float), ("cost_ms", ctypes.c_float),
                ("merge_ms", ctypes.c_float), ("commit_ms", ctypes.c_float),
                ("vote_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
                ("cost_launches", ctypes.c_int32), ("rescore_rounds", ctypes.c_int32),
                ("unschedulable", ctypes.c_int32), ("commit_rounds", ctypes.c_int32),
                ("rescored_pods", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_c = ctypes
_V = _c.c_void_p
_I = _c.c_int32
_CTX = _c.c_void_p

# name -> (restype, argtypes); mirrors include/nas.h one to one
SIGNATURES = {
    "nas_version": (_I, []),
    "nas_debug_counters": (_I, [_V, _I]),
    "nas_create": (_I, [_c.POINTER(_V), _c.POINTER(NasConfig)]),
    "nas_destroy": (None, [_CTX]),
    "nas_last_error": (_c.c_char_p, [_CTX]),
    "nas_get_timings": (_I, [_CTX, _c.POINTER(NasTimings)]),
    "nas_set_option": (_I, [_CTX, _I, _c.c_int64]),
    "nas_upload_snapshot": (_I, [_CTX, _V, _V, _V, _V, _V, _V, _I, _I]),
    "nas_upload_orders": (_I, [_CTX, _V, _V, _I]),
    "nas_upload_pod_orders": (_I, [_CTX, _V, _V, _I]),
    "nas_score_reference": (_I, [_CTX, _V, _V, _V, _I, _V, _V]),
    "nas_upload_snapshot_shard": (_I, [_CTX, _V, _V, _V, _V, _V, _V, _I, _I, _I, _I]),
    "nas_vote_partials": (_I, [_CTX, _V, _V, _I, _V]),
    "nas_vote_merge": (_I, [_CTX, _V, _I, _I, _V, _V]),
    "nas_upload_latency": (_I, [_CTX, _V, _I, _I]),
    "nas_upload_capacity": (_I, [_CTX, _V, _V, _V, _I]),
    "nas_reset_capacity": (_I, [_CTX]),
    "nas_get_capacity": (_I, [_CTX, _V, _V, _V, _I]),
    "nas_upload_pods": (_I, [_CTX, _V, _V, _V, _I]),
    "nas_upload_traffic_dense": (_I, [_CTX, _V, _I, _I, _I]),
    "nas_upload_traffic_csr": (_I, [_CTX, _V, _V, _V, _I, _I, _I, _c.c_int64]),
    "nas_filter": (_I, [_CTX, _V]),
    "nas_score": (_I, [_CTX]),
    "nas_place": (_I, [_CTX, _V, _V, _V]),
    "nas_get_candidates": (_I, [_CTX, _V, _V, _V, _V, _V]),
    "nas_comm_unique_id": (_I, [_V]),
    "nas_comm_init": (_I, [_CTX, _V, _I, _I]),
    "nas_local_group_create": (_I, [_I, _c.POINTER(_V)]),
    "nas_local_group_destroy": (None, [_V]),
    "nas_comm_init_local": (_I, [_CTX, _V, _I]),
    "nas_set_shard": (_I, [_CTX, _I, _I]),
    "nas_get_candidate_keys": (_I, [_CTX, _V, _V]),
    "nas_score_range": (_I, [_CTX, _I, _I]),
    "nas_get_candidate_keys_range": (_I, [_CTX, _I, _I, _V, _V]),
    "nas_set_candidate_keys": (_I, [_CTX, _I, _I, _V, _V]),
    "nas_commit": (_I, [_CTX, _I, _V, _V, _V, _V]),
    "nas_synth_snapshots": (_I, [_CTX, _c.c_uint64, _I, _I]),
    "nas_synth_snapshots_shard": (_I, [_CTX, _c.c_uint64, _I, _I, _I, _I]),
    "nas_read_snapshot": (_I, [_CTX, _I, _V, _V, _V, _V, _V, _V]),
    "nas_synth_cluster": (_I, [_CTX, _c.c_uint64, _I, _I, _I, _I]),
    "nas_set_batch": (_I, [_CTX, _I]),
    "nas_synth_batch": (_I, [_CTX, _c.c_uint64, _I, _I, _I, _I, _I]),
    "nas_read_inputs": (_I, [_CTX, _I, _I, _V, _V, _V, _V, _V, _V, _V, _V]),
}

_LIB = None


def lib():
    """Load libnas.so (raises if it was not built -- never falls back)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NasError(NAS_ERR_HIP, f"{LIB_PATH} not built: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def ptr(a):
    """Host pointer of a contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data_as(_V)


def as_c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)
