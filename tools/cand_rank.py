"""Where in its candidate list each pod's placement sits (C3 pipelined pass,
and a single-chunk score + commit from fresh capacity)."""
import json, os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from kubernetesnetawarescheduler_amd import Engine
N, P = 10000, 100000
def ranks(e, node):
    keys, bounds = e.candidate_keys_range(0, P)
    kn = (keys & np.uint64(0xFFFFFFFF)).astype(np.int64)
    m = kn == node[:, None]
    r = np.where(m.any(1), m.argmax(1), 8)
    return {int(k): int(v) for k, v in zip(*np.unique(r, return_counts=True))}
with Engine(0) as e:
    e.synth_cluster(0xC3, N, P, "i8", peers=8)
    e.reset_capacity()
    node = e.place()[0]
    print("pass", json.dumps(ranks(e, np.asarray(node))))
    e.reset_capacity()
    e.score_range(0, P)
    nd = np.zeros(P, np.int32)
    e.reset_capacity()
    stop = e.commit(0, nd)
    print("single", stop, json.dumps(ranks(e, nd)))
