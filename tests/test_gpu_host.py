"""The C++ host mirror's control loop (libnas_host.so) driving the GPU engine:
Schedule / findNodesThatFit / prioritize / findBestNode / Bind / Event
(scheduler.go:189-394) against an in-memory cluster, checked against the
oracle's literal vote loop on the metrics the mirror ingested, and the
network-aware batch path (nas_place) against the oracle's sequential greedy.
"""
import numpy as np
import pytest

import oracle
from hostfix import exporter_body, iperf_report
from kubernetesnetawarescheduler_amd import Engine
from kubernetesnetawarescheduler_amd import hostlib as H

pytestmark = pytest.mark.gpu

NAMES = ["ubuntu", "raspiworker0", "raspiworker1", "raspiworker2", "raspiworker3"]
URLS = ["http://192.168.1.137:9100/metrics", "http://192.168.1.132:9100/metrics",
        "http://192.168.1.135:9100/metrics", "http://192.168.1.133:9100/metrics",
        "http://192.168.1.134:9100/metrics"]


def reference_cluster(rng, order=None):
    bodies, files, snap = {}, {}, {k: [] for k in ("cpu", "mem", "rx", "tx", "bw", "disk")}
    freqs = [6e8, 1.2e9, 1.5e9, 1.8e9]
    for name, url in zip(NAMES, URLS):
        body = exporter_body(name, rng.choice(freqs, 4), 9.26e8 if name != "ubuntu" else 8.26e9,
                             float(rng.integers(1e8, 9e8)), int(rng.integers(0, 2e6)),
                             int(rng.integers(0, 2e6)), int(rng.integers(0, 4)))
        bodies[url] = body
        cpu, mem, rx, tx, disk = H.node_metrics(body, name)
        bw = 0.0
        if name != "ubuntu":
            b = float(rng.uniform(8e7, 9.5e7))
            path = f"/home/{name}.json"
            files[path] = iperf_report(b)
            bw = b
        for k, v in zip(("cpu", "mem", "rx", "tx", "bw", "disk"), (cpu, mem, rx, tx, bw, disk)):
            snap[k].append(v)
    return H.FakeCluster(nodes=NAMES, bodies=bodies, files=files, order=order), snap


def test_reference_topology_panics_at_raspiworker3():
    """As shipped, getNetworkBandwith("raspiworker3") opens "" (no entry in
    the map of :505-510) and Streams[0] panics: the Go process would crash on
    its first pod.  The mirror reports the same panic and drops the pod."""
    rng = np.random.default_rng(0)
    cl, _ = reference_cluster(rng)
    cl.files = {"/home/192.168.1.133.json": iperf_report(9e7),
                "/home/192.168.1.134.json": iperf_report(9.1e7),
                "/home/192.168.1.135.json": iperf_report(9.2e7)}
    with Engine(0) as e:
        s = H.HostScheduler(e, cl)
        assert s.enqueue("default", "p0", uid="u0")
        kind, pod, node, msg = s.schedule_one()
    assert kind == "PANICKED" and "index out of range [0] with length 0" in msg
    assert cl.bindings == []


@pytest.mark.parametrize("seed", range(6))
def test_schedule_one_matches_oracle_vote(seed):
    rng = np.random.default_rng(seed)
    o1 = rng.permutation(5)
    o2 = rng.permutation(6)
    cl, snap = reference_cluster(rng, order=lambda n: (o1, o2))
    with Engine(0) as e:
        s = H.HostScheduler(e, cl)
        for name in NAMES[1:]:
            s.set_iperf_path(name, f"/home/{name}.json")
        assert s.enqueue("default", "p0", uid="u0")
        assert not s.enqueue("default", "bound", node_name="raspiworker1")  # :173 filter
        assert not s.enqueue("default", "other", scheduler_name="default-scheduler")
        kind, pod, node, msg = s.schedule_one()
    best, _, _ = oracle.vote(snap, o1, o2)
    want = "none" if best == -2 else "" if best == -1 else NAMES[best]
    assert pod == "default/p0" and node == want
    assert kind == "BOUND" and cl.bindings == [("default", "p0", want)]
    assert cl.events[0][3] == f"Assigned pod p0 to {want}\n"


def test_schedule_batch_each_pod_its_own_map_order():
    rng = np.random.default_rng(42)
    orders = [(rng.permutation(5), rng.permutation(6)) for _ in range(12)]
    it = iter(orders)
    cl, snap = reference_cluster(rng, order=lambda n: next(it))
    with Engine(0) as e:
        s = H.HostScheduler(e, cl)
        for name in NAMES[1:]:
            s.set_iperf_path(name, f"/home/{name}.json")
        for i in range(12):
            s.enqueue("ns", f"p{i}", uid=f"u{i}")
        out = s.schedule_batch(12)
    assert len(out) == 12
    for (kind, pod, node, _), (o1, o2) in zip(out, orders):
        best, _, _ = oracle.vote(snap, o1, o2)
        assert node == ("none" if best == -2 else NAMES[best]) and kind == "BOUND"


def test_list_and_bind_errors_drop_the_pod():
    rng = np.random.default_rng(3)
    cl, _ = reference_cluster(rng)
    with Engine(0) as e:
        s = H.HostScheduler(e, cl)
        for name in NAMES[1:]:
            s.set_iperf_path(name, f"/home/{name}.json")
        s.enqueue("ns", "a")
        s.enqueue("ns", "b")
        cl.list_error = "connection refused"
        assert s.schedule_one()[0] == "LIST_ERROR"
        cl.list_error, cl.bind_error = None, "node not found"
        kind, _, _, msg = s.schedule_one()
        assert (kind, msg) == ("BIND_ERROR", "node not found")
        assert s.schedule_one()[0] == "NO_POD"
    assert cl.events == []


def test_place_pending_matches_oracle():
    """Network-aware path: pods with requests and peers, pairwise latency from
    iperf reports, capacities from the cluster; placements and binds equal the
    oracle's sequential greedy on the same WA / L / capacity."""
    rng = np.random.default_rng(7)
    n, P = 40, 150
    nodes = [f"node{i}" for i in range(n)]
    bps = rng.uniform(8e7, 2e9, (n, n))
    reports = [[None if i == j else iperf_report(bps[i, j]) for j in range(n)] for i in range(n)]
    L = H.latency_matrix(reports)
    cap = {nd: (int(rng.integers(500, 2000)), int(rng.integers(400_000, 2_000_000)), 3)
           for nd in nodes}
    bound = {f"ns/srv{i}": nodes[int(rng.integers(0, n))] for i in range(30)}
    cl = H.FakeCluster(nodes=nodes, capacity=cap, bound=dict(bound))
    pods = []
    for p in range(P):
        peers = [(f"ns/srv{int(rng.integers(0, 30))}", int(rng.integers(1, 400)))
                 for _ in range(int(rng.integers(0, 5)))]
        peers.append((f"ns/pending{p}", 9))  # an unbound peer is skipped
        pods.append((f"p{p}", int(rng.integers(1, 540)), int(rng.integers(7_464, 303_749)), peers))
    with Engine(0) as e:
        s = H.HostScheduler(e, cl)
        s.set_latency(nodes, L)
        for name, c, m, peers in pods:
            s.enqueue("ns", name, cpu_milli=c, mem_kib=m, peers=peers)
        out = s.place_pending()
    WA = np.zeros((P, n), np.int32)
    for p, (_, _, _, peers) in enumerate(pods):
        for q, w in peers:
            if q in bound:
                WA[p, nodes.index(bound[q])] += w
    assert WA.max() > 127  # aggregates beyond int8: exact int32 traffic, never saturated
    free = np.array([cap[nd] for nd in nodes], np.int32)
    req = np.array([[c, m, 1] for _, c, m, _ in pods], np.int32)
    want, _, _ = oracle.place(WA, L, req, free, "i8")
    assert len(out) == P
    for (kind, pod, node, _), w in zip(out, want):
        if w < 0:
            assert kind == "UNSCHEDULABLE" and node == ""
        else:
            assert kind == "BOUND" and node == nodes[w]
    assert (want < 0).any() and (want >= 0).any()


def test_place_pending_f32_measured_latency():
    """The fp32 path end to end: iperf reports -> unquantised microseconds per
    MB (nas_host_latency_matrix_us) -> NAS_DT_F32 placement of the queued pods;
    equal to the fp64 sequential oracle on the same float L / traffic."""
    rng = np.random.default_rng(11)
    n, P = 48, 200
    nodes = [f"node{i}" for i in range(n)]
    bps = rng.uniform(8e7, 2e9, (n, n))
    reports = [[None if i == j else iperf_report(bps[i, j]) for j in range(n)] for i in range(n)]
    L = H.latency_matrix(reports, us=True)
    assert L.dtype == np.float32
    cap = {nd: (int(rng.integers(500, 2000)), int(rng.integers(400_000, 2_000_000)), 3)
           for nd in nodes}
    bound = {f"ns/srv{i}": nodes[int(rng.integers(0, n))] for i in range(40)}
    cl = H.FakeCluster(nodes=nodes, capacity=cap, bound=dict(bound))
    pods = []
    for p in range(P):
        peers = [(f"ns/srv{int(rng.integers(0, 40))}", int(rng.integers(1, 400)))
                 for _ in range(int(rng.integers(1, 6)))]
        pods.append((f"p{p}", int(rng.integers(1, 540)), int(rng.integers(7_464, 303_749)), peers))
    with Engine(0) as e:
        s = H.HostScheduler(e, cl)
        s.set_latency(nodes, L)  # float32: the fp32 path
        for name, c, m, peers in pods:
            s.enqueue("ns", name, cpu_milli=c, mem_kib=m, peers=peers)
        out = s.place_pending()
    WA = np.zeros((P, n), np.float64)
    for p, (_, _, _, peers) in enumerate(pods):
        for q, w in peers:
            WA[p, nodes.index(bound[q])] += w
    free = np.array([cap[nd] for nd in nodes], np.int32)
    req = np.array([[c, m, 1] for _, c, m, _ in pods], np.int32)
    want, _, _ = oracle.place(WA.astype(np.float32), L, req, free, "f32")
    got = [nodes.index(node) if kind == "BOUND" else -1 for kind, _, node, _ in out]
    assert got == want.tolist()
    assert (want < 0).any() and (want >= 0).any()
