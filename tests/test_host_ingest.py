"""Host mirror ingest (libnas_host.so, kubernetesnetawarescheduler_amd/host/):
Go strconv / encoding/json / slicing semantics of scheduler.go:396-555 and
the pairwise latency matrix.  CPU only.

Parity is unpinned by the reference's own tests (it has none, and Go is absent
here): expected values are derived by hand from Go's published strconv and
encoding/json behaviour and from the reference's statements, cited per case.
"""
import json
import math

import numpy as np
import pytest

from hostfix import exporter_body, go_g, iperf_report
from kubernetesnetawarescheduler_amd import hostlib as H

f32 = lambda x: float(np.float32(x))  # noqa: E731


# ------------------------------------------------- strconv.ParseFloat(s, 32)
@pytest.mark.parametrize("s,value,err", [
    ("1.2e+09", 1.2e9, 0),
    ("6e+08", 6e8, 0),
    ("0.1", f32(0.1), 0),                 # float32-rounded, widened to float64
    ("1_000", 1000.0, 0),                 # Go float literal syntax allows '_' between digits
    ("1__0", 0.0, 1), ("_1", 0.0, 1), ("1_", 0.0, 1), ("1_.5", 0.0, 1),
    ("0x1p-2", 0.25, 0), ("0X1.8P1", 3.0, 0), ("0x_1p0", 1.0, 0), ("0x1_p0", 0.0, 1),
    ("0x1.8", 0.0, 1),                    # hexadecimal mantissa needs a 'p' exponent
    ("0x", 0.0, 1), ("0xp1", 0.0, 1),
    ("inf", math.inf, 0), ("+Inf", math.inf, 0), ("-infinity", -math.inf, 0),
    ("infin", 0.0, 1), ("+nan", 0.0, 1), ("infinityx", 0.0, 1),
    ("1e39", math.inf, 2), ("-1e39", -math.inf, 2),   # overflow: +-Inf with ErrRange
    ("3.4028235e38", f32(3.4028235e38), 0), ("3.4028236e38", math.inf, 2),
    ("1e-50", 0.0, 0),                    # underflow is not an error
    ("1.4e-45", f32(1.4e-45), 0),         # smallest denormal
    ("", 0.0, 1), (" 1", 0.0, 1), ("1 ", 0.0, 1), ("1.", 1.0, 0), (".5", 0.5, 0), (".", 0.0, 1),
    ("1e", 0.0, 1), ("1e+", 0.0, 1), ("e5", 0.0, 1), ("1e1_0", 1e10, 0), ("--1", 0.0, 1),
    ("1.2.3", 0.0, 1), ("0.000000001e9", 1.0, 0),
    ("1.5\nnode_cpu_scaling_frequency_hertz{cpu=\"4\"} 6e+08", 0.0, 1),
])
def test_parse_float32(s, value, err):
    v, e = H.parse_float(s, 32)
    assert e == err
    assert v == value or (math.isnan(v) and math.isnan(value))


def test_parse_float_nan_and_bits64():
    v, e = H.parse_float("NaN", 32)
    assert e == 0 and math.isnan(v)
    assert H.parse_float("0.1", 64) == (0.1, 0)
    assert H.parse_float("1e39", 64) == (1e39, 0)
    assert H.parse_float("1e309", 64) == (math.inf, 2)


def test_parse_float32_random_decimals():
    """Short decimal strings against numpy's float32 rounding (the double
    rounding through float64 cannot bite at <= 9 significant digits here)."""
    rng = np.random.default_rng(5)
    for _ in range(3000):
        m = int(rng.integers(1, 10 ** int(rng.integers(1, 9))))
        e = int(rng.integers(-30, 30))
        s = f"{m}e{e}"
        v, err = H.parse_float(s, 32)
        assert err == 0 and v == float(np.float32(float(s))), s


# ----------------------------------------------------------- strconv.Atoi
@pytest.mark.parametrize("s,value,err", [
    ("123", 123, 0), ("+5", 5, 0), ("-0", 0, 0), ("007", 7, 0),
    ("1_000", 0, 1),        # base 10 given: no underscores
    ("1.234567e+06", 0, 1),  # how node-exporter prints counters >= 1e6
    ("", 0, 1), ("+", 0, 1), (" 1", 0, 1), ("12a", 0, 1), ("0x10", 0, 1),
    ("9223372036854775807", 9223372036854775807, 0),
    ("-9223372036854775808", -9223372036854775808, 0),
    ("9223372036854775808", 9223372036854775807, 2),
    ("-9223372036854775809", -9223372036854775808, 2),
    ("99999999999999999999x", 9223372036854775807, 2),  # ParseUint stops at the overflow
    ("123456789012345678", 123456789012345678, 0),       # 18 chars: Atoi's fast path
])
def test_atoi(s, value, err):
    assert H.atoi(s) == (value, err)


# ------------------------------------------------------- node metric getters
def test_node_metrics_raspi():
    body = exporter_body("raspiworker0", [6e8, 1.2e9, 1.5e9, 6e8], 926_000_000, 500_000_000,
                         rx=123_456, tx=999_999, disk=3)
    cpu, mem, rx, tx, disk = H.node_metrics(body, "raspiworker0")
    assert cpu == (f32(6e8) + f32(1.2e9) + f32(1.5e9) + f32(6e8)) / 4           # :441
    assert mem == 100 - ((f32(5e8) * 100) / f32(9.26e8))                          # :460
    assert (rx, tx, disk) == (123_456, 999_999, 3)


def test_node_metrics_quirks():
    # counters >= 1e6 print as 1.234567e+06: Atoi fails, the getters return 0
    # (:474-479, :493-499); an 8-core node makes the 4th cpu substring span
    # cpu 3..7 and fail to parse, so cpu3 := cpu2 (:436-439)
    body = exporter_body("ubuntu", [1e9, 1.1e9, 1.3e9, 2e9, 2e9, 2e9, 2e9, 2e9], 8.26e9, 4.1e9,
                         rx=1_234_567, tx=2_000_000, disk=0, extra_disks=[("sda1", 4)])
    cpu, mem, rx, tx, disk = H.node_metrics(body, "ubuntu")
    assert go_g(1_234_567) == "1.234567e+06"
    assert cpu == (f32(1e9) + f32(1.1e9) + f32(1.3e9) + f32(1.3e9)) / 4
    assert (rx, tx) == (0, 0)
    assert disk == 0  # "0\nnode_disk_io_now{device=\"sda1\"} 4" does not Atoi
    assert mem == 100 - ((f32(4.1e9) * 100) / f32(8.26e9))


def test_node_metrics_zero_total_memory():
    body = exporter_body("raspiworker1", [1e9] * 4, 0, 0, 1, 2, 3)
    _, mem, _, _, _ = H.node_metrics(body, "raspiworker1")
    assert math.isnan(mem)  # 100 - (0*100)/0 in float64


def test_node_metrics_wrong_interface_name():
    # a raspi body read with the master's names: the enp3s0f1 markers are
    # missing, Index = -1, low = 54 > high -> Go panics
    body = exporter_body("raspiworker2", [1e9] * 4, 1e9, 5e8, 1, 2, 3)
    with pytest.raises(H.GoPanicError, match="slice bounds out of range"):
        H.node_metrics(body, "ubuntu")


def test_node_metrics_missing_marker_panics():
    body = exporter_body("raspiworker2", [1e9] * 4, 1e9, 5e8, 1, 2, 3)
    with pytest.raises(H.GoPanicError, match=r"\[:-2\]"):
        H.node_metrics(body.replace("max_hrts", "max_hertz"), "raspiworker2")  # node-exporter >= 0.18.1
    with pytest.raises(H.GoPanicError):
        H.node_metrics("", "raspiworker2")


# ----------------------------------------------------- json.Unmarshal(Iperf)
def test_iperf_report():
    assert H.iperf_receiver(iperf_report(9.4e7, 9.5e7)) == (9.4e7, 9.5e7, 1, True)


def _end(streams_json):
    return '{"end": {"streams": %s}}' % streams_json


@pytest.mark.parametrize("doc,receiver,n,valid", [
    ("", 0.0, 0, False),                                      # empty file (failed os.Open)
    ("{", 0.0, 0, False),
    ('{"end": {"streams": [{"receiver": {"bits_per_second": 1}}]},}', 0.0, 0, False),  # trailing comma
    ('{"title": "a\tb"}', 0.0, 0, False),                     # a raw control byte (0x09) in a string
    ('[1, 2]', 0.0, 0, True),                                  # not an object: type error, zero struct
    ("null", 0.0, 0, True),
    (_end('[]'), 0.0, 0, True),
    (_end('null'), 0.0, 0, True),
    (_end('{"receiver": {}}'), 0.0, 0, True),                  # wrong kind: skipped
    (_end('[{"receiver": {"bits_per_second": 5e7}}]'), 5e7, 1, True),
    (_end('[{"Receiver": {"Bits_Per_Second": 5e7}}]'), 5e7, 1, True),   # case-insensitive keys
    ('{"END": {"STREAMS": [{"RECEIVER": {"BITS_PER_SECOND": 7}}]}}', 7.0, 1, True),
    ('{"end": {"\\u017ftreams": [{"receiver": {"bit\\u017f_per_\\u017fecond": 8}}]}}', 8.0, 1, True),
    ('{"end": {"s\\u0074reams": [{"receiver": {"bits_per_second": 9}}]}}', 9.0, 1, True),  # escaped key
    (_end('[{"receiver": {"bits_per_second": "5e7"}}]'), 0.0, 1, True),  # string: type error
    (_end('[{"receiver": {"bits_per_second": 1e400}}]'), 0.0, 1, True),  # overflows float64
    (_end('[{"receiver": {"bits_per_second": 3, "bits_per_second": 4}}]'), 4.0, 1, True),  # last wins
    (_end('[{"receiver": {"bits_per_second": 3, "bits_per_second": null}}]'), 3.0, 1, True),
    (_end('[{"receiver": {"bits_per_second": 3}}, {"receiver": {"bits_per_second": 6}}]'), 3.0, 2, True),
    # a repeated "end" merges into the same struct; a repeated "streams" decodes
    # into the existing elements (merging), then truncates
    ('{"end": {"streams": [{"receiver": {"bits_per_second": 1}}, {}]},'
     ' "end": {"streams": [{"sender": {"bits_per_second": 2}}]}}', 1.0, 1, True),
    ('{"end": {"streams": [{"receiver": {"bits_per_second": 1}}]},'
     ' "end": {"streams": []}}', 0.0, 0, True),
    ('{"end": {"streams": [{"receiver": {"bits_per_second": 1}}]}, "end": null}', 1.0, 1, True),
    ('{"end": {"streams": [{"receiver": {"bits_per_second": 1}}]}, "end": {"streams": null}}',
     0.0, 0, True),
    ('{"end": {"streams": [{"receiver": {"bits_per_second": -0.0}}]}} ', 0.0, 1, True),
    ('\n {"end": {"streams": [{"receiver": {"bits_per_second": 12}}]}}\r\n', 12.0, 1, True),
    ('{"end": {"streams": [{"receiver": {"bits_per_second": 01}}]}}', 0.0, 0, False),  # leading zero
    ('{"end": {"streams": [{"receiver": {"bits_per_second": .5}}]}}', 0.0, 0, False),
    ('{"end": {"streams": [{"receiver": {"bits_per_second": 5}}]}}{}', 0.0, 0, False),  # two values
    ('{"t": "\\x"}', 0.0, 0, False),                          # bad escape
    ('{"t": "\xff\xfe"}', 0.0, 0, True),                      # invalid UTF-8 is accepted
    ('{"t": "\\ud800"}', 0.0, 0, True),                       # lone surrogate is accepted
])
def test_iperf_go_decoding(doc, receiver, n, valid):
    r, _, ns, ok = H.iperf_receiver(doc.encode("latin-1") if "\xff" in doc else doc)
    assert (ok, ns) == (valid, n)
    assert r == receiver


def test_iperf_nesting_depth():
    ok_doc = "[" * 10000 + "]" * 10000
    bad_doc = "[" * 10001 + "]" * 10001
    assert H.iperf_receiver(ok_doc)[3] is True
    assert H.iperf_receiver(bad_doc)[3] is False


def test_iperf_stale_elements_within_capacity():
    """Truncation keeps the slice's backing array: a later, longer "streams"
    decodes into the stale tail elements (Go's reflect.Value.SetLen)."""
    doc = ('{"end": {"streams": [{"receiver": {"bits_per_second": 1}}, '
           '{"receiver": {"bits_per_second": 2}}]}, '
           '"end": {"streams": [{"sender": {"bits_per_second": 3}}]}, '
           '"end": {"streams": [{}, {}]}}')
    r, s, n, ok = H.iperf_receiver(doc)
    assert (r, s, n, ok) == (1.0, 3.0, 2, True)


# ------------------------------------------------------- pairwise latency
@pytest.mark.parametrize("bps,ms", [(9.4e7, 86), (1e8, 80), (1e9, 8), (1e10, 1), (8e9, 1),
                                    (1e6, 127), (0.0, 127), (-5.0, 127), (float("nan"), 127),
                                    (float("inf"), 1)])
def test_latency_from_bps(bps, ms):
    assert H.latency_from_bps(bps) == ms


def test_latency_matrix_pairs():
    n = 4
    rng = np.random.default_rng(1)
    bps = rng.uniform(5e7, 2e9, (n, n))
    reports = [[None if i == j else iperf_report(bps[i, j]) for j in range(n)] for i in range(n)]
    reports[0][3] = "{broken"      # invalid report: 127 in that direction
    reports[2][1] = None           # missing
    L = H.latency_matrix(reports)
    want = np.zeros((n, n), np.int64)
    d = np.ceil(8e9 / bps).clip(1, 127)
    d[0, 3] = d[2, 1] = 127
    for i in range(n):
        for j in range(n):
            if i != j:
                want[i, j] = max(d[i, j], d[j, i])
    assert (L == want).all() and (L == L.T).all() and (np.diag(L) == 0).all()


@pytest.mark.parametrize("bps,us", [(1e8, 80000.0), (8e9, 1000.0), (1e12, 8.0),
                                    (0.0, 1e7), (-1.0, 1e7), (float("nan"), 1e7),
                                    (float("inf"), 0.0), (1.0, 1e7)])
def test_latency_us_from_bps(bps, us):
    assert H.latency_us_from_bps(bps) == np.float32(us)


def test_latency_matrix_us_unquantised():
    """The fp32 path keeps the measurement: 8e12 / bps microseconds per MB as
    float, the slower direction, 1e7 us for unusable pairs."""
    n = 5
    rng = np.random.default_rng(2)
    bps = rng.uniform(5e7, 2e9, (n, n))
    reports = [[None if i == j else iperf_report(bps[i, j]) for j in range(n)] for i in range(n)]
    reports[1][4] = "{broken"
    L = H.latency_matrix(reports, us=True)
    d = (8e12 / bps).astype(np.float32)
    d[1, 4] = 1e7
    want = np.maximum(d, d.T)
    np.fill_diagonal(want, 0)
    assert L.dtype == np.float32 and (L == want).all()
    assert len(np.unique(L[L > 0])) > n  # not quantised to a few levels


def test_host_abi_symbols():
    """Every symbol include/nas_host.h declares is exported and bound."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "nas_host.h")).read()
    declared = set(re.findall(r"\b(nas_host_\w+)\s*\(", hdr))
    assert declared == set(H.SIGNATURES), declared ^ set(H.SIGNATURES)
    L = H.hostlib()
    for name in declared:
        assert hasattr(L, name)
    json.dumps(sorted(declared))


# ------------------------------------------- snapshot refresh (batch ingest)
def test_snapshot_from_bodies_equals_per_node_and_thread_count_free():
    """nas_host_snapshot_from_bodies: every node equal to nas_host_node_metrics
    on its own (a panicking node reports NAS_HOST_PANIC and zeros), for 1, 3
    and 16 worker threads."""
    rng = np.random.default_rng(3)
    names, bodies = [], []
    for i in range(700):
        name = "ubuntu" if i % 97 == 0 else f"raspiworker{i}"
        body = exporter_body(name, rng.choice([6e8, 1.2e9, 1.5e9, 1.8e9], 4),
                             float(rng.integers(5e8, 9e9)), float(rng.integers(1e8, 5e8)),
                             int(rng.integers(0, 3e6)), int(rng.integers(0, 3e6)),
                             int(rng.integers(0, 9)))
        if i % 113 == 5:
            body = body.replace("node_disk_io_now", "node_disk_io_later")  # marker missing: panic
        names.append(name)
        bodies.append(body)
    want = []
    for b, n in zip(bodies, names):
        try:
            want.append((0,) + H.node_metrics(b, n))
        except H.GoPanicError:
            want.append((H.NAS_HOST_PANIC, 0.0, 0.0, 0, 0, 0))
    assert any(w[0] == H.NAS_HOST_PANIC for w in want)
    for threads in (1, 3, 16):
        got = H.snapshot_from_bodies(bodies, names, threads)
        for i, w in enumerate(want):
            g = (int(got["status"][i]), got["cpu"][i], got["mem"][i], int(got["rx"][i]),
                 int(got["tx"][i]), int(got["disk"][i]))
            assert g == w, (threads, i)
