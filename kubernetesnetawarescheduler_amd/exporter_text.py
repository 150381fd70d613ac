"""Synthetic node-exporter /metrics text and iperf3 -J reports shaped like
the ones the reference parsed (scheduler.go:34-117, :396-549) -- input
generators for the host-ingest tests and bench.py's host leg.

Node-exporter 0.18.0 (the version whose cpufreq collector exported the
misspelt node_cpu_scaling_frequency_max_hrts the reference slices up to,
scheduler.go:420) prints samples with Go's strconv.FormatFloat(v, 'g', -1,
64): shortest digits, exponent form from 1e+06 up -- which is why large
packet counters reach strconv.Atoi as "1.234567e+06" and become 0.
"""
import json

import numpy as np


def go_g(v):
    """strconv.FormatFloat(v, 'g', -1, 64)."""
    v = float(v)
    if v == 0:
        return "0"
    if np.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if np.isnan(v):
        return "NaN"
    sign = "-" if v < 0 else ""
    r = repr(abs(v))  # shortest round-trip digits, like Go's
    mant, _, e = r.partition("e")
    exp10 = int(e) if e else 0
    ip, _, fp = mant.partition(".")
    digits = (ip + fp).lstrip("0")
    # decimal point position relative to the digit string
    if ip.strip("0"):
        dp = len(ip.lstrip("0")) + exp10
    else:
        dp = exp10 - (len(fp) - len(fp.lstrip("0")))
    digits = digits.rstrip("0") or "0"
    x = dp - 1
    eprec = 6  # shortest formatting decides %e vs %f with precision 6
    if x < -4 or x >= eprec:
        m = digits[0] + ("." + digits[1:] if len(digits) > 1 else "")
        return f"{sign}{m}e{'+' if x >= 0 else '-'}{abs(x):02d}"
    if dp <= 0:
        return f"{sign}0.{'0' * -dp}{digits}"
    if dp >= len(digits):
        return f"{sign}{digits}{'0' * (dp - len(digits))}"
    return f"{sign}{digits[:dp]}.{digits[dp:]}"


def exporter_body(node, freqs, mem_total, mem_avail, rx, tx, disk, extra_disks=()):
    """node-exporter 0.18.0 text (the parts the reference reads, in the
    exporter's sorted order).  `node` == "ubuntu" uses the master's names
    (enp3s0f1, sda/sr0), otherwise a Raspberry Pi's (eth0, mmcblk0)."""
    iface = "enp3s0f1" if node == "ubuntu" else "eth0"
    dev, nxt = ("sda", "sr0") if node == "ubuntu" else ("mmcblk0", "mmcblk0p1")
    L = ["# HELP node_boot_time_seconds Node boot time, in unixtime.",
         "# TYPE node_boot_time_seconds gauge", "node_boot_time_seconds 1.57e+09",
         "# HELP node_cpu_scaling_frequency_hertz Current scaled cpu thread frequency in hertz.",
         "# TYPE node_cpu_scaling_frequency_hertz gauge"]
    for i, f in enumerate(freqs):
        L.append(f'node_cpu_scaling_frequency_hertz{{cpu="{i}"}} {go_g(f)}')
    L += ["# HELP node_cpu_scaling_frequency_max_hrts Maximum scaled cpu thread frequency in hertz.",
          "# TYPE node_cpu_scaling_frequency_max_hrts gauge"]
    for i, f in enumerate(freqs):
        L.append(f'node_cpu_scaling_frequency_max_hrts{{cpu="{i}"}} 1.8e+09')
    L += ["# HELP node_disk_io_now The number of I/Os currently in progress.",
          "# TYPE node_disk_io_now gauge",
          f'node_disk_io_now{{device="{dev}"}} {go_g(disk)}']
    for d, v in extra_disks:
        L.append(f'node_disk_io_now{{device="{d}"}} {go_g(v)}')
    L += [f'node_disk_io_now{{device="{nxt}"}} 0',
          "# HELP node_memory_MemAvailable_bytes Memory information field MemAvailable_bytes.",
          "# TYPE node_memory_MemAvailable_bytes gauge",
          f"node_memory_MemAvailable_bytes {go_g(mem_avail)}",
          "# HELP node_memory_MemFree_bytes Memory information field MemFree_bytes.",
          "# TYPE node_memory_MemFree_bytes gauge", "node_memory_MemFree_bytes 1e+08",
          "# HELP node_memory_MemTotal_bytes Memory information field MemTotal_bytes.",
          "# TYPE node_memory_MemTotal_bytes gauge",
          f"node_memory_MemTotal_bytes {go_g(mem_total)}",
          "# HELP node_memory_Mlocked_bytes Memory information field Mlocked_bytes.",
          "# TYPE node_memory_Mlocked_bytes gauge", "node_memory_Mlocked_bytes 0",
          "# HELP node_network_receive_packets_total Network device statistic receive_packets.",
          "# TYPE node_network_receive_packets_total counter",
          'node_network_receive_packets_total{device="cni0"} 1234',
          f'node_network_receive_packets_total{{device="{iface}"}} {go_g(rx)}',
          'node_network_receive_packets_total{device="flannel.1"} 77',
          "# HELP node_network_transmit_packets_total Network device statistic transmit_packets.",
          "# TYPE node_network_transmit_packets_total counter",
          'node_network_transmit_packets_total{device="cni0"} 4321',
          f'node_network_transmit_packets_total{{device="{iface}"}} {go_g(tx)}',
          'node_network_transmit_packets_total{device="flannel.1"} 88', ""]
    return "\n".join(L)


def iperf_report(receiver_bps, sender_bps=None, host="192.168.1.133"):
    """An iperf3 -J report (the fields of scheduler.go:34-117 that matter)."""
    sender_bps = receiver_bps * 1.01 if sender_bps is None else sender_bps
    s = {"socket": 5, "start": 0, "end": 10.0, "seconds": 10.0, "bytes": int(receiver_bps * 10 / 8),
         "bits_per_second": sender_bps, "retransmits": 0, "snd_cwnd": 85336, "omitted": False}
    r = dict(s, bits_per_second=receiver_bps)
    r.pop("retransmits")
    return json.dumps({
        "start": {"connected": [{"socket": 5, "local_host": "10.244.1.5", "local_port": 41234,
                                 "remote_host": host, "remote_port": 5201}],
                  "version": "iperf 3.6", "system_info": "Linux",
                  "timestamp": {"time": "Mon, 01 Jul 2019 10:00:00 GMT", "timesecs": 1561975200},
                  "connecting_to": {"host": "iperf3-server", "port": 5201}, "cookie": "x",
                  "tcp_mss_default": 1448,
                  "test_start": {"protocol": "TCP", "num_streams": 1, "blksize": 131072, "omit": 0,
                                 "duration": 10, "bytes": 0, "blocks": 0, "reverse": 0}},
        "intervals": [{"streams": [s], "sum": s}],
        "end": {"streams": [{"sender": s, "receiver": r}], "sum_sent": s, "sum_received": r,
                "cpu_utilization_percent": {"host_total": 1.5, "host_user": 0.5,
                                            "host_system": 1.0, "remote_total": 2.0,
                                            "remote_user": 1.0, "remote_system": 1.0}},
        "title": "Client on 192.168.1.135"})
