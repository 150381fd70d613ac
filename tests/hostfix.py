"""Fixtures for the host-mirror tests (the generators live in the package, so
bench.py's host leg uses the same ones)."""
from kubernetesnetawarescheduler_amd.exporter_text import exporter_body, go_g, iperf_report  # noqa: F401
