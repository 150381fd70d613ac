"""ASan + UBSan build of the repo's CPU code ("an ASan/UBSan CPU
build of oracle/ and host/").

tests/sanitize/san_driver.cpp links the host mirror's parsing code
(host/go_semantics.cpp, go_json.cpp, ingest.cpp, latency.cpp -- everything
in libnas_host.so that does not call the GPU library) and the whole oracle
(oracle/oracle.c, gomap.cpp), all compiled with
-fsanitize=address,undefined -fno-sanitize-recover=all, and drives them over
the fixture node-exporter body and iperf3 report, every prefix and thousands
of byte mutations of both, and random small oracle workloads with internal
cross-checks.  Any sanitizer report makes the run exit nonzero.  (The HIP
kernels cannot run under a sanitizer: GPU ASan is not available on the
pool.)
"""
import os
import shutil
import subprocess

import pytest

from hostfix import exporter_body, iperf_report

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "kubernetesnetawarescheduler_amd", "host")
ORACLE = os.path.join(ROOT, "oracle")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None,
                    reason="needs gcc/g++")
def test_asan_ubsan_host_and_oracle(tmp_path):
    objs = []
    for src in ["go_semantics.cpp", "go_json.cpp", "ingest.cpp", "latency.cpp"]:
        o = tmp_path / (src + ".o")
        subprocess.run(["g++", "-std=c++17", *SAN, "-I", HOST, "-c", os.path.join(HOST, src),
                        "-o", str(o)], check=True)
        objs.append(str(o))
    o = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-std=c11", "-fopenmp", "-fno-fast-math", *SAN, "-c",
                    os.path.join(ORACLE, "oracle.c"), "-o", str(o)], check=True)
    objs.append(str(o))
    o = tmp_path / "gomap.o"
    subprocess.run(["g++", "-std=c++17", "-fno-fast-math", *SAN, "-c",
                    os.path.join(ORACLE, "gomap.cpp"), "-o", str(o)], check=True)
    objs.append(str(o))
    exe = tmp_path / "san_driver"
    subprocess.run(["g++", "-std=c++17", *SAN, "-fopenmp", "-I", HOST,
                    os.path.join(ROOT, "tests", "sanitize", "san_driver.cpp"), *objs, "-o", str(exe)],
                   check=True)
    body = tmp_path / "metrics.txt"
    body.write_text(exporter_body("raspiworker0", [6e8, 1.2e9, 1.5e9, 6e8], 926_000_000,
                                  500_000_000, rx=123_456, tx=999_999, disk=3))
    rep = tmp_path / "iperf.json"
    rep.write_text(iperf_report(9.4e7))
    env = dict(os.environ, OMP_NUM_THREADS="2",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe), str(body), "raspiworker0", str(rep)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "SAN OK" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
