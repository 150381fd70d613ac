"""Kernel timeline of one nas_place pass in a rocprofv3 --kernel-trace
directory: start / end / duration (us, from the pass's first launch) and HW
queue of every kernel, to see the pipeline (scoring streams, commit stream).
By default the 4th pass from the end: bench.py's last timed step (its last
three steps run with stage timings on, whose extra timing events put ~10 us
gaps in front of the commits that the timed steps do not have).
usage: python tools/pass_timeline.py TRACE_DIR [PASS_FROM_END]"""
import csv
import glob
import re
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for f in glob.glob(sys.argv[1] + "/**/*.db", recursive=True):  # rocprofv3's default (rocpd) output
    import sqlite3
    con = sqlite3.connect(f)
    rows += [{"Start_Timestamp": a, "End_Timestamp": b, "Kernel_Name": n, "Queue_Id": q, "Grid_Size_X": g}
             for a, b, n, q, g in con.execute("select start, end, name, queue_id, grid_x from kernels")]
def kname(n):
    m = re.search(r"(k_[a-z0-9_]+|__amd_[a-zA-Z_]+|ncclDevKernel[a-zA-Z_0-9]*|Cijk_[A-Za-z0-9]+)", n)
    return m.group(1) if m else n[:24]


ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             kname(r["Kernel_Name"]),
             r["Queue_Id"], r["Grid_Size_X"]) for r in rows)


def pass_start(i):
    # with the LDS commit the first chunks' scoring launches precede the init
    while i > 0 and ks[i - 1][2] in ("k_cost_topk", "k_fit") and ks[i][0] - ks[i - 1][0] < 2_000_000:
        i -= 1
    return i


starts = [pass_start(i) for i, k in enumerate(ks) if k[2] == "k_pass_init"]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 4
back = min(back, len(starts))
a = starts[-back]
b = starts[-back + 1] if back > 1 else len(ks)
base = ks[a][0]
for s, e, n, q, g in ks[a:b]:
    print(f"{(s - base) / 1e3:9.1f} {(e - base) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{q} {n} {g}")
