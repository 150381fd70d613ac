"""Where one nas_place pass spends its time, from a rocprofv3 --kernel-trace
directory: the pass's span, busy time (some kernel running) vs idle gaps,
and per kernel name the launches and summed duration.  The pass is picked
like tools/pass_timeline.py (PASS_FROM_END, default 4: bench.py's last timed
step).  usage: python tools/pass_breakdown.py TRACE_DIR [PASS_FROM_END]"""
import collections
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
             kname(r["Kernel_Name"]))
            for r in rows)


def pass_start(i):
    while i > 0 and ks[i - 1][2] in ("k_cost_topk", "k_fit") and ks[i][0] - ks[i - 1][0] < 2_000_000:
        i -= 1
    return i


starts = [pass_start(i) for i, k in enumerate(ks) if k[2] == "k_pass_init"]
back = min(int(sys.argv[2]) if len(sys.argv) > 2 else 4, len(starts))
a = starts[-back]
b = starts[-back + 1] if back > 1 else len(ks)
sel = ks[a:b]
t0, t1 = sel[0][0], max(e for _, e, _ in sel)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in sel:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"pass span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us, "
      f"{len(sel)} launches")
agg = collections.defaultdict(lambda: [0, 0])
for s, e, n in sel:
    agg[n][0] += 1
    agg[n][1] += e - s
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {n:24s} {c:5d} launches {d / 1e3:10.1f} us")
