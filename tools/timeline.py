"""Timeline of one nas_place step from a rocprofv3 --kernel-trace CSV:
per-kernel busy time, first/last timestamps of the last step, and the gaps.
usage: python tools/timeline.py TRACE_DIR"""
import csv
import re
import glob
import sys


def _short(name):
    m = re.search(r"(k_[a-z0-9_]+?)(E|I|\(|<|$)", name)
    return m.group(1) if m else name[:24]


def main(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                  _short(r["Kernel_Name"])) for r in rows))
    # steps begin at the first k_fit after a gap > 200 us
    starts = [i for i, k in enumerate(ks) if k[2] == "k_fit" and (i == 0 or k[0] - ks[i - 1][1] > 200_000)]
    last = ks[starts[-2]:starts[-1]] if len(starts) > 1 else ks
    t0 = last[0][0]
    busy = {}
    for s, e, n in last:
        busy.setdefault(n, [0, 0, 1e18, 0])
        b = busy[n]
        b[0] += e - s; b[1] += 1; b[2] = min(b[2], s - t0); b[3] = max(b[3], e - t0)
    print(f"step span {(last[-1][1] - t0) / 1e3:.1f} us, {len(last)} kernels")
    for n, (tot, c, f, l) in sorted(busy.items(), key=lambda x: -x[1][0]):
        print(f"{n:24s} calls {c:4d} busy {tot / 1e3:9.1f} us  first {f / 1e3:8.1f}  last-end {l / 1e3:8.1f}")
    print("commit launches (start, end) us:")
    for s, e, n in last:
        if n == "k_commit":
            print(f"  {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  ({(e - s) / 1e3:.1f})")


if __name__ == "__main__":
    main(sys.argv[1])
