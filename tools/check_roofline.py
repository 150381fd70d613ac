"""Reproduce bench.py's roofline numbers from a rocprofv3 kernel trace of the
same command (tools/prof_bench.sh runs `rocprofv3 --kernel-trace --stats --
python3 bench.py ...`).

For every roofline object in the bench JSON line (the headline, and the
C3_bf16 / C2_f32 / C5 configs), the launches it timed with HIP events are the
LAST `launches` dispatches of k_cost_topk with that dtype template and grid
(bench.py issues them after any placement pass of the same shape).  This
prints, per roofline, the bench's mean launch time, the rocprof mean of
those dispatches, their relative difference, and frac recomputed from the
rocprof duration.

usage: python tools/check_roofline.py BENCH_JSON TRACE_CSV [--nodes 10000 --pods 100000]
"""
import argparse
import csv
import json
import sys

BM = BN = 256
DT = {"i8": 1, "bf16": 2, "f32": 4}


def cdiv(a, b):
    return -(-a // b)


def grid_x(nodes, pods, batch=1):
    """grid x (threads) of a full launch: the wide tile (256 x 384, 768
    threads) for one cluster of >= 32,768 padded pods or any cluster batch,
    else 256 x 256 / 512 (nas_api.hip wide_ok)."""
    if batch > 1 or cdiv(pods, BN) * BN >= 32768:
        return cdiv(nodes, BM) * cdiv(cdiv(pods, BN) * BN, 384) * 768
    return cdiv(nodes, BM) * cdiv(pods, BN) * 512


def expected(name, cfg, nodes, pods):
    """(template dtype id, grid x threads, grid y) of the roofline's launch."""
    if name in ("headline", "C3_fullrange"):
        return DT["i8"], grid_x(nodes, pods), 1
    if name == "C3_bf16":
        return DT["bf16"], grid_x(nodes, pods), 1
    if name == "C2_f32":  # the fp32 split runs the bf16 kernel
        return DT["bf16"], grid_x(1000, 10000), 1
    if name == "C5":  # first launch of the wide + narrow pair (score_batch)
        return DT["i8"], cdiv(5000, BM) * (cdiv(5000, BN) * BN // 768 * 2) * 768, 64
    raise KeyError(name)


def c5_narrow_grid():
    """the narrow launch behind C5's wide one: 256 x 256 tiles over the pods
    past the last multiple of 768 (5,120 padded pods: 512 of them)"""
    pp = cdiv(5000, BN) * BN
    return cdiv(5000, BM) * ((pp - pp // 768 * 768) // BN) * 512


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench_json")
    ap.add_argument("trace_csv")
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--pods", type=int, default=100000)
    a = ap.parse_args()
    with open(a.bench_json) as f:
        line = [ln for ln in f.read().splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    with open(a.trace_csv) as f:
        rows = [r for r in csv.DictReader(f) if "k_cost_topk<" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    roofs = {"headline": out.get("roofline")}
    for k, v in out.get("configs", {}).items():
        if isinstance(v, dict) and "roofline" in v:
            roofs[k] = v["roofline"]
    res = {}
    for name, rf in roofs.items():
        if not rf or "launch_ms" not in rf:
            continue
        dt, gx, gy = expected(name, out.get("config", {}), a.nodes, a.pods)
        tag = f"k_cost_topk<{dt},"
        ds = [r for r in rows if tag in r["Kernel_Name"] and int(r["Grid_Size_X"]) == gx
              and int(r["Grid_Size_Y"]) == gy]
        n = int(rf.get("launches", 3))
        if len(ds) < n:
            res[name] = {"error": f"{len(ds)} matching dispatches, bench timed {n}"}
            continue
        sel = ds[-n:]
        if name == "headline" and "C3_fullrange" in roofs:
            # the full-range config's launches (same kernel and grid: one
            # untimed, then its timed ones) come after the headline's
            n_fr = int(roofs["C3_fullrange"].get("launches", 3)) + 1
            sel = ds[-n_fr - n:-n_fr]
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in sel]
        if name == "C5":  # the bench's span covers the wide launch and the narrow one behind it
            nx = [r for r in rows if tag in r["Kernel_Name"] and int(r["Grid_Size_X"]) == c5_narrow_grid()
                  and int(r["Grid_Size_Y"]) == gy]
            if len(nx) < n:
                res[name] = {"error": f"{len(nx)} narrow dispatches, bench timed {n}"}
                continue
            ms = [(int(b["End_Timestamp"]) - int(a["Start_Timestamp"])) * 1e-6
                  for a, b in zip(ds[-n:], nx[-n:])]
        prof = sum(ms) / n
        ops = rf.get("ops_per_launch")
        peak = rf["peak"]
        res[name] = {"bench_launch_ms": rf["launch_ms"], "rocprof_mean_ms": prof,
                     "rel_diff": (rf["launch_ms"] - prof) / prof, "dispatches": n,
                     "bench_frac": rf["frac"],
                     "rocprof_frac": ops / (prof * 1e-3) / 1e12 / peak if ops else None}
    json.dump(res, sys.stdout, indent=1)
    print()
    # 2% on full launches; sub-millisecond launches (C2_f32: 0.17 ms) jitter more
    bad = [k for k, v in res.items()
           if "error" in v or abs(v["rel_diff"]) > (0.02 if v["rocprof_mean_ms"] >= 1 else 0.05)]
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
