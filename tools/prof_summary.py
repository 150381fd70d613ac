"""Summarise tools/prof_bench.sh output into one JSON (the file committed as
profiles/rNN_*_prof_summary.json):

  stats     per-kernel calls / average / share from the kernel-trace stats of
            the bench command (trace_bench) and of the placement leg
            (trace_place);
  roofline  tools/check_roofline.py's comparison (bench HIP-event launch
            time vs rocprof mean of the same dispatches);
  pmc       per kernel, the LARGEST dispatch of the scoring leg (--only
            score: the full-size k_fit / k_cost_topk / k_merge launches):
            HBM bytes = FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md
            HBM/rocprofv3 section; FETCH_SIZE is in KB) + WRITE_SIZE (KB), and
            from the SQ group: MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
            (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), wait / active shares of
            SQ_WAVE_CYCLES, LDS instructions, effective clock = GRBM_GUI_ACTIVE
            / 8 / the trace's mean duration of that kernel at that grid.

usage: python tools/prof_summary.py OUTDIR"""
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    head = name.replace("(anonymous namespace)", "anon").split("(")[0]
    return head.split("<")[0].replace("void ", "").split("::")[-1]


def per_dispatch(d):
    """{(dispatch id, short kernel, grid): {counter: summed value}}"""
    per = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        key = (int(r["Dispatch_Id"]), short(r["Kernel_Name"]), int(r.get("Grid_Size", 0) or 0),
               r["Kernel_Name"])
        c = per.setdefault(key, {})
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def main(d):
    res = {"stats": {}, "roofline": None, "pmc": {}}
    for leg in ("bench", "place"):
        st = rows(f"{d}/trace_{leg}/**/*kernel_stats.csv")
        res["stats"][leg] = {short(r["Name"]): {"calls": int(r["Calls"]),
                                                "avg_ms": float(r["AverageNs"]) / 1e6,
                                                "pct": float(r["Percentage"])} for r in st}
    cr = os.path.join(d, "check_roofline.json")
    if os.path.exists(cr):
        with open(cr) as f:
            res["roofline"] = json.load(f)
    # mean kernel durations of the headline grid in the bench trace (for the clock)
    dur = {}
    for r in rows(f"{d}/trace_bench/**/*kernel_trace.csv"):
        # (full name: the int8 and bf16 instantiations share a grid at C3)
        k = (r["Kernel_Name"],
             int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r.get("Grid_Size_Z", 1) or 1))
        dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    merged = {}
    for sub in ("pmc1", "pmc2", "pmc3"):
        for (disp, kern, grid, full), c in per_dispatch(os.path.join(d, sub)).items():
            if kern not in ("k_cost_topk", "k_fit", "k_merge"):
                continue
            # the largest dispatch per kernel: by the counter that scales with work
            score = c.get("GRBM_GUI_ACTIVE", 0) + c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)
            m = merged.setdefault(kern, {})
            if score >= m.get(sub + "_score", -1):
                m[sub + "_score"] = score
                m[sub] = c
                if sub == "pmc1":
                    m["grid"] = (full, grid)
    for kern, m in merged.items():
        out = {}
        sq = m.get("pmc1", {})
        if sq.get("SQ_WAVE_CYCLES"):
            w = sq["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in sq:
                    out[k + "_frac"] = sq[k] / w
        if sq.get("GRBM_GUI_ACTIVE"):
            gui = sq["GRBM_GUI_ACTIVE"] / 8.0
            out["GRBM_GUI_ACTIVE_per_xcd"] = gui
            out["mfma_busy_frac"] = sq.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui * 1024)
            out["SQ_INSTS_LDS"] = sq.get("SQ_INSTS_LDS")
            # the bench trace's dispatches of the same kernel at the same grid
            # as the profiled one (the largest grid overall is C4's or C5's)
            big = dur.get(m.get("grid", ("", -1)))
            if big:
                mean_s = sum(big) / len(big)
                # GRBM_GUI_ACTIVE counts the whole counter window of the
                # dispatch (set-up and drain included), so for a short kernel
                # it overstates the clock (k_fit, 34 us: "3.08 GHz" on a
                # 2.4 GHz part in round 2): only quoted from 100 us up
                if mean_s >= 100e-6:
                    out["effective_clock_ghz"] = gui / mean_s / 1e9
                else:
                    out["effective_clock_ghz"] = None
                    out["effective_clock_note"] = (
                        f"kernel {mean_s * 1e6:.1f} us: GRBM_GUI_ACTIVE spans the counter window "
                        "beyond the kernel, not a clock measurement below 100 us")
        fetch = m.get("pmc2", {}).get("FETCH_SIZE")
        write = m.get("pmc3", {}).get("WRITE_SIZE")
        if fetch is not None:
            out["FETCH_SIZE_kb"] = fetch
            out["fetch_bytes"] = fetch * 1024 * 2
        if write is not None:
            out["WRITE_SIZE_kb"] = write
            out["write_bytes"] = write * 1024
        if fetch is not None and write is not None:
            out["hbm_bytes"] = out["fetch_bytes"] + out["write_bytes"]
        res["pmc"][kern] = out
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
