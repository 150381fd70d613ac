"""Summarise rocprofv3 --pmc passes (one directory per run): per dispatch the
sum of each counter over its instances, then derived figures -- effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time, MI355X_MICROARCH.md DVFS note),
MFMA busy % (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * CUs * SIMDs...)
as fractions of the SQ wave cycles) and wait shares.
usage: python tools/pmc_table.py DIR [DIR ...]"""
import csv
import glob
import json
import os
import sys


def load(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (r["Dispatch_Id"], r["Kernel_Name"].split("(")[0][-60:])
                c = per.setdefault(key, {})
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def main(dirs):
    out = {}
    for d in dirs:
        for (disp, kern), c in sorted(load(d).items(), key=lambda x: int(x[0][0])):
            row = dict(c)
            if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
                w = c["SQ_WAVE_CYCLES"]
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    if k in c:
                        row[k + "_frac"] = c[k] / w
            if "GRBM_GUI_ACTIVE" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                # MFMA busy cycles summed over SIMDs vs GUI-active cycles x SIMDs (256 CU x 4)
                gui = c["GRBM_GUI_ACTIVE"] / 8.0
                row["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 1024)
            out.setdefault(os.path.basename(d.rstrip("/")), []).append({"dispatch": disp, "kernel": kern, **row})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
