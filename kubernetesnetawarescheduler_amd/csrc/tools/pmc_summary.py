"""Summarise rocprofv3 --pmc CSVs (per kernel dispatch, counters summed over
dimensions) from the directories given on the command line."""
import collections
import csv
import glob
import sys

agg = collections.OrderedDict()
for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0][-40:], int(r["Dispatch_Id"]))
            agg.setdefault(k, collections.OrderedDict())
            agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for (name, disp), cs in agg.items():
    if "fillBuffer" in name or "copyBuffer" in name:
        continue
    print(name, disp)
    for c, v in cs.items():
        print(f"    {c:32s} {v:.6g}")
