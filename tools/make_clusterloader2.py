"""Extract the (Cpu cores, Mem bytes) rows of the reference's clusterloader2
resource summaries (datasets/clusterloader2/{90,110,130}containers/*.json:
percentile blocks "100"/"50"/"90"/"99" x 17 control-plane containers) into
kubernetesnetawarescheduler_amd/data/clusterloader2_requests.json -- data
only, the empirical pod-request distribution of BASELINE config C2 (SURVEY.md
§8(d)).  Run once where /root/reference exists; the output is committed.

  python tools/make_clusterloader2.py
"""
import glob
import json
import os

REF = "/root/reference/datasets/clusterloader2"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "kubernetesnetawarescheduler_amd", "data", "clusterloader2_requests.json")


def main():
    rows = []
    for f in sorted(glob.glob(f"{REF}/*/*.json")):
        run, name = f.split("/")[-2], os.path.basename(f)
        with open(f) as fh:
            d = json.load(fh)
        for pct in sorted(d):
            for r in d[pct]:
                rows.append({"run": run, "file": name, "percentile": pct,
                             "container": r["Name"], "cpu_cores": r["Cpu"], "mem_bytes": r["Mem"]})
    with open(OUT, "w") as fh:
        json.dump({"source": "pablojara/kubernetesNetAwareScheduler datasets/clusterloader2/*/*.json",
                   "rows": rows}, fh, indent=0)
    print(f"wrote {len(rows)} rows to {OUT}")


if __name__ == "__main__":
    main()
