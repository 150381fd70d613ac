"""One line per run of a tools/ab_lib.sh output directory (A_i.json / B_i.json):
pass ms, full-launch ms and roofline frac, fit launch, rescore rounds --
the text committed under profiles/ for a same-box A/B.
usage: python tools/ab_summary.py OUTDIR [label A] [label B]"""
import glob
import json
import os
import sys


def main(d, *labels):
    for f in sorted(glob.glob(os.path.join(d, "[A-F]_*.json"))):
        try:
            p = json.load(open(f))
        except (ValueError, OSError):
            print(os.path.basename(f), "unreadable")
            continue
        k = os.path.basename(f)[0]
        tag = labels["ABCDEF".index(k)] if "ABCDEF".index(k) < len(labels) else k
        rf = p.get("roofline", {})
        fr = p.get("fit_roofline", {})
        cf = p.get("configs", {})
        extra = " ".join(f"{k}={v['ms_per_step']:.3f}ms" + (f"/frac {v['roofline']['frac']:.4f}" if 'roofline' in v else "")
                         for k, v in cf.items())
        print(f"{os.path.basename(f):10s} {tag:28s} pass {p.get('ms_per_step', float('nan')):.3f} ms"
              f"  launch {rf.get('launch_ms', float('nan')):.3f} ms frac {rf.get('frac', float('nan')):.4f}"
              f"  fit {fr.get('launch_ms', float('nan')) * 1e3:.1f} us"
              f"  rescores {p.get('rescore_rounds')}  {extra}")


if __name__ == "__main__":
    main(*sys.argv[1:])
