"""Kernel timeline of the last nas_place pass in a rocprofv3 --kernel-trace
directory: start / end / duration (us, from the pass's k_pass_init) and HW
queue of every kernel, to see the pipeline (scoring streams, commit stream).
usage: python tools/pass_timeline.py TRACE_DIR"""
import csv,glob,re,sys
rows=[]
for f in glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True):
    rows+=list(csv.DictReader(open(f)))
ks=sorted((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),re.search(r"(k_[a-z0-9_]+|__amd_[a-zA-Z_]+|ncclDevKernel[a-zA-Z_0-9]*)",r["Kernel_Name"]).group(1),r["Queue_Id"],r["Grid_Size_X"]) for r in rows)
pi=[k for k in ks if k[2]=="k_pass_init"]
start=pi[-1][0]
sel=[k for k in ks if k[0]>=start]
base=start
for s,e,n,q,g in sel:
    print(f"{(s-base)/1e3:9.1f} {(e-base)/1e3:9.1f} {(e-s)/1e3:7.1f} q{q} {n} {g}")
