"""Kernel timeline of the last nas_place pass in a rocprofv3 --kernel-trace
directory: start / end / duration (us, from the pass's first launch) and HW
queue of every kernel, to see the pipeline (scoring streams, commit stream).
usage: python tools/pass_timeline.py TRACE_DIR"""
import csv,glob,re,sys
rows=[]
for f in glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True):
    rows+=list(csv.DictReader(open(f)))
ks=sorted((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),re.search(r"(k_[a-z0-9_]+|__amd_[a-zA-Z_]+|ncclDevKernel[a-zA-Z_0-9]*)",r["Kernel_Name"]).group(1),r["Queue_Id"],r["Grid_Size_X"]) for r in rows)
pi=[i for i,k in enumerate(ks) if k[2]=="k_pass_init"]
i=pi[-1]
# with the LDS commit the first chunks' scoring launches precede the init
while i>0 and ks[i-1][2] in ("k_cost_topk","k_fit") and ks[i][0]-ks[i-1][0]<2_000_000:
    i-=1
start=ks[i][0]
sel=[k for k in ks if k[0]>=start]
base=start
for s,e,n,q,g in sel:
    print(f"{(s-base)/1e3:9.1f} {(e-base)/1e3:9.1f} {(e-s)/1e3:7.1f} q{q} {n} {g}")
