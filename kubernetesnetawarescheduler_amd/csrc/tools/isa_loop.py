"""Main-loop census of a k_cost_topk instantiation in a device assembly dump
(hipcc --cuda-device-only -S k_cost.hip -o k.s): per MFMA-carrying loop,
its instruction counts (MFMA, scratch spills, LDS reads, global loads,
waits, VALU).  usage: python tools/isa_loop.py MANGLED_SUBSTRING k.s [k2.s]"""
import re,sys
def fn(path, key):
    s=open(path).read()
    for m in re.finditer(r'^(_Z\S*k_cost_topk\S*):', s, re.M):
        n=m.group(1)
        if key not in n: continue
        start=m.start(); end=s.index('.Lfunc_end', start)
        lines=s[start:end].split('\n')
        # split into blocks
        blocks=[]; cur=None
        for l in lines:
            mm=re.match(r'^(\.LBB\d+_\d+):\s*(;.*)?$', l)
            if mm:
                cur={'name':mm.group(1),'cmt':mm.group(2) or '','ins':[]}; blocks.append(cur); continue
            if cur is not None: cur['ins'].append(l)
        loops={}
        for b in blocks:
            h=None
            if 'Loop Header' in b['cmt']: h=b['name'][1:]
            mm=re.search(r'Header=(BB\d+_\d+)', b['cmt'])
            if mm: h=mm.group(1)
            if h: loops.setdefault(h,[]).append(b)
        for h,bs in loops.items():
            ins=[l for b in bs for l in b['ins']]
            c=lambda pat: sum(1 for l in ins if re.search(pat,l))
            if c('v_mfma')==0: continue
            print(path.split('/')[-1], n[-60:-30], h, 'lines',len(ins),'mfma',c('v_mfma'),'scratch',c('scratch_'),'ds_read',c('ds_read'),'gload',c('global_load'),'waitcnt',c('s_waitcnt'),'valu',c(r'^\s+v_(?!mfma)'))
for p in sys.argv[2:]: fn(p, sys.argv[1])
