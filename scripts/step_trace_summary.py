#!/usr/bin/env python3
"""Per-step summary of a rocprofv3 --marker-trace --kernel-trace run of the routed
step (scripts/trace_bench.sh): kernels and ROCTX phases between consecutive
`serve.plan` markers, plus the timeline of the last step.

usage: step_trace_summary.py TRACE_DIR [STEPS] [STEP_MARKER]
STEP_MARKER: the ROCTX range that starts a step (default serve.plan, the routed step;
hbm.lookup_coalesced for the one-GPU step)."""
import csv,sys,re
from collections import defaultdict
d=sys.argv[1]; nsteps=int(sys.argv[2]) if len(sys.argv)>2 else 10
marker=sys.argv[3] if len(sys.argv)>3 else 'serve.plan'
m=list(csv.DictReader(open(d+'/bench_marker_api_trace.csv')))
k=list(csv.DictReader(open(d+'/bench_kernel_trace.csv')))
def short(n):
    n=re.sub(r"\(anonymous namespace\)::","",n); n=re.sub(r"^void ","",n)
    mm=re.match(r"([\w:]+(<[^()]*?>)?)",n); b=mm.group(1) if mm else n
    if b.startswith("at::") or b.startswith("rocprim"): b=b.split("<")[0]
    return b.replace("shellac::","")[:60]
plans=sorted(int(r['Start_Timestamp']) for r in m if r['Function']==marker)
print(len(plans),'plan markers')
st=plans[-nsteps-1:]
ks=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp']),short(r['Kernel_Name']),
           r.get('Queue_Id',''),r.get('Stream_Id','')) for r in k)
tot=defaultdict(lambda:[0,0])
t0,t1=st[0],st[-1]
for s,e,n,_,_ in ks:
    if t0<=s<t1: tot[n][0]+=1; tot[n][1]+=e-s
busy=sum(v[1] for v in tot.values())
print(f"wall/step {(t1-t0)/1e3/nsteps:.1f} us, busy {busy/1e3/nsteps:.1f} us")
for n,(c,dd) in sorted(tot.items(),key=lambda x:-x[1][1])[:40]:
    print(f"{dd/1e3/nsteps:8.1f} us {c/nsteps:5.1f}x  {n}")
# phases
ph=defaultdict(int)
for r in m:
    s=int(r['Start_Timestamp']);e=int(r['End_Timestamp'])
    if t0<=s<t1: ph[r['Function']]+=e-s
for p,v in sorted(ph.items(),key=lambda x:-x[1]): print(f"{v/1e3/nsteps:8.1f} us host  {p}")
# timeline of last step
print("--- last step timeline")
a,b=st[-2],st[-1]
prev=a
for s,e,n,q,sid in ks:
    if a<=s<b:
        print(f"{(s-a)/1e3:8.1f} {(e-s)/1e3:7.1f} gap {(s-prev)/1e3:6.1f} q{q:>3} s{sid:>3} {n}"); prev=max(prev,e)
# STEP_TABLE=1: one line per step (wall, then the busiest kernels' time in that step)
import os
if os.environ.get("STEP_TABLE"):
    top=[n for n,_ in sorted(tot.items(),key=lambda x:-x[1][1])[:8]]
    print("--- per step (us): wall | "+" | ".join(top))
    for i in range(len(st)-1):
        a,b=st[i],st[i+1]; row=defaultdict(int)
        for s,e,n,_,_ in ks:
            if a<=s<b: row[n]+=e-s
        print(f"{(b-a)/1e3:7.1f} | "+" | ".join(f"{row[n]/1e3:6.1f}" for n in top))
# SPAN=n: every kernel of the last n steps on one GPU clock (origin: the first k_coalesce
# among them), with its queue: the cross-stream hand-offs and in-queue gaps of the chains
if os.environ.get("SPAN"):
    nspan=int(os.environ["SPAN"]); a=st[-nspan-1]; b=st[-1]
    sel=[x for x in ks if a<=x[0]<b]
    org=next((s for s,e,n,q,sid in sel if n.startswith("k_coalesce")),sel[0][0] if sel else 0)
    print(f"--- last {nspan} steps on the GPU clock (origin: first k_coalesce)")
    lastq={}
    for s,e,n,q,sid in sel:
        g=(s-lastq[q])/1e3 if q in lastq else float('nan')
        print(f"{(s-org)/1e3:8.1f} {(e-org)/1e3:8.1f} {(e-s)/1e3:7.1f} qgap {g:6.1f} q{q:>3} {n}")
        lastq[q]=max(lastq.get(q,0),e)
