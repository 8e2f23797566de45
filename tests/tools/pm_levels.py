"""Package-merge level statistics of a bench frame's four Huffman tables (test
infrastructure; CPU only): symbols per table, the unlimited Huffman depth, and the
first level from which package-merge's merged lists stop changing (None: they
change up to the limit).  The oracle gives the frame's quantised blocks.
  python tests/tools/pm_levels.py [frame]      (3840x2160 synthetic, 4:4:4, q90)
[length_limited.rs:37-134, symbol_counting.rs:55-94]"""
import heapq
import os
import sys

import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dmmt-jpeg-encoder_amd')]
import oracle
from oracle.synth import synthetic
import dmmt_jpeg
w,h=3840,2160
rgb=synthetic(w,h,frame=int(sys.argv[1]) if len(sys.argv)>1 else 0)
sub=0; q=90
luma,chroma=dmmt_jpeg.quality_tables(q)
co=oracle.forward(rgb,255,sub,luma,chroma,threads=8)  # zigzag blocks in emission order
co=co.reshape(-1,64).astype(np.int64)
nb=co.shape[0]; bpm=3; nl=1
comp=np.arange(nb)%bpm; tab=np.where(comp<nl,0,1)
# DC
dc=co[:,0]
def cat(v):
    a=np.abs(v); c=np.zeros_like(a)
    nz=a>0; c[nz]=np.floor(np.log2(a[nz])).astype(np.int64)+1
    return c
hist=[np.zeros(256,np.int64) for _ in range(4)]  # 0 lumaDC 1 lumaAC 2 chromaDC 3 chromaAC
for cidx in range(3):
    d=dc[comp==cidx]; diff=np.diff(np.concatenate([[0],d]))
    t=0 if cidx==0 else 2
    np.add.at(hist[t], cat(diff), 1)
ac=co[:,1:]; nzm=ac!=0
for t,sel in ((1,tab==0),(3,tab==1)):
    a=ac[sel]; m=nzm[sel]
    rows,cols=np.nonzero(m)
    # previous nonzero col per row
    prev=np.full(len(cols),-1); same=np.r_[False, rows[1:]==rows[:-1]]
    prev[same]=cols[:-1][same[1:]] if len(cols)>1 else prev[same]
    run=cols-prev-1
    zrl=run>>4
    sym=((run&15)<<4)|cat(a[rows,cols])
    np.add.at(hist[t], sym, 1)
    hist[t][0xF0]+=zrl.sum()
    last=np.full(m.shape[0],-1); last[rows]=cols  # rows ascending so last assignment wins
    hist[t][0]+=(last<62).sum()
def pm_levels(freqs,limit=15):
    import heapq
    leaves=[(f,0) for f in freqs]; levels=[leaves]
    for _ in range(1,limit):
        prev=levels[-1]
        pk=[(prev[2*i][0]+prev[2*i+1][0],1) for i in range(len(prev)//2)]
        levels.append(list(heapq.merge(pk,leaves)))
    return levels
for t in range(4):
    f=sorted([x for x in hist[t] if x>0])
    L=pm_levels(f)
    conv=None
    for k in range(1,len(L)):
        if L[k]==L[k-1]: conv=k; break
    # unconstrained huffman depth
    import heapq
    hp=[(x,0) for x in f]; heapq.heapify(hp)
    while len(hp)>1:
        a=heapq.heappop(hp); b=heapq.heappop(hp); heapq.heappush(hp,(a[0]+b[0],max(a[1],b[1])+1))
    print('table',t,'n',len(f),'min',f[0],'max',f[-1],'huffman depth',hp[0][1],'levels identical from',conv)
