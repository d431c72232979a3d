#!/usr/bin/env python3
"""Per lookup position of the bench step (CPU only): the fraction of the 128-B pyramid lines (w8 tiles layout)
that the previous lookup did not read, and the fraction of lookup waves (64 slots x level x row part,
corr_lookup.hip grid) that touch at least one such line, for the bench, reverse and shift coordinate
orders of tools/lookup_context.py.  usage: python tools/lookup_wave_miss.py"""
import sys, os, numpy as np
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, _R); sys.path.insert(0, os.path.join(_R, 'raft-meets-dicl_amd'))
import bench
from rmd import ops
H,W,B,R=55,128,8,4
_,_,co=bench.synthetic(B,8,H,W,12,1234,'cpu'); co=co.numpy()
slot=ops.tiles_slots(H,W).numpy()
LV=[(55,128,2,4,16),(27,64,2,4,16),(13,32,1,4,8),(6,16,1,2,4)]
PR=3
def touch(c):
    """returns dict level-> (keys array, wave ids array) per touched line per lane-part"""
    out=[]
    for l,(lh,lw,th,tw,cb) in enumerate(LV):
        spl=128//cb
        x=c[:,0].reshape(B,-1)/2**l; y=c[:,1].reshape(B,-1)/2**l
        x0=np.floor(x).astype(np.int64)-R; y0=np.floor(y).astype(np.int64)-R
        sl=np.broadcast_to(slot[None],(B,H*W))
        bb=np.broadcast_to(np.arange(B)[:,None],(B,H*W))
        for part in range(3):
            bb0=min(part*PR, 2*R+1-PR)
            for jj in range(PR+1):
                yy=y0+bb0+jj
                for k in range(2*R+2):
                    xx=x0+k
                    ok=(yy>=0)&(yy<lh)&(xx>=0)&(xx<lw)
                    ty=yy[ok]//th; tx=xx[ok]//tw
                    key=(((l*B+bb[ok])*64+ty)*64+tx)*100000+sl[ok]//spl
                    wave=((l*3+part)*B+bb[ok])*1000+sl[ok]//64
                    out.append((key,wave))
    k=np.concatenate([a for a,_ in out]); w=np.concatenate([b for _,b in out])
    return k,w
def stats(seq):
    prev=None; res=[]
    for c in seq:
        k,w=touch(c)
        if prev is None: res.append((1.0,1.0)); prev=np.unique(k); continue
        new=~np.isin(k,prev)
        uk=np.unique(k)
        frac_lines=1-np.isin(uk,prev).mean()
        waves=np.unique(w); wm=np.unique(w[new])
        res.append((round(frac_lines,4), round(wm.size/waves.size,3)))
        prev=uk
    return res
print("bench", stats([co[i] for i in range(12)]))
print("rev", stats([co[11-i] for i in range(12)]))
print("shift", stats([co[0]+0.02*i for i in range(12)]))
