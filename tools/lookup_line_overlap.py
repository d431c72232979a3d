#!/usr/bin/env python3
"""Fraction of each bench-step lookup's 128-B pyramid lines (w8 tiles layout: 2x4 / 2x4 / 1x4 / 1x2 target
chunks, 8 / 8 / 16 / 32 query slots per line) that the previous lookup read (CPU only; bench.synthetic
cfg2 coords).  usage: python tools/lookup_line_overlap.py"""
import sys, numpy as np, torch
import os; _R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, _R); sys.path.insert(0, os.path.join(_R, 'raft-meets-dicl_amd'))
import bench
from rmd import ops
H,W,B,R=55,128,8,4
f1,f2,co=bench.synthetic(B,8,H,W,12,1234,'cpu')
co=co.numpy()
slot=ops.tiles_slots(H,W).numpy()   # pixel -> slot
LV=[(55,128,2,4,16),(27,64,2,4,16),(13,32,1,4,8),(6,16,1,2,4)]
def lines(c):
    keys=[]
    for l,(lh,lw,th,tw,cb) in enumerate(LV):
        spl=128//cb
        x=c[:,0].reshape(B,-1)/2**l; y=c[:,1].reshape(B,-1)/2**l
        x0=np.floor(x).astype(np.int64)-R; y0=np.floor(y).astype(np.int64)-R
        sl=np.broadcast_to(slot[None],(B,H*W))//spl
        bb=np.broadcast_to(np.arange(B)[:,None],(B,H*W))
        for j in range(2*R+2):
            yy=y0+j
            for k in range(2*R+2):
                xx=x0+k
                ok=(yy>=0)&(yy<lh)&(xx>=0)&(xx<lw)
                ty=yy[ok]//th; tx=xx[ok]//tw
                key=(((l*B+bb[ok])*64+ty)*64+tx)*100000+sl[ok]
                keys.append(np.unique(key))
    return np.unique(np.concatenate(keys))
S=[lines(co[i]) for i in range(12)]
U=S[0]
for i in range(12):
    prev = np.intersect1d(S[i],S[i-1]).size/S[i].size if i else 0
    anyp = np.intersect1d(S[i],U).size/S[i].size if i else 0
    print(i, S[i].size*128/1e6, "MB", "overlap prev %.3f"%prev, "any earlier %.3f"%anyp)
    U=np.union1d(U,S[i])
print("union MB", U.size*128/1e6)
