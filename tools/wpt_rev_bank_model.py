#!/usr/bin/env python3
"""Bank-model estimate (MI355X_MICROARCH.md LDS table) of the ds_read_b128
conflicts of the config-4 WPT reverse tile (wpt_rev_tile1<16,256,4096,6>):
per level, the average extra LDS cycles per 16-lane group read.  The couples
sit at a 16-B lane stride, so only the lane groups that straddle a packet
window boundary conflict; deep levels (short windows) pay most."""
import sys
L=16; Q=L//2; T=4096; K=6; NT=256
PAD = '--pad' in sys.argv  # Wpt1RevGeo::stride(l, true)
def c(l):
    cc=0
    for k in range(l): cc=((cc//2+(Q-1))+1)&~1
    return cc
def ln(l): return (T>>l)+c(l)
def ncw(l): return (ln(l-1)//2+1)//2
def stride(l):
    if not PAD or l < 1 or l >= K: return ln(l)
    want=(ncw(l)+(ncw(l)&1))%16; st=ln(l)
    while st%16!=want: st+=2
    return st
G=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G=G+[[x+32 for x in g] for g in G]
tot_extra=0; tot=0
for l in range(K,0,-1):
    li=stride(l); lo=ln(l-1); NW=1<<(l-1); NPW=lo//2; NCW=(NPW+1)//2; NC=NW*NCW
    off=c(l)-c(l-1)//2; sh=(off-(Q-1))&1; NR=(Q+3)&~1
    R=(NC+NT-1)//NT
    ex=0; n=0
    for r in range(R):
        for w in range(NT//64):
            lanes=[]
            for lane in range(64):
                k=w*64+lane+r*NT
                if k>=NC: lanes.append(None); continue
                s=k//NCW; ml=2*(k%NCW)
                st=off+ml-(Q-1)-sh
                lanes.append((2*s)*li+st)   # doubles, a operand
            for j in range(0,NR,2):
                for base in (0,):  # a; d is +li (same pattern shift)
                    for g in G:
                        sl=[ (lanes[x]+j)//2 % 16 for x in g if lanes[x] is not None]
                        if not sl: continue
                        from collections import Counter
                        ways=max(Counter(sl).values())
                        ex+=ways-1; n+=1
    print('level',l,'li',li,'NCW',NCW,'R',R,'avg extra cycles per group-read',round(ex/max(n,1),3))
