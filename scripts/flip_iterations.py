"""Profiling aid: flip-loop iterations of the SMA kernel per 64 bars for walk windows of 64,
128 and 256 bars (a wave iterates the max over its 64 lanes of flips per window), from oracle
trade lists of config-2 symbols with the kernel's column-major lane mapping."""
import sys, numpy as np
sys.path.insert(0,'oracle'); sys.path.insert(0,'.')
import orc_ffi as F
fast=list(range(4,43,2)); slow=list(range(50,241,10)); nf=len(fast); ns=len(slow)
B=2520; P=nf*ns
rng=range(0,12)
it={64:[],128:[],256:[]}
for s in rng:
    c=F.gen(0x5EED,s,B,0)[3]
    flips=np.zeros((P,B),bool)
    for j in range(P):
        kf=j%nf; ks=j//nf
        r=F.sma(c,fast[kf],slow[ks],252,trades_cap=200)
        tr=r[1] if isinstance(r,tuple) else None
        for t in tr:
            flips[j,t['entry_bar']]=True; flips[j,t['exit_bar']]=True
    for T in it:
        nt=(B+T-1)//T
        pad=np.zeros((P,nt*T),bool); pad[:,:B]=flips
        cnt=pad.reshape(P,nt,T).sum(2)
        for w in range(0,P,64):
            it[T].append(cnt[w:w+64].max(0).sum())
    mean=flips.sum()/P
print("mean flips per lane", mean)
for T in it: print(T, "iterations per wave over series", np.mean(it[T]), "per 64 bars", np.mean(it[T])/ (B/64))
