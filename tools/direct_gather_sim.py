"""Cache lines per 64-row chunk of k_direct on the nonSU2 N26 sector, by
gather kind: spin-up hops stay in the chunk's block, spin-down hops and the
nonSU2 spin-flip hybridisation (ed_model.hpp gen_row, stored/Himp_bath.f90:
253-310) reach other blocks.  400 random full chunks, 128-B lines.

    python tools/direct_gather_sim.py > profiles/r4/direct_n26s_gather_sim.txt
"""
import numpy as np, itertools, math, random
NS=13; N=13
# rank tables per up popcount class: rank[c][pattern]
from math import comb
ranks={}
pats_by_c={c:[] for c in range(NS+1)}
for p in range(1<<NS):
    pats_by_c[bin(p).count('1')].append(p)
rank=np.zeros(1<<NS,dtype=np.int64)
for c,l in pats_by_c.items():
    for i,p in enumerate(l): rank[p]=i
# block offsets: blocks idw in increasing order; block idw holds up patterns of popcount N - pc(idw)
off={}
o=0
for idw in range(1<<NS):
    nu=N-bin(idw).count('1')
    if 0<=nu<=NS:
        off[idw]=o; o+=comb(NS,nu)
print("dim",o)
def row(idw,up): return off[idw]+rank[up]
random.seed(1)
imp=0; baths=range(1,NS)
tot={'up':0,'dn':0,'flip':0}; cnt={'up':0,'dn':0,'flip':0}
blocks=[b for b in off if comb(NS,N-bin(b).count('1'))>=64]
for _ in range(400):
    idw=random.choice(blocks)
    nu=N-bin(idw).count('1')
    ups=pats_by_c[nu]
    s=random.randrange(0,len(ups)-63)
    chunk=ups[s:s+64]
    for k in baths:
        # up hop imp<->bath k (spin up): target (idw, up^(1|1<<k)) if bits differ
        t=[row(idw,u^(1|1<<k)) for u in chunk if ((u>>0)&1)!=((u>>k)&1)]
        if t: tot['up']+=len({x*8//128 for x in t}); cnt['up']+=1
        # dn hop: target (idw^(1|1<<k), up) if dn bits differ -> whole chunk if fires (uniform)
        if ((idw>>0)&1)!=((idw>>k)&1):
            t=[row(idw^(1|1<<k),u) for u in chunk]
            tot['dn']+=len({x*8//128 for x in t}); cnt['dn']+=1
        # flips: imp up <-> bath dn k ; imp dn <-> bath up k
        t=[]
        for u in chunk:
            if (u&1) and not (idw>>k)&1: t.append(row(idw|(1<<k), u&~1))
            elif not (u&1) and (idw>>k)&1: t.append(row(idw&~(1<<k), u|1))
        if t: tot['flip']+=len({x*8//128 for x in t}); cnt['flip']+=1
        t=[]
        for u in chunk:
            if (idw&1) and not (u>>k)&1: t.append(row(idw&~1, u|(1<<k)))
            elif not (idw&1) and (u>>k)&1: t.append(row(idw|1, u&~(1<<k)))
        if t: tot['flip']+=len({x*8//128 for x in t}); cnt['flip']+=1
for k in tot: print(k, "ops per chunk", round(cnt[k]/400,2), "lines per op", round(tot[k]/max(cnt[k],1),1), "lines per chunk", round(tot[k]/400,1))

# ---- block order: an LRU model of each XCD's 4 MiB L2 at block granularity
# (k_direct sweeps the blocks of its eighth of the chunks in idw order; a
# block's gathers touch itself, its 12 spin-down and 13 spin-flip neighbours)
import collections  # noqa: E402

size = {idw: comb(NS, N - bin(idw).count('1')) * 8 if 0 <= N - bin(idw).count('1') <= NS else 0
        for idw in range(1 << NS)}
vbytes = sum(size.values())
masks = [1 << k for k in range(NS)] + [1 | (1 << k) for k in range(1, NS)]


def l2_fetch(order, cap=4 << 20, nx=8):
    fetched = 0
    for p in np.array_split(np.array(order), nx):
        c, used = collections.OrderedDict(), 0
        for b in p:
            for r in [int(b)] + [int(b) ^ m for m in masks]:
                if r in c:
                    c.move_to_end(r)
                else:
                    fetched += size[r]
                    c[r] = 1
                    used += size[r]
                    while used > cap:
                        k, _ = c.popitem(last=False)
                        used -= size[k]
    return fetched


ident = list(range(1 << NS))
gray = [i ^ (i >> 1) for i in range(1 << NS)]
shuf = ident[:]
random.shuffle(shuf)
print(f"block-order L2 model (v = {vbytes / 1e6:.1f} MB):")
for name, o in (("idw order (k_direct)", ident), ("Gray-code sequence", gray), ("random", shuf)):
    f = l2_fetch(o)
    print(f"  {name:22s} {f / 1e9:.3f} GB fetched = {f / vbytes:.2f} reads of v")
