"""Locality bound of the one-pass stored H·v on the Nlevels=28 (7,7) sector.

Model of k_spmv_pk's down-spin gathers at the granularity of V rows (the
DimDw x DimUp view of v, one row = 3,432 doubles = 27 KB): a 64-row wave of
block iw reads its own row (up hops) and the 7 rows iw' of its down-spin
neighbours (impurity <-> bath hops).  Each XCD sweeps its part of the blocks
with an LRU L2 of W rows (4 MiB = ~150 rows); every miss is one V row fetched
from the Infinity Cache / HBM.  Printed: row fetches for the reference (rank)
order, reverse Cuthill-McKee, a greedy cache-aware order, a partition by three
bath bits, and the lower bound (distinct rows each XCD must touch at least
once).  One fetch per row per XCD is the best any one-pass order can do.

    python tools/l2_order_sim.py [--vbytes 8|16] > profiles/r4/stored_l2_order_sim_{real,complex}.txt

--vbytes 16: complex(8) vectors — a V row is 54 KB, the 4 MiB L2 holds ~75.
"""
import argparse
import collections

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import reverse_cuthill_mckee

NS, N = 14, 7                     # levels per spin, particles (Norb=1, Nbath=13, half filling)
pats = [p for p in range(1 << NS) if bin(p).count("1") == N]   # build_sector rank order
idx = {p: i for i, p in enumerate(pats)}
NB = len(pats)
nbr = [[idx[p ^ 1 ^ (1 << k)] for k in range(1, NS) if (p & 1) != ((p >> k) & 1)] for p in pats]


def fetches(parts, W):
    tot = 0
    for part in parts:
        cache = collections.OrderedDict()
        for b in part:
            for r in [b] + nbr[b]:
                if r in cache:
                    cache.move_to_end(r)
                else:
                    tot += 1
                    cache[r] = 1
                    if len(cache) > W:
                        cache.popitem(last=False)
    return tot


def greedy(part, W):
    rem, cache, out, cur = set(part), collections.OrderedDict(), [], part[0]
    while rem:
        if cur not in rem:
            cand = {q for r in list(cache)[-40:] for q in nbr[r] if q in rem} or set(list(rem)[:50])
            cur = max(cand, key=lambda q: sum(r in cache for r in [q] + nbr[q]))
        rem.discard(cur)
        out.append(cur)
        for r in [cur] + nbr[cur]:
            if r in cache:
                cache.move_to_end(r)
            else:
                cache[r] = 1
                if len(cache) > W:
                    cache.popitem(last=False)
        cur = -1
    return out


def distinct(parts):
    return sum(len({r for b in p for r in [b] + nbr[b]}) for p in parts)


ap = argparse.ArgumentParser()
ap.add_argument("--vbytes", type=int, default=8)
args = ap.parse_args()
ROWB = NB * args.vbytes               # bytes of one V row
W = (4 << 20) // ROWB                 # rows one XCD's L2 holds
ident = np.arange(NB)
A = csr_matrix((np.ones(7 * NB), ([i for i in range(NB) for _ in nbr[i]], [j for l in nbr for j in l])),
               shape=(NB, NB))
rcm = reverse_cuthill_mckee(A, symmetric_mode=True)
rank_parts = np.array_split(ident, 8)
cls = collections.defaultdict(list)
for i, p in enumerate(pats):
    cls[(p >> 11) & 7].append(i)
cls_parts = [cls[k] for k in range(8)]
print(f"V rows: {NB} (one row = {ROWB / 1024:.0f} KB, {args.vbytes}-B elements); L2 model: {W} rows per XCD; 8 XCDs")
fr = fetches(rank_parts, W)
print(f"rank order (k_spmv_pk):        {fr:6d} row fetches = {fr / NB:.2f} reads of v, "
      f"excess {(fr - NB) * ROWB / 1e9:.3f} GB")
print(f"reverse Cuthill-McKee:         {fetches(np.array_split(rcm, 8), W):6d}")
print(f"rank parts, greedy order:      {fetches([greedy(list(p), W) for p in rank_parts], W):6d}")
print(f"3-bath-bit parts, greedy:      {fetches([greedy(p, W) for p in cls_parts], W):6d}")
print(f"lower bound, rank parts:       {distinct(rank_parts):6d} (distinct rows per XCD, summed)")
print(f"lower bound, 3-bath-bit parts: {distinct(cls_parts):6d}")
print(f"own-bytes model (v read once): {NB:6d}")
