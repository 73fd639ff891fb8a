"""Numpy restatement of the degeneracy-probe screen (probe_screen, ed_lib.hip)
on configs[3] sectors: steps until the screen decides "none below the cut"
with the tolerance test (theta converged to 1e-5) and with the residual-
interval test (theta - |beta_k s_k| > cut), and steps until a missed copy
(one vector of a degenerate pair left unlocked) is flagged below the cut.

    python tests/probe_rule_study.py
"""
import sys, os, numpy as np, scipy.sparse as sp, scipy.sparse.linalg as sla
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0]=[ROOT,os.path.join(ROOT,'dmft-ed_amd'),os.path.join(ROOT,'tests')]
from golden.golden_configs import c4_config
from oracle.oracle import Oracle
def H_of(cfg,q):
    o=Oracle(cfg); hm=o.build_sector(*q); rp,c,v=o.build_csr(hm)
    n=len(hm); return sp.csr_matrix((np.real(v),c,rp),shape=(n,n))
def screen(H, L, cut, tol=1e-5, maxs=400, seed=1):
    n=H.shape[0]; rng=np.random.default_rng(seed)
    v=rng.uniform(-1,1,n); v-=L@(L.T@v); v-=L@(L.T@v); v/=np.linalg.norm(v)
    V=[v]; al=[]; be=[]; res={}
    vp=np.zeros(n); b=0.0
    for k in range(maxs):
        w=H@v - b*vp
        a=v@w; w-=a*v
        w-=L@(L.T@w)
        Vm=np.array(V).T; w-=Vm@(Vm.T@w)
        b=np.linalg.norm(w); al.append(a); be.append(b)
        vp=v; v=w/b; V.append(v)
        if (k+1)%10==0:
            T=np.diag(al)+np.diag(be[:-1],1)+np.diag(be[:-1],-1)
            e,Z=np.linalg.eigh(T); th=e[0]; r=abs(be[-1]*Z[-1,0])
            if th<cut:
                res.setdefault('below',k+1); break
            if 'loose' not in res and th - r > cut: res['loose']=k+1
            if r <= tol*max(3.6e-11,abs(th)): res['strict']=k+1; break
    return res
for bath in ('random','flat'):
    cfg=c4_config(bath)
    for q in [(2,3),(3,4),(4,5),(3,3),(5,5),(4,4)]:
        H=H_of(cfg,q); n=H.shape[0]
        w,X=sla.eigsh(H,k=8,which='SA',tol=1e-12); o=np.argsort(w); w=w[o]; X=X[:,o]
        cut=w[5]-1e-9*max(1,abs(w[5]))
        r_full=screen(H,X[:,:6],cut)
        # drop one copy of the lowest degenerate pair if any
        deg=[i for i in range(5) if abs(w[i+1]-w[i])<1e-8]
        extra=''
        if deg:
            keep=[i for i in range(6) if i!=deg[0]+1]
            r_miss=screen(H,X[:,keep],cut)
            extra=f' miss-case {r_miss}'
        print(bath,q,n,'w6-w7 gap %.3g'%(w[6]-w[5]),r_full,extra,flush=True)
