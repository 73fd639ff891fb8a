"""Model configurations used by the parity tests (small enough for the oracle).

Each case: (name, EDConfig factory, list of sectors (q1, q2)).  Together they
exercise every term of ED_HAMILTONIAN/stored/*.f90: impurity hops, nonSU2
spin-flip impHloc, Jx/Jp, replica bath hops, superconducting pairs,
hybridisation, spin-flip hybridisation; normal/hybrid/replica baths.
"""
import numpy as np

from edgpu.params import EDConfig, init_dmft_bath, make_config, random_bath


def _hloc(Nspin, Norb, seed, cplx=False, offdiag=True, spinflip=False):
    rng = np.random.default_rng(seed)
    h = np.zeros((Nspin, Nspin, Norb, Norb), dtype=np.complex128)
    for s in range(Nspin):
        a = rng.normal(size=(Norb, Norb))
        if cplx:
            a = a + 1j * rng.normal(size=(Norb, Norb))
        a = 0.5 * (a + a.conj().T)
        if not offdiag:
            a = np.diag(np.diag(a))
        h[s, s] = 0.3 * a
    if spinflip and Nspin == 2:
        b = 0.1 * (rng.normal(size=(Norb, Norb)) + (1j * rng.normal(size=(Norb, Norb)) if cplx else 0))
        h[0, 1] = b
        h[1, 0] = b.conj().T
    return h


def c2():      # configs[1]: Norb=1 Nbath=7 flat bath, half filling (4,4)
    return make_config(Norb=1, Nbath=7)


def c5():      # configs[4]: nonSU2 Norb=1 Nbath=6
    return make_config(Norb=1, Nbath=6, Nspin=2, ed_mode="nonsu2")


def normal_rand():
    cfg = make_config(Norb=2, Nbath=3, Nspin=2, Uloc=(2.0, 1.5, 0.0), Ust=1.0, Jh=0.3,
                      xmu=0.2, bath="random", seed=7)
    cfg.impHloc = _hloc(2, 2, 1)
    return cfg


def normal_jh():   # spin exchange + pair hopping (Jhflag)
    cfg = make_config(Norb=2, Nbath=2, Nspin=1, Uloc=(2.0, 2.0, 0.0), Ust=1.2, Jh=0.4,
                      Jx=0.4, Jp=0.3, bath="random", seed=3)
    cfg.impHloc = _hloc(1, 2, 2)
    return cfg


def normal_3orb():
    cfg = make_config(Norb=3, Nbath=1, Nspin=2, Uloc=(2.0, 1.8, 1.6), Ust=1.1, Jh=0.25,
                      Jx=0.25, Jp=0.25, hfmode=False, xmu=0.3, bath="random", seed=11)
    cfg.impHloc = _hloc(2, 3, 4)
    return cfg


def hybrid():
    cfg = make_config(Norb=2, Nbath=4, Nspin=1, bath_type="hybrid", Uloc=(2.0, 2.0, 0.0),
                      Ust=1.0, Jh=0.2, bath="random", seed=5)
    cfg.impHloc = _hloc(1, 2, 6)
    return cfg


def replica_cplx():
    cfg = EDConfig(Norb=2, Nbath=2, Nspin=1, bath_type="replica", Uloc=(2.0, 1.0, 0.0),
                   Ust=0.8, Jh=0.2)
    cfg.impHloc = _hloc(1, 2, 8, cplx=True)
    b = init_dmft_bath(cfg)
    rng = np.random.default_rng(9)
    for k in range(cfg.Nbath):
        a = rng.normal(size=(2, 2)) + 1j * rng.normal(size=(2, 2))
        b.h[0, 0, :, :, k] = 0.5 * (a + a.conj().T)
        b.vr[k] = 0.4 + 0.1 * (k + 1)   # real, as init_dmft_bath sets it (dmft_aux.f90:144)
    cfg.bath = b
    return cfg


def replica_cplx_vr():
    """Complex replica hybridisation vr: the reference conjugates it in BOTH
    hopping directions (stored/Himp_bath.f90:20 and :32), so its stored H is
    complex-symmetric in that block, not Hermitian (and directMatVec_cc uses the
    unconjugated value).  Parity target = the stored semantics."""
    cfg = replica_cplx()
    for k in range(cfg.Nbath):
        cfg.bath.vr[k] = 0.4 + 0.1j * (k + 1)
    return cfg


def nonsu2_rand():
    cfg = make_config(Norb=2, Nbath=2, Nspin=2, ed_mode="nonsu2", Uloc=(2.0, 1.0, 0.0),
                      Ust=0.7, Jh=0.1, Jx=0.1, Jp=0.1, bath="random", seed=13)
    cfg.impHloc = _hloc(2, 2, 10, cplx=True, spinflip=True)
    return cfg


def nonsu2_replica():
    cfg = EDConfig(Norb=1, Nbath=3, Nspin=2, ed_mode="nonsu2", bath_type="replica")
    cfg.impHloc = _hloc(2, 1, 12, cplx=True, spinflip=True)
    b = init_dmft_bath(cfg)
    rng = np.random.default_rng(14)
    for k in range(cfg.Nbath):
        a = rng.normal(size=(2, 2)) + 1j * rng.normal(size=(2, 2))
        a = 0.5 * (a + a.conj().T)
        b.h[:, :, 0, 0, k] = a
        b.vr[k] = 0.3 + 0.05 * k
    cfg.bath = b
    return cfg


def _soc(lam, Norb=3):
    """lam * L.S in the Lz basis iorb -> m = Lzdiag = (-1, +1, 0) (ED_VARS_GLOBAL.f90:207):
    h[s, s', a, b] multiplies c+_{a s} c_{b s'}; conserves twoJz = 2Lz + 2Sz."""
    m = (-1, 1, 0)
    io = {mm: i for i, mm in enumerate(m)}
    h = np.zeros((2, 2, Norb, Norb), dtype=np.complex128)
    for a in range(Norb):
        h[0, 0, a, a] += 0.5 * lam * m[a]
        h[1, 1, a, a] -= 0.5 * lam * m[a]
    for mm in (-1, 0):                      # L+ S- /2 : c+_{m+1,dn} c_{m,up}
        a, b = io[mm + 1], io[mm]
        h[1, 0, a, b] += 0.5 * lam * np.sqrt(2.0)
        h[0, 1, b, a] += 0.5 * lam * np.sqrt(2.0)
    return h


def nonsu2_jz():
    """Jz_basis sectors (n, twoJz): t2g (Norb=3) replica bath, spin-orbit
    coupling in the Lz basis on the impurity and in every bath replica."""
    cfg = EDConfig(Norb=3, Nbath=1, Nspin=2, ed_mode="nonsu2", bath_type="replica",
                   Uloc=(2.0, 2.0, 2.0), Ust=1.2, Jh=0.4, xmu=1.0, Jz_basis=True)
    cfg.impHloc = _soc(0.35)
    for s in range(2):
        for a in range(3):
            cfg.impHloc[s, s, a, a] += (-0.1, 0.15, 0.05)[a]
    b = init_dmft_bath(cfg)
    for k in range(cfg.Nbath):
        b.h[..., k] = _soc(0.2 + 0.1 * k)
        for s in range(2):
            for a in range(3):
                b.h[s, s, a, a, k] += 0.3 - 0.2 * a + 0.5 * k
        b.vr[k] = 0.45 + 0.1 * k
    cfg.bath = b
    return cfg


def superc():
    cfg = make_config(Norb=1, Nbath=4, Nspin=1, ed_mode="superc", deltasc=0.15, bath="random",
                      seed=17)
    return cfg


def superc_2orb():
    cfg = make_config(Norb=2, Nbath=2, Nspin=1, ed_mode="superc", Uloc=(2.0, 2.0, 0.0), Ust=1.0,
                      Jh=0.3, Jx=0.3, Jp=0.3, deltasc=0.1, bath="random", seed=19)
    cfg.impHloc = _hloc(1, 2, 20)
    return cfg


CASES = [
    ("c2", c2, [(4, 4), (3, 5), (0, 8)]),
    ("c5", c5, [(7, 0), (6, 0)]),
    ("normal_rand", normal_rand, [(4, 4), (3, 5), (2, 1)]),
    ("normal_jh", normal_jh, [(3, 3), (2, 4)]),
    ("normal_3orb", normal_3orb, [(3, 3), (2, 4)]),
    ("hybrid", hybrid, [(3, 3), (4, 2)]),
    ("replica_cplx", replica_cplx, [(3, 3), (2, 4)]),
    ("nonsu2_rand", nonsu2_rand, [(6, 0), (5, 0)]),
    ("nonsu2_replica", nonsu2_replica, [(4, 0), (3, 0)]),
    ("nonsu2_jz", nonsu2_jz, [(6, 0), (6, 2), (5, 1), (7, -3)]),
    ("superc", superc, [(0, 0), (1, 0), (-2, 0)]),
    ("superc_2orb", superc_2orb, [(0, 0), (1, 0)]),
]
