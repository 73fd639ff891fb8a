"""Impurity Green's function by Lanczos continued fraction, normal mode.

Mirrors build_gf_normal / lanc_build_gf_normal_c / add_to_lanczos_gf_normal
(ED_GF_NORMAL.f90:18-92, 116-260, 580-632) for the diagonal components
G_{aa,ss}.  Per kept state |gs> (energy E_i), orbital a, spin s:

  * seed  c+_{a s}|gs>  in sector getCDGsector(s, isector)  and
          c_{a s}|gs>   in sector getCsector(s, isector),
    built on the GPU (ed_sector_apply_op, the vvinit loop :159-174);
  * norm2 = <seed|seed>, seed /= sqrt(norm2);
  * nlanc = min(jdim, lanc_nGFiter) steps of sp_lanc_tridiag on the GPU
    (device-resident plain Lanczos from a device start vector);
  * poles: eigenvalues and squared first eigenvector components of the
    tridiagonal (diag alfa, subdiag beta(2:)) by `ed_tridiag_poles` (implicit
    QL on the first row of Z, the tql2 iteration), weight norm2/Z * Z(1,j)^2,
    G(iw_n) += w/(iw_n - isign*(E_j - E_i)), G(w) += w/(w + i eps - isign*(E_j - E_i))
    with w_n = pi/beta (2n-1) and w = linspace(wini, wfin, Lreal)
    (allocate_grids, ED_AUX_FUNX.f90:449-461).
The pole sums of all seeds run in one device kernel (ed_gf_add_poles) into
G arrays kept in HBM, in the serial job order and the reference's per-pole
addition order; the frequency grids are uploaded once per build and G is
copied to the host (or all-reduced on the device) once at the end.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import check
from .diag import StateList, is_complex_vector
from .hamiltonian import Sector
from .params import EDConfig
from .sectors import c_sector, cdg_sector, setup_pointers


@dataclass
class GFOptions:
    """ED_INPUT_VARS defaults (ED_INPUT_VARS.f90:126-173)."""

    lanc_nGFiter: int = 200
    Lmats: int = 5000
    Lreal: int = 5000
    beta: float = 1000.0
    eps: float = 0.01
    wini: float = -5.0
    wfin: float = 5.0
    threshold: float = 1e-13      # sp_lanc_tridiag breakdown test (.repo/PLAIN_LANCZOS.f90:27)
    sparse_H: bool = True         # ed_sparse_H
    # seeds solved concurrently on one GPU (host threads, each with its own
    # device sectors); contributions are added to G in job order, so the
    # result is bit-identical to the serial loop
    workers: int = 4
    # seeds grouped by target sector: one sector build and one batched
    # persistent Lanczos launch per group (one workgroup per seed,
    # ed_sector_lanc_tridiag_batch); bit-identical to the per-seed runs
    batch: bool = True


def matsubara(beta: float, L: int) -> np.ndarray:
    return np.pi / beta * (2.0 * np.arange(1, L + 1) - 1.0)


def realaxis(wini: float, wfin: float, L: int) -> np.ndarray:
    return np.linspace(wini, wfin, L)


def tridiag_poles(alfa: np.ndarray, beta: np.ndarray, n: int, first_row: bool = False):
    """Eigenvalues of tridiag(alfa(1:n), beta(2:n)) and squared first components
    (tql2 / eigh of add_to_lanczos_gf_*, ED_GF_NONSU2.f90:936, ED_GF_NORMAL.f90:
    612-618): `ed_tridiag_poles`, the implicit-QL iteration carrying only the
    first row of the eigenvector matrix (O(n^2)).  first_row: return the
    components Z(1,j) themselves instead of their squares."""
    a = np.ascontiguousarray(alfa[:n], dtype=np.float64)
    b = np.zeros(n, dtype=np.float64)
    b[1:n] = beta[1:n]
    E = np.empty(n, dtype=np.float64)
    z2 = np.empty(n, dtype=np.float64)
    z1 = np.empty(n, dtype=np.float64)
    check(_lib.load().ed_tridiag_poles(n, a.ctypes.data, b.ctypes.data, E.ctypes.data, z2.ctypes.data,
                                       z1.ctypes.data), "ed_tridiag_poles")
    return (E, z1) if first_row else (E, z2)


class PoleSums:
    """Device side of add_to_lanczos_gf_normal / _nonsu2 (ED_GF_NORMAL.f90:
    620-631, ED_GF_NONSU2.f90:936-950): the frequency grids are uploaded once,
    G lives in HBM as (Nspin, Nspin, Norb, L) complex arrays, and `add` queues
    one continued fraction (its poles from ed_tridiag_poles) for component
    (ispin, jspin, iorb).  `flush` sums every queued fraction in one launch of
    ed_gf_add_poles, in queue order and pole by pole (the reference's order of
    additions into G(i))."""

    def __init__(self, nspin: int, norb: int, wm: np.ndarray, wr: np.ndarray, eps: float, device: int):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("the Green's function pole sum runs on the GPU (no host fallback)")
        self.dev = torch.device("cuda", device)
        self.nspin, self.norb, self.eps = nspin, norb, float(eps)
        self.wm = torch.from_numpy(np.ascontiguousarray(wm, dtype=np.float64)).to(self.dev)
        self.wr = torch.from_numpy(np.ascontiguousarray(wr, dtype=np.float64)).to(self.dev)
        self.Gm = torch.zeros((nspin, nspin, norb, len(wm)), dtype=torch.complex128, device=self.dev)
        self.Gr = torch.zeros((nspin, nspin, norb, len(wr)), dtype=torch.complex128, device=self.dev)
        self._q = []

    def add(self, comp, peso_bz, Ei: float, E: np.ndarray, z: np.ndarray, isign: int) -> None:
        ispin, jspin, iorb = comp
        c = (ispin * self.nspin + jspin) * self.norb + iorb
        pb = complex(peso_bz)
        self._q.append((c, pb.real, pb.imag, float(Ei), int(isign), np.asarray(E, np.float64),
                        np.asarray(z, np.float64)))

    def flush(self) -> None:
        import torch

        if not self._q:
            return
        q, self._q = self._q, []
        npole = np.array([len(t[5]) for t in q], dtype=np.int32)
        E = np.ascontiguousarray(np.concatenate([t[5] for t in q]))
        z = np.ascontiguousarray(np.concatenate([t[6] for t in q]))
        pb = np.ascontiguousarray(np.array([[t[1], t[2]] for t in q], dtype=np.float64).reshape(-1))
        ei = np.array([t[3] for t in q], dtype=np.float64)
        sg = np.array([t[4] for t in q], dtype=np.int32)
        comp = np.array([t[0] for t in q], dtype=np.int32)
        st = torch.cuda.current_stream(self.dev)
        P = ctypes.c_void_p
        check(_lib.load().ed_gf_add_poles(len(q), P(npole.ctypes.data), P(E.ctypes.data), P(z.ctypes.data),
                                          P(pb.ctypes.data), P(ei.ctypes.data), P(sg.ctypes.data),
                                          P(comp.ctypes.data), P(self.wm.data_ptr()), self.wm.numel(),
                                          P(self.wr.data_ptr()), self.wr.numel(), self.eps,
                                          P(self.Gm.data_ptr()), P(self.Gr.data_ptr()), P(st.cuda_stream)),
              "ed_gf_add_poles")

    def to_host(self, Gm: np.ndarray, Gr: np.ndarray) -> None:
        """Add the device G into the host (Nspin, Nspin, Norb, Norb, L) arrays."""
        gm, gr = self.Gm.cpu().numpy(), self.Gr.cpu().numpy()
        for o in range(self.norb):
            Gm[:, :, o, o] += gm[:, :, o]
            Gr[:, :, o, o] += gr[:, :, o]


def _seed(src: Sector, dst: Sector, op: int, terms, vec: np.ndarray, cplx: bool):
    """Seed sum_t coef_t * op_{level_t}|vec> on the device (first term assigned,
    the rest accumulated, as the vvinit loops of ED_GF_NORMAL/ED_GF_NONSU2);
    returns (normalised seed, norm2)."""
    import torch

    real = not cplx
    dt = torch.float64 if real else torch.complex128
    dev = f"cuda:{src.device}"
    if isinstance(vec, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(vec.astype(np.float64 if real else np.complex128))).to(dev)
    else:                                   # state vector kept in HBM by the farm
        x = vec.to(device=dev, dtype=dt).contiguous()
    y = torch.empty(dst.dim, dtype=dt, device=dev)
    st = torch.cuda.current_stream(x.device)
    L = _lib.load()
    vt = 0 if real else 1
    xp, yp, sp = ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(st.cuda_stream)
    (lvl0, c0), rest = terms[0], terms[1:]
    assert c0 == 1
    check(L.ed_sector_apply_op(src.handle, dst.handle, op, lvl0, vt, xp, yp, sp), "ed_sector_apply_op")
    for lvl, c in rest:
        check(L.ed_sector_apply_op_acc(src.handle, dst.handle, op, lvl, float(np.real(c)), float(np.imag(c)),
                                       vt, xp, yp, sp), "ed_sector_apply_op_acc")
    norm2 = float(torch.sum(y.abs() ** 2).item())
    if norm2 > 0:
        y = y / np.sqrt(norm2)
    y = y.contiguous()
    st.synchronize()   # the seed is complete for the library's stream (no device-wide sync:
    return y, norm2    # other threads may be capturing graphs)


def _tridiag_dev(S: Sector, seed, nlanc: int, real: bool, threshold: float):
    a = np.zeros(nlanc)
    b = np.zeros(nlanc)
    n = ctypes.c_int32()
    check(_lib.load().ed_sector_lanc_tridiag_dev(S.handle, 0 if real else 1,
                                                 ctypes.c_void_p(seed.data_ptr()), nlanc, threshold,
                                                 a.ctypes.data_as(ctypes.c_void_p),
                                                 b.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)),
          "ed_sector_lanc_tridiag_dev")
    return a, b, int(n.value)


def _target(cfg: EDConfig, sec, op: int, ispin: int, iorb: int = 0):
    return cdg_sector(cfg, sec, ispin, iorb) if op == 1 else c_sector(cfg, sec, ispin, iorb)


class _SectorCache:
    """Device sectors reused across the seeds of one GF build (the reference
    rebuilds them per seed with build_Hv_sector / delete_Hv_sector)."""

    def __init__(self, cfg, gopt, device):
        self.cfg, self.gopt, self.device, self.d = cfg, gopt, device, {}

    def get(self, sec, hamiltonian: bool) -> Sector:
        key = (sec.q1, sec.q2, hamiltonian)
        if key not in self.d:
            stored = hamiltonian and self.gopt.sparse_H
            self.d[key] = Sector(self.cfg, sec.q1, sec.q2, stored=stored, direct=not stored,
                                 real=self.cfg.is_real(), device=self.device)
        return self.d[key]

    def close(self):
        for S in self.d.values():
            S.close()
        self.d.clear()


def mixed_pairs(cfg: EDConfig):
    """(ispin, jspin, iorb) of the spin-off-diagonal nonsu2 components
    (build_gf_nonsu2 ED_GF_NONSU2.f90:39-48 normal/hybrid: all of them;
    :203-217 replica: only where dmft_bath%mask(ispin,jspin,iorb,iorb,:) is set,
    i.e. |Re or Im impHloc(ispin,jspin,iorb,iorb)| > 1e-6, init_dmft_bath_mask
    ED_BATH/dmft_aux.f90:261-302)."""
    if cfg.ed_mode != "nonsu2":
        return []
    Nsp, No = cfg.Nspin, cfg.Norb
    out = []
    for s1 in range(Nsp):
        for s2 in range(Nsp):
            for o in range(No):
                if s1 == s2:
                    continue
                if cfg.bath_type == "replica":
                    h = 0j if cfg.impHloc is None else cfg.impHloc[s1, s2, o, o]
                    if not (abs(h.real) > 1e-6 or abs(h.imag) > 1e-6):
                        continue
                out.append((s1, s2, o))
    return out


def _job_list(cfg: EDConfig, states: StateList):
    """Every (component, kept state, seed spec) of build_gf in the serial
    accumulation order: diagonal components (ispin, iorb), then for nonSU2 the
    mixed seeds (ispin != jspin, iorb).  A seed spec is (op, isign, spin of the
    first level, [(level, coef)], weight)."""
    Ns, No, Nsp = cfg.Ns, cfg.Norb, cfg.Nspin
    site = lambda o, s: o + s * Ns          # impIndex(iorb,ispin), 0-based bit
    chans = []
    for ispin in range(Nsp):
        for iorb in range(No):
            i = site(iorb, ispin)
            chans.append(((ispin, ispin, iorb), ("diag", ispin, iorb),
                          [(1, +1, ispin, [(i, 1)], 1.0), (0, -1, ispin, [(i, 1)], 1.0)]))
    pairs = mixed_pairs(cfg)
    if pairs:
        if cfg.Jz_basis:
            # the reference builds the second term of a mixed seed in the sector
            # of (jorb,jspin) (ED_GF_NONSU2.f90:576-584), a different Jz sector
            raise NotImplementedError("mixed nonsu2 seeds in the Jz basis")
        for ispin, jspin, iorb in pairs:
            i, j = site(iorb, ispin), site(iorb, jspin)
            chans.append(((ispin, jspin, iorb), ("mix", ispin, jspin, iorb), [
                (1, +1, ispin, [(i, 1), (j, 1)], 1.0),         # (c+_i + c+_j)|gs>      :571-595
                (0, -1, ispin, [(i, 1), (j, 1)], 1.0),         # (c_i + c_j)|gs>        :654-678
                (1, +1, ispin, [(i, 1), (j, 1j)], 1j),         # (c+_i + i c+_j)|gs>    :739-763, cnorm2=i*norm2
                (0, -1, ispin, [(i, 1), (j, -1j)], 1j),        # (c_i - i c_j)|gs>      :823-847
            ]))
    secs = setup_pointers(cfg)
    jobs = []
    for comp, tag, seeds in chans:
        for k, isec in enumerate(states.sectors):
            sec = secs[isec - 1]
            for spec in seeds:
                jsec = _target(cfg, sec, spec[0], spec[2], comp[2])
                if jsec is not None:
                    jobs.append((comp, tag, k, spec, sec, jsec))
    return jobs, pairs


def _run_job(cfg, states, gopt, job, cache, poles, record, zeta):
    """One tridiagonalisation; its poles are queued on `poles` (PoleSums)."""
    comp, tag, k, (op, isign, ispin, terms, weight), sec, jsec = job
    e_i, vec = states.energies[k], states.vectors[k]
    if vec is None:
        raise ValueError("the Green's function needs the state vectors (keep_vectors=True)")
    cplx = (not cfg.is_real()) or is_complex_vector(vec) or any(np.imag(c) != 0 for _, c in terms)
    HI, HJ = cache.get(sec, False), cache.get(jsec, True)
    seed, norm2 = _seed(HI, HJ, op, terms, vec, cplx)
    if norm2 == 0.0:
        return
    nlanc = min(HJ.dim, gopt.lanc_nGFiter)
    a, b, n = _tridiag_dev(HJ, seed, nlanc, not cplx, gopt.threshold)
    # the reference diagonalises all nlanc entries (unset ones stay 0)
    E, z = tridiag_poles(a, b, nlanc, first_row=True)
    if record is not None:
        record.append(dict(channel=tag, isector=states.sectors[k], op=op, norm2=norm2, alfa=a, beta=b,
                           nlanc=n))
    poles.add(comp, weight * norm2 / zeta, e_i, E, z, isign)


def _tridiag_batch(S: Sector, seeds, nlanc: int, real: bool, threshold: float):
    """sp_lanc_tridiag of every seed (rows of the contiguous `seeds` tensor) on S."""
    k = seeds.shape[0]
    a = np.zeros((k, nlanc))
    b = np.zeros((k, nlanc))
    n = np.zeros(k, dtype=np.int32)
    check(_lib.load().ed_sector_lanc_tridiag_batch(S.handle, 0 if real else 1, k,
                                                   ctypes.c_void_p(seeds.data_ptr()), nlanc, threshold,
                                                   a.ctypes.data_as(ctypes.c_void_p),
                                                   b.ctypes.data_as(ctypes.c_void_p),
                                                   n.ctypes.data_as(ctypes.c_void_p)),
          "ed_sector_lanc_tridiag_batch")
    return a, b, n


def _run_jobs_batched(cfg, states, gopt, jobs, todo, device, poles, zeta, record=None):
    """The seed loop grouped by (target sector, vector type): each group's
    seeds are built on the device and tridiagonalised in one batched launch;
    the poles are queued in job order (the serial loop's sequence of
    additions)."""
    import torch

    torch.cuda.set_device(device)
    cache = _SectorCache(cfg, gopt, device)
    groups = {}
    for n in todo:
        comp, tag, k, (op, isign, ispin, terms, weight), sec, jsec = jobs[n]
        vec = states.vectors[k]
        if vec is None:
            raise ValueError("the Green's function needs the state vectors (keep_vectors=True)")
        cplx = (not cfg.is_real()) or is_complex_vector(vec) or any(np.imag(c) != 0 for _, c in terms)
        groups.setdefault((jsec.q1, jsec.q2, cplx), []).append(n)
    fracs = {}
    try:
        for (_, _, cplx), members in groups.items():
            live, seeds, norms = [], [], []
            for n in members:
                comp, tag, k, (op, isign, ispin, terms, weight), sec, jsec = jobs[n]
                HI, HJ = cache.get(sec, False), cache.get(jsec, True)
                seed, norm2 = _seed(HI, HJ, op, terms, states.vectors[k], cplx)
                if norm2 == 0.0:
                    continue
                live.append(n)
                seeds.append(seed)
                norms.append(norm2)
            if not live:
                continue
            HJ = cache.get(jobs[live[0]][5], True)
            nlanc = min(HJ.dim, gopt.lanc_nGFiter)
            stacked = torch.stack(seeds).contiguous()
            # the library copies the seeds on the sector's own (non-blocking)
            # stream: the stack kernel on torch's stream must be complete first
            torch.cuda.current_stream(stacked.device).synchronize()
            a, b, nl = _tridiag_batch(HJ, stacked, nlanc, not cplx, gopt.threshold)
            for q, n in enumerate(live):
                comp, tag, k, (op, isign, ispin, terms, weight), sec, jsec = jobs[n]
                E, z = tridiag_poles(a[q], b[q], nlanc, first_row=True)
                if record is not None:
                    record.append((n, dict(channel=tag, isector=states.sectors[k], op=op, norm2=norms[q],
                                           alfa=a[q], beta=b[q], nlanc=int(nl[q]))))
                fracs[n] = (comp, weight * norms[q] / zeta, states.energies[k], E, z, isign)
    finally:
        cache.close()
    for n in todo:
        if n in fracs:
            poles.add(*fracs[n])


def _run_jobs_threaded(cfg, states, gopt, jobs, todo, device, poles, zeta):
    """The seed loop on `gopt.workers` host threads (one sector cache per
    thread); each job's poles are queued in job order afterwards — the same
    sequence of additions as the serial loop."""
    import threading
    from concurrent.futures import ThreadPoolExecutor

    import torch

    local = threading.local()
    caches, lock = [], threading.Lock()

    def init():
        torch.cuda.set_device(device)   # the current device is per thread
        local.cache = _SectorCache(cfg, gopt, device)
        with lock:
            caches.append(local.cache)

    class _Rec:
        def __init__(self):
            self.q = []

        def add(self, *a):
            self.q.append(a)

    def work(n):
        r = _Rec()
        _run_job(cfg, states, gopt, jobs[n], local.cache, r, None, zeta)
        return r.q

    order = sorted(todo, key=lambda n: -jobs[n][5].dim)   # longest first
    try:
        with ThreadPoolExecutor(max_workers=min(gopt.workers, len(todo)), initializer=init) as ex:
            futs = {n: ex.submit(work, n) for n in order}
            for n in todo:
                for fr in futs[n].result():
                    poles.add(*fr)
    finally:
        for c in caches:
            c.close()


def _dist():
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


def build_gf(cfg: EDConfig, states: StateList, gopt: Optional[GFOptions] = None, device: int = 0,
             record: Optional[list] = None, owners: Optional[List[int]] = None, runner=None):
    """impGmats, impGreal (Nspin, Nspin, Norb, Norb, L) for ed_mode normal
    (diagonal components, build_gf_normal) and nonsu2 (build_gf_nonsu2,
    ED_GF_NONSU2.f90:18-333, bath_type normal/hybrid: diagonal components plus
    the spin-off-diagonal ones from the mixed seeds and the 0.5*(G - (1+i)G_ii -
    (1+i)G_jj) recombination).

    Seed farm: with a process group initialised, the (component, state, seed)
    jobs are split over ranks (longest first by target dimension), each rank
    sums its poles into its own G, and one all_reduce adds the G arrays
    (2 x L complex numbers per component — no collective inside a job).  State
    vectors missing on a rank (farm_diag keeps them on their owner) are
    broadcast from `owners` first.  `runner(cfg, states, gopt, job, wm, wr,
    G_m, G_r, zeta)` replaces the device job (the CPU tests pass the oracle's)."""
    gopt = gopt or GFOptions()
    if cfg.ed_mode == "superc":
        raise NotImplementedError("superc Green's function (ED_GF_SUPERC) is outside this hot path")
    No, Nsp = cfg.Norb, cfg.Nspin
    wm = matsubara(gopt.beta, gopt.Lmats)
    wr = realaxis(gopt.wini, gopt.wfin, gopt.Lreal)
    Gm = np.zeros((Nsp, Nsp, No, No, gopt.Lmats), dtype=np.complex128)
    Gr = np.zeros((Nsp, Nsp, No, No, gopt.Lreal), dtype=np.complex128)
    dist = _dist()
    rank = dist.get_rank() if dist else 0
    world = dist.get_world_size() if dist else 1
    if dist and owners is not None:
        from .farm import broadcast_vector

        vecs = list(states.vectors)
        for k, isec in enumerate(states.sectors):
            dim = setup_pointers(cfg)[isec - 1].dim
            cplx = not cfg.is_real() or is_complex_vector(vecs[k])
            flag = [cplx]
            dist.broadcast_object_list(flag, src=owners[k])
            vecs[k] = broadcast_vector(vecs[k], owners[k], dim, flag[0], device)
        states = StateList(list(states.energies), list(states.sectors), vecs)
    jobs, pairs = _job_list(cfg, states)
    if world > 1:
        from .farm import lpt_partition

        costs = [float(min(j[5].dim, gopt.lanc_nGFiter)) * j[5].dim for j in jobs]
        mine = set(lpt_partition(costs, world)[rank])
    else:
        mine = set(range(len(jobs)))
    zeta = float(states.size)       # T=0: zeta_function = state_list%size (ED_DIAG.f90:411)
    todo = [n for n in range(len(jobs)) if n in mine]
    poles = PoleSums(Nsp, No, wm, wr, gopt.eps, device) if runner is None else None
    if runner is None and gopt.batch:
        rec = [] if record is not None else None
        _run_jobs_batched(cfg, states, gopt, jobs, todo, device, poles, zeta, rec)
        if record is not None:
            record.extend(r for _, r in sorted(rec, key=lambda t: t[0]))
    elif runner is None and record is None and gopt.workers > 1 and len(todo) > 1:
        _run_jobs_threaded(cfg, states, gopt, jobs, todo, device, poles, zeta)
    else:
        cache = _SectorCache(cfg, gopt, device)
        try:
            for n in todo:
                job = jobs[n]
                ispin, jspin, iorb = job[0]
                g_m, g_r = Gm[ispin, jspin, iorb, iorb], Gr[ispin, jspin, iorb, iorb]
                if runner is None:
                    _run_job(cfg, states, gopt, job, cache, poles, record, zeta)
                else:
                    runner(cfg, states, gopt, job, wm, wr, g_m, g_r, zeta)
        finally:
            cache.close()
    if poles is not None:
        poles.flush()
    if world > 1:
        import torch

        if poles is not None and dist.get_backend() == "nccl":
            for t in (poles.Gm, poles.Gr):            # device G, summed over ranks in HBM
                dist.all_reduce(torch.view_as_real(t))
        elif poles is not None:
            for t in (poles.Gm, poles.Gr):
                h = torch.view_as_real(t).cpu()
                dist.all_reduce(h)
                torch.view_as_real(t).copy_(h)
        else:
            for G in (Gm, Gr):
                t = torch.view_as_real(torch.from_numpy(G))   # (re, im) pairs: plain f64 sum
                dist.all_reduce(t)
                G[...] = torch.view_as_complex(t).numpy()
    if poles is not None:
        poles.to_host(Gm, Gr)
    for ispin, jspin, iorb in pairs:               # build_gf_nonsu2 :35-48
        for G in (Gm, Gr):
            G[ispin, jspin, iorb, iorb] = 0.5 * (G[ispin, jspin, iorb, iorb]
                                                 - (1 + 1j) * G[ispin, ispin, iorb, iorb]
                                                 - (1 + 1j) * G[jspin, jspin, iorb, iorb])
    return Gm, Gr


def build_gf_normal(cfg: EDConfig, states: StateList, gopt: Optional[GFOptions] = None,
                    device: int = 0, record: Optional[list] = None):
    """build_gf_normal (ED_GF_NORMAL.f90:18-92), diagonal components."""
    if cfg.ed_mode != "normal":
        raise ValueError("build_gf_normal needs ed_mode='normal'")
    rec = [] if record is not None else None
    Gm, Gr = build_gf(cfg, states, gopt, device, rec)
    if record is not None:
        for r in rec:
            _, ispin, iorb = r["channel"]
            record.append(dict(r, ispin=ispin, iorb=iorb))
    return Gm, Gr
