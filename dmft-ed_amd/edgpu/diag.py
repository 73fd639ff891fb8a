"""Sector loop of the impurity diagonalisation: ed_diag_c (ED_DIAG.f90:49-251).

For every symmetry sector (reference isector order):
  * Neigen / Nitermax / Nblock as ED_DIAG.f90:88-97;
  * dim <= max(lanc_dim_threshold, MpiSize) or Neigen == dim: dense path —
    H dumped from the device sector (sp_dump_matrix) and diagonalised with
    LAPACK on the host, as the reference does on its master rank (:187-212);
  * lanc_method="lanczos": device-resident plain Lanczos (sp_lanc_eigh, :173-180);
  * lanc_method="arpack" : sp_eigh (:145-167) replaced by a device
    thick-restart Lanczos (ed_sector_eigh): Krylov basis in HBM, CGS2
    reorthogonalisation kernels, only the ncv x ncv projected matrix on host.
The T=0 state list follows :217-236 (gs_threshold window, 10*gs_threshold
reset).  Sectors can be restricted (the farm hands each rank its subset);
`state_list` replays the list logic in isector order over gathered
eigenvalues, so a farmed run reproduces the serial list exactly.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np

from .hamiltonian import Sector
from .params import EDConfig
from .sectors import Sector as SectorId
from .sectors import diag_sectors


@dataclass
class DiagOptions:
    """ED_INPUT_VARS defaults (ED_INPUT_VARS.f90:166-176, :179)."""

    lanc_method: str = "arpack"
    lanc_nstates_sector: int = 6
    lanc_niter: int = 512
    lanc_ncv_factor: int = 3
    lanc_ncv_add: int = 5
    lanc_tolerance: float = 1e-12
    lanc_dim_threshold: int = 256
    gs_threshold: float = 1e-9
    mpi_size: int = 1
    keep_vectors: bool = True
    # Lanczos / thick-restart eigenvectors stay in HBM (torch tensors on the
    # sector's GPU) and nothing crosses PCIe unless a caller asks for host
    # copies: to_host(vec) turns any state vector into a numpy array.  With
    # device_vectors=False every vector is a host numpy array, as before.
    device_vectors: bool = True
    # device vectors: after the T=0 state list is formed only its states are
    # retained and SectorResult.vectors of every sector becomes None (the
    # farm's HBM budget); retain_all=True keeps every sector's (dim, Neigen)
    # block in SectorResult.vectors as well
    retain_all: bool = False
    # sectors solved concurrently on one GPU (host threads, one HIP stream per
    # sector; ctypes releases the GIL): small sectors are launch-latency bound
    workers: int = 8
    # of those, this many take the smallest pending sector instead of the
    # largest (single-rank schedule; at least one worker stays on the largest):
    # the launch-latency-bound small sectors run beside the HBM-bound large
    # ones instead of after them.  configs[3] on one MI355X, alternating runs:
    # 6 → median 0.707 s, 0 (largest first for all) → 0.752 s; 2 or 4 within
    # noise of 0 (gpurun_out r6sw*)
    small_workers: int = 6
    # each worker thread keeps one HIP stream for every sector it solves
    # (False: every sector creates and destroys a private stream)
    worker_streams: bool = True
    # ED_OPT_* kernel alternatives (Sector.set_options names) for every sector
    # of the diagonalisation (A/B runs; the defaults are the measured best)
    kernel_options: Tuple[str, ...] = ()
    # concurrent sectors' working sets (Krylov basis + stored H, estimated by
    # `working_set_bytes`) are admitted up to this many MB, so that the bases
    # being streamed by the Gram-Schmidt sweeps stay in the 256 MB Infinity
    # Cache instead of evicting each other to HBM; a sector larger than the
    # budget runs when nothing else big is in flight.  0: no limit.
    cache_budget_mb: float = 0.0
    # thick-restart sectors of at most this many rows (real H, stored) are
    # solved together by one host thread through ed_sectors_eigh_batch beside
    # the other workers; 0: every sector alone (ed_sector_eigh).  The library
    # gives the sectors of up to 2,640 rows one workgroup each (one launch per
    # restart cycle for all of them: configs[3]'s 36 in 17 ms instead of 138
    # ms one after the other) and runs the larger ones in lockstep (every
    # kernel of a Krylov step carries that step of all of them).  configs[3]
    # farm, one box, alternating runs (gpurun_out r6bm2): cap
    # 2,640 median 0.652 s, 33,000 0.638 s, 60,000 0.594 s (the 52 sectors of
    # 4,356-52,272 rows in lockstep beside the workers' large sectors); every
    # sector in lockstep 0.81-0.96 s (its tail of few sectors is serial)
    batch_max_dim: int = 60000
    # multi-rank farms: "dynamic" — every rank's workers take the next sector
    # (largest cost first) from one global counter in the process group's
    # key-value store, so the ranks finish together whatever the cost
    # model's error; "lpt" — the static longest-processing-time partition
    farm_schedule: str = "dynamic"


@dataclass
class SectorResult:
    isector: int
    q: Tuple[int, int]
    dim: int
    eigenvalues: np.ndarray          # the Neigen lowest (or all, dense)
    neigen: int
    vectors: Optional[np.ndarray] = None   # (dim, Neigen) host copy, if kept
    method: str = ""


@dataclass
class StateList:
    """state_list at T=0: energies, sectors and (optionally) vectors."""

    energies: List[float] = field(default_factory=list)
    sectors: List[int] = field(default_factory=list)
    vectors: List[Optional[np.ndarray]] = field(default_factory=list)

    @property
    def emin(self) -> float:
        return min(self.energies)

    @property
    def size(self) -> int:
        return len(self.energies)


def lanczos_params(dim: int, opt: DiagOptions) -> Tuple[int, int, int]:
    """(Neigen, Nitermax, Nblock), ED_DIAG.f90:88-97 (neigen_sector from
    setup_pointers: min(dim, lanc_nstates_sector))."""
    neigen_sector = min(dim, opt.lanc_nstates_sector)
    if opt.lanc_method == "lanczos":
        return 1, min(dim, opt.lanc_niter), 1
    neigen = min(dim, neigen_sector)
    nitermax = min(dim, opt.lanc_niter)
    nblock = min(dim, opt.lanc_ncv_factor * max(neigen, opt.lanc_nstates_sector) + opt.lanc_ncv_add)
    return neigen, nitermax, nblock


def to_host(vec):
    """A state vector as a host numpy array (device tensors are copied back)."""
    if vec is None or isinstance(vec, np.ndarray):
        return vec
    return vec.detach().cpu().numpy()


def is_complex_vector(vec) -> bool:
    if vec is None:
        return False
    if isinstance(vec, np.ndarray):
        return np.iscomplexobj(vec)
    return bool(vec.is_complex())


def _start_vector(dim: int, cplx: bool) -> np.ndarray:
    i = np.arange(1, dim + 1, dtype=np.float64)
    return (np.sin(i) + 1j * np.cos(3.0 * i)) if cplx else np.sin(i)


_tls = None


def _worker_stream(opt: DiagOptions, device: int):
    """The calling thread's own stream on `device` (DiagOptions.worker_streams),
    created on first use and reused for every sector the thread solves."""
    global _tls
    import torch

    if not opt.worker_streams or not torch.cuda.is_available():
        return None
    if _tls is None:
        import threading

        _tls = threading.local()
    d = getattr(_tls, "streams", None)
    if d is None:
        d = _tls.streams = {}
    if device not in d:
        d[device] = torch.cuda.Stream(device=device)
    return d[device]


def solve_sector(cfg: EDConfig, sec: SectorId, opt: DiagOptions, device: int = 0) -> SectorResult:
    dim = sec.dim
    st = _worker_stream(opt, device)
    neigen, nitermax, nblock = lanczos_params(dim, opt)
    lanc_solve = not (neigen == dim or dim <= max(opt.lanc_dim_threshold, opt.mpi_size))
    real = cfg.is_real()
    q = (sec.q1, sec.q2)
    if not lanc_solve:
        with Sector(cfg, sec.q1, sec.q2, stored=True, real=real, device=device,
                    options=opt.kernel_options, stream=st) as S:
            rp, cols, vals = S.dump_csr()
        H = np.zeros((dim, dim), dtype=np.complex128)
        rows = np.repeat(np.arange(dim), np.diff(rp))
        np.add.at(H, (rows, cols), vals)
        if real:
            H = H.real
        w, v = np.linalg.eigh(H)
        vec = v[:, :neigen] if opt.keep_vectors else None
        return SectorResult(sec.isector, q, dim, w, neigen, vec, "dense")
    with Sector(cfg, sec.q1, sec.q2, stored=True, real=real, device=device,
                options=opt.kernel_options, stream=st) as S:
        if opt.lanc_method == "lanczos":
            e0, vec, _ = S.lanc_eigh(nitermax=nitermax, threshold=opt.lanc_tolerance,
                                     v0=_start_vector(dim, not real), vector=opt.keep_vectors,
                                     on_device=opt.device_vectors)
            vecs = vec[:, None] if vec is not None else None
            return SectorResult(sec.isector, q, dim, np.array([e0]), 1, vecs, "lanczos")
        if neigen >= dim:
            raise ValueError("arpack path needs Neigen < dim")
        ncv = min(max(nblock, neigen + 1), 64, dim)   # device basis limit (ed_gpu.h)
        w, v, _, _ = S.eigh(neigen=neigen, ncv=ncv, maxit=max(nitermax, 10),
                            tol=opt.lanc_tolerance, v0=_start_vector(dim, not real),
                            vectors=opt.keep_vectors, on_device=opt.device_vectors)
        order = np.argsort(w)
        if np.any(order != np.arange(len(w))):      # (the device solver returns them ascending)
            w = w[order]
            v = v[:, order] if v is not None else None
        return SectorResult(sec.isector, q, dim, w, neigen, v if opt.keep_vectors else None, "arpack")


def batchable(cfg: EDConfig, sec: SectorId, opt: DiagOptions) -> bool:
    """A sector `solve_batch` takes: thick-restart (arpack) path, real H,
    at most opt.batch_max_dim rows, a Krylov basis of at most 32 columns."""
    if opt.batch_max_dim <= 0 or opt.lanc_method != "arpack" or not cfg.is_real():
        return False
    neigen, _, nblock = lanczos_params(sec.dim, opt)
    if neigen == sec.dim or sec.dim <= max(opt.lanc_dim_threshold, opt.mpi_size):
        return False
    ncv = min(max(nblock, neigen + 1), 64, sec.dim)
    return sec.dim <= opt.batch_max_dim and ncv <= 32 and neigen + 2 <= 32


def solve_batch(cfg: EDConfig, secs: List[SectorId], opt: DiagOptions, device: int = 0) -> List[SectorResult]:
    """The arpack path of `solve_sector` for many small sectors at once
    (ed_sectors_eigh_batch; the same start vector, Neigen, Nblock, Nitermax
    and tolerance per sector, ED_DIAG.f90:88-167).  Results in `secs` order."""
    from .hamiltonian import eigh_batch

    st = _worker_stream(opt, device)
    groups: Dict[Tuple[int, int], List[int]] = {}
    for k, sec in enumerate(secs):
        neigen, nitermax, nblock = lanczos_params(sec.dim, opt)
        ncv = min(max(nblock, neigen + 1), 64, sec.dim)
        groups.setdefault((neigen, ncv), []).append(k)
    out: List[Optional[SectorResult]] = [None] * len(secs)
    from concurrent.futures import ThreadPoolExecutor

    def build(k):   # on the pool thread's own stream (the build synchronises it)
        return Sector(cfg, secs[k].q1, secs[k].q2, stored=True, real=True, device=device,
                      options=opt.kernel_options, stream=_worker_stream(opt, device))

    # the sector builds (a few ms of small launches and host syncs each) on
    # opt.workers threads, then one batch call, then the frees in parallel
    with ThreadPoolExecutor(max_workers=max(1, opt.workers)) as ex:
        for (neigen, ncv), ks in groups.items():
            maxit = [max(lanczos_params(secs[k].dim, opt)[1], 10) for k in ks]
            futs = [ex.submit(build, k) for k in ks]
            hs: List[Sector] = []
            try:
                for f in futs:
                    hs.append(f.result())
                res, _ = eigh_batch(hs, neigen, ncv, maxit, opt.lanc_tolerance,
                                    [_start_vector(h.dim, False) for h in hs], vectors=opt.keep_vectors,
                                    on_device=opt.device_vectors, stream=st, fallback=False)
            finally:
                for f in futs:
                    if f.exception() is None and f.result() not in hs:
                        hs.append(f.result())
                list(ex.map(lambda h: h.close(), hs))
            # the sectors the batch left (a missed degenerate copy to probe, an
            # invariant subspace, ...): the per-sector solve on the pool's threads
            redo = [k for k, r in zip(ks, res) if r[2] < 0]
            again = dict(zip(redo, ex.map(lambda k: solve_sector(cfg, secs[k], opt, device), redo)))
            for k, (w, v, _, _) in zip(ks, res):
                if k in again:
                    out[k] = again[k]
                    continue
                sec = secs[k]
                out[k] = SectorResult(sec.isector, (sec.q1, sec.q2), sec.dim, w, neigen,
                                      v if opt.keep_vectors else None, "arpack")
    return out


def state_list(results: Iterable[SectorResult], opt: DiagOptions) -> StateList:
    """T=0 state list, ED_DIAG.f90:224-235, replayed in isector order."""
    sl = StateList()
    oldzero = 1000.0
    for r in sorted(results, key=lambda r: r.isector):
        for i in range(r.neigen):
            enemin = float(r.eigenvalues[i])
            vec = r.vectors[:, i] if r.vectors is not None else None
            if enemin < oldzero - 10.0 * opt.gs_threshold:
                oldzero = enemin
                sl = StateList()
                sl.energies.append(enemin); sl.sectors.append(r.isector); sl.vectors.append(vec)
            elif abs(enemin - oldzero) <= opt.gs_threshold:
                oldzero = min(oldzero, enemin)
                sl.energies.append(enemin); sl.sectors.append(r.isector); sl.vectors.append(vec)
    return sl


def retain_state_vectors(sl: StateList, results: Iterable[SectorResult],
                         drop_blocks: bool = True) -> StateList:
    """Keep only the state list's vectors (ED_DIAG.f90:220-236 stores just
    those): each kept device vector is cloned out of its sector's (neigen, dim)
    block and (drop_blocks) every sector result drops its device block, so the
    HBM held after the diagonalisation is the kept states alone.  Host (numpy)
    blocks are never dropped."""
    vecs = [v.clone() if (v is not None and not isinstance(v, np.ndarray)) else v for v in sl.vectors]
    if not drop_blocks:
        return StateList(list(sl.energies), list(sl.sectors), vecs)
    for r in results:
        if r.vectors is not None and not isinstance(r.vectors, np.ndarray):
            r.vectors = None
    return StateList(list(sl.energies), list(sl.sectors), vecs)


def working_set_bytes(cfg: EDConfig, sec: SectorId, opt: DiagOptions) -> float:
    """Device bytes a sector's solve streams repeatedly: the Krylov basis
    (Nblock columns), the packed stored H (4 B per element, ~1 + Norb*Nbath
    per row) and the O(dim) vectors (diagonal, residual, scratch)."""
    _, _, nblock = lanczos_params(sec.dim, opt)
    vs = 8 if cfg.is_real() else 16
    return float(sec.dim) * (nblock * vs + 4.0 * (1 + cfg.Norb * cfg.Nbath) + 4 * vs)


def solve_many(cfg: EDConfig, secs: List[SectorId], opt: DiagOptions, device: int = 0,
               solver=None, cost=None, take_global=None, batch_solver=None) -> List[SectorResult]:
    """Solve a list of sectors on one GPU with `opt.workers` host threads,
    largest first (`opt.small_workers` of them smallest first); results in
    the order of `secs` (each sector's result does not depend on the
    schedule).  With `opt.cache_budget_mb` a worker takes
    the largest pending sector whose working set fits beside those in flight
    (a sector larger than the budget only when nothing else big runs), else
    waits for one to finish.

    take_global: the farm's multi-rank work queue — a callable returning the
    next index into `secs` (already in schedule order) or None; the result
    list then holds the sectors this process solved, None elsewhere.  The
    cache budget applies to the single-rank and LPT schedules only: a worker
    on the global queue takes the next index unconditionally (a warning says
    so when a budget is set).

    batch_solver: solves the `batchable` sectors together in one more thread
    beside the workers (default: solve_batch with the library's own solver;
    opt.batch_max_dim = 0 turns it off); not on the multi-rank queue, where
    farm_diag deals the batchable sectors to the ranks itself."""
    solver = solver or solve_sector
    if batch_solver is None and solver is solve_sector:
        batch_solver = solve_batch
    import threading

    if take_global is not None:
        if opt.cache_budget_mb > 0:
            import warnings

            warnings.warn("DiagOptions.cache_budget_mb is not applied on the multi-rank dynamic queue "
                          "(farm_schedule='lpt' applies it per rank)", RuntimeWarning, stacklevel=2)
        out_g: List[Optional[SectorResult]] = [None] * len(secs)
        errs: List[BaseException] = []

        def gworker():
            while not errs:
                i = take_global()
                if i is None:
                    return
                try:
                    out_g[i] = solver(cfg, secs[i], opt, device)
                except BaseException as e:  # noqa: BLE001 - re-raised below
                    errs.append(e)
                    return

        ths = [threading.Thread(target=gworker, daemon=True) for _ in range(max(1, min(opt.workers, len(secs))))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]
        return out_g
    if batch_solver is not None and opt.batch_max_dim > 0 and take_global is None:
        bidx = [i for i, s in enumerate(secs) if batchable(cfg, s, opt)]
        if len(bidx) > 1:
            bset = set(bidx)
            ridx = [i for i in range(len(secs)) if i not in bset]
            opt_nb = replace(opt, batch_max_dim=0)
            rest, bres = with_batch(cfg, [secs[i] for i in bidx], opt, device,
                                    lambda: solve_many(cfg, [secs[i] for i in ridx], opt_nb, device,
                                                       solver=solver, cost=cost), batch_solver)
            out_b: List[Optional[SectorResult]] = [None] * len(secs)
            for i, r in zip(bidx, bres):
                out_b[i] = r
            for i, r in zip(ridx, rest):
                out_b[i] = r
            return out_b
    if opt.workers <= 1 or len(secs) <= 1:
        return [solver(cfg, sec, opt, device) for sec in secs]

    order = sorted(range(len(secs)), key=lambda i: -(cost(secs[i]) if cost else secs[i].dim))
    budget = opt.cache_budget_mb * 1e6
    # (sectors below 16 MB are not counted: they fit the cache beside anything)
    ws = [working_set_bytes(cfg, s, opt) if budget > 0 else 0.0 for s in secs]
    ws = [w if w >= 16e6 else 0.0 for w in ws]
    out: List[Optional[SectorResult]] = [None] * len(secs)
    err: List[BaseException] = []
    pending = list(order)
    used = [0.0]
    cv = threading.Condition()

    def take(small: bool) -> Optional[int]:
        with cv:
            while pending and not err:
                ks = range(len(pending) - 1, -1, -1) if small else range(len(pending))
                for k in ks:
                    i = pending[k]
                    if ws[i] == 0.0 or used[0] + ws[i] <= budget or used[0] == 0.0:
                        used[0] += ws[i]
                        return pending.pop(k)
                cv.wait()
            return None

    def worker(small: bool):
        while True:
            i = take(small)
            if i is None:
                return
            try:
                out[i] = solver(cfg, secs[i], opt, device)
            except BaseException as e:  # noqa: BLE001 - re-raised by the caller
                with cv:
                    err.append(e)
            finally:
                with cv:
                    used[0] -= ws[i]
                    if used[0] < 1.0:
                        used[0] = 0.0
                    cv.notify_all()

    nw = min(opt.workers, len(secs))
    threads = [threading.Thread(target=worker, args=(w < min(opt.small_workers, nw - 1),), daemon=True)
               for w in range(nw)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if err:
        raise err[0]
    return out


def with_batch(cfg: EDConfig, bsecs: List[SectorId], opt: DiagOptions, device: int, fn, batch_solver=None):
    """Run fn() (the other sectors' workers) while one more host thread
    solves `bsecs` with batch_solver (solve_batch); returns (fn(), batch
    results)."""
    import threading

    batch_solver = batch_solver or solve_batch
    box: List = [None, None]

    def run():
        try:
            box[0] = batch_solver(cfg, bsecs, opt, device)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            box[1] = e

    th = threading.Thread(target=run, daemon=True)
    th.start()
    try:
        rest = fn()
    finally:
        th.join()
    if box[1] is not None:
        raise box[1]
    return rest, box[0]


def ed_diag(cfg: EDConfig, opt: Optional[DiagOptions] = None,
            sectors: Optional[Iterable[int]] = None, device: int = 0):
    """Diagonalise all (or the given) sectors; returns (results, state_list)."""
    opt = opt or DiagOptions()
    secs = diag_sectors(cfg)
    pick = set(sectors) if sectors is not None else None
    todo = [sec for sec in secs if pick is None or sec.isector in pick]
    results = solve_many(cfg, todo, opt, device)
    return results, retain_state_vectors(state_list(results, opt), results, drop_blocks=not opt.retain_all)


def eigenvalues_table(results: Iterable[SectorResult]) -> Dict[int, np.ndarray]:
    """eigenvalues_list.ed content (ED_DIAG.f90:238-242): Neigen per sector."""
    return {r.isector: np.asarray(r.eigenvalues[: r.neigen]) for r in results}
