"""Sector / seed farm over ranks: one process per GPU, torch.distributed.

The reference loops over sectors on every rank and splits each sector's rows
across MPI ranks, with an MPI_Allgatherv of the whole vector on every H·v
(ED_HAMILTONIAN_STORED_HxV.f90:147-197).  Sectors are independent
(ED_DIAG.f90:71-249), so here whole sectors go to ranks instead:

  * a dynamic schedule (default at N > 1): every rank's worker threads take
    the next sector, largest modelled cost first, from one global counter in
    the process group's key-value store (an atomic add per sector — no
    collective, no data), so the ranks finish together even where the cost
    model is off; or the static longest-processing-time partition by that
    model (`DiagOptions.farm_schedule = "lpt"`);
  * each rank diagonalises its sectors on its own GPU — no collective in the
    data path;
  * one all_gather of the per-sector eigenvalues (KB), after which every rank
    replays the T=0 state-list logic in isector order, so the result is
    identical to the serial loop;
  * ground-state vectors stay on their owner rank; `broadcast_vector` ships one
    to every rank (RCCL broadcast over xGMI, 16*dim bytes) for the
    Green's-function seed farm.

The collective backend is whatever process group is initialised (nccl = RCCL
on the GPU box, gloo in the CPU tests).
"""
from __future__ import annotations

from dataclasses import replace
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from .diag import DiagOptions, SectorResult, StateList, lanczos_params, retain_state_vectors, state_list
from .params import EDConfig
from .sectors import Sector as SectorId
from .sectors import diag_sectors


def _dist():
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


def sector_cost(cfg: EDConfig, sec: SectorId, opt: DiagOptions) -> float:
    """Work model in seconds of one MI355X: a fixed cost per sector (build,
    launches, host syncs) plus a part proportional to the H·v work.
    Dense sectors: 2 ms + dim^3 x 1e-10 (LAPACK); Lanczos sectors: 7.0 ms +
    9.1e-12 x Nitermax x dim x (1 + elements per row), elements/row ~ 1 +
    Norb*Nbath.  Least-squares fit to the 136 serial Lanczos sector times of
    configs[3] (create + eigh + close; round 6 with the converged-and-interval
    screen seeded by the next Ritz vector: profiles/r6/farm_c4_serial_stats.json,
    the first sector's one-off library warm-up left out; round 5: 6.7 ms +
    9.8e-12 with the residual-interval exit; round 4: 8.0 ms +
    9.8e-12, earlier 8.5 ms + 1.18e-11, round 3: 9.4 ms + 1.13e-11, round 2:
    11.2 ms + 1.34e-11): small Lanczos sectors are dominated by the fixed
    part, which a purely proportional model gave to the ranks holding many
    of them.  Only ratios matter (LPT, and the dynamic schedule's order)."""
    neigen, nitermax, _ = lanczos_params(sec.dim, opt)
    if neigen == sec.dim or sec.dim <= max(opt.lanc_dim_threshold, opt.mpi_size):
        return 2e-3 + float(sec.dim) ** 3 * 1e-10
    per_row = 1.0 + cfg.Norb * cfg.Nbath
    return 7.0e-3 + 9.06e-12 * float(nitermax) * sec.dim * per_row


def lpt_partition(costs: Sequence[float], nranks: int) -> List[List[int]]:
    """Longest processing time first: items (indices) to the least-loaded rank."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    loads = [0.0] * nranks
    parts: List[List[int]] = [[] for _ in range(nranks)]
    for i in order:
        r = min(range(nranks), key=lambda k: (loads[k], k))
        parts[r].append(i)
        loads[r] += costs[i]
    return [sorted(p) for p in parts]


class FarmResult:
    def __init__(self, states: StateList, owners: List[int], tables: Dict[int, np.ndarray],
                 local: Dict[int, SectorResult], assignment: List[List[int]]):
        self.states = states          # vectors present only for states owned by this rank
        self.owners = owners          # rank owning each state's vector
        self.eigenvalues = tables     # isector -> Neigen eigenvalues (all ranks)
        self.local = local            # isector -> SectorResult solved here
        self.assignment = assignment  # rank -> isectors


def farm_diag(cfg: EDConfig, opt: Optional[DiagOptions] = None, *, device: int = 0,
              sectors: Optional[Sequence[int]] = None,
              solver: Optional[Callable[[EDConfig, SectorId, DiagOptions, int], SectorResult]] = None,
              batch_solver: Optional[Callable[[EDConfig, List[SectorId], DiagOptions, int], List[SectorResult]]] = None
              ) -> FarmResult:
    """ed_diag over all ranks of the default process group (or serially).
    solver: one sector's solve (default solve_sector); batch_solver: the
    `batchable` small sectors' joint solve (default solve_batch with the
    default solver, none with another solver unless given)."""
    from .diag import batchable, solve_batch, solve_many, solve_sector, with_batch

    opt = opt or DiagOptions()
    solver = solver or solve_sector
    if batch_solver is None and solver is solve_sector:
        batch_solver = solve_batch
    dist = _dist()
    rank = dist.get_rank() if dist else 0
    world = dist.get_world_size() if dist else 1
    secs = [s for s in diag_sectors(cfg) if sectors is None or s.isector in set(sectors)]
    local: Dict[int, SectorResult] = {}
    dynamic = bool(dist and world > 1 and opt.farm_schedule == "dynamic")
    # dynamic queue: the small sectors solve_batch takes are dealt to the
    # ranks up front (LPT on the cost model: the same on every rank), each
    # rank's share in one batch beside its queue workers; the queue holds
    # the others
    bsecs: List[SectorId] = []
    if dynamic and batch_solver is not None and opt.batch_max_dim > 0:
        bsecs = [s for s in secs if batchable(cfg, s, opt)]
        if len(bsecs) > 1:
            bset = {s.isector for s in bsecs}
            secs_q = [s for s in secs if s.isector not in bset]
        else:
            bsecs, secs_q = [], secs
    else:
        secs_q = secs
    costs = [sector_cost(cfg, s, opt) for s in secs_q]
    take = _global_queue(dist, len(secs_q)) if dynamic else None
    if take is not None:
        order = sorted(range(len(secs_q)), key=lambda i: (-costs[i], i))   # the same on every rank
        qsecs = [secs_q[i] for i in order]
        opt_q = replace(opt, batch_max_dim=0)
        bparts = lpt_partition([sector_cost(cfg, s, opt) for s in bsecs], world)
        mine_b = [bsecs[i] for i in bparts[rank]]
        run_q = lambda: solve_many(cfg, qsecs, opt_q, device, solver=solver, take_global=take)  # noqa: E731
        if len(mine_b) > 0:
            rq, rb = with_batch(cfg, mine_b, opt, device, run_q, batch_solver)
        else:
            rq, rb = run_q(), []
        for r in list(rq) + list(rb):
            if r is not None:
                local[r.isector] = r
        assignment = None   # from the gathered tables below
    else:
        parts = lpt_partition(costs, world)
        assignment = [[secs[i].isector for i in p] for p in parts]
        mine = [secs[i] for i in parts[rank]]
        for r in solve_many(cfg, mine, opt, device, solver=solver, cost=lambda s: sector_cost(cfg, s, opt),
                            batch_solver=batch_solver):
            local[r.isector] = r
    # gather eigenvalues (tiny) from every rank
    mine = {k: (v.q, v.dim, v.neigen, np.asarray(v.eigenvalues[: max(v.neigen, 1)])) for k, v in local.items()}
    if dist:
        allt: List[Optional[dict]] = [None] * world
        dist.all_gather_object(allt, mine)
    else:
        allt = [mine]
    merged: Dict[int, tuple] = {}
    owner_of: Dict[int, int] = {}
    for rk, t in enumerate(allt):
        for k, v in t.items():
            if k in merged:
                raise RuntimeError(f"farm_diag: sector {k} solved by ranks {owner_of[k]} and {rk}")
            merged[k] = v
            owner_of[k] = rk
    missing = sorted({s.isector for s in secs} - set(merged))
    if missing:
        raise RuntimeError(f"farm_diag: sectors {missing[:8]} (of {len(missing)}) solved by no rank")
    if assignment is None:
        assignment = [sorted(k for k, o in owner_of.items() if o == r) for r in range(world)]
    shadows = []
    for k, (q, dim, neigen, ev) in merged.items():
        loc = local.get(k)
        shadows.append(SectorResult(k, q, dim, ev, neigen, loc.vectors if loc is not None else None))
    states = retain_state_vectors(state_list(shadows, opt), list(local.values()), drop_blocks=not opt.retain_all)
    owners = [owner_of[s] for s in states.sectors]
    tables = {k: v[3] for k, v in merged.items()}
    return FarmResult(states, owners, tables, local, assignment)


_QUEUE_CALLS = [0]
_QUEUE_STORE: list = []      # [store] once connected, [None] once found unusable
QUEUE_FALLBACK: list = []    # reasons the dynamic schedule fell back to LPT (for logs / tests)


def _queue_store(dist):
    """A client of the job's rendezvous key-value server, through the public
    torch.distributed.TCPStore API: MASTER_ADDR:MASTER_PORT is the server that
    torchrun's agent (or rank 0's env:// init) keeps alive for the whole job.
    Every rank connects as a client (is_master=False); keys live under the
    prefix "edgpu_farm/<TORCHELASTIC_RUN_ID>/<TORCHELASTIC_RESTART_COUNT>/" (the
    agent's store outlives an elastic restart; each farm call's counter key
    is moreover unique, _global_queue).  None (and the reason recorded) when the variables are
    absent or the connection fails: the farm then runs the static LPT
    partition, which needs no store."""
    if _QUEUE_STORE:
        return _QUEUE_STORE[0]
    import datetime
    import os
    import sys

    addr, port = os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")
    store, why = None, None
    if not addr or not port:
        why = "MASTER_ADDR/MASTER_PORT not set (process group not from env://)"
    else:
        try:
            tcp = dist.TCPStore(addr, int(port), is_master=False, timeout=datetime.timedelta(seconds=60))
            run = os.environ.get("TORCHELASTIC_RUN_ID", "none")
            attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
            store = dist.PrefixStore(f"edgpu_farm/{run}/{attempt}/", tcp)
        except Exception as e:   # noqa: BLE001 - any connection failure means: no dynamic queue
            why = f"TCPStore({addr}:{port}) client failed: {type(e).__name__}: {e}"
    if store is None:
        QUEUE_FALLBACK.append(why)
        print(f"edgpu.farm: dynamic sector queue unavailable ({why}); using the LPT partition",
              file=sys.stderr, flush=True)
    _QUEUE_STORE.append(store)
    return store


def _global_queue(dist, n: int):
    """Work queue over the ranks of the default group: `take()` returns the
    next of n indices (0, 1, ...) or None.  One counter key per farm call
    (every rank makes the same sequence of farm_diag calls, so the keys
    agree); the store's add is atomic, each index goes to exactly one taker.
    The key carries a token rank 0 draws and all-reduces per call, so a
    counter left on the store by an earlier call or job attempt is never
    reused.  A barrier first, so no rank takes from the counter of a call the others
    have not reached.  Returns None when no store is reachable (every rank
    decides the same way: a collective agreement on the store's availability
    precedes the first use, so ranks never mix the two schedules)."""
    import threading
    import uuid

    import torch

    store = _queue_store(dist)
    # [store reachable (MIN over ranks), rank 0's random token (the others add
    # 0)]: a counter key no earlier call — nor an earlier incarnation of this
    # job on the same store — can have used; one all_reduce per flag
    ok = torch.tensor([1 if store is not None else 0], dtype=torch.int64)
    tok = torch.tensor([uuid.uuid4().int & ((1 << 62) - 1) if dist.get_rank() == 0 else 0], dtype=torch.int64)
    if dist.get_backend() == "nccl":
        ok, tok = ok.cuda(), tok.cuda()
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        return None
    dist.all_reduce(tok, op=dist.ReduceOp.SUM)
    _QUEUE_CALLS[0] += 1
    key = f"queue_{_QUEUE_CALLS[0]}_{int(tok.item()):x}"
    dist.barrier()
    lock = threading.Lock()   # one store client per process: serialise its use
    done = [False]

    def take():
        if done[0]:
            return None
        with lock:
            i = int(store.add(key, 1)) - 1
        if i >= n:
            done[0] = True
            return None
        return i
    return take


def broadcast_vector(vec, owner: int, dim: int, cplx: bool, device: Optional[int] = None):
    """Ship one eigenvector from its owner to every rank.  nccl (RCCL over
    xGMI): the device tensor is broadcast in place and stays in HBM on every
    rank (a host array on the owner is uploaded first).  gloo (CPU tests):
    host tensors, returned as numpy."""
    dist = _dist()
    if dist is None:
        return vec
    import torch

    dt = torch.complex128 if cplx else torch.float64
    on_gpu = dist.get_backend() == "nccl"
    dev = torch.device("cuda", device if device is not None else torch.cuda.current_device()) if on_gpu \
        else torch.device("cpu")
    if dist.get_rank() == owner:
        if isinstance(vec, np.ndarray):
            t = torch.from_numpy(np.ascontiguousarray(vec).astype(np.complex128 if cplx else np.float64))
        else:
            t = vec
        t = t.to(device=dev, dtype=dt).contiguous()
    else:
        t = torch.empty(dim, dtype=dt, device=dev)
    dist.broadcast(t, src=owner)
    return t if on_gpu else t.numpy()
