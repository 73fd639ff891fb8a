"""Sector farm logic on CPU: LPT partition, world_size-2 gloo runs reproduce the
serial state list exactly, vector broadcast over the process group."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from edgpu.diag import DiagOptions
from edgpu.farm import farm_diag, lpt_partition, sector_cost
from edgpu.params import make_config
from edgpu.sectors import setup_pointers


def test_lpt_partition_balances_c4():
    cfg = make_config(Norb=2, Nbath=5)           # configs[3]: 169 sectors
    opt = DiagOptions()
    secs = setup_pointers(cfg)
    costs = [sector_cost(cfg, s, opt) for s in secs]
    for n in (1, 2, 4, 8):
        parts = lpt_partition(costs, n)
        assert sorted(i for p in parts for i in p) == list(range(len(secs)))
        loads = [sum(costs[i] for i in p) for p in parts]
        # LPT bound: max load <= mean + largest item
        assert max(loads) <= sum(costs) / n + max(costs) + 1e-9
        if n == 8:
            assert max(loads) / (sum(costs) / n) < 1.05   # ~8x achievable


@pytest.mark.parametrize("budget_mb", [0.0, 300.0])
def test_solve_many_cache_budget(budget_mb):
    """solve_many's scheduler: results in input order whatever the schedule;
    with a cache budget the working sets counted in flight never exceed it
    except for one sector alone (configs[3], a sleeping fake solver)."""
    import threading
    import time

    from edgpu.diag import SectorResult, solve_many, working_set_bytes

    cfg = make_config(Norb=2, Nbath=5)
    opt = DiagOptions(workers=8, cache_budget_mb=budget_mb)
    secs = setup_pointers(cfg)
    ws = {s.isector: working_set_bytes(cfg, s, opt) for s in secs}
    lock = threading.Lock()
    live, peaks = {}, []

    def solver(c, sec, o, device):
        w = ws[sec.isector] if ws[sec.isector] >= 16e6 else 0.0
        with lock:
            live[sec.isector] = w
            peaks.append((sum(live.values()), sum(1 for v in live.values() if v > 0)))
        time.sleep(1e-3 + 2e-11 * sec.dim)
        with lock:
            del live[sec.isector]
        return SectorResult(sec.isector, (sec.q1, sec.q2), sec.dim, np.zeros(1), 1)

    out = solve_many(cfg, secs, opt, solver=solver, cost=lambda s: sector_cost(cfg, s, opt))
    assert [r.isector for r in out] == [s.isector for s in secs]
    big = sum(1 for v in ws.values() if v >= 16e6)
    assert big >= 4                                   # the test has something to schedule
    if budget_mb > 0:
        assert all(tot <= budget_mb * 1e6 or n == 1 for tot, n in peaks)
    else:
        assert max(n for _, n in peaks) > 1


@pytest.mark.parametrize("small", [0, 2])
def test_solve_many_small_workers(small):
    """DiagOptions.small_workers: that many workers start from the cheapest
    pending sector, the rest from the most expensive; results in input order
    and each sector solved once either way."""
    import threading
    import time

    from edgpu.diag import SectorResult, solve_many

    cfg = make_config(Norb=2, Nbath=5)
    opt = DiagOptions(workers=4, small_workers=small)
    secs = setup_pointers(cfg)
    cost = {s.isector: sector_cost(cfg, s, opt) for s in secs}
    lock = threading.Lock()
    started = []
    gate = threading.Barrier(4)

    def solver(c, sec, o, device):
        with lock:
            started.append(sec.isector)
            first = len(started) <= 4
        if first:
            gate.wait(timeout=30)   # the four first picks are made before any finishes
        time.sleep(2e-4)
        return SectorResult(sec.isector, (sec.q1, sec.q2), sec.dim, np.zeros(1), 1)

    out = solve_many(cfg, secs, opt, solver=solver, cost=lambda s: cost[s.isector])
    assert [r.isector for r in out] == [s.isector for s in secs]
    assert sorted(started) == sorted(s.isector for s in secs)
    ranked = sorted(cost, key=lambda k: -cost[k])
    first = set(started[:4])
    assert set(ranked[:4 - small]) <= first
    if small:
        assert set(ranked[-small:]) <= first    # the cheapest ones start at once
    else:
        assert first == set(ranked[:4])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_batch(cfg, secs, opt, device):
    """Stand-in for solve_batch on CPU: the oracle solver per sector, tagged."""
    from oracle_solver import solve_sector_oracle

    out = []
    for s in secs:
        r = solve_sector_oracle(cfg, s, opt, device)
        r.method = "batch"
        out.append(r)
    return out


def _worker(rank, world, port, q, cfg_kw, method, schedule="dynamic", init="env", batch=False):
    import torch.distributed as dist
    from oracle_solver import solve_sector_oracle
    from edgpu.farm import QUEUE_FALLBACK, broadcast_vector

    if init in ("env", "stale"):
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:   # a file rendezvous: no MASTER_ADDR/PORT, so no key-value server to reach
        os.environ.pop("MASTER_ADDR", None)
        os.environ.pop("MASTER_PORT", None)
        dist.init_process_group("gloo", rank=rank, world_size=world, init_method=init)
    cfg = make_config(**cfg_kw)
    if init == "stale":
        # counters an earlier attempt of the job left on the agent's store
        # under the old fixed keys (queue_1, queue_2, ...): exhausted
        import datetime

        if rank == 0:
            tcp = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=30))
            old = dist.PrefixStore("edgpu_farm/none/0/", tcp)
            for k in range(1, 4):
                old.add(f"queue_{k}", 10_000)
        dist.barrier()
    res = farm_diag(cfg, DiagOptions(lanc_method=method, farm_schedule=schedule), solver=solve_sector_oracle,
                    batch_solver=_oracle_batch if batch else None)
    if init == "stale":   # a second farm call in the same job takes a fresh counter too
        res = farm_diag(cfg, DiagOptions(lanc_method=method, farm_schedule=schedule), solver=solve_sector_oracle)
    gs_owner = res.owners[0]
    v = res.states.vectors[0] if rank == gs_owner else None
    dim = [s for s in setup_pointers(cfg) if s.isector == res.states.sectors[0]][0].dim
    vb = broadcast_vector(v, gs_owner, dim, cplx=True)
    q.put((rank, res.states.energies, res.states.sectors, res.owners, res.assignment,
           float(np.linalg.norm(vb)), list(QUEUE_FALLBACK),
           sorted(k for k, r in res.local.items() if r.method == "batch")))
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(world, cfg_kw, method, schedule, init="env", batch=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, cfg_kw, method, schedule, init, batch))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


@pytest.mark.parametrize("world,init", [(4, "env"), (2, "file"), (2, "stale")])
def test_gloo_dynamic_queue(world, init, tmp_path):
    """The dynamic sector queue through the public TCPStore client: 4 ranks
    (processes) take sectors from one counter and reproduce the serial state
    list; with a file rendezvous (no MASTER_ADDR/PORT) every rank falls back
    to the LPT partition, says why, and still reproduces it; with exhausted
    counters left on the store by an earlier job attempt ("stale") each call
    still takes a fresh per-call key and solves every sector."""
    from oracle_solver import solve_sector_oracle

    cfg_kw, method = dict(Norb=1, Nbath=5), "lanczos"
    cfg = make_config(**cfg_kw)
    serial = farm_diag(cfg, DiagOptions(lanc_method=method), solver=solve_sector_oracle)
    init_arg = init if init in ("env", "stale") else f"file://{tmp_path}/rdzv"
    out = _run_ranks(world, cfg_kw, method, "dynamic", init_arg)
    for rank, en, secs, owners, assignment, vnorm, fallback, _ in out:
        assert secs == serial.states.sectors
        np.testing.assert_allclose(en, serial.states.energies, rtol=0, atol=1e-12)
        assert abs(vnorm - 1.0) < 1e-10
        if init in ("env", "stale"):
            assert fallback == []
        else:
            assert len(fallback) == 1 and "MASTER_ADDR" in fallback[0]
    assign = out[0][4]
    assert all(o[4] == assign for o in out)
    assert sorted(i for a in assign for i in a) == sorted(s.isector for s in setup_pointers(cfg))
    if init == "file":    # LPT: every rank got work
        assert all(len(a) > 0 for a in assign)


@pytest.mark.parametrize("schedule", ["dynamic", "lpt"])
@pytest.mark.parametrize("cfg_kw,method", [
    (dict(Norb=1, Nbath=4), "arpack"),                 # configs[0]: all sectors dense
    (dict(Norb=1, Nbath=5), "lanczos"),                # sectors > 256 through the Lanczos branch
    (dict(Norb=1, Nbath=3, Nspin=2, ed_mode="nonsu2"), "arpack"),
])
def test_gloo_farm_matches_serial(cfg_kw, method, schedule):
    from oracle_solver import solve_sector_oracle

    cfg = make_config(**cfg_kw)
    serial = farm_diag(cfg, DiagOptions(lanc_method=method), solver=solve_sector_oracle)
    out = _run_ranks(2, cfg_kw, method, schedule)
    for rank, en, secs, owners, assignment, vnorm, fallback, _ in out:
        assert fallback == []
        assert secs == serial.states.sectors
        np.testing.assert_allclose(en, serial.states.energies, rtol=0, atol=1e-12)
        assert abs(vnorm - 1.0) < 1e-10           # broadcast delivered the owner's unit vector
    # the assignment covers every sector once, the same on both ranks (LPT:
    # both ranks got work; the dynamic queue gives work to whoever takes it)
    assign = out[0][4]
    assert out[1][4] == assign
    if schedule == "lpt":
        assert all(len(a) > 0 for a in assign)
    assert sorted(i for a in assign for i in a) == sorted(s.isector for s in setup_pointers(cfg))


@pytest.mark.parametrize("schedule", ["dynamic", "lpt"])
def test_gloo_farm_with_batch(schedule):
    """Two ranks with the small-sector batch (a CPU stand-in batch solver):
    the dynamic queue deals the batchable sectors to the ranks up front (LPT
    on the cost model) and queues the others; the LPT schedule batches each
    rank's share beside its workers.  Every sector solved exactly once, the
    serial state list reproduced, both ranks batched some sectors."""
    from oracle_solver import solve_sector_oracle

    from edgpu.diag import batchable

    cfg_kw, method = dict(Norb=1, Nbath=5), "arpack"
    cfg = make_config(**cfg_kw)
    opt = DiagOptions(lanc_method=method)
    nb = sum(1 for s in setup_pointers(cfg) if batchable(cfg, s, opt))
    assert nb >= 4
    serial = farm_diag(cfg, opt, solver=solve_sector_oracle)
    out = _run_ranks(2, cfg_kw, method, schedule, batch=True)
    for rank, en, secs, owners, assignment, vnorm, fallback, batched in out:
        assert secs == serial.states.sectors
        np.testing.assert_allclose(en, serial.states.energies, rtol=0, atol=1e-12)
        assert len(batched) > 0
    assert sum(len(o[7]) for o in out) == nb
    assign = out[0][4]
    assert sorted(i for a in assign for i in a) == sorted(s.isector for s in setup_pointers(cfg))


def _gf_worker(rank, world, port, q, cfg_kw):
    import torch.distributed as dist
    from oracle_gf import oracle_job_runner
    from oracle_solver import solve_sector_oracle
    from edgpu.gf import GFOptions, build_gf

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = make_config(**cfg_kw)
    res = farm_diag(cfg, DiagOptions(lanc_method="lanczos"), solver=solve_sector_oracle)
    Gm, Gr = build_gf(cfg, res.states, GFOptions(Lmats=64, Lreal=64), owners=res.owners,
                      runner=oracle_job_runner)
    q.put((rank, Gm, Gr))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg_kw", [
    dict(Norb=1, Nbath=5, bath="random", seed=5),                       # normal, 2 seeds/state
    dict(Norb=1, Nbath=3, Nspin=2, ed_mode="nonsu2", bath="random", seed=2),  # 12 seeds/state
])
def test_gloo_gf_seed_farm_matches_serial(cfg_kw):
    """GF seed farm: jobs split over 2 gloo ranks (state vectors broadcast from
    their farm owner, G all-reduced) equal the serial oracle build."""
    from oracle_gf import build_gf_oracle
    from oracle_solver import solve_sector_oracle
    from edgpu.gf import GFOptions

    cfg = make_config(**cfg_kw)
    serial = farm_diag(cfg, DiagOptions(lanc_method="lanczos"), solver=solve_sector_oracle)
    Gm0, Gr0 = build_gf_oracle(cfg, serial.states, GFOptions(Lmats=64, Lreal=64))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gf_worker, args=(r, 2, port, q, cfg_kw)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, Gm, Gr in out:
        assert np.max(np.abs(Gm - Gm0)) / np.max(np.abs(Gm0)) < 1e-12
        assert np.max(np.abs(Gr - Gr0)) / np.max(np.abs(Gr0)) < 1e-12
