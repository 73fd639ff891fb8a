"""Within-sector multi-GPU H·v.

The reference splits one sector's rows over MPI ranks and all-gathers the
whole vector before every product (ED_HAMILTONIAN.f90:55-62,
ED_HAMILTONIAN_STORED_HxV.f90:147-197: spMatVec_mpi_cc).  For the normal-mode
Hamiltonian without Jx/Jp the sector factorises,

    H = D + Hup (x) 1 + 1 (x) Hdw      on the DimDw x DimUp view of v,

so a rank that owns down rows [w0, w0+nw) applies D and the up-spin hops to
its own block, and the down-spin hops — which mix rows — run on the
transposed view, where each rank owns up columns [u0, u0+nu):

    y  = rows(x)                                  ed_sector_kron_rows (HIP)
    z  = strip(x)                                 all_to_all over RCCL/xGMI
    yz = cols(z)                                  ed_sector_kron_cols (HIP)
    y += unstrip(yz)                              all_to_all

The strip is the DimDw x nu block of the rank's up columns, row-major: the
row blocks an all-to-all delivers are already in that order, so neither
exchange needs a transpose (only a column slice/scatter of the local block).

Each H·v moves 2·(P-1)/P of the local block per rank instead of the
reference's full-vector Allgatherv (P·x the local block), and every rank
holds only its 1/P of v.  `dist_lanczos` runs the plain recurrence
(.repo/PLAIN_LANCZOS.f90:87-118) on the split vector with two all-reduces of
scalars per step.

Any other sector (superc, nonsu2, Jx/Jp, Jz_basis ...) uses `DistRowSector`:
the reference's own layout — each rank builds rows [r0, r0+n) of the stored
(or matrix-free generic) H on its GPU (ed_sector_create_rows).  Instead of
spMatVec_mpi_cc's whole-vector Allgatherv it exchanges a halo: at
construction every rank lists the columns its rows refer to
(ed_sector_col_mask), sends each owner the list of its entries it needs, and
per H·v one all-to-all moves exactly those entries, scattered into a
full-length scratch vector before the local product (same values at every
column the rows read: bit-identical to the Allgatherv product).

The collective backend is the default process group (nccl = RCCL on the GPU
box; gloo in the CPU tests, where `ops` injects reference factor products).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import check


def _dist():
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


def split(n: int, parts: int) -> Tuple[List[int], List[int]]:
    """Contiguous near-even split: (starts, counts)."""
    base, extra = divmod(n, parts)
    counts = [base + (1 if p < extra else 0) for p in range(parts)]
    starts = [int(x) for x in np.concatenate([[0], np.cumsum(counts)[:-1]])]
    return starts, counts


class DeviceKronOps:
    """The two factor products on the GPU (ed_sector_kron_rows / _cols)."""

    accumulates = True   # cols(..., into=y) adds in place

    def __init__(self, S):
        self.S = S
        self.dimup = int(S.info.dimup)
        self.dimdw = int(S.info.dimdw)

    def _args(self, x, y):
        import torch

        st = torch.cuda.current_stream(x.device)
        return ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(st.cuda_stream)

    def rows(self, w0: int, nw: int, x):
        import torch

        y = torch.empty_like(x)
        xp, yp, sp = self._args(x, y)
        vt = 1 if x.is_complex() else 0
        check(_lib.load().ed_sector_kron_rows(self.S.handle, vt, w0, nw, xp, yp, sp), "ed_sector_kron_rows")
        return y

    def cols(self, u0: int, nu: int, xt, into=None):
        """Hdw on the strip; into: add to this tensor in place (same layout)."""
        import torch

        yt = torch.empty_like(xt) if into is None else into
        xp, yp, sp = self._args(xt, yt)
        vt = 1 if xt.is_complex() else 0
        check(_lib.load().ed_sector_kron_cols(self.S.handle, vt, u0, nu, xp, yp, 0 if into is None else 1, sp),
              "ed_sector_kron_cols")
        return yt


class DistKronSector:
    """One sector split by down rows over the ranks of the default process
    group (or serial).  Vectors are 1-D torch tensors holding this rank's
    nw x DimUp block (row-major = the reference's row order)."""

    def __init__(self, cfg=None, q1: int = 0, q2: int = 0, *, device: int = 0, real: Optional[bool] = None,
                 ops=None):
        import torch

        dist = _dist()
        self.rank = dist.get_rank() if dist else 0
        self.world = dist.get_world_size() if dist else 1
        self._S = None
        if ops is None:
            from .hamiltonian import Sector

            real = cfg.is_real() if real is None else real
            self._S = Sector(cfg, q1, q2, stored=False, direct=True, real=real, device=device)
            if not self._S.info.kron:
                self._S.close()
                raise ValueError("within-sector split needs the Kronecker form (normal mode, no Jx/Jp)")
            ops = DeviceKronOps(self._S)
            self.dtype = torch.float64 if real else torch.complex128
            self.device = torch.device("cuda", device)
        else:
            self.dtype = getattr(ops, "dtype", torch.complex128)
            self.device = getattr(ops, "device", torch.device("cpu"))
        self.ops = ops
        self.du, self.dd = ops.dimup, ops.dimdw
        self.w0, self.nw = split(self.dd, self.world)
        self.u0, self.nu = split(self.du, self.world)
        self.comm_cpu = dist is not None and dist.get_backend() != "nccl"

    # ------------------------------------------------------------- layout
    @property
    def local_rows(self) -> Tuple[int, int]:
        return self.w0[self.rank], self.nw[self.rank]

    @property
    def local_dim(self) -> int:
        return self.nw[self.rank] * self.du

    def scatter(self, v_full):
        """This rank's block of a full vector (tests, start vectors)."""
        w0, nw = self.local_rows
        return v_full[w0 * self.du:(w0 + nw) * self.du].contiguous()

    def gather(self, v_loc):
        """Full vector on every rank (tests only: the point is not to need it)."""
        import torch

        dist = _dist()
        if dist is None:
            return v_loc
        m = max(self.nw) * self.du           # equal-size all_gather (gloo needs it): pad
        pad = torch.zeros(m, dtype=v_loc.dtype, device=v_loc.device)
        pad[:v_loc.numel()] = v_loc
        parts = [torch.empty(m, dtype=v_loc.dtype, device=v_loc.device) for _ in self.nw]
        if self.comm_cpu:
            cpu = [p.cpu() for p in parts]
            dist.all_gather(cpu, pad.cpu())
            parts = [p.to(v_loc.device) for p in cpu]
        else:
            dist.all_gather(parts, pad)
        parts = [p[:n * self.du] for p, n in zip(parts, self.nw)]
        return torch.cat(parts)

    # ------------------------------------------------------ communication
    def _a2a(self, send, in_splits, out_splits):
        import torch

        dist = _dist()
        if dist is None:
            return send
        recv = torch.empty(sum(out_splits), dtype=send.dtype, device=send.device)
        if self.comm_cpu:
            r = recv.cpu()
            dist.all_to_all_single(r, send.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits)
            return r.to(send.device)
        dist.all_to_all_single(recv, send, output_split_sizes=out_splits, input_split_sizes=in_splits)
        return recv

    def to_cols(self, x):
        """Row block (nw_r x du) -> the DimDw x nu_r strip of this rank's up
        columns.  Block q of the send buffer is X[:, cols of q]; what arrives
        from ranks 0..P-1 (down rows in rank order) is the strip row-major."""
        import torch

        r, P = self.rank, self.world
        if P == 1:
            return x
        X = x.view(self.nw[r], self.du)
        send = torch.cat([X[:, self.u0[q]:self.u0[q] + self.nu[q]].reshape(-1) for q in range(P)])
        return self._a2a(send, [self.nw[r] * self.nu[q] for q in range(P)],
                         [self.nw[q] * self.nu[r] for q in range(P)])

    def to_rows(self, yz):
        """DimDw x nu_r strip -> this rank's row block: the strip's row block q
        goes to rank q as is; the blocks received are scattered into columns."""
        import torch

        r, P = self.rank, self.world
        if P == 1:
            return yz
        recv = self._a2a(yz, [self.nw[q] * self.nu[r] for q in range(P)],
                         [self.nw[r] * self.nu[q] for q in range(P)])
        Y = torch.empty(self.nw[r], self.du, dtype=yz.dtype, device=yz.device)
        off = 0
        for q in range(P):
            n = self.nw[r] * self.nu[q]
            Y[:, self.u0[q]:self.u0[q] + self.nu[q]] = recv[off:off + n].view(self.nw[r], self.nu[q])
            off += n
        return Y.reshape(-1)

    # ----------------------------------------------------------------- H·v
    def hxv(self, x):
        """H·v on the split vector (spMatVec_mpi_cc semantics)."""
        r = self.rank
        y = self.ops.rows(self.w0[r], self.nw[r], x)
        if self.world == 1 and getattr(self.ops, "accumulates", False):
            # one rank: the strip is the whole view, so the down-spin sum goes
            # straight into y (no exchange, no separate add)
            return self.ops.cols(0, self.du, x, into=y)
        yt = self.ops.cols(self.u0[r], self.nu[r], self.to_cols(x))
        return y + self.to_rows(yt)

    def close(self):
        if self._S is not None:
            self._S.close()
            self._S = None


def mpi_split(n: int, parts: int) -> Tuple[List[int], List[int]]:
    """build_Hv_sector's row split (ED_HAMILTONIAN.f90:55-62): mpiQ = n/parts
    rows per rank, the remainder on the last rank."""
    q = n // parts
    starts = [r * q for r in range(parts)]
    counts = [q + (n % parts if r == parts - 1 else 0) for r in range(parts)]
    return starts, counts


class DistRowSector:
    """One sector split by rows over the ranks of the default process group,
    any ed_mode (build_Hv_sector with MpiStatus, ED_HAMILTONIAN.f90:55-62,
    `mpi_split`).
    Vectors are 1-D tensors holding this rank's rows; H·v applies the local
    rows with global columns to a full-length vector that holds this rank's
    entries and the halo — the entries of other ranks its rows refer to,
    received by one all-to-all (halo=True, default) — or the whole
    all-gathered vector (halo=False: spMatVec_mpi_cc's Allgatherv,
    STORED_HxV.f90:175-189).  `hxv_rows` (injectable, CPU tests) maps a
    whole vector to the local rows of H·v; `cols_needed` then lists the
    global columns those rows refer to."""

    def __init__(self, cfg=None, q1: int = 0, q2: int = 0, *, device: int = 0, real: Optional[bool] = None,
                 stored: bool = True, hxv_rows=None, dim: Optional[int] = None, dtype=None,
                 halo: bool = True, cols_needed=None):
        import torch

        dist = _dist()
        self.rank = dist.get_rank() if dist else 0
        self.world = dist.get_world_size() if dist else 1
        self._S = None
        if hxv_rows is None:
            from .hamiltonian import Sector
            from .sectors import sector_dim

            real = cfg.is_real() if real is None else real
            dim = sector_dim(cfg, q1, q2)
            r0, n = mpi_split(dim, self.world)
            self._S = Sector(cfg, q1, q2, stored=stored, direct=not stored, real=real, device=device,
                             rows=(r0[self.rank], n[self.rank]))
            self.dtype = torch.float64 if real else torch.complex128
            self.device = torch.device("cuda", device)
            S = self._S

            def hxv_rows(v):
                y = torch.empty(S.nrows, dtype=v.dtype, device=v.device)
                S.hxv_dev(v, y)
                return y

            if halo and self.world > 1:
                mask = torch.empty((dim + 31) // 32, dtype=torch.int32, device=self.device)
                st = torch.cuda.current_stream(self.device)
                check(_lib.load().ed_sector_col_mask(S.handle, ctypes.c_void_p(mask.data_ptr()),
                                                     ctypes.c_void_p(st.cuda_stream)), "ed_sector_col_mask")
                bits = np.unpackbits(mask.cpu().numpy().view(np.uint8), bitorder="little")
                cols_needed = np.flatnonzero(bits[:dim])
        else:
            self.dtype = dtype or torch.complex128
            self.device = torch.device("cpu")
        self.dim = dim
        self.r0, self.n = mpi_split(dim, self.world)
        self._rows = hxv_rows
        self.comm_cpu = dist is not None and dist.get_backend() != "nccl"
        self.halo = bool(halo and self.world > 1)
        if self.halo:
            if cols_needed is None:
                raise ValueError("halo exchange needs the columns the local rows refer to")
            self._setup_halo(np.asarray(cols_needed, dtype=np.int64))

    # ----------------------------------------------------------------- halo
    def _a2a(self, send, in_splits, out_splits):
        import torch

        dist = _dist()
        recv = torch.empty(sum(out_splits), dtype=send.dtype, device=send.device)
        if self.comm_cpu:
            r = recv.cpu()
            dist.all_to_all_single(r, send.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits)
            return r.to(send.device)
        dist.all_to_all_single(recv, send, output_split_sizes=out_splits, input_split_sizes=in_splits)
        return recv

    def _setup_halo(self, cols):
        """Who needs which of my entries: every rank sends each owner the
        (sorted) global columns it needs from it; the owner keeps them as
        local indices.  Two all-to-alls, once per sector."""
        import torch

        P, r = self.world, self.rank
        lo, hi = self.r0[r], self.r0[r] + self.n[r]
        cols = np.unique(cols)
        cols = cols[(cols < lo) | (cols >= hi)]
        starts = np.asarray(self.r0, dtype=np.int64)
        owner = np.searchsorted(starts, cols, side="right") - 1
        need = [cols[owner == q] for q in range(P)]
        cnt = torch.tensor([len(x) for x in need], dtype=torch.int64, device=self.device)
        got = self._a2a(cnt, [1] * P, [1] * P).cpu().numpy()
        req = torch.from_numpy(np.concatenate(need).astype(np.int64)).to(self.device)
        want = self._a2a(req, [len(x) for x in need], [int(c) for c in got])
        self._send_idx = (want - lo).to(torch.int64)           # my entries, grouped by destination rank
        self._send_splits = [int(c) for c in got]
        self._recv_splits = [len(x) for x in need]
        self._halo_cols = req                                    # global columns, in arrival order
        self._xfull = None
        self.halo_size = int(req.numel())

    def _with_halo(self, x):
        import torch

        if self._xfull is None or self._xfull.dtype != x.dtype:
            self._xfull = torch.zeros(self.dim, dtype=x.dtype, device=x.device)
        recv = self._a2a(x.index_select(0, self._send_idx), self._send_splits, self._recv_splits)
        r0, n = self.local_rows
        self._xfull[r0:r0 + n] = x
        self._xfull.index_copy_(0, self._halo_cols, recv)
        return self._xfull

    @property
    def local_rows(self) -> Tuple[int, int]:
        return self.r0[self.rank], self.n[self.rank]

    @property
    def local_dim(self) -> int:
        return self.n[self.rank]

    def scatter(self, v_full):
        r0, n = self.local_rows
        return v_full[r0:r0 + n].contiguous()

    def gather(self, v_loc):
        """Allgatherv of the split vector (equal-size all_gather of padded
        blocks: RCCL and gloo both take it)."""
        import torch

        dist = _dist()
        if dist is None:
            return v_loc
        m = max(self.n)
        pad = torch.zeros(m, dtype=v_loc.dtype, device=v_loc.device)
        pad[:v_loc.numel()] = v_loc
        parts = [torch.empty(m, dtype=v_loc.dtype, device=v_loc.device) for _ in self.n]
        if self.comm_cpu:
            cpu = [p.cpu() for p in parts]
            dist.all_gather(cpu, pad.cpu())
            parts = [p.to(v_loc.device) for p in cpu]
        else:
            dist.all_gather(parts, pad)
        return torch.cat([p[:k] for p, k in zip(parts, self.n)])

    def hxv(self, x):
        if self.halo:
            return self._rows(self._with_halo(x))
        return self._rows(self.gather(x))

    def close(self):
        if self._S is not None:
            self._S.close()
            self._S = None


def _allreduce_sum(t):
    dist = _dist()
    if dist is None:
        return t
    if dist.get_backend() != "nccl":
        c = t.cpu()
        dist.all_reduce(c)
        return c.to(t.device)
    dist.all_reduce(t)
    return t


def dist_lanczos(ds, v0_loc, nitermax: int, threshold: float = 1e-13):
    """sp_lanc_tridiag on the split vector: (alfa, beta, nlanc); beta[0] = 0,
    beta[k+1] couples k, k+1 (.repo/PLAIN_LANCZOS.f90:87-118, 154-180)."""
    import torch

    v = v0_loc.clone()
    nrm = _allreduce_sum(torch.sum(torch.abs(v) ** 2).reshape(1).to(torch.float64))
    v = v / torch.sqrt(nrm).to(v.dtype)
    vo = torch.zeros_like(v)
    b = 0.0
    alfa = np.zeros(nitermax)
    beta = np.zeros(nitermax + 1)
    n = 0
    for it in range(nitermax):
        w = ds.hxv(v) - b * vo
        a = float(_allreduce_sum(torch.sum(torch.conj(v) * w).real.reshape(1).to(torch.float64)).item())
        w = w - a * v
        b = float(torch.sqrt(_allreduce_sum(torch.sum(torch.abs(w) ** 2).reshape(1).to(torch.float64))).item())
        alfa[it] = a
        beta[it + 1] = b
        n = it + 1
        if abs(b) < threshold:
            break
        vo = v
        v = w / b
    return alfa, beta, n
