"""Within-sector split kernels (ed_sector_kron_rows / _cols):
the two-pass Kronecker kernels serve the split on sectors that have the
two-pass tables (k_kron_up on a rank's row block, k_kron_dw on a DimDw x nu
column strip with row length nu).  Same products in the same order as the
one-thread-per-row k_kron_rows / k_kron_cols: bit-identical, for every row
block / strip of a 3-rank split, real and complex vectors, with and without
accumulation into the strip.  kron2=True builds the two-pass tables on these
small sectors; the split_simple option selects the simple kernels."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _call(S, fn, vt, a, b, x, y, acc=None):
    from edgpu import _lib
    from edgpu._lib import check

    L = _lib.load()
    st = torch.cuda.current_stream()
    args = [S.handle, vt, a, b, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr())]
    if acc is not None:
        args.append(acc)
    args.append(ctypes.c_void_p(st.cuda_stream))
    check(getattr(L, fn)(*args), fn)


@pytest.mark.parametrize("cfg_kw,q", [
    (dict(Norb=1, Nbath=7, bath="random", seed=3), (4, 4)),
    (dict(Norb=2, Nbath=4, bath="random", seed=4), (3, 6)),       # DimUp != DimDw
])
@pytest.mark.parametrize("cvec", [False, True])
def test_split_kernels_bit_identical(cfg_kw, q, cvec):
    from edgpu.dist import split
    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config

    cfg = make_config(**cfg_kw)
    with Sector(cfg, q[0], q[1], stored=False, direct=True, real=True, kron2=True) as S:
        du, dd = int(S.info.dimup), int(S.info.dimdw)
        vt = 1 if cvec else 0
        i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
        x = torch.complex(torch.sin(i), torch.cos(3 * i)) if cvec else torch.sin(i)
        X = x.view(dd, du)
        w0s, nws = split(dd, 3)
        u0s, nus = split(du, 3)
        for w0, nw in zip(w0s, nws):
            xb = X[w0:w0 + nw].reshape(-1).contiguous()
            out = []
            for simple in (False, True):
                S.set_options(*(("split_simple",) if simple else ()))
                y = torch.empty_like(xb)
                _call(S, "ed_sector_kron_rows", vt, w0, nw, xb, y)
                out.append(y)
            torch.cuda.synchronize()
            assert torch.equal(out[0], out[1]), f"rows [{w0},{w0 + nw})"
        for u0, nu in zip(u0s, nus):
            z = X[:, u0:u0 + nu].contiguous().reshape(-1)
            seed = torch.cos(torch.arange(z.numel(), dtype=torch.float64, device="cuda")).to(z.dtype)
            for acc in (0, 1):
                out = []
                for simple in (False, True):
                    S.set_options(*(("split_simple",) if simple else ()))
                    yz = seed.clone()
                    _call(S, "ed_sector_kron_cols", vt, u0, nu, z, yz, acc)
                    out.append(yz)
                torch.cuda.synchronize()
                assert torch.equal(out[0], out[1]), f"cols [{u0},{u0 + nu}) acc={acc}"
        S.set_options()
        # and the assembled split product equals the whole-sector H·v to rounding
        y_full = torch.empty_like(x)
        S.hxv_dev(x, y_full, path=2)
        Y = torch.empty(dd, du, dtype=x.dtype, device="cuda")
        for w0, nw in zip(w0s, nws):
            yb = torch.empty(nw * du, dtype=x.dtype, device="cuda")
            _call(S, "ed_sector_kron_rows", vt, w0, nw, X[w0:w0 + nw].reshape(-1).contiguous(), yb)
            Y[w0:w0 + nw] = yb.view(nw, du)
        for u0, nu in zip(u0s, nus):
            z = X[:, u0:u0 + nu].contiguous().reshape(-1)
            yz = torch.empty_like(z)
            _call(S, "ed_sector_kron_cols", vt, u0, nu, z, yz, 0)
            Y[:, u0:u0 + nu] += yz.view(dd, nu)
        torch.cuda.synchronize()
        ref = y_full.cpu().numpy()
        got = Y.reshape(-1).cpu().numpy()
        assert np.max(np.abs(got - ref)) <= 1e-13 * np.max(np.abs(ref))
