"""CPU tests of the host logic and of the C-ABI library's exports (no GPU calls)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from edgpu.params import EDConfig, EdParams, init_dmft_bath, make_config
from edgpu.sectors import c_sector, cdg_sector, setup_pointers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ed_gpu.h")
LIB = os.path.join(ROOT, "dmft-ed_amd", "libedgpu.so")


def test_flat_bath_literal_values():
    """init_dmft_bath, ED_BATH/dmft_aux.f90:103-135."""
    b = init_dmft_bath(EDConfig(Norb=1, Nbath=7))
    np.testing.assert_allclose(b.e[0, 0], [-2, -2 + 2 / 3, -2 + 4 / 3, 0, 2 - 4 / 3, 2 - 2 / 3, 2])
    np.testing.assert_allclose(b.v[0, 0], 1 / np.sqrt(7))
    b = init_dmft_bath(EDConfig(Norb=1, Nbath=4))
    np.testing.assert_allclose(b.e[0, 0], [-2, -1e-3, 1e-3, 2])
    b = init_dmft_bath(EDConfig(Norb=2, Nbath=6, Nspin=2, ed_mode="nonsu2"))
    np.testing.assert_allclose(b.e[1, 1], [-2, -1, -1e-3, 1e-3, 1, 2])
    np.testing.assert_allclose(b.u, 0.1 * b.v)
    b = init_dmft_bath(EDConfig(Norb=1, Nbath=5, ed_mode="superc"))
    np.testing.assert_allclose(b.d, 0.02)
    np.testing.assert_allclose(b.v, max(0.1, 1 / np.sqrt(5)))
    b = init_dmft_bath(EDConfig(Norb=2, Nbath=3, bath_type="replica"))
    assert b.h.shape == (1, 1, 2, 2, 3) and np.all(b.vr == 0.5)


def test_dimensions_and_sectors():
    pins = {"c1": (make_config(Norb=1, Nbath=4), 36, 100),
            "c4": (make_config(Norb=2, Nbath=5), 169, 853776)}
    for cfg, nsec, maxdim in pins.values():
        secs = setup_pointers(cfg)
        assert len(secs) == nsec
        assert max(s.dim for s in secs) == maxdim
    cfg = make_config(Norb=1, Nbath=6, Nspin=2, ed_mode="nonsu2")
    secs = setup_pointers(cfg)
    assert len(secs) == 2 * cfg.Ns + 1 and sum(s.dim for s in secs) == 2 ** (2 * cfg.Ns)
    s7 = [s for s in secs if s.q1 == 7][0]
    assert cdg_sector(cfg, s7, 0).q1 == 8 and c_sector(cfg, s7, 1).q1 == 6
    cfg = make_config(Norb=1, Nbath=3, ed_mode="superc")
    assert sum(s.dim for s in setup_pointers(cfg)) == 2 ** (2 * cfg.Ns)


def test_params_struct_layout():
    """ctypes mirror matches the C struct size computed by the C compiler."""
    src = '#include "%s"\n#include <stdio.h>\nint main(){printf("%%zu",sizeof(ed_params));}' % HEADER
    exe = "/tmp/_edp_size"
    subprocess.run(["gcc", "-x", "c", "-", "-o", exe], input=src, text=True, check=True)
    size = int(subprocess.run([exe], capture_output=True, text=True, check=True).stdout)
    assert size == ctypes.sizeof(EdParams)
    p = make_config(Norb=2, Nbath=3, Uloc=(2.0, 1.0, 0.0)).to_ctypes()
    assert p.norb == 2 and p.nbath == 3 and p.uloc[1] == 1.0


def test_config_checks():
    with pytest.raises(ValueError):
        EDConfig(Norb=1, Nbath=3, Nspin=1, ed_mode="nonsu2").check()
    with pytest.raises(ValueError):
        EDConfig(Norb=1, Nbath=20).check()   # Ns=21 > 16-level limit


def test_library_exports_every_header_symbol():
    """libedgpu.so exports each entry point declared in include/ed_gpu.h."""
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "dmft-ed_amd"), "libedgpu.so"], check=True)
    decl = re.findall(r"^\s*(?:int|const char\*)\s+(ed_\w+)\s*\(", open(HEADER).read(), re.M)
    assert len(decl) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\s[TW]\s+(\w+)$", out, re.M))
    missing = [d for d in decl if d not in exported]
    assert not missing, missing
    from edgpu._lib import SIGNATURES
    assert set(decl) == set(SIGNATURES)
    lib = ctypes.CDLL(LIB)              # loads without a GPU
    for d in decl:
        assert hasattr(lib, d)


def test_option_names_match_header_bits():
    """Every ED_OPT_* bit of include/ed_gpu.h has its Python name in
    edgpu._lib.OPTIONS (Sector(options=...) / DiagOptions.kernel_options) with
    the same value, and the library accepts exactly those bits."""
    from edgpu._lib import OPTIONS

    bits = {m.group(1).lower(): int(m.group(2), 16)
            for m in re.finditer(r"#define\s+ED_OPT_(\w+)\s+(0x[0-9a-fA-F]+)", open(HEADER).read())}
    assert bits == OPTIONS
    assert len(set(bits.values())) == len(bits)
    mask = 0
    for v in bits.values():
        assert v & (v - 1) == 0  # one bit each
        mask |= v
    src = open(os.path.join(ROOT, "dmft-ed_amd", "csrc", "ed_lib.hip")).read()
    assert re.search(r"if \(opts & ~kOptKnown\) return fail\(ED_ERR_ARG", src)
    m = re.search(r"kOptKnown =([^;]+);", src)
    names = re.findall(r"ED_OPT_(\w+)", m.group(1))
    assert {n.lower() for n in names} == set(bits) and len(names) == len(bits)  # exactly the defined bits


def test_fortran_shim_compiles_and_binds():
    """The Fortran module builds and references every bound C symbol it declares."""
    d = os.path.join(ROOT, "dmft-ed_amd", "fortran")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "dmft-ed_amd"), "fortran"], check=True)
    out = subprocess.run(["nm", "-D", "--undefined-only", os.path.join(d, "ed_gpu_driver")],
                         capture_output=True, text=True).stdout
    for sym in ("ed_gpu_hxv", "ed_gpu_init", "ed_gpu_build_sector", "ed_gpu_lanc_eigh",
                "ed_gpu_lanc_tridiag", "ed_gpu_delete_sector", "ed_gpu_vecdim"):
        assert re.search(r"\sU\s+%s$" % sym, out, re.M), sym


def test_tridiag_poles_host_matches_tql2_and_lapack():
    """ed_tridiag_poles (host code of the C-ABI library, no device call): the
    first-row implicit QL is bit-identical to the oracle's tql2
    (ED_GF_SHARED.f90:76-214) and agrees with LAPACK dstev (the normal-mode
    eigh, ED_GF_NORMAL.f90:612-618) to 1e-12 on GF-sized tridiagonals."""
    from scipy.linalg import eigh_tridiagonal

    from edgpu.gf import tridiag_poles
    from oracle.oracle import tql2

    rng = np.random.default_rng(7)
    for n in (1, 2, 5, 64, 200):
        a = rng.normal(size=n)
        b = np.concatenate([[0.0], np.abs(rng.normal(size=n - 1))])
        E, z2 = tridiag_poles(a, b, n)
        assert np.all(np.diff(E) >= 0)
        assert abs(z2.sum() - 1.0) < 1e-13
        if n == 1:
            assert E[0] == a[0] and z2[0] == 1.0
            continue
        W, Z, ierr = tql2(a.copy(), b.copy())
        assert ierr == 0
        np.testing.assert_array_equal(E, W)
        np.testing.assert_array_equal(z2, Z[0] ** 2)
        w, z = eigh_tridiagonal(a, b[1:], lapack_driver="stev")
        np.testing.assert_allclose(E, w, atol=1e-12)
        np.testing.assert_allclose(z2, z[0] ** 2, atol=1e-12)
    # split tridiagonal (a zero off-diagonal: invariant subspace of the seed)
    a = np.array([1.0, -2.0, 0.5, 3.0])
    b = np.array([0.0, 0.7, 0.0, 0.2])
    E, z2 = tridiag_poles(a, b, 4)
    np.testing.assert_allclose(z2.sum(), 1.0, atol=1e-15)
    assert np.count_nonzero(z2 > 1e-30) == 2


def test_mpi_split_matches_reference_formula():
    """ed_gpu_mpi_split = build_Hv_sector's split (ED_HAMILTONIAN.f90:55-62):
    MpiQ = Dim/MpiSize, the last rank also takes mod(Dim, MpiSize); ranks may
    hold no rows when Dim < MpiSize.  Pure host arithmetic (no GPU call)."""
    import ctypes

    from edgpu import _lib

    L = _lib.load()
    for dim, P in [(4900, 1), (4900, 3), (4900, 8), (5, 8), (0, 2), (853776, 7)]:
        rows = []
        for r in range(P):
            r0, n = ctypes.c_int64(), ctypes.c_int64()
            assert L.ed_gpu_mpi_split(dim, r, P, ctypes.byref(r0), ctypes.byref(n)) == 0
            q, rem = dim // P, (dim % P if r == P - 1 else 0)
            assert (r0.value, n.value) == (r * q, q + rem)
            rows.append((r0.value, n.value))
        assert sum(n for _, n in rows) == dim
        assert all(rows[i][0] + rows[i][1] == rows[i + 1][0] for i in range(P - 1))
