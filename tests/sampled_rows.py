"""Oracle parity on sampled rows of a full-size sector (test helper).

The Nlevels=28 sectors (dim 11.8 M) are the roofline workloads; their whole
CSR is not built on the host, so a GPU H·v there is checked on row ranges:
the oracle builds rows [r0, r0+n) of ed_buildH_c's CSR against the whole map
(oracle/ed_oracle.c orc_build_csr_rows; ED_HAMILTONIAN_STORED_HxV.f90:28-113)
and each sampled element of y must lie within `tol` of the row's absolute sum
sum_j |H_ij x_j| of spMatVec_cc's value (STORED_HxV.f90:132-143) — the
rounding bound of any summation order.
"""
import numpy as np

BLOCK = 1024


def sample_starts(dim, nblocks=16, block=BLOCK, seed=0):
    """First and last rows plus random ranges: >= 10^4 rows at nblocks=16."""
    rng = np.random.default_rng(seed)
    starts = {0, dim - block}
    while len(starts) < nblocks:
        starts.add(int(rng.integers(0, dim - block)))
    return sorted(starts)


def check_rows(orc, hmap, x, y, starts, block=BLOCK, tol=1e-13):
    """Worst |y - ref| / bound over the sampled rows; asserts it is <= tol."""
    x = np.asarray(x)
    y = np.asarray(y)
    worst = 0.0
    nrows = 0
    for r0 in starts:
        rp, cols, vals = orc.build_csr_rows(hmap, r0, block)
        rows = np.repeat(np.arange(block), np.diff(rp))
        v = vals.real if np.isrealobj(x) else vals
        ref = np.zeros(block, dtype=np.result_type(v, x))
        np.add.at(ref, rows, v * x[cols])
        bound = np.zeros(block)
        np.add.at(bound, rows, np.abs(vals) * np.abs(x[cols]))
        err = np.abs(y[r0:r0 + block] - ref)
        worst = max(worst, float(np.max(err / np.maximum(bound, 1e-300))))
        nrows += block
    assert nrows >= 10_000
    assert worst <= tol, worst
    return worst
