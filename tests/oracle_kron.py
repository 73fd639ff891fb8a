"""Kronecker factors of a normal-mode sector from the oracle CSR (test
infrastructure): H = D + Hup (x) 1 + 1 (x) Hdw on the DimDw x DimUp view
(row i = iw*DimUp + iu, the reference's build_sector order).  Used to give
the CPU (gloo) tests of edgpu.dist reference factor products."""
import numpy as np
import scipy.sparse as sp
import torch

from oracle.oracle import Oracle


def oracle_factors(cfg, q1, q2):
    orc = Oracle(cfg)
    hmap = orc.build_sector(q1, q2)
    rp, cols, vals = orc.build_csr(hmap)
    dim = len(hmap)
    H = sp.csr_matrix((vals, cols, rp), shape=(dim, dim))
    mask = (1 << cfg.Ns) - 1
    ups = np.unique(hmap & mask)
    dws = np.unique(hmap >> cfg.Ns)
    du, dd = len(ups), len(dws)
    assert du * dd == dim
    D = H.diagonal().reshape(dd, du)
    Hup = H[0:du, 0:du].tolil()
    Hup.setdiag(0)
    Hdw = H[np.arange(dd) * du][:, np.arange(dd) * du].tolil()
    Hdw.setdiag(0)
    return H, D, Hup.tocsr(), Hdw.tocsr(), du, dd


class NumpyKronOps:
    """CPU stand-in for DeviceKronOps built from oracle factors."""

    def __init__(self, D, Hup, Hdw, du, dd):
        self.D, self.Hup, self.Hdw = D, Hup, Hdw
        self.dimup, self.dimdw = du, dd
        self.dtype = torch.complex128
        self.device = torch.device("cpu")

    def rows(self, w0, nw, x):
        X = x.numpy().reshape(nw, self.dimup)
        Y = self.D[w0:w0 + nw] * X + (self.Hup @ X.T).T
        return torch.from_numpy(np.ascontiguousarray(Y).reshape(-1))

    def cols(self, u0, nu, z):
        Z = z.numpy().reshape(self.dimdw, nu)
        return torch.from_numpy(np.ascontiguousarray(self.Hdw @ Z).reshape(-1))
