"""edgpu — MI355X-native Lanczos H·v hot path of dmft-ed (host mirror).

Modules:
  params      EDConfig / bath initialisation / the ed_params C struct
  sectors     symmetry-sector tables (setup_pointers_*)
  hamiltonian Sector handle + build_Hv_sector / spHtimesV_cc mirror; its
              lanc_eigh / lanc_tridiag / eigh methods are the device
              sp_lanc_eigh / sp_lanc_tridiag / sp_eigh replacements
  diag        ed_diag sector loop (single GPU) and the T=0 state list
  farm        sector farm over ranks (torch.distributed / RCCL)
  gf          Green's functions (normal, nonSU2): device seeds, Lanczos, poles
  dist        one sector over ranks (row split + Allgatherv; Kronecker all-to-all)

Importing this package does not touch the GPU; the HIP library is loaded on
first use and its absence is an error (no CPU fallback).
"""
from .params import EDConfig, make_config, init_dmft_bath, random_bath  # noqa: F401
from .sectors import setup_pointers  # noqa: F401

__all__ = ["EDConfig", "make_config", "init_dmft_bath", "random_bath", "setup_pointers"]
