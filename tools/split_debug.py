"""Sector info of the configs[1] sector with and without the two-segment form."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401

from cases import c2  # noqa: E402
from edgpu.hamiltonian import Sector  # noqa: E402

for split in (None, False, True):
    for real in (True, False):
        try:
            with Sector(c2(), 4, 4, stored=True, real=real, split=split) as S:
                i = S.info
                print(f"split={split} real={real}: dim={i.dim} nnz={i.nnz} padded={i.padded} packed={i.packed} "
                      f"npdict={i.npdict} split={i.split} far={i.split_far} uni={i.split_far_uniform} "
                      f"flags={i.flags:#x}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"split={split} real={real}: {type(e).__name__}: {e}", flush=True)
