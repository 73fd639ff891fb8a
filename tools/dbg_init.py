"""Diagnose: HIP error state left by ed_sector_eigh before torch initialises HIP."""
import ctypes, sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd")]
import numpy as np
from edgpu.params import make_config
from edgpu.hamiltonian import Sector
hip = ctypes.CDLL("libamdhip64.so")
n = ctypes.c_int()
print("count before", hip.hipGetDeviceCount(ctypes.byref(n)), n.value, flush=True)
cfg = make_config(Norb=1, Nbath=7)
mode = sys.argv[1]
with Sector(cfg, 4, 4, stored=True, real=True) as S:
    if mode == "eigh":
        print(S.eigh()[0])
    elif mode == "lanc":
        print(S.lanc_eigh(vector=False)[0])
    else:
        print(S.hxv(np.ones(S.dim))[:3])
print("peek", hip.hipPeekAtLastError(), flush=True)
print("count after", hip.hipGetDeviceCount(ctypes.byref(n)), n.value, flush=True)
import torch
print("torch count", torch.cuda.device_count(), flush=True)
torch.cuda.init()
print("ok", flush=True)
