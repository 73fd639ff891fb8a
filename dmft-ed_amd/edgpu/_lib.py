"""Loader for the in-tree HIP library ``dmft-ed_amd/libedgpu.so``.

There is no CPU fallback: if the library is missing or cannot be loaded the
import fails loudly (the product path must never silently run elsewhere).
"""
from __future__ import annotations

import ctypes
import os
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG_ROOT, "libedgpu.so")

ED_STORED, ED_DIRECT, ED_REAL = 0x1, 0x2, 0x4
ED_NO_PACK, ED_KRON2_OFF, ED_KRON2_ON, ED_NO_SPLIT, ED_SPLIT_ON = 0x10, 0x20, 0x40, 0x80, 0x100
ED_FUSED_ON, ED_NO_FUSED = 0x200, 0x400
ED_BATCH_NO_FALLBACK = 0x1   # ed_sectors_eigh_batch flags
# kernel alternatives of a built sector (ed_sector_set_options, include/ed_gpu.h)
OPTIONS = {
    "no_persist": 0x001, "persist_stored": 0x002, "no_preg": 0x004, "no_pkron": 0x008,
    "split_simple": 0x020, "no_batch": 0x040, "eigh_no_verify": 0x080,
    "trlan_unfused": 0x100, "trlan_nofold": 0x200, "no_graph": 0x800,
    "trlan_nolocal": 0x1000, "trlan_nosolo": 0x2000, "trlan_fullupd": 0x4000,
    "stored_exact": 0x100000, "eigh_fullprobe": 0x200000, "no_fused": 0x400000, "eigh_nohint": 0x800000,
}
ED_OK = 0
ERRORS = {1: "ED_ERR_ARG", 2: "ED_ERR_STATE", 3: "ED_ERR_HIP", 4: "ED_ERR_OOM",
          5: "ED_ERR_UNSUPPORTED"}

# Every entry point of include/ed_gpu.h with its ctypes signature.
_P = ctypes.c_void_p
_i32, _i64, _f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
SIGNATURES = {
    "ed_sector_create": ([_P, _i32, _i32, _i32, _i32, _P, _P], ctypes.c_int),
    "ed_sector_create_rows": ([_P, _i32, _i32, _i32, _i64, _i64, _i32, _P, _P], ctypes.c_int),
    "ed_sector_destroy": ([_P], ctypes.c_int),
    "ed_sector_set_options": ([_P, _i32], ctypes.c_int),
    "ed_sector_get_info": ([_P, _P], ctypes.c_int),
    "ed_sector_hxv_dev": ([_P, _i32, _P, _P, _P], ctypes.c_int),
    "ed_sector_hxv_dev_path": ([_P, _i32, _i32, _P, _P, _P], ctypes.c_int),
    "ed_sector_hxv": ([_P, _i32, _P, _P], ctypes.c_int),
    "ed_sector_col_mask": ([_P, _P, _P], ctypes.c_int),
    "ed_sector_map": ([_P, _P], ctypes.c_int),
    "ed_sector_dump_csr": ([_P, _P, _P, _P], ctypes.c_int),
    "ed_sector_lanc_tridiag": ([_P, _i32, _P, _i32, _f64, _P, _P, _P], ctypes.c_int),
    "ed_sector_lanc_eigh": ([_P, _i32, _P, _i32, _f64, _i32, _P, _P, _P], ctypes.c_int),
    "ed_sector_lanc_run": ([_P, _i32, _P, _i32, _P, _P, _P, _P], ctypes.c_int),
    "ed_sector_lanc_mode": ([_P, _i32, _i32], ctypes.c_int),
    "ed_gpu_eigh": ([_i32, _i32, _i32, _f64, _P, _P, _P, _P], ctypes.c_int),
    "ed_sector_kron_rows": ([_P, _i32, _i64, _i64, _P, _P, _P], ctypes.c_int),
    "ed_sector_kron_cols": ([_P, _i32, _i64, _i64, _P, _P, _i32, _P], ctypes.c_int),
    "ed_sector_eigh": ([_P, _i32, _i32, _i32, _i32, _f64, _P, _P, _P, _P, _P], ctypes.c_int),
    "ed_sectors_eigh_batch": ([_P, _i32, _i32, _i32, _P, _f64, _P, _P, _P, _P, _P, _P, _i32, _P], ctypes.c_int),
    "ed_sector_sell_view": ([_P, _P], ctypes.c_int),
    "ed_sector_apply_op": ([_P, _P, _i32, _i32, _i32, _P, _P, _P], ctypes.c_int),
    "ed_sector_apply_op_acc": ([_P, _P, _i32, _i32, _f64, _f64, _i32, _P, _P, _P], ctypes.c_int),
    "ed_sector_lanc_tridiag_dev": ([_P, _i32, _P, _i32, _f64, _P, _P, _P], ctypes.c_int),
    "ed_sector_lanc_tridiag_batch": ([_P, _i32, _i32, _P, _i32, _f64, _P, _P, _P], ctypes.c_int),
    "ed_tridiag_poles": ([_i32, _P, _P, _P, _P, _P], ctypes.c_int),
    "ed_gf_add_poles": ([_i32, _P, _P, _P, _P, _P, _P, _P, _P, _i32, _P, _i32, _f64, _P, _P, _P],
                        ctypes.c_int),
    "ed_gpu_init": ([_P], ctypes.c_int),
    "ed_gpu_set_device": ([_i32], ctypes.c_int),
    "ed_gpu_build_sector": ([_i32, _i32, _i32, _P], ctypes.c_int),
    "ed_gpu_vecdim": ([_P], ctypes.c_int),
    "ed_gpu_hxv": ([_P, _P, _P], ctypes.c_int),
    "ed_gpu_build_sector_rows": ([_i32, _i32, _i32, _i64, _i64, _P], ctypes.c_int),
    "ed_gpu_mpi_split": ([_i64, _i32, _i32, _P, _P], ctypes.c_int),
    "ed_gpu_hxv_mpi": ([_P, _P, _P], ctypes.c_int),
    "ed_gpu_dump_csr": ([_P, _P, _P], ctypes.c_int),
    "ed_gpu_lanc_eigh": ([_i32, _f64, _i32, _P, _P, _P], ctypes.c_int),
    "ed_gpu_lanc_tridiag": ([_P, _i32, _f64, _P, _P, _P], ctypes.c_int),
    "ed_gpu_delete_sector": ([], ctypes.c_int),
    "ed_gpu_finalize": ([], ctypes.c_int),
    "ed_gpu_last_error": ([], ctypes.c_char_p),
    "ed_gpu_current_sector": ([_P], ctypes.c_int),
}


class SectorInfo(ctypes.Structure):
    _fields_ = [("dim", _i64), ("nnz", _i64), ("padded", _i64), ("ns", _i32), ("mode", _i32),
                ("q1", _i32), ("q2", _i32), ("flags", _i32), ("kron", _i32),
                ("dimup", _i64), ("dimdw", _i64), ("device_bytes", _i64),
                ("packed", _i32), ("npdict", _i32), ("row0", _i64), ("nrows", _i64),
                ("split", _i32), ("pad_", _i32), ("split_far", _i64), ("split_far_uniform", _i64),
                ("split_bytes", _i64), ("split_list_bytes", _i64),
                ("fused", _i32), ("pad2_", _i32), ("fused_far", _i64), ("fused_far_uniform", _i64),
                ("fused_bytes", _i64)]


class EDGPUError(RuntimeError):
    pass


_lib = None


def load():
    """Load libedgpu.so (raises if absent: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EDGPUError(
                f"HIP library {LIB_PATH} not built: run __graft_entry__.build() "
                "(there is deliberately no CPU fallback)")
        # torch ships its own libamdhip64 beside the /opt/rocm one this library
        # links; when ours takes the device first, torch's later initialisation
        # can find no free hardware queue ("No HIP GPUs are available").  Let
        # torch initialise first; the Fortran/C users never load torch.
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != ED_OK:
        msg = load().ed_gpu_last_error().decode(errors="replace")
        raise EDGPUError(f"{what}: {ERRORS.get(rc, rc)}: {msg}")
