"""ctypes binding of libsanta_hip.so (the C-ABI declared in include/santa_hip.h).

This is the binding a maintainer of the reference would add.
There is no fallback: if the shared library is missing the import fails
loudly, and every device entry point needs a ROCm GPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SANTA_HIP_LIB") or os.path.join(_HERE, "libsanta_hip.so")

SH_OK = 0
SH_ERR_INFEASIBLE = -1
SH_ERR_ARGS = -2
SH_ERR_HIP = -3
SH_MODE_SINGLE = 0
SH_MODE_TWINS = 1
SH_MODE_TRIPLETS = 2  # extension: 3-slot triplet units (the reference only asserts them)
SH_COMPAT_TIEBREAK = 1
SH_FLAG_EXACT_ARGMIN = 2
SH_FLAG_BUILD_ONLY = 4
SH_FLAG_LDS_TILE = 8
SH_FLAG_SW_TILE = 16  # retired: the C-ABI refuses it (SH_ERR_ARGS)
SH_FLAG_VT_TILE = 32
SH_FLAG_TIMING = 64
SH_FLAG_SP_TILE = 128
SH_FLAG_SP1 = 256
SH_FLAG_TEST_RANGE = 512  # test hook: every register-tile block goes to the fallback launch
SH_FLAG_NO_APPLY = 1024  # solve without writing the gift types (overlapping blocks allowed)
SH_FLAG_SP2 = 2048  # retired (round 4): the C-ABI refuses it (SH_ERR_ARGS)
SH_FLAG_DT_TILE = 4096  # force the dense-tile one-wave kernel (santa_dt_kernel)
SH_FLAG_BIG_ROWS = 8192  # singles n > 256: force the row-rebuild kernel (santa_big_kernel)
SH_ERRF_ROWS = 1
SH_ERRF_INFEASIBLE = 2
SH_ERRF_TYPE = 4
SH_DESIGN_SPARSE = 0
SH_DESIGN_LDS_TILE = 1
SH_DESIGN_SW_TILE = 2
SH_DESIGN_VT_TILE = 3
SH_DESIGN_TWINS = 4
SH_DESIGN_LARGE = 5
SH_DESIGN_SPARSE2 = 6
SH_DESIGN_SPARSE3 = 7
SH_DESIGN_DT_TILE = 8
SH_DESIGN_LARGE_LB = 9
SH_DESIGN_NAMES = {0: "santa_sp_kernel (1-wave sparse LDS tile)", 1: "santa_block_kernel (4-wave LDS byte tile)",
                   2: "(retired: santa_sw_kernel)", 3: "santa_vt_kernel (4-wave register tile)",
                   4: "santa_block_kernel (twins, 4-wave code-pair tile)",
                   5: "santa_big_kernel (row rebuilt from the wishlist)",
                   6: "(retired: santa_sp2_kernel)",
                   7: "santa_sp3_kernel (1-wave sparse register tile built in-kernel, 32-bit lattice keys)",
                   8: "santa_dt_kernel (LDS byte tile built by 4 waves, solved by 1 wave, 32-bit lattice keys)",
                   9: "santa_lb_kernel (each wave's candidate row staged as a gift-type cost table in LDS, "
                      "32-bit lattice keys)"}
SH_MAX_N = 1024
SH_MAX_N_SANTA = 4096

_ERRF_TEXT = {SH_ERRF_ROWS: "a block's child ids out of [0, nc)",
              SH_ERRF_INFEASIBLE: "an infeasible solve",
              SH_ERRF_TYPE: "a block's current gift type out of [0, ng)"}


def describe_error_flags(flags: int) -> str:
    """The SH_ERRF_* bits of sh_ctx_error_flags as text (unknown bits by value)."""
    parts = [t for b, t in _ERRF_TEXT.items() if flags & b]
    rest = flags & ~sum(_ERRF_TEXT)
    if rest:
        parts.append(f"unknown bits {rest:#x}")
    return "; ".join(parts) or "none"


_P = ctypes.c_void_p
_I = ctypes.c_int
_U64 = ctypes.c_uint64
_I64 = ctypes.c_int64
_U = ctypes.c_uint

# name -> (restype, argtypes); mirrors include/santa_hip.h one to one.
SIGNATURES = {
    "sh_last_error": (ctypes.c_char_p, []),
    "sh_version": (_I, []),
    "sh_ctx_create": (_I, [ctypes.POINTER(_P), _I, _P, _I, _P, _I, _I, _I, _I]),
    "sh_ctx_destroy": (None, [_P]),
    "sh_sample_blocks": (_I, [_U64, _U64, _I, _I, _I, _I, _I, _P, _P]),
    "sh_sample_blocks_undo": (_I, [_U64, _U64, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "sh_solve_blocks": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _P, _U, _P]),
    "sh_solve_round": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _P, _P, _U, _P]),
    "sh_score": (_I, [_P, _P, _P, _P]),
    "sh_ctx_error_flags": (_I, [_P, _P]),
    "sh_ctx_mailbox": (ctypes.POINTER(ctypes.c_int64), [_P]),
    "sh_publish_delta": (_I, [_P, _P, _I, _I64, _P]),
    "sh_ctx_fallback_steps": (_I, [_P, _P]),
    "sh_solve_design": (_I, [_P, _I, _I, _I, _U]),
    "sh_resident_blocks": (_I, [_P, _I, _I, _I, _U]),
    "sh_ctx_set_sparse_budget": (_I, [_P, _I]),
    "sh_pack_types": (_I, [_P, _P, _I, _P, _P]),
    "sh_unpack_types": (_I, [_P, _P, _I, _P, _I, _P]),
    "lsap_solve_batched_i64": (_I, [_P, _I, _I, _P, _P, _U, _P]),
    "lsap_solve_batched_i32": (_I, [_P, _I, _I, _P, _P, _U, _P]),
    "lsap_solve_batched_f64": (_I, [_P, _I, _I, _P, _P, _U, _P]),
    "lsap_solve_batched_hash": (_I, [_U64, _I64, _I, _I, _P, _P, _U, _P]),
    "sh_gen_synthetic": (_I, [_U64, _I, _I, _I, _I, _I, _P, _P, _P]),
}


class RoundExt(ctypes.Structure):
    """sh_round_ext (include/santa_hip.h): sh_solve_round's undo record,
    next-round sampler arguments and mailbox publish."""
    _fields_ = [("d_undo", ctypes.c_void_p), ("next_rows", ctypes.c_void_p),
                ("next_seed", ctypes.c_uint64), ("next_round", ctypes.c_uint64),
                ("next_lo", ctypes.c_int), ("next_count", ctypes.c_int), ("next_stride", ctypes.c_int),
                ("next_B", ctypes.c_int), ("publish", ctypes.c_int), ("publish_slot", ctypes.c_int),
                ("publish_seq", ctypes.c_int64)]


class SantaHipError(RuntimeError):
    """A C-ABI call returned a negative status."""

    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C mpi-hungarian-method_amd/csrc` "
                "or __graft_entry__.build(); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return lib().sh_last_error().decode(errors="replace")


def check(rc: int, where: str) -> int:
    if rc < 0:
        msg = last_error()
        if rc == SH_ERR_INFEASIBLE:
            raise ValueError(f"cost matrix is infeasible ({where}: {msg})")
        if rc == SH_ERR_ARGS:
            raise ValueError(f"{where}: {msg}")
        raise SantaHipError(rc, where, msg)
    return rc
