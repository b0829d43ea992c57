"""ctypes binding of libgelim.so (the C++/HIP core, ``csrc/``).

The Python layer never re-implements numerics: every op goes through this
library, CPU ops included.  Loading is strict — if the shared library is
missing the import raises, so a GPU run can never silently fall back to an
eager PyTorch path.  Build it with ``python __graft_entry__.py build`` (or
``cmake -S csrc -B build -G Ninja && ninja -C build``).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_LIB_DIR = Path(__file__).resolve().parent / "lib"
_LIB_PATH = _LIB_DIR / "libgelim.so"

# error codes (gelim.h)
OK, E_ARG, E_IO, E_HIP, E_SINGULAR, E_NOMEM, E_THREAD = 0, -1, -2, -3, -4, -5, -6
PIVOT_ZERO, PIVOT_PARTIAL = 0, 1
CPU_SEQ, CPU_OMP, CPU_PTH_V1, CPU_PTH_V2, CPU_PTH_V3 = 0, 1, 2, 3, 4
GPU_BLOCKED, GPU_PIVOT = 0, 1
MM_NAIVE_ROW, MM_NAIVE_ELEM, MM_MFMA = 0, 1, 2


class GelimError(RuntimeError):
    """A libgelim call failed; ``code`` is the GELIM_E_* value."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class SingularMatrixError(GelimError):
    """Zero pivot: the reference prints 'The matrix is singular' and exits."""


_i64, _i32, _int, _dbl, _vp = C.c_int64, C.c_int32, C.c_int, C.c_double, C.c_void_p
_u64 = C.c_uint64
_PROTOS = {
    "gelim_last_error": (C.c_char_p, []),
    "gelim_version": (C.c_char_p, []),
    "gelim_build_digest": (C.c_char_p, []),
    "gelim_dat_size": (_i64, [C.c_char_p]),
    "gelim_dat_read": (_int, [C.c_char_p, _vp, _i64, _i64]),
    "gelim_matrix_gen": (_int, [_i64, C.c_char_p]),
    "gelim_init_synthetic_f64": (None, [_vp, _i64, _vp, _i64]),
    "gelim_init_random_f64": (None, [_vp, _i64, _i64, _u64]),
    "gelim_init_rhs_f64": (None, [_vp, _i64, _vp, _i64]),
    "gelim_error_metric": (_dbl, [_vp, _i64]),
    "gelim_cpu_gauss": (_int, [_vp, _i64, _vp, _i64, _int, _int, _int, _int]),
    "gelim_cpu_max_threads": (_int, []),
    "gelim_cpu_backsub_unit": (None, [_vp, _i64, _vp, _vp, _i64]),
    "gelim_cpu_matmul_f32": (None, [_vp, _vp, _vp, _i64, _int, _int]),
    "gelim_init_matmul_f32": (None, [_vp, _vp, _i64]),
    "gelim_cpu_panel_factor": (_int, [_vp, _i64, _i64, _i64, _i64, _int, _vp, _vp]),
    "gelim_cpu_swap_trsm": (_int, [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64]),
    "gelim_cpu_gemm_update": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64]),
    "gelim_gpu_device_count": (_int, []),
    "gelim_gpu_set_device": (_int, [_int]),
    "gelim_gpu_sync": (_int, [_vp]),
    "gelim_gpu_side_stream_create": (_int, [C.POINTER(C.c_void_p)]),
    "gelim_gpu_stream_destroy": (_int, [_vp]),
    "gelim_gpu_stream_probe": (_int, [_vp]),
    "gelim_gpu_stream_create_probed": (_int, [C.POINTER(C.c_void_p), _vp, _i32]),
    "gelim_gpu_probe_kernel": (_int, [_vp, _vp, _i32, _i64]),
    "gelim_rccl_load": (_int, [C.c_char_p]),
    "gelim_rccl_version": (_int, []),
    "gelim_rccl_unique_id": (_int, [_vp]),
    "gelim_rccl_comm_create": (_int, [C.POINTER(C.c_void_p), _vp, _i32, _i32]),
    "gelim_rccl_comm_destroy": (_int, [_vp, _i32]),
    "gelim_rccl_async_error": (_int, [_vp]),
    "gelim_rccl_bcast": (_int, [_vp, _vp, _i64, _i32, _i32, _vp]),
    "gelim_rccl_allreduce": (_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp]),
    "gelim_rccl_allgather": (_int, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "gelim_rccl_sendrecv": (_int, [_vp, _vp, _i64, _i32, _vp, _i64, _i32, _i32, _vp]),
    "gelim_gpu_stream_priority_range": (_int, [_vp]),
    "gelim_gpu_side_stream_stats": (None, [_vp]),
    "gelim_gpu_init_synthetic": (_int, [_vp, _i64, _i64, _vp]),
    "gelim_gpu_init_synthetic_f32": (_int, [_vp, _i64, _i64, _vp]),
    "gelim_gpu_init_random": (_int, [_vp, _i64, _i64, _u64, _vp]),
    "gelim_gpu_init_rhs": (_int, [_vp, _i64, _i64, _vp]),
    "gelim_gpu_error_metric": (_int, [_vp, _i64, _vp, _vp]),
    "gelim_gpu_panel_factor": (_int, [_vp, _i64, _i64, _i64, _i64, _int, _vp, _vp, _vp]),
    "gelim_gpu_panel_max_rows": (_i64, [_i64]),
    "gelim_gpu_swap_trsm": (_int, [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp]),
    "gelim_gpu_gemm_update": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp]),
    "gelim_gpu_dgemm": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _dbl, _vp]),
    "gelim_gpu_dgemm_capped": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _dbl, _int, _vp]),
    "gelim_gpu_dgemm_grouped": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _dbl, _int, _int, _vp]),
    "gelim_gpu_leaf_factor": (_int, [_vp, _i64, _i64, _i64, _int, _vp, _vp, _vp, _vp]),
    "gelim_gpu_leaf_factor_ws": (_int, [_vp, _i64, _i64, _i64, _int, _vp, _vp, _vp, _vp, _int, _vp]),
    "gelim_gpu_leaf_workspace_bytes": (_i64, []),
    "gelim_gpu_leaf_participants": (_i32, [_i64]),
    "gelim_mixed_max_n": (_i64, []),
    "gelim_gpu_matvec": (_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gelim_mixed_padded": (_i64, [_i64]),
    "gelim_mixed_plan_create": (_vp, [_i64, _vp, _vp]),
    "gelim_mixed_plan_create2": (_vp, [_i64, _vp, _vp, _int]),
    "gelim_mixed_solve_error": (_int, [_vp, _vp]),
    "gelim_mixed_reset_error": (_int, [_vp, _vp]),
    "gelim_rbt_block_inverse": (_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gelim_rbt_vec": (_int, [_vp, _i64, _i64, _i64, _vp, _int, _vp, _i64, _vp]),
    "gelim_drbt_transform": (_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _int, _int, _vp, _vp, _vp]),
    "gelim_gpu_dgemm_bm": (_int, [_vp, _i64, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _dbl, _int, _int,
                                  _vp]),
    "gelim_drbt_super_solve": (_int, [_vp, _i64, _vp, _int, _vp, _vp, _vp, _int, _vp]),
    "gelim_rbt_block_solve": (_int, [_vp, _i64, _vp, _int, _vp, _vp, _vp, _int, _vp, _vp]),
    "gelim_drbt_gemv": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _dbl, _vp]),
    "gelim_drbt_matvec_abs": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "gelim_gpu_dgemm_thin": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _dbl, _int, _int, _vp]),
    "gelim_gpu_dgemm_ex": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _dbl, _int, _int, _vp]),
    "gelim_mixed_debug_ptrs": (_i64, [_vp, _vp]),
    "gelim_mixed_debug_copy": (_int, [_vp, _vp, _i64]),
    "gelim_mixed_plan_np": (_i64, [_vp]),
    "gelim_mixed_solve": (_int, [_vp, _vp, _i64, _vp, _int, _vp, _vp, _vp]),
    "gelim_gpu_residual_cw": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "gelim_mixed_plan_destroy": (None, [_vp]),
    "gelim_drbt_exec_create": (_vp, []),
    "gelim_drbt_exec_destroy": (None, [_vp]),
    "gelim_drbt_factor": (_int, [_vp, _vp]),
    "gelim_drbt_chain_products": (_int, [_vp, _vp, _vp, _vp, _vp, _int, _vp]),
    "gelim_drbt_side_cap": (_int, []),
    "gelim_drbt_args_layout": (_i64, [_i32]),
    "gelim_mixed_factor": (_int, [_vp, _vp, _i64, _vp]),
    "gelim_mixed_apply": (_int, [_vp, _vp, _i64, _vp, _vp]),
    "gelim_gpu_leaf_max_rows": (_i64, []),
    "gelim_debug_leaf_stamps": (_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gelim_gpu_laswp_trsm": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp]),
    "gelim_dist_pair_slot": (_i64, []),
    "gelim_dist_panel_factor": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _int, _vp, _vp, _vp, _vp, _int, _i64, _vp,
                                       _vp]),
    "gelim_dist_panel_apply": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _vp, _int, _int,
                                      _vp]),
    "gelim_dist_net_ints": (_i64, []),
    "gelim_dist_panel_compose": (_int, [_i64, _i64, _int, _vp, _vp, _vp]),
    "gelim_dist_side_cap": (_int, [_i64]),
    "gelim_gpu_panel_trsm": (_int, [_vp, _i64, _i64, _i64, _vp, _i64, _int, _vp]),
    "gelim_gpu_laswp_panel": (_int, [_vp, _i64, _i64, _i64, _int, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "gelim_gpu_laswp_net": (_int, [_vp, _i64, _i64, _i64, _int, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _int, _vp]),
    "gelim_gpu_backsub": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _int, _vp]),
    "gelim_gauss_plan_create": (_vp, [_i64, _int, _int, _int, _int]),
    "gelim_gauss_plan_resolve": (_int, [_vp, _vp, _vp, _vp]),
    "gelim_gpu_residual": (_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gelim_gauss_plan_destroy": (None, [_vp]),
    "gelim_gauss_plan_lda": (_i64, [_vp]),
    "gelim_gauss_plan_work": (_vp, [_vp]),
    "gelim_gpu_memcpy_d2h": (_int, [_vp, _vp, _i64, _vp]),
    "gelim_gauss_plan_solve": (_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "gelim_gauss_plan_info": (_int, [_vp, _vp]),
    "gelim_gpu_matmul_f32": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _int, _vp]),
    "gelim_gpu_matmul_f32_ex": (_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "gelim_init_random_block_f64": (None, [_vp, _i64, _i64, _i64, _i64, _i64, _u64]),
    "gelim_gpu_init_random_block": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _u64, _vp]),
}

_lib: C.CDLL | None = None


def library_path() -> Path:
    return _LIB_PATH


def lib() -> C.CDLL:
    """Load libgelim.so once (raises ImportError with a build hint if absent)."""
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise ImportError(
                f"libgelim.so not found at {_LIB_PATH}; build it with "
                "`python __graft_entry__.py build` (cmake -S csrc -B build -G Ninja)"
            )
        handle = C.CDLL(os.fspath(_LIB_PATH), mode=C.RTLD_GLOBAL)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def last_error() -> str:
    msg = lib().gelim_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "") -> int:
    """Raise on a negative libgelim return code."""
    if rc is not None and rc < 0:
        msg = f"{what}: {last_error()}" if what else last_error()
        if rc == E_SINGULAR:
            raise SingularMatrixError(rc, msg)
        raise GelimError(rc, msg)
    return rc


def version() -> str:
    return lib().gelim_version().decode()


# the files csrc/cmake/source_digest.cmake hashes (relative to csrc/)
_DIGEST_GLOBS = ("core/**/*.cpp", "cpu/**/*.cpp", "comm/**/*.hip", "hip/**/*.hip", "hip/**/*.h", "include/**/*.h",
                 "tools/**/*.cpp")


def build_digest() -> str:
    """The source digest compiled into the loaded libgelim.so."""
    return lib().gelim_build_digest().decode()


def source_digest(csrc: Path | None = None) -> str:
    """The same digest (csrc/cmake/source_digest.cmake) of the sources in the
    tree beside this package: equal to build_digest() when the loaded
    library was built from them."""
    import hashlib

    root = Path(csrc) if csrc is not None else Path(__file__).resolve().parents[1] / "csrc"
    files = sorted({p.relative_to(root).as_posix() for g in _DIGEST_GLOBS for p in root.glob(g) if p.is_file()})
    lines = "".join(f"{f} {hashlib.sha256((root / f).read_bytes()).hexdigest()}\n" for f in files)
    return hashlib.sha256(lines.encode()).hexdigest()
