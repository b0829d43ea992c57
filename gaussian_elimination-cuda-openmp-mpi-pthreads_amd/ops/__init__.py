"""Ops: thin tensor-level wrappers over the native kernels."""
from . import gauss, init, lu, matmul  # noqa: F401
from .lu import backsub, gemm_update, panel_factor, swap_trsm  # noqa: F401
from .matmul import cpu_matmul, matmul as gpu_matmul  # noqa: F401
