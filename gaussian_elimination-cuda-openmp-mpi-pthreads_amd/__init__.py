"""gelim — MI355X-native dense Gaussian elimination and matrix multiply.

A from-scratch re-design, for AMD Instinct MI355X (gfx950 / CDNA4), of the
capabilities of svdeepak99/Gaussian_Elimination-CUDA-OpenMP-MPI-Pthreads:

  * Gaussian elimination (forward elimination + back substitution) on the
    synthetic "internal" system or reference `.dat` files, with the reference's
    pivoting rules, on the GPU (blocked LU on fp64 MFMA, or the per-pivot
    algorithm) or with the reference CPU strategies (seq / OpenMP /
    Pthreads V1-V3);
  * fp32 matrix multiply: naive parity kernels and an MFMA tiled GEMM, plus the
    reference sequential/OpenMP loops;
  * multi-GPU versions of both over RCCL (one process per GPU).

Layers: `_native` (ctypes over libgelim.so: C++17 + HIP), `ops` (tensor-level
kernels), `models` (GaussSolver, MatMul), `parallel` (communicator,
distributed solvers), `utils` (IO, timers, reports).  Import as `gelim`.
"""
from . import _native  # noqa: F401,E402
from . import utils  # noqa: F401,E402
from . import ops  # noqa: F401,E402
from . import models  # noqa: F401,E402
from . import parallel  # noqa: F401,E402
from ._native import GelimError, SingularMatrixError, version  # noqa: F401,E402
from .models import GaussSolver, MatMul, blocked_solve_, solve  # noqa: F401,E402
from .ops.init import augment_with_rhs, random_system, synthetic_system  # noqa: F401,E402

__version__ = "0.1.0"
