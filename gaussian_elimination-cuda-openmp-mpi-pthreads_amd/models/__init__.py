"""Models: the two workloads of the reference as solver objects."""
from .gauss_solver import GaussSolver, blocked_solve_, solve  # noqa: F401
from .matmul import MatMul, MatMulTiming  # noqa: F401
