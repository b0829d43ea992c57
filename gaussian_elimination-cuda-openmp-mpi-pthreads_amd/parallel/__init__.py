"""Multi-GPU layer: communicator (RCCL / gloo), distributed Gauss (partial
pivoting and the randomised block-LDU engine), distributed matmul."""
from . import comm, dist_gauss, dist_matmul, dist_rbt, emulated  # noqa: F401
from .comm import Communicator, destroy, init_from_env  # noqa: F401
from .dist_gauss import ColumnLayout, DistributedGauss  # noqa: F401
from .dist_rbt import DistributedRBT  # noqa: F401
from .dist_matmul import allgather_matmul, ring_matmul, summa_matmul  # noqa: F401
from .emulated import EmulatedComm, make_world, run_emulated  # noqa: F401
