"""`import gelim` — importable alias of the framework package, whose on-disk
directory name (`gaussian_elimination-cuda-openmp-mpi-pthreads_amd/`) is not a
valid Python identifier.  The real package is imported once and registered
under this name together with all of its submodules, so `gelim.ops.lu` and
`gaussian_elimination-...amd.ops.lu` are the same module objects."""
import importlib
import sys
from pathlib import Path

_REAL = "gaussian_elimination-cuda-openmp-mpi-pthreads_amd"
_root = str(Path(__file__).resolve().parent.parent)
if _root not in sys.path:
    sys.path.insert(0, _root)
_pkg = importlib.import_module(_REAL)
for _name, _mod in list(sys.modules.items()):
    if _name == _REAL or _name.startswith(_REAL + "."):
        sys.modules["gelim" + _name[len(_REAL):]] = _mod
sys.modules[__name__] = _pkg
