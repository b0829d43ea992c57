"""Factor one random system with the randomised no-pivoting engine a few
times (a short workload for rocprofv3 PMC passes over its kernels).

  python scripts/rbt_factor_only.py [--backend hip-rbt|hip-mixed] N [reps]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

args = sys.argv[1:]
backend = "hip-rbt"
if args and args[0] == "--backend":
    backend, args = args[1], args[2:]
n = int(args[0]) if args else 2048
reps = int(args[1]) if len(args) > 1 else 3
dev = torch.device("cuda:0")
lib = gelim._native.lib()
aug = gelim.random_system(n, seed=n, device=dev)
s = gelim.GaussSolver(n, backend=backend, device=dev)
for _ in range(reps):
    gelim._native.check(lib.gelim_mixed_factor(s._mixed, ptr(aug), aug.stride(0), stream_handle(dev)), "factor")
torch.cuda.synchronize()
print("factored", backend, n, reps)
s.close()
