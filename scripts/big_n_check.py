"""Single-GPU blocked solves past the old 32768-row leaf cap: each order is
solved twice (first call, then a timed replay), checked against the exact
solution x_i = i + 1 and by the fp64 residual ||b - A x|| / (||A|| ||x||)
(native kernel), and -- up to n = 46340, where n^2 still fits an int32 --
compared with fp64 torch.linalg.solve on the GPU (rocSOLVER).  Past that
order the rocSOLVER factorisation is not used: n = 70000 through
torch.linalg.solve aborted in rocBLAS ("Could not initialize Tensile host")
and left the GPU faulted (round 3, after our solve had returned).

  python scripts/big_n_check.py 40000 70000
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402


def main() -> None:
    dev = torch.device("cuda:0")
    lib = gelim._native.lib()
    for n in [int(a) for a in sys.argv[1:]]:
        aug = gelim.random_system(n, seed=n, device=dev)
        s = gelim.GaussSolver(n, backend="hip", device=dev)
        t0 = time.perf_counter()
        x = s.solve(aug, check=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        x = s.solve(aug, check=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        err = gelim.ops.gauss.error_metric(x)
        s.close()
        r = torch.empty(n, dtype=torch.float64, device=dev)
        gelim._native.check(lib.gelim_gpu_residual(gelim.utils.tensors.ptr(aug), aug.stride(0), n,
                                                   gelim.utils.tensors.ptr(x), gelim.utils.tensors.ptr(r),
                                                   gelim.utils.tensors.stream_handle(dev)), "residual")
        anorm = aug[:, :n].abs().sum(1).max().item()
        res = (r.abs().max() / (anorm * x.abs().max())).item()
        line = (f"n={n}: first {t1 - t0:.3f} s, replay {t2 - t1:.3f} s ({(2 / 3) * n ** 3 / (t2 - t1) * 1e-12:.1f} "
                f"TFLOP/s), err vs exact {err:.2e}, scaled residual {res:.2e}, "
                f"first leaf participants {lib.gelim_gpu_leaf_participants(n)}")
        if n <= 46340:
            ref = torch.linalg.solve(aug[:, :n], aug[:, n].clone())
            line += f", rel diff vs torch.linalg.solve {((x - ref).abs().max() / ref.abs().max()).item():.2e}"
            del ref
        print(line, flush=True)
        del aug, r, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
