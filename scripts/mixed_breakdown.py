"""Where the mixed-precision solve spends its time: RBT + fp32 LU, one
correction apply (RBT vectors + forward + back substitution), one fp64
mat-vec, and the whole solve with its GMRES iteration count.

  python scripts/mixed_breakdown.py 2048 8192
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


dev = torch.device("cuda:0")
lib = gelim._native.lib()
sh = stream_handle(dev)
for n in [int(a) for a in sys.argv[1:]]:
    aug = gelim.random_system(n, seed=n, device=dev)
    s = gelim.GaussSolver(n, backend="hip-mixed", device=dev)
    ld = aug.stride(0)
    t_fac = timed(lambda: lib.gelim_mixed_factor(s._mixed, ptr(aug), ld, sh))
    r = aug[:, n].contiguous()
    d = torch.empty(n, dtype=torch.float64, device=dev)
    t_app = timed(lambda: lib.gelim_mixed_apply(s._mixed, ptr(r), 1, ptr(d), sh), reps=20)
    t_mv = timed(lambda: lib.gelim_gpu_matvec(ptr(aug), ld, n, ptr(r), ptr(d), sh), reps=20)
    t_all = timed(lambda: s.solve(aug), reps=3)
    print(f"n={n}: factor {t_fac:.2f} ms, apply {t_app:.3f} ms, matvec {t_mv:.3f} ms, solve {t_all:.2f} ms "
          f"({s.last_steps} corrections, {s.last_inner} GMRES iterations)", flush=True)
    s.close()
