"""Where the randomised no-pivoting solves spend their time: RBT + LU, one
correction apply (RBT vectors + forward + back substitution), one fp64
mat-vec, and the whole solve with its correction / GMRES iteration counts and
its error (vs the exact x_i = i + 1) next to the fp64 partial-pivoting engine.

  python scripts/mixed_breakdown.py [--backend hip-mixed|hip-rbt] 2048 8192
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
args = sys.argv[1:]
backend = "hip-mixed"
if args and args[0] == "--backend":
    backend, args = args[1], args[2:]
for n in [int(a) for a in args]:
    aug = gelim.random_system(n, seed=n, device=dev)
    s = gelim.GaussSolver(n, backend=backend, device=dev)
    ld = aug.stride(0)
    t_fac = timed(lambda: lib.gelim_mixed_factor(s._mixed, ptr(aug), ld, sh))
    r = aug[:, n].contiguous()
    d = torch.empty(n, dtype=torch.float64, device=dev)
    t_app = timed(lambda: lib.gelim_mixed_apply(s._mixed, ptr(r), 1, ptr(d), sh), reps=20)
    t_mv = timed(lambda: lib.gelim_gpu_matvec(ptr(aug), ld, n, ptr(r), ptr(d), sh), reps=20)
    t_all = timed(lambda: s.solve(aug), reps=3)
    err = gelim.ops.gauss.error_metric(s.solve(aug))
    ref = gelim.GaussSolver(n, backend="hip", device=dev)
    t_ref = timed(lambda: ref.solve(aug), reps=3)
    err_ref = gelim.ops.gauss.error_metric(ref.solve(aug))
    print(f"{backend} n={n}: factor {t_fac:.2f} ms, apply {t_app:.3f} ms, matvec {t_mv:.3f} ms, solve {t_all:.2f} ms "
          f"({s.last_steps} corrections, {s.last_inner} GMRES iterations, fallback={s.last_fallback}), "
          f"error {err:.2e} | fp64 partial pivoting {t_ref:.2f} ms, error {err_ref:.2e}", flush=True)
    s.close()
    ref.close()
