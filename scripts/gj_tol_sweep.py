"""hip-rbt on the systems the seed study found hard (profiles/rbt_seeds_r6.txt)
under different probe tolerances of the block inverse (lu_mixed.hip
kGjTol; inf = never the pivoted Gauss-Jordan, < 0 = always): corrections,
final componentwise backward error, fallback, time; and the distribution of
the per-block probe errors |D A x - x| / |x| of the unpivoted inverses."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402

dev = torch.device("cuda:0")
lib = gelim._native.lib()
E = torch.finfo(torch.float64).eps
default = lib.gelim_debug_gj_tol(1.0)
lib.gelim_debug_gj_tol(default)
errs = torch.zeros(256, dtype=torch.float64, device=dev)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
seeds = [int(a) for a in sys.argv[2:]] or [18, 3, 28, 52, 6, 11, 0, 1]
s = gelim.GaussSolver(n, backend="hip-rbt", device=dev)
for seed in seeds:
    aug = gelim.random_system(n, seed=seed, device=dev)
    lib.gelim_debug_gj_tol(float("inf"))
    lib.gelim_debug_gj_errors(errs.data_ptr())
    errs.zero_()
    s.solve(aug)
    torch.cuda.synchronize()
    lib.gelim_debug_gj_errors(None)
    e = errs[: n // 128].cpu()
    print(f"seed {seed}: probe errors of the {n // 128} unpivoted inverses: max {e.max().item():.2e}, "
          f">1e-11: {(e > 1e-11).sum().item()}, >1e-10: {(e > 1e-10).sum().item()}, >1e-9: {(e > 1e-9).sum().item()}",
          flush=True)
    for tol in (float("inf"), 1e-8, 1e-9, 1e-10, default, -1.0):
        lib.gelim_debug_gj_tol(tol)
        s.solve(aug)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x = s.solve(aug)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"   tol {tol:8.1e}: corrections {s.last_steps}  berr {s.last_berr / E:10.2f} eps  fallback "
              f"{'yes' if s.last_fallback else 'no ':3s}  {dt * 1e3:7.2f} ms  error {gelim.ops.gauss.error_metric(x):.2e}",
              flush=True)
lib.gelim_debug_gj_tol(default)
s.close()
