"""Classic fp64 refinement (native gelim_mixed_solve) on the fp32-trailing
factor of hip-mixed: corrections needed, time, error -- vs GMRES-IR.

  python scripts/mixed_classic_ir.py 2048 4096 8192
"""
import ctypes
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

dev = torch.device("cuda:0")
lib = gelim._native.lib()
sh = stream_handle(dev)
for n in [int(a) for a in sys.argv[1:]]:
    aug = gelim.random_system(n, seed=n, device=dev)
    s = gelim.GaussSolver(n, backend="hip-mixed", device=dev)
    x = torch.empty(n, dtype=torch.float64, device=dev)
    st, be = ctypes.c_int(0), ctypes.c_double(0.0)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = lib.gelim_mixed_solve(s._mixed, ptr(aug), aug.stride(0), ptr(x), 20, ctypes.byref(st), ctypes.byref(be), sh)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
    print(f"hip-mixed classic IR n={n}: rc={rc} corrections={st.value} berr={be.value:.2e} time {dt:.2f} ms "
          f"error {gelim.ops.gauss.error_metric(x):.2e}", flush=True)
    s.close()
