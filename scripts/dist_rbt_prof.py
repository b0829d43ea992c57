"""One rank of the distributed randomised solver (parallel/dist_rbt.py) on the
distributed SCHEDULE (single_fast_path=False): wall time per solve and, under
rocprofv3 --kernel-trace, the per-kernel durations the 8-rank critical-path
estimate is built from (scripts/dist_rbt_critical_path.py).

  rocprofv3 --kernel-trace -d gpurun_out/drbt -o run -- python3 scripts/dist_rbt_prof.py 8192
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.parallel import DistributedRBT  # noqa: E402
from gelim.parallel.comm import Communicator  # noqa: E402


def micro():
    """Uncontended kernel times of the distributed engine's critical-path
    pieces (CUDA events over 50 back-to-back calls): the 128 x 128 block
    inverse, the super-block solve for P = 1, 2, 4, 8 blocks, the GEMV."""
    import ctypes  # noqa: F401

    from gelim.utils.tensors import ptr, stream_handle

    dev = torch.device("cuda:0")
    lib = gelim._native.lib()
    sh = stream_handle(dev)
    g = torch.Generator(device=dev).manual_seed(0)

    def timed(fn, reps=50):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    blk = torch.randn(128, 130, dtype=torch.float64, device=dev, generator=g)[:, :128] + 16 * torch.eye(
        128, dtype=torch.float64, device=dev)
    dinv = torch.empty(128, 128, dtype=torch.float64, device=dev)
    info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
    t = timed(lambda: lib.gelim_rbt_block_inverse(ptr(blk), blk.stride(0), 0, ptr(dinv), ptr(info), sh))
    print(f"block inverse 128 x 128: {t:.1f} us", flush=True)
    for P in (1, 2, 4, 8):
        S = 128 * P
        Fs = torch.randn(S, S, dtype=torch.float64, device=dev, generator=g)
        Ds = torch.randn(P, 128, 128, dtype=torch.float64, device=dev, generator=g)
        rhs = torch.randn(S, dtype=torch.float64, device=dev, generator=g)
        x = torch.empty(S, dtype=torch.float64, device=dev)
        y = torch.empty(S, dtype=torch.float64, device=dev)
        t = timed(lambda: lib.gelim_drbt_super_solve(ptr(Fs), S, ptr(Ds), P, ptr(rhs), ptr(x), ptr(y), 0, sh))
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        t2 = timed(lambda: lib.gelim_rbt_block_solve(ptr(Fs), S, ptr(Ds), P, ptr(rhs), ptr(x), ptr(y), 0, ptr(err), sh))
        t3 = timed(lambda: lib.gelim_rbt_block_solve(ptr(Fs), S, ptr(Ds), P, ptr(rhs), ptr(x), None, 1, ptr(err), sh))
        print(f"super-block solve, P = {P} (S = {S}): one-workgroup kernel {t:.1f} us, persistent block solve "
              f"lower {t2:.1f} / upper {t3:.1f} us (err {int(err.item())})", flush=True)
    A = torch.randn(8192, 130, dtype=torch.float64, device=dev, generator=g)[:, :128]
    xv = torch.randn(128, dtype=torch.float64, device=dev, generator=g)
    yv = torch.zeros(8192, dtype=torch.float64, device=dev)
    t = timed(lambda: lib.gelim_drbt_gemv(ptr(A), A.stride(0), 8192, 128, ptr(xv), ptr(yv), 1.0, sh))
    print(f"gemv 8192 x 128: {t:.1f} us", flush=True)
    X = torch.randn(8192 * 128, dtype=torch.float64, device=dev, generator=g)
    M = torch.randn(8192, 1026, dtype=torch.float64, device=dev, generator=g)
    t = timed(lambda: X.view(8192, 128).copy_(M[:, 128:256]))
    print(f"column pack 8192 x 128 (8.4 MB): {t:.1f} us", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--micro":
        return micro()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    dev = torch.device("cuda:0")
    c = Communicator(0, 1, dev, "none")
    for fast in (True, False):
        d = DistributedRBT(c, n, single_fast_path=fast)
        ts = []
        for _ in range(3):
            loc = d.generate_random(seed=99)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x = d.solve_(loc)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"n={n} fast_path={fast}: solve {min(ts) * 1e3:.2f} ms (best of 3), error "
              f"{gelim.ops.gauss.error_metric(x):.2e}, corrections {d.last_steps}, fallback {d.last_fallback}",
              flush=True)
        d.close()


if __name__ == "__main__":
    main()
