"""Isolated timings of the wide-panel LU pieces on one GPU (hipEvent around
each launch) and the leaf's in-kernel phase stamps.

  python scripts/leaf_bench.py [m]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim import _native  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main() -> None:
    m = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 8192
    dev = torch.device("cuda:0")
    lib = _native.lib()
    sh = stream_handle(dev)
    lda = m + 8
    A0 = torch.rand(m, lda, dtype=torch.float64, device=dev) * 2 - 1
    A = A0.clone()
    ws = torch.zeros(int(lib.gelim_gpu_leaf_workspace_bytes()) // 8, dtype=torch.float64, device=dev)
    ipiv = torch.zeros(m + 64, dtype=torch.int32, device=dev)
    pairs = torch.zeros(256, dtype=torch.int32, device=dev)
    info = torch.zeros(4, dtype=torch.int32, device=dev)

    counter = [0]

    def leaf():
        # a fresh leaf counter per call, as in a solve: granules are tagged with
        # it, so a rerun can never read the previous run's (identical) granules
        # as current and skip the exchange waits
        A.copy_(A0)
        counter[0] += 1
        _native.check(lib.gelim_gpu_leaf_factor_ws(ptr(A), lda, m, 0, 1, ptr(ipiv), ptr(pairs), ptr(info), ptr(ws),
                                                   counter[0], sh), "leaf")

    def copy_only():
        A.copy_(A0)

    t_leaf = timeit(leaf) - timeit(copy_only)
    print(f"leaf m={m} ("
          f"{lib.gelim_gpu_leaf_participants(m)} participants): {t_leaf:.1f} us ({t_leaf / 32:.2f} us/column)")
    if "--time-only" in sys.argv:
        return
    leaf()
    torch.cuda.synchronize()

    def laswp():
        _native.check(lib.gelim_gpu_laswp_trsm(ptr(A), lda, 0, 0, 32, m + 1, 32, m, ptr(pairs), sh), "laswp")

    print(f"laswp+trsm (swap only) over {m + 1} columns, {pairs[0].item()} pairs: {timeit(laswp):.1f} us")

    def trsm():
        _native.check(lib.gelim_gpu_laswp_trsm(ptr(A), lda, 0, 0, 32, m + 1, m + 1, m, None, sh), "trsm")

    print(f"trsm only over {m + 1} columns: {timeit(trsm):.1f} us")
    # phase stamps
    P = int(lib.gelim_gpu_leaf_participants(m))
    st = torch.zeros(P * 32 * 8, dtype=torch.int64, device=dev)
    A.copy_(A0)
    _native.check(lib.gelim_debug_leaf_stamps(ptr(A), lda, m, ptr(ws), ptr(st), sh), "stamps")
    torch.cuda.synchronize()
    s = st.view(P, 32, 8).cpu()
    names = ["argmax", "publish", "keysweep", "rowload", "prow", "update"]
    for wg in (0, P - 1):
        print(f"participant {wg}: shader cycles per phase (avg over columns; column 0; column 31)")
        d = (s[wg, :, 1:7] - s[wg, :, 0:6]).double()
        for i, nme in enumerate(names):
            print(f"  {nme:8s} avg {d[:, i].mean().item():8.0f}  col0 {d[0, i].item():8.0f}  col31 {d[31, i].item():8.0f}")
        tot = (s[wg, 1:, 0] - s[wg, :-1, 0]).double()
        sw = s[wg, :, 7]
        print(f"  column-to-column avg {tot.mean().item():.0f} cycles; key sweeps/column "
              f"{(sw % 256).double().mean().item():.1f}, row loads/column {(sw // 256).double().mean().item():.1f}")


if __name__ == "__main__":
    main()
