"""Accuracy and time of the 128 x 128 block inverse (lu_mixed.hip
diag_inv_pair_kernel) against LAPACK's (torch.linalg.inv) on well- and
ill-conditioned blocks: max |D A - I| and the kernel time (events, 50
back-to-back launches).  Round 6: the pair Gauss-Jordan without the uniform
form's cancellation."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

dev = torch.device("cuda:0")
lib = gelim._native.lib()
g = torch.Generator().manual_seed(3)


def blocks():
    A = torch.randn(128, 128, generator=g, dtype=torch.float64)
    yield "randn", A.clone()
    yield "dominant", A + 16 * torch.eye(128, dtype=torch.float64)
    Q, _ = torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))
    yield "rbt_like_1e4", Q @ torch.diag(torch.logspace(0, 4, 128, dtype=torch.float64)) @ Q.T + 0.1 * A
    Q, _ = torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))
    yield "rbt_like_1e6", Q @ torch.diag(torch.logspace(0, 6, 128, dtype=torch.float64)) @ Q.T + 0.01 * A
    yield "zero", torch.zeros(128, 128, dtype=torch.float64)


for name, A in blocks():
    Ag = A.to(dev)
    cond = torch.linalg.cond(A).item() if A.abs().max() > 0 else float("inf")
    D = torch.empty_like(Ag)
    info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
    sh = stream_handle(dev)
    gelim._native.check(lib.gelim_rbt_block_inverse(ptr(Ag), 128, 0, ptr(D), ptr(info), sh), "inv")
    torch.cuda.synchronize()
    r = (D.cpu() @ A - torch.eye(128, dtype=torch.float64)).abs().max().item()
    rl = (torch.linalg.inv(A) @ A - torch.eye(128, dtype=torch.float64)).abs().max().item() if cond < 1e300 else 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        lib.gelim_rbt_block_inverse(ptr(Ag), 128, 0, ptr(D), ptr(info), sh)
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:14s} cond {cond:9.2e}  |DA-I| {r:8.2e}  (LAPACK {rl:8.2e})  info {info.item():#x}  "
          f"{e0.elapsed_time(e1) / 50 * 1e3:6.1f} us", flush=True)
