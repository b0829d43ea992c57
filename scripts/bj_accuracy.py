import os, sys
sys.path.insert(0, '/root/repo')
import torch, gelim
from gelim.utils.tensors import ptr, stream_handle
dev = torch.device('cuda:0'); lib = gelim._native.lib(); sh = stream_handle(dev)
g = torch.Generator().manual_seed(1)
for kind in ("dominant", "randn", "rbt_like"):
    A = torch.randn(128, 128, generator=g, dtype=torch.float64)
    if kind == "dominant": A += 64 * torch.eye(128, dtype=torch.float64)
    elif kind == "rbt_like":
        Q, _ = torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))
        A = Q @ torch.diag(torch.logspace(0, 4, 128, dtype=torch.float64)) @ Q.T + 0.1 * A
    Ag = A.to(dev)
    cond = torch.linalg.cond(A).item()
    line = f"{kind:9s} cond {cond:9.2e}"
    for form in ("0", "1", "2"):
        os.environ["GELIM_GJ_BLOCKED"] = form
        D = torch.empty(128, 128, dtype=torch.float64, device=dev)
        info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
        lib.gelim_rbt_block_inverse(ptr(Ag), 128, 0, ptr(D), ptr(info), sh); torch.cuda.synchronize()
        r = (D.cpu() @ A - torch.eye(128, dtype=torch.float64)).abs().max().item()
        line += f" | form {form}: |DA-I| {r:.2e}"
    print(line, flush=True)
