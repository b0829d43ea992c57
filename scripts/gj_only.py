"""Run the 128 x 128 block inverse (gelim_rbt_block_inverse) 20 times, for
PMC passes over that one kernel (scripts/pmc_gj.sh)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

dev = torch.device("cuda:0")
lib = gelim._native.lib()
sh = stream_handle(dev)
g = torch.Generator(device=dev).manual_seed(0)
blk = torch.randn(128, 130, dtype=torch.float64, device=dev, generator=g)[:, :128] + 16 * torch.eye(
    128, dtype=torch.float64, device=dev)
dinv = torch.empty(128, 128, dtype=torch.float64, device=dev)
info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
for _ in range(20):
    gelim._native.check(lib.gelim_rbt_block_inverse(ptr(blk), blk.stride(0), 0, ptr(dinv), ptr(info), sh), "inv")
torch.cuda.synchronize()
print("ok")
