"""Host time of torch.cuda.is_current_stream_capturing() while the legacy
default stream runs a 1 s kernel (why the RCCL watchdog keeps its own
capture flag)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from gelim import _native  # noqa: E402
from gelim.utils.tensors import dedicated_stream, ptr  # noqa: E402

dev = torch.device("cuda:0")
lib = _native.lib()
words = torch.zeros(2, dtype=torch.int32, device=dev)
torch.cuda.synchronize()
for name, st in (("default", torch.cuda.current_stream(dev)), ("dedicated", dedicated_stream(dev, "comm"))):
    words.zero_()
    torch.cuda.synchronize()
    _native.check(lib.gelim_gpu_probe_kernel(st.cuda_stream, ptr(words), 0, 100_000_000), "probe")
    with torch.cuda.stream(st):
        a = time.perf_counter()
        c = torch.cuda.is_current_stream_capturing()
        print(f"is_current_stream_capturing() on the {name} stream behind a 1 s kernel: {time.perf_counter() - a:.4f} s"
              f" ({c})", flush=True)
    torch.cuda.synchronize()
