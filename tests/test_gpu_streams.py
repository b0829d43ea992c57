"""Lookahead side streams and the hardware queues behind them (runtime.hip
side_stream_create / gelim_gpu_stream_probe, utils/tensors.py side_stream):
a side stream must run concurrently with the default stream, and the probe
must tell a stream that shares the default stream's queue from one that
does not (profiles/hw_queues_r4.txt)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_probe_detects_a_shared_queue(gelim, cuda):
    """The default stream probed against itself is the shared-queue case
    (the waiting kernel times out before the flag is set): 0."""
    from gelim import _native

    with torch.cuda.device(cuda):
        assert _native.lib().gelim_gpu_stream_probe(torch.cuda.default_stream(cuda).cuda_stream) == 0


def test_side_stream_runs_beside_default(gelim, cuda):
    from gelim import _native
    from gelim.utils.tensors import side_stream, side_stream_stats

    s = side_stream(cuda)
    assert side_stream(cuda) is s  # one per process and device: solvers made in a loop add no streams
    before = side_stream_stats()
    assert s.cuda_stream != torch.cuda.default_stream(cuda).cuda_stream
    with torch.cuda.device(cuda):
        assert _native.lib().gelim_gpu_stream_probe(s.cuda_stream) == 1
    after = side_stream_stats()
    assert after[0] == before[0] + 1
    # work on it is ordinary stream work
    with torch.cuda.stream(s):
        x = torch.arange(1000, dtype=torch.float64, device=cuda).mul_(2)
    s.synchronize()
    assert x.sum().item() == 999000.0


def test_unprobed_side_streams_still_solve(gelim, cuda, monkeypatch):
    """GELIM_SIDE_PROBE=0 (plain streams): the plans' lookahead schedules
    give the same bits, only the concurrency guarantee is gone."""
    n = 3000
    aug = gelim.random_system(n, seed=12, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x0 = s.solve(aug.clone()).cpu()
    s.close()
    monkeypatch.setenv("GELIM_SIDE_PROBE", "0")
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x1 = s.solve(aug.clone()).cpu()
    s.close()
    assert torch.equal(x0, x1)


def test_dedicated_streams_pairwise_concurrent(gelim, cuda):
    """The side and comm streams (parallel/comm.py issues collectives on the
    latter) each run beside the default stream and beside each other: a
    bounded waiter on one is released by a setter on the other."""
    from gelim import _native
    from gelim.utils.tensors import dedicated_stream, ptr

    lib = _native.lib()
    side = dedicated_stream(cuda, "side")
    comm = dedicated_stream(cuda, "comm")
    assert dedicated_stream(cuda, "comm") is comm
    streams = {"default": torch.cuda.default_stream(cuda), "side": side, "comm": comm}
    for a, sa in streams.items():
        for b, sb in streams.items():
            if a == b:
                continue
            w = torch.zeros(2, dtype=torch.int32, device=cuda)
            torch.cuda.synchronize(cuda)
            assert lib.gelim_gpu_probe_kernel(sa.cuda_stream, ptr(w), 0, 500000) == 0
            assert lib.gelim_gpu_probe_kernel(sb.cuda_stream, ptr(w), 1, 0) == 0
            torch.cuda.synchronize(cuda)
            assert int(w[1].item()) == 1, f"{b} does not run beside {a}"


def test_dedicated_stream_roles_are_distinct_and_cached(gelim, cuda):
    from gelim.utils.tensors import dedicated_stream

    a = dedicated_stream(cuda, "side")
    b = dedicated_stream(cuda, "comm")
    assert a is dedicated_stream(cuda, "side") and b is dedicated_stream(cuda, "comm")
    assert a.cuda_stream != b.cuda_stream
    assert torch.cuda.default_stream(cuda).cuda_stream not in (a.cuda_stream, b.cuda_stream)
