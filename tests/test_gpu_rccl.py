"""The RCCL transport on the one MI355X: a ONE-rank `nccl` process group
(init_from_env(force_pg=True)) drives every distributed schedule, so each
broadcast / all_gather / all_reduce / batched p2p is a real RCCL call issued
on the communicator's dedicated stream and ordered against the main and
lookahead side streams by events -- the path an 8-GPU node runs, minus the
links.  Each result must equal, bit for bit, the same schedule on the plain
one-rank communicator (no collective at all): a one-rank collective leaves
the data unchanged, so any difference is an ordering bug (a stream reading a
buffer before its collective landed).

The stream check: a bounded waiter kernel occupies the side stream while a
broadcast is issued and the main stream waits on it; the setter queued after
the broadcast must release the waiter, i.e. the collective does not share the
side stream's hardware queue (the lookahead would otherwise serialise).

Reference: the MPI collectives these replace,
OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:130-206."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = Path(__file__).resolve().parent


@pytest.fixture(scope="module")
def rccl_run(tmp_path_factory, cuda):
    out = tmp_path_factory.mktemp("rccl")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    code = f"import dist_worker; dist_worker.rccl_one_rank({str(out)!r})"
    proc = subprocess.run([sys.executable, "-u", "-c", code], cwd=HERE, env=env, capture_output=True, text=True,
                          timeout=300)
    resf = out / "res.json"
    assert resf.exists(), f"rc={proc.returncode}\n{proc.stdout[-3000:]}\n{proc.stderr[-3000:]}"
    res = json.loads(resf.read_text())
    keep = HERE.parent / "gpurun_out"
    if keep.is_dir():  # on the GPU box: the record travels back with the call
        (keep / "rccl_one_rank_res.json").write_text(resf.read_text())
    assert res.get("ok"), res.get("traceback", res)
    return out, res


def test_rccl_group_is_real(rccl_run):
    _, res = rccl_run
    assert res["backend"] == "nccl" and res["pg"] and res["initialized"] and res["native"]
    assert res["pg_backend"] == "nccl" and res["world"] == 1


def test_rccl_collectives_beside_side_stream(rccl_run):
    _, res = rccl_run
    assert res["overlap_own_stream"] and res["overlap_torch_stream"], res
    s = res["streams"]
    assert len({s["side"], s["comm"], s["default"]}) == 3


@pytest.mark.parametrize("tag", ["gauss_la_tail0", "gauss_la", "gauss_serial"])
def test_rccl_dist_gauss_bitwise(rccl_run, gelim, tag):
    out, res = rccl_run
    r = res[tag]
    assert r["bitwise"] and r["torch_path_bitwise"], r
    if tag == "gauss_la_tail0":
        assert r["panels"] >= 4
    x = torch.load(out / f"{tag}.pt")
    aug = gelim.random_system(2048, seed=41, device="cuda:0").double().cpu()
    ref = torch.linalg.solve(aug[:, :2048], aug[:, 2048])
    assert torch.allclose(x, ref, rtol=1e-7, atol=1e-7)


def test_rccl_dist_rbt_bitwise(rccl_run, gelim):
    out, res = rccl_run
    r = res["rbt"]
    assert r["bitwise"], r
    # the graph-replayed schedule (factorisation + applies captured once, RCCL
    # collectives inside the graph) gives the eager schedule's bits
    assert r["graph_rccl"] and r["graph_none"] and not r["graph_torch_path"], r
    assert r["replay_equals_eager"], r
    assert r["fallback"] is None
    assert r["berr"] <= 4 * torch.finfo(torch.float64).eps  # the strict rule (round 6: accurate block inverses)
    x = torch.load(out / "rbt.pt")
    aug = gelim.random_system(2048, seed=43, device="cuda:0").double().cpu()
    ref = torch.linalg.solve(aug[:, :2048], aug[:, 2048])
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-9


def test_rccl_dist_matmul_bitwise(rccl_run):
    _, res = rccl_run
    assert res["matmul_allgather"]["bitwise"] and res["matmul_allgather"]["rel"] < 1e-5
    assert res["matmul_summa"]["bitwise"]
    assert res["matmul_summa"]["subgroup_backend"] == "nccl" and res["matmul_summa"]["subgroup_pg"]


def test_rccl_p2p_self(rccl_run):
    _, res = rccl_run
    assert res["p2p_self"]["ok"], res["p2p_self"]


@pytest.mark.parametrize("op", ["bcast", "allreduce_sum", "allreduce_max", "allreduce_min", "allgather", "sendrecv"])
@pytest.mark.parametrize("dtype", ["torch.float64", "torch.float32", "torch.int32", "torch.int64", "torch.uint8"])
def test_native_rccl_ops(rccl_run, op, dtype):
    """libgelim's own RCCL communicator (csrc/comm/rccl_comm.hip, torch's
    librccl.so, the id through the process group's store): each collective
    in each supported dtype, one rank, on the current stream."""
    _, res = rccl_run
    assert res["native_ops"][f"{op}_{dtype}"], res["native_ops"]


@pytest.fixture(scope="module")
def watchdog_run(tmp_path_factory, cuda):
    out = tmp_path_factory.mktemp("rccl_wd")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    code = f"import dist_worker; dist_worker.rccl_watchdog({str(out)!r})"
    proc = subprocess.run([sys.executable, "-u", "-c", code], cwd=HERE, env=env, capture_output=True, text=True,
                          timeout=120)
    resf = out / "res.json"
    assert resf.exists(), f"rc={proc.returncode}\n{proc.stdout[-3000:]}\n{proc.stderr[-3000:]}"
    res = json.loads(resf.read_text())
    keep = HERE.parent / "gpurun_out"
    if keep.is_dir():
        (keep / "rccl_watchdog_res.json").write_text(resf.read_text())
    assert res.get("ok"), res.get("traceback", res)
    assert proc.returncode == 0, proc.stderr[-2000:]  # the process exits cleanly after the abort
    return res


def test_rccl_watchdog_wait_point(watchdog_run):
    """A collective stuck behind a 2 s kernel, watchdog timeout 0.5 s: the
    guarded host wait raises CommFailure within ~1 s, every native
    communicator is aborted, and the next collective raises at once
    (gauss_mpi/gauss_internal_input.c:289-297 has no handler)."""
    r = watchdog_run["wait_point"]
    assert watchdog_run["native"]
    assert r["raised"], r
    assert 0.4 <= r["after_s"] <= 1.5, r
    assert r["later_call_raised"] and r["native_left_later"] == 0, r


def test_rccl_watchdog_async(watchdog_run):
    """The same stall with the main thread outside any wait point: the
    watchdog thread raises CommFailure in it."""
    r = watchdog_run["async"]
    assert r["raised"], r
    assert 0.4 <= r["after_s"] <= 1.5, r
    assert r["native_left_later"] == 0, r
