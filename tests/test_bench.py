"""bench.py's launch contract on CPU ranks (gloo): `python bench.py --gpus N`
without a torchrun environment starts N ranks itself (as a child torchrun,
the counterpart of the reference's `mpirun -np P`,
OpenMP_and_MPI/README.txt:23,46) and rank 0's ONE JSON line reports the
world size that actually joined."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _bench(*args, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return r


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks():
    r = _bench("--gpus", "2", "--headline-only", "--n", "96", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stdout + r.stderr
    j = _line(r.stdout)
    assert j["world_size"] == 2 and j["n_gpus"] == 2
    assert j["backend"] == "gloo"
    assert j["launcher"].startswith("self")
    assert j["steps"] == 2 and j["warmup"] == 1
    assert j["max_error"] < 1e-10
    assert j["value"] > 0 and abs(j["ms_per_step"] - 1e3 * j["value"]) < 1e-9


def test_bench_single_rank_cpu():
    r = _bench("--headline-only", "--n", "64", "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stdout + r.stderr
    j = _line(r.stdout)
    assert j["world_size"] == 1 and j["backend"] == "none" and j["launcher"] == "single process"
    # the sequential Gauss denominator is timed in every run (SURVEY.md §6 caveat)
    assert j["host_seq"]["source"].startswith("gauss_64_s measured in this run") or \
        "measured in this run" in j["host_seq"]["source"]
    assert j["host_seq"]["gauss_64_s"] > 0


def test_bench_world_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3", "--headline-only", "--n", "32"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
