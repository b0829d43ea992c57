"""Host code under sanitizers: every CPU backend and CPU
building block of libgelim, built with ASan+UBSan (all backends, OpenMP
included) and with TSan (the pthreads V1/V2/V3 backends — libgomp is not
TSan-instrumented, so OpenMP regions would only give false positives).
The reference's Pthreads V3 overflows its stack at -t > 32 and has a racy
condvar barrier; ours runs 40 pinned threads clean."""
import shutil
import subprocess

import pytest

from conftest import REF_DATA, ROOT

SRC = ["core/errors.cpp", "core/io.cpp", "core/init.cpp", "cpu/gauss_cpu.cpp", "cpu/matmul_cpu.cpp",
       "tools/sanitize_check.cpp"]


def _build(tmp_path, flags, name):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    out = tmp_path / name
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fopenmp", "-fno-omit-frame-pointer", *flags,
           "-I", str(ROOT / "csrc" / "include"), *[str(ROOT / "csrc" / s) for s in SRC], "-o", str(out), "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return out


def test_asan_ubsan_all_backends(tmp_path):
    exe = _build(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "asan")
    args = [str(exe), "all"]
    if (REF_DATA / "matrix_10.dat").exists():
        args.append(str(REF_DATA / "matrix_10.dat"))
    r = subprocess.run(args, capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "OMP_NUM_THREADS": "4"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize_check all: ok" in r.stdout
    assert "runtime error" not in r.stderr


def test_tsan_pthreads_backends(tmp_path):
    exe = _build(tmp_path, ["-fsanitize=thread"], "tsan")
    r = subprocess.run([str(exe), "pthreads"], capture_output=True, text=True, timeout=300,
                       env={"TSAN_OPTIONS": "halt_on_error=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ThreadSanitizer" not in r.stderr
