"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the host C / C++ code (sanitizers),
on the CPU: the product path's CSV writer / reader (trajectory_generation_amd/csrc/dataset_csv.cpp) and the C oracle
(oracle/traj_oracle.c, riccati_ipm.c), each driven by a harness under tests/sanitize/ and built with
-fsanitize=address,undefined -fno-sanitize-recover (any report fails the run; leaks are reported at exit).  The
GPU kernels are out of reach here: GPU sanitizers are not available on this pool."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:strict_string_checks=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, **kw)
    assert r.returncode == 0, (cmd, r.stdout[-3000:], r.stderr[-3000:])
    return r


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_dataset_csv_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "san_csv")
    _run(["g++", *SAN, "-std=c++17", "-pthread", "-o", exe,
          os.path.join(ROOT, "trajectory_generation_amd", "csrc", "dataset_csv.cpp"),
          os.path.join(HERE, "sanitize", "san_csv.cpp")])
    r = _run([exe, str(tmp_path)], env=ENV)
    assert "san_csv ok" in r.stdout and "ERROR" not in r.stderr


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "san_oracle")
    _run(["gcc", *SAN, "-fopenmp", "-ffp-contract=off", "-o", exe,
          os.path.join(ROOT, "oracle", "traj_oracle.c"), os.path.join(ROOT, "oracle", "riccati_ipm.c"),
          os.path.join(HERE, "sanitize", "san_oracle.c"), "-lm"])
    r = _run([exe], env=ENV)
    assert "san_oracle ok" in r.stdout and "ERROR" not in r.stderr
