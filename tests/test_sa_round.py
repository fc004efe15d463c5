"""The device's superaccumulator rounding (csrc/sa_round.h sa_round_fast, used by
finalize_round for the dangling mass, residual and rank sum) must equal the bit-loop form it
replaced, bit for bit.  Host-compiled with g++ (the header is plain C++ outside hipcc)."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "page-rank-and-tfidf-using-apache-spark_amd" / "csrc"


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sa_round_fast_equals_bit_loop(tmp_path):
    exe = tmp_path / "sa_round_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(CSRC),
                    str(ROOT / "tests" / "native" / "sa_round_check.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe), "600000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok 600000")
