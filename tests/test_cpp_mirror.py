"""The reference's unit tests restated in C++ against include/onc_rpc.hpp
(tests/cpp/test_mirror.cpp), executed on the GPU codec."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_mirror")
VECTORS = os.path.join(ROOT, "tests", "golden", "vectors.json")


def test_cpp_mirror_header_compiles():
    """The mirror header builds against the C ABI (build() compiles it)."""
    assert os.path.exists(os.path.join(ROOT, "include", "onc_rpc.hpp"))
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True,
                       capture_output=True, timeout=600)
    assert os.path.exists(BIN)


@pytest.mark.gpu
def test_cpp_mirror_reference_tests():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True, timeout=600)
    r = subprocess.run([BIN, VECTORS], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout
