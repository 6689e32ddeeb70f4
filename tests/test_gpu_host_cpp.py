"""Runs the C++ host-mirror tests (tests/cpp/test_host.cpp): the reference's own tests restated
in C++ over rust-crdt_amd/host/crdts.hpp, every merge on the GPU through the C ABI."""
import os
import subprocess

import pytest

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "test_host")


def test_host_binary_is_built():
    assert os.path.exists(BIN), "build with `make -C rust-crdt_amd` (or __graft_entry__.build())"


@pytest.mark.gpu
def test_cpp_host_mirror_on_gpu():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr
    assert "0 failed" in r.stdout
