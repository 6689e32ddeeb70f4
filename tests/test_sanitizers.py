"""CPU sanitizer runs ("hipcc -fsanitize=address on the CPU oracle + host code";
VERDICT r2 #8).  Three builds, all CPU-only:

  * the oracle (oracle/ref_fold.cpp) under ASan + UBSan (`make -C oracle asan`), loaded through
    ORACLE_LIB by a pytest child with libasan / libubsan preloaded: the oracle KATs and twin tests
    run against it;
  * the sharded entry points' host bookkeeping (rust-crdt_amd/csrc/shard_host.hpp: agreement headers,
    Orswot regrouping, the LWW prefix, the Map flag exchange), g++ -fsanitize=address,undefined
    (tests/cpp/test_shard_host.cpp);
  * the C++ host mirror's host-only paths (rust-crdt_amd/host/crdts.hpp: interning, dense encode /
    decode, host CmRDT::apply), hipcc with -Xarch_host -fsanitize=... (tests/cpp/test_host_sanitize.cpp).
A sanitizer report aborts the program (-fno-sanitize-recover / halt_on_error), failing the test."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _gcc_lib(name):
    return subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True, capture_output=True)
    lib = os.path.join(ROOT, "oracle", "build", "liboracle_asan.so")
    env = dict(os.environ, LD_PRELOAD=f"{_gcc_lib('libasan.so')}:{_gcc_lib('libubsan.so')}",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", ORACLE_LIB=lib)
    probe = ("import sys, ctypes; sys.path.insert(0, %r); import oracle as O; "
             "assert O.lib()._name.endswith('liboracle_asan.so'); ctypes.CDLL(None).__asan_init; print('asan ok')"
             % os.path.join(ROOT, "oracle"))
    r = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "asan ok" in r.stdout, r.stderr[-3000:]
    tests = [os.path.join(ROOT, "tests", t) for t in ("test_oracle_kat.py", "test_oracle_twins.py",
                                                      "test_oracle_map_dense.py", "test_oracle_orswot_apply.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:xdist", "-p", "no:cacheprovider", *tests],
                       env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_shard_host_bookkeeping_under_asan_ubsan(tmp_path):
    exe = tmp_path / "test_shard_host"
    subprocess.run(["g++", "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "rust-crdt_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "test_shard_host.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "all checks passed" in r.stdout, r.stderr[-3000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_host_mirror_under_asan_ubsan(tmp_path):
    exe = tmp_path / "test_host_sanitize"
    subprocess.run([HIPCC, "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", "-Xarch_host", "-fsanitize=address",
                    "-Xarch_host", "-fsanitize=undefined", "-Xarch_host", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "rust-crdt_amd", "host"),
                    os.path.join(ROOT, "tests", "cpp", "test_host_sanitize.cpp"), "-o", str(exe)],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "all checks passed" in r.stdout, r.stderr[-3000:]
