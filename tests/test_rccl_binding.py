"""libcrdt_gpu binds RCCL at run time (csrc/shard.hip): it does not link librccl, and
in a torch process it binds the librccl.so.1 torch already loaded, so the library's communicator
and torch.distributed run on ONE RCCL of one version.  CPU-only: crdt_ctx_comm_note binds and reads
the version without touching a GPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rust-crdt_amd", "libcrdt_gpu.so")

PROBE = r"""
import ctypes, json, sys
pre = sys.argv[1]
if pre == "torch":
    import torch
lib = ctypes.CDLL(sys.argv[2])
lib.crdt_ctx_comm_note.restype = ctypes.c_char_p
rt, hd = ctypes.c_int(), ctypes.c_int()
lib.crdt_ctx_comm_note(None, ctypes.byref(rt), ctypes.byref(hd))
maps = [l.split()[-1] for l in open("/proc/self/maps") if "librccl" in l]
out = {"runtime": rt.value, "header": hd.value, "rccl_files": sorted(set(maps))}
if pre == "torch":
    v = torch.cuda.nccl.version()
    out["torch"] = v[0] * 10000 + v[1] * 100 + v[2]
print(json.dumps(out))
"""


def _probe(pre, env=None):
    r = subprocess.run([sys.executable, "-c", PROBE, pre, LIB], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr
    import json
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_library_does_not_link_rccl():
    r = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True, check=True)
    needed = [ln for ln in r.stdout.splitlines() if "NEEDED" in ln]
    assert needed and not any("rccl" in ln for ln in needed), needed


def test_binds_one_rccl_without_torch():
    out = _probe("none")
    assert out["runtime"] >= 21800
    assert len(out["rccl_files"]) == 1


def test_binds_torchs_rccl_inside_torch():
    out = _probe("torch")
    assert out["runtime"] == out["torch"], out  # the library and torch.distributed share one RCCL
    assert len(out["rccl_files"]) == 1, out


def test_explicit_rccl_path():
    path = "/opt/rocm/lib/librccl.so.1"
    if not os.path.exists(path):
        import pytest
        pytest.skip("no /opt/rocm RCCL")
    out = _probe("none", env=dict(os.environ, CRDT_RCCL_LIB=path))
    assert out["runtime"] >= 21800 and any(f.startswith("/opt/rocm") for f in out["rccl_files"]), out
