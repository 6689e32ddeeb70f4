"""CPU checks of the C-ABI boundary: the library loads and exports every declared symbol
(no compute calls without a GPU), and the product raises instead of falling back."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "crdt_gpu.h")
LIB = os.path.join(ROOT, "rust-crdt_amd", "libcrdt_gpu.so")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(crdt_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared()
    for t in ("vclock", "gcounter", "pncounter", "gset"):
        assert f"crdt_{t}_lub_many" in names and f"crdt_{t}_merge_batch" in names
    assert "crdt_lwwreg_lub_many" in names and "crdt_orswot_lub_many" in names
    assert "crdt_map_lub_many" in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build with `make -C rust-crdt_amd`"
    lib = ctypes.CDLL(LIB)
    for name in declared():
        assert hasattr(lib, name), name
    import crdts_gpu._abi as abi
    assert sorted(abi.EXPORTS) == declared()
    lib.crdt_version.restype = ctypes.c_char_p
    assert lib.crdt_version() == b"0.1.0"
    lib.crdt_build_target.restype = ctypes.c_char_p
    assert lib.crdt_build_target() == b"gfx950"


def test_code_objects_are_gfx950():
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_ctx_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("host has a GPU")
    import crdts_gpu
    with pytest.raises(crdts_gpu.CrdtGpuUnavailable):
        crdts_gpu.Context(0)


def test_ctypes_struct_layout_matches_header():
    import crdts_gpu._abi as abi
    # 4 dims + ptr + 2 strides + ptr + 3 strides + 3 ptrs = 14 eight-byte fields
    assert ctypes.sizeof(abi.OrswotBatch) == 14 * 8
    assert ctypes.sizeof(abi.OrswotOut) == 4 * 8
    # 5 dims + 4 x (ptr + 2 strides) + def_off + 3 ptrs = 21; out: Vout, Vstate + 8 ptrs = 10
    assert ctypes.sizeof(abi.MapBatch) == 21 * 8
    assert ctypes.sizeof(abi.MapOut) == 10 * 8
