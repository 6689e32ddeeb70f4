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
    assert lib.crdt_version() == b"0.8.0"
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
    assert ctypes.sizeof(abi.MapCounterBatch) == 18 * 8
    assert ctypes.sizeof(abi.MapCounterOut) == 6 * 8
    assert ctypes.sizeof(abi.MapOrswotBatch) == 17 * 8
    assert ctypes.sizeof(abi.MapOrswotOut) == 11 * 8  # (+ Vd, ABI 8)
    assert ctypes.sizeof(abi.MapOrswotStates) == 12 * 8
    assert ctypes.sizeof(abi.MapNestedStates) == 16 * 8 and ctypes.sizeof(abi.MapNestedOut) == 15 * 8


HOST_CAPABLE = ({f"crdt_{t}_{op}" for t in ("vclock", "gcounter", "pncounter", "gset", "lwwreg", "orswot", "map")
                 for op in ("lub_many", "merge_batch")}
                | {"crdt_map_counter_lub_many", "crdt_map_orswot_lub_many", "crdt_map_nested_lub_many"})
CTX_ONLY = {"crdt_ctx_destroy", "crdt_ctx_set_stream", "crdt_ctx_synchronize", "crdt_ctx_set_timing",
            "crdt_ctx_timing", "crdt_ctx_timing_reset", "crdt_ctx_tune", "crdt_ctx_set_mem_kind",
            "crdt_ctx_comm_init", "crdt_ctx_comm_destroy", "crdt_ctx_comm_info", "crdt_ctx_mem_kind",
            "crdt_ctx_comm_init_ops", "crdt_device_alloc", "crdt_device_free"}  # (allocation, no compute)


def test_every_compute_entry_point_guards_host_mode():
    """CRDT_MEM_HOST (include/crdt_gpu.h) is honoured by the lattice / lwwreg entry points only;
    every other entry point taking a ctx must refuse it (CRDT_DEVICE_MEM_ONLY as its first
    statement) rather than read host pointers as device memory."""
    import glob
    pat = re.compile(r'^(?:extern "C" )?int\s+(crdt_\w+)\(([^)]*)\)\s*\{\n(.*?)\n', re.M | re.S)
    seen = set()
    for f in glob.glob(os.path.join(ROOT, "rust-crdt_amd", "csrc", "*.*")):
        for m in pat.finditer(open(f).read()):
            name, args, first = m.group(1), m.group(2), m.group(3).strip()
            if "crdt_ctx *ctx" not in args:
                continue
            seen.add(name)
            if name in HOST_CAPABLE:
                assert ("CRDT_CHECK_CTX" in first or "_dispatch(ctx" in first or first.startswith("return crdt_")
                        or "_host(ctx" in first or "mem_kind == CRDT_MEM_HOST" in first), name
            elif name.endswith("_sharded") or name.endswith("_sharded_doff"):
                # collective: the host-mode refusal is part of the agreed validation status (every
                # rank must learn it), so it is not the first statement (csrc/shard.hip); the Orswot
                # and Map pairs share an impl that makes that check
                body = open(f).read()[m.end(2):]
                body = body[:body.index("\n}\n")]
                impl = re.match(r"return (lattice_sharded|orswot_sharded_impl|map_sharded_impl)\(", first)
                if not impl:  # (round 5: the value-typed Maps validate their batch first, then the impl)
                    impl = re.search(r"return (vmap_sharded_impl)\(", body)
                assert impl or "device_mem_only(ctx, what)" in body, name
                if impl:
                    src = open(f).read()
                    i = src.index(f"static int {impl.group(1)}(")
                    assert "device_mem_only(ctx, what)" in src[i:src.index("\n}\n", i)], impl.group(1)
            elif name not in CTX_ONLY:
                assert first.startswith("CRDT_DEVICE_MEM_ONLY(ctx);"), (f, name)
    assert HOST_CAPABLE <= seen and len(seen) > 50
