"""ctypes binding of libcrdt_gpu.so (include/crdt_gpu.h).

This is the only way the package reaches the kernels.  There is no CPU fallback: if the
library is missing or no HIP device is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # rust-crdt_amd/
LIB_PATH = os.environ.get("CRDT_GPU_LIB", os.path.join(PKG_ROOT, "libcrdt_gpu.so"))

CRDT_OK = 0
CRDT_EINVAL = -1
CRDT_EHIP = -2
CRDT_ENOMEM = -3
CRDT_EUNSUPPORTED = -4
CRDT_ECOMM = -5
CRDT_UNIQUE_ID_BYTES = 128
CRDT_ACCUMULATE = 0x1
CRDT_MEM_DEVICE = 0
CRDT_ABI_VERSION = 8  # include/crdt_gpu.h
CRDT_MEM_HOST = 1
CRDT_KIND = {"vclock": 1, "gcounter": 2, "pncounter": 3, "gset": 4}
CRDT_RED_MAX, CRDT_RED_MIN, CRDT_RED_SUM = 0, 1, 2

# Every symbol declared in include/crdt_gpu.h (checked by tests/test_abi.py).
EXPORTS = (
    "crdt_ctx_create", "crdt_ctx_destroy", "crdt_ctx_set_stream", "crdt_ctx_synchronize",
    "crdt_last_error", "crdt_version", "crdt_abi_version", "crdt_build_target", "crdt_ctx_set_timing",
    "crdt_ctx_timing", "crdt_ctx_timing_reset", "crdt_ctx_tune",
    "crdt_vclock_lub_many", "crdt_vclock_merge_batch",
    "crdt_gcounter_lub_many", "crdt_gcounter_merge_batch",
    "crdt_pncounter_lub_many", "crdt_pncounter_merge_batch",
    "crdt_gset_lub_many", "crdt_gset_merge_batch",
    "crdt_lwwreg_lub_many", "crdt_lwwreg_merge_batch",
    "crdt_orswot_lub_many", "crdt_orswot_apply_batch", "crdt_map_lub_many",
    "crdt_vclock_pair_op", "crdt_vclock_partial_cmp", "crdt_vclock_cmp_matrix", "crdt_gcounter_read",
    "crdt_pncounter_read", "crdt_vclock_apply_batch", "crdt_gcounter_apply_batch",
    "crdt_pncounter_apply_batch", "crdt_gset_apply_batch",
    "crdt_synth_fill", "crdt_synth_orswot", "crdt_synth_orswot_rm", "crdt_synth_map",
    "crdt_comm_unique_id", "crdt_ctx_comm_init", "crdt_ctx_comm_destroy", "crdt_ctx_comm_info",
    "crdt_vclock_lub_many_sharded", "crdt_gcounter_lub_many_sharded", "crdt_pncounter_lub_many_sharded",
    "crdt_gset_lub_many_sharded", "crdt_orswot_lub_many_sharded",
    "crdt_lwwreg_lub_many_sharded", "crdt_map_lub_many_sharded",
    "crdt_vclock_ingest", "crdt_pncounter_ingest", "crdt_gset_ingest", "crdt_lwwreg_ingest", "crdt_orswot_ingest",
    "crdt_vclock_egress", "crdt_pncounter_egress", "crdt_gset_egress", "crdt_lwwreg_egress", "crdt_orswot_egress",
    "crdt_orswot_forget_batch", "crdt_map_forget_batch", "crdt_map_apply_batch",
    "crdt_orswot_merge_batch", "crdt_map_merge_batch",
    "crdt_ctx_set_mem_kind", "crdt_ctx_mem_kind", "crdt_host_alloc", "crdt_host_free",
    "crdt_device_alloc", "crdt_device_free",
    "crdt_lub_many_multi", "crdt_lub_many_multi_sharded", "crdt_map_ingest", "crdt_map_egress",
    "crdt_ctx_comm_init_ops", "crdt_ctx_comm_note",
    "crdt_mvreg_lub_many", "crdt_mvreg_merge_batch", "crdt_mvreg_apply_batch",
    "crdt_orswot_lub_many_doff", "crdt_map_lub_many_doff",
    "crdt_orswot_lub_many_sharded_doff", "crdt_map_lub_many_sharded_doff", "crdt_map_counter_lub_many", "crdt_map_orswot_lub_many",
    "crdt_map_nested_lub_many", "crdt_map_counter_lub_many_sharded", "crdt_map_orswot_lub_many_sharded",
    "crdt_map_nested_lub_many_sharded", "crdt_map_counter_forget_batch", "crdt_map_orswot_forget_batch",
    "crdt_map_counter_apply_batch", "crdt_map_orswot_apply_batch",
    "crdt_map_nested_apply_batch", "crdt_map_nested_forget_batch", "crdt_map_nested_ingest", "crdt_map_nested_egress",
    "crdt_map_counter_merge_batch", "crdt_map_orswot_merge_batch", "crdt_map_nested_merge_batch",
    "crdt_map_counter_ingest", "crdt_map_counter_egress", "crdt_map_orswot_ingest", "crdt_map_orswot_egress",
)


class CrdtGpuError(RuntimeError):
    """A libcrdt_gpu call returned a negative status."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} -> {code}: {msg}")
        self.code = code


class CrdtGpuUnavailable(RuntimeError):
    """libcrdt_gpu.so is not built (or not loadable): there is no CPU fallback."""


P = ctypes.c_void_p
S = ctypes.c_size_t
U64 = ctypes.c_uint64


class OrswotBatch(ctypes.Structure):
    _fields_ = [
        ("G", S), ("R", S), ("M", S), ("A", S),
        ("clock", P), ("clock_rstride", S), ("clock_gstride", S),
        ("entries", P), ("entry_mstride", S), ("entry_rstride", S), ("entry_gstride", S),
        ("def_off", ctypes.POINTER(S)), ("def_clock", P), ("def_members", P),
    ]


class OrswotOut(ctypes.Structure):
    _fields_ = [("clock", P), ("entries", P), ("def_keep", P), ("def_members", P)]


class OrswotStates(ctypes.Structure):  # crdt_orswot_states
    _fields_ = [
        ("N", S), ("M", S), ("A", S), ("Dcap", S),
        ("clock", P), ("clock_stride", S), ("entries", P), ("entry_mstride", S), ("entry_sstride", S),
        ("def_clock", P), ("def_members", P), ("def_count", P),
    ]


class OrswotOps(ctypes.Structure):  # crdt_orswot_ops
    _fields_ = [
        ("n_ops", S), ("op_off", P), ("kind", P), ("actor", P), ("counter", P), ("rm_row", P),
        ("rm_clock", P), ("n_rm_rows", S), ("mem_off", P), ("mem", P), ("n_mem", S),
    ]


class OrswotShardedOut(ctypes.Structure):  # crdt_orswot_sharded_out
    _fields_ = [("clock", P), ("entries", P), ("def_cap", S), ("def_clock", P), ("def_members", P),
                ("def_group", P), ("ndef", ctypes.POINTER(S))]


class MapStates(ctypes.Structure):  # crdt_map_states
    _fields_ = [("N", S), ("K", S), ("A", S), ("V", S), ("clock", P), ("clock_stride", S), ("ec", P),
                ("ec_stride", S), ("vclk", P), ("vclk_stride", S), ("vval", P), ("vval_stride", S)]


class MapCounterStates(ctypes.Structure):  # crdt_map_counter_states
    _fields_ = [("N", S), ("K", S), ("A", S), ("W", S), ("clock", P), ("clock_stride", S), ("ec", P),
                ("ec_stride", S), ("val", P), ("val_stride", S)]


class MapOrswotStates(ctypes.Structure):  # crdt_map_orswot_states
    _fields_ = [("N", S), ("K", S), ("M", S), ("A", S), ("clock", P), ("ec", P), ("oc", P), ("ent", P),
                ("vd_n", P), ("vd_clock", P), ("vd_mem", P), ("Vd", S)]


class MapNestedStates(ctypes.Structure):  # crdt_map_nested_states
    _fields_ = [("N", S), ("K", S), ("K2", S), ("A", S), ("clock", P), ("ec", P), ("ic", P), ("iec", P), ("ivc", P),
                ("ivv", P), ("nval", P), ("id_n", P), ("id_clock", P), ("id_keys", P), ("Id", S), ("Vs", S)]


class MapNestedOps(ctypes.Structure):  # crdt_map_nested_ops
    _fields_ = [("n_ops", S), ("op_off", P), ("kind", P), ("actor", P), ("counter", P), ("key", P), ("ikind", P),
                ("iactor", P), ("icounter", P), ("ikey", P), ("val", P), ("ikeys", P), ("clk_row", P),
                ("clk_pool", P), ("n_clk_rows", S), ("key_off", P), ("keys", P), ("n_keys", S)]


class MapCounterOps(ctypes.Structure):  # crdt_map_counter_ops
    _fields_ = [("n_ops", S), ("op_off", P), ("kind", P), ("actor", P), ("counter", P), ("key", P), ("vactor", P),
                ("vcounter", P), ("vdir", P), ("clk_row", P), ("clk_pool", P), ("n_clk_rows", S), ("key_off", P),
                ("keys", P), ("n_keys", S)]


class MapOrswotOps(ctypes.Structure):  # crdt_map_orswot_ops
    _fields_ = [("n_ops", S), ("op_off", P), ("kind", P), ("actor", P), ("counter", P), ("key", P), ("vkind", P),
                ("vactor", P), ("vcounter", P), ("clk_row", P), ("clk_pool", P), ("n_clk_rows", S), ("key_off", P),
                ("keys", P), ("n_keys", S), ("mem_off", P), ("mems", P), ("n_mems", S)]


class MapOps(ctypes.Structure):  # crdt_map_ops
    _fields_ = [("n_ops", S), ("op_off", P), ("kind", P), ("actor", P), ("counter", P), ("key", P), ("val", P),
                ("clk_row", P), ("clk_pool", P), ("n_clk_rows", S), ("key_off", P), ("keys", P),
                ("n_keys", S)]


class MapDeferred(ctypes.Structure):  # crdt_map_deferred
    _fields_ = [("clock", P), ("keys", P), ("count", P), ("Dcap", S)]


class LubSegment(ctypes.Structure):  # crdt_lub_segment
    _fields_ = [("kind", ctypes.c_int), ("in_", P), ("G", S), ("R", S), ("A", S), ("row_stride", S),
                ("group_stride", S), ("out", P), ("out_stride", S), ("flags", ctypes.c_uint)]


class MVRegStates(ctypes.Structure):  # crdt_mvreg_states
    _fields_ = [("N", S), ("A", S), ("V", S), ("vclk", P), ("vclk_stride", S), ("vval", P), ("vval_stride", S)]


class MVRegBatch(ctypes.Structure):  # crdt_mvreg_batch
    _fields_ = [("G", S), ("R", S), ("A", S), ("V", S), ("vclk", P), ("vclk_rstride", S), ("vclk_gstride", S),
                ("vval", P), ("vval_rstride", S), ("vval_gstride", S)]


class MVRegOut(ctypes.Structure):  # crdt_mvreg_out
    _fields_ = [("Vout", S), ("Vstate", S), ("vclk", P), ("vval", P), ("nval", P), ("flags", P)]


class MVRegOps(ctypes.Structure):  # crdt_mvreg_ops
    _fields_ = [("n_ops", S), ("op_off", P), ("clk_row", P), ("clk_pool", P), ("n_clk_rows", S), ("val", P)]


# crdt_comm_ops: the caller's own collectives (host buffers)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                ctypes.c_int)


class CommOps(ctypes.Structure):  # crdt_comm_ops
    _fields_ = [("user", P), ("allgather", ALLGATHER_FN), ("allreduce_u64", ALLREDUCE_FN)]


class MapBatch(ctypes.Structure):  # crdt_map_batch
    _fields_ = [
        ("G", S), ("R", S), ("K", S), ("A", S), ("V", S),
        ("clock", P), ("clock_rstride", S), ("clock_gstride", S),
        ("ec", P), ("ec_rstride", S), ("ec_gstride", S),
        ("vclk", P), ("vclk_rstride", S), ("vclk_gstride", S),
        ("vval", P), ("vval_rstride", S), ("vval_gstride", S),
        ("def_off", ctypes.POINTER(S)), ("def_row", P), ("def_clock", P), ("def_keys", P),
    ]


class MapCounterBatch(ctypes.Structure):  # crdt_map_counter_batch
    _fields_ = [
        ("G", S), ("R", S), ("K", S), ("A", S), ("W", S),
        ("clock", P), ("clock_rstride", S), ("clock_gstride", S),
        ("ec", P), ("ec_rstride", S), ("ec_gstride", S),
        ("val", P), ("val_rstride", S), ("val_gstride", S),
        ("def_off", ctypes.POINTER(S)), ("def_row", P), ("def_clock", P), ("def_keys", P),
    ]


class MapCounterOut(ctypes.Structure):  # crdt_map_counter_out
    _fields_ = [("clock", P), ("ec", P), ("val", P), ("flags", P), ("def_keep", P), ("def_keys", P)]


class MapOrswotBatch(ctypes.Structure):  # crdt_map_orswot_batch
    _fields_ = [
        ("G", S), ("R", S), ("K", S), ("M", S), ("A", S),
        ("clock", P), ("ec", P), ("oc", P), ("ent", P),
        ("vd_off", P), ("vd_clock", P), ("vd_mem", P),
        ("def_off", ctypes.POINTER(S)), ("def_row", P), ("def_clock", P), ("def_keys", P), ("Dv", S),
    ]


class MapOrswotOut(ctypes.Structure):  # crdt_map_orswot_out
    _fields_ = [("clock", P), ("ec", P), ("oc", P), ("ent", P), ("vd_n", P), ("vd_clock", P), ("vd_mem", P),
                ("flags", P), ("def_keep", P), ("def_keys", P), ("Vd", S)]


class MapNestedBatch(ctypes.Structure):  # crdt_map_nested_batch
    _fields_ = [
        ("G", S), ("R", S), ("K", S), ("K2", S), ("V", S), ("A", S),
        ("clock", P), ("ec", P), ("ic", P), ("iec", P), ("ivc", P), ("ivv", P),
        ("id_off", P), ("id_clock", P), ("id_keys", P), ("Di", S),
        ("def_off", ctypes.POINTER(S)), ("def_row", P), ("def_clock", P), ("def_keys", P),
    ]


class MapNestedOut(ctypes.Structure):  # crdt_map_nested_out
    _fields_ = [("clock", P), ("ec", P), ("ic", P), ("iec", P), ("ivc", P), ("ivv", P), ("nval", P), ("id_n", P),
                ("id_clock", P), ("id_keys", P), ("flags", P), ("def_keep", P), ("def_keys", P), ("Id", S), ("Vs", S)]


class MapOut(ctypes.Structure):  # crdt_map_out
    _fields_ = [("Vout", S), ("Vstate", S), ("clock", P), ("ec", P), ("vclk", P), ("vval", P), ("nval", P),
                ("flags", P), ("def_keep", P), ("def_keys", P)]


_SIGS = {
    "crdt_ctx_create": ([ctypes.c_int, ctypes.POINTER(P)], ctypes.c_int),
    "crdt_ctx_destroy": ([P], ctypes.c_int),
    "crdt_ctx_set_stream": ([P, P], ctypes.c_int),
    "crdt_ctx_synchronize": ([P], ctypes.c_int),
    "crdt_last_error": ([P], ctypes.c_char_p),
    "crdt_version": ([], ctypes.c_char_p),
    "crdt_abi_version": ([], ctypes.c_int),
    "crdt_build_target": ([], ctypes.c_char_p),
    "crdt_ctx_set_timing": ([P, ctypes.c_int], ctypes.c_int),
    "crdt_ctx_timing": ([P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64)], ctypes.c_int),
    "crdt_ctx_timing_reset": ([P], ctypes.c_int),
    "crdt_ctx_tune": ([P, ctypes.c_char_p], ctypes.c_int),
    "crdt_ctx_set_mem_kind": ([P, ctypes.c_int], ctypes.c_int),
    "crdt_ctx_mem_kind": ([P], ctypes.c_int),
    "crdt_host_alloc": ([S, ctypes.POINTER(P)], ctypes.c_int),
    "crdt_host_free": ([P], ctypes.c_int),
    "crdt_device_alloc": ([P, S, ctypes.POINTER(P)], ctypes.c_int),
    "crdt_device_free": ([P, P], ctypes.c_int),
    "crdt_lub_many_multi": ([P, ctypes.POINTER(LubSegment), S], ctypes.c_int),
    "crdt_lub_many_multi_sharded": ([P, ctypes.POINTER(LubSegment), S], ctypes.c_int),
    "crdt_map_ingest": ([P, P, P, P, P, ctypes.POINTER(MapStates), ctypes.POINTER(MapDeferred), P], ctypes.c_int),
    "crdt_map_egress": ([P, ctypes.POINTER(MapStates), ctypes.POINTER(MapDeferred), P, P, P, P, S,
                         ctypes.POINTER(S)], ctypes.c_int),
    "crdt_synth_fill": ([P, P, S, S, S, S, U64, ctypes.c_int], ctypes.c_int),
    "crdt_synth_orswot": ([P, P, P, S, S, S, S, U64, U64], ctypes.c_int),
    "crdt_synth_orswot_rm": ([P, P, S, S, S, P, P, P], ctypes.c_int),
    "crdt_synth_map": ([P, P, P, P, P, S, S, S, S, S, U64, U64, P, P, P], ctypes.c_int),
    "crdt_lwwreg_lub_many": ([P, P, P, S, S, S, P, P, P, ctypes.c_uint], ctypes.c_int),
    "crdt_lwwreg_merge_batch": ([P, P, P, P, P, S, P], ctypes.c_int),
    "crdt_orswot_lub_many": ([P, ctypes.POINTER(OrswotBatch), ctypes.POINTER(OrswotOut)], ctypes.c_int),
    "crdt_orswot_apply_batch": ([P, ctypes.POINTER(OrswotStates), ctypes.POINTER(OrswotOps), P], ctypes.c_int),
    "crdt_map_lub_many": ([P, ctypes.POINTER(MapBatch), ctypes.POINTER(MapOut)], ctypes.c_int),
    "crdt_orswot_lub_many_doff": ([P, ctypes.POINTER(OrswotBatch), P, S, ctypes.POINTER(OrswotOut), P], ctypes.c_int),
    "crdt_map_lub_many_doff": ([P, ctypes.POINTER(MapBatch), P, S, ctypes.POINTER(MapOut)], ctypes.c_int),
    "crdt_vclock_pair_op": ([P, ctypes.c_int, P, P, P, S, S, S, S, S], ctypes.c_int),
    "crdt_vclock_partial_cmp": ([P, P, P, S, S, S, S, P], ctypes.c_int),
    "crdt_vclock_cmp_matrix": ([P, P, S, S, S, P], ctypes.c_int),
    "crdt_gcounter_read": ([P, P, S, S, S, P], ctypes.c_int),
    "crdt_pncounter_read": ([P, P, S, S, S, P], ctypes.c_int),
    "crdt_vclock_apply_batch": ([P, P, S, S, S, P, P, P, S, P], ctypes.c_int),
    "crdt_gcounter_apply_batch": ([P, P, S, S, S, P, P, P, S, P], ctypes.c_int),
    "crdt_pncounter_apply_batch": ([P, P, S, S, S, P, P, P, P, S, P], ctypes.c_int),
    "crdt_gset_apply_batch": ([P, P, S, S, S, P, P, S, P], ctypes.c_int),
}
_SIGS.update({
    "crdt_map_nested_apply_batch": ([P, ctypes.POINTER(MapNestedStates), P, P, P, S, ctypes.POINTER(MapNestedOps), P],
                                    ctypes.c_int),
    "crdt_map_nested_forget_batch": ([P, ctypes.POINTER(MapNestedStates), P, S, P, P, S, P], ctypes.c_int),
    "crdt_map_nested_ingest": ([P, P, P, P, P, P, ctypes.POINTER(MapNestedStates), ctypes.POINTER(MapDeferred), P],
                               ctypes.c_int),
    "crdt_map_nested_egress": ([P, ctypes.POINTER(MapNestedStates), ctypes.POINTER(MapDeferred), P, P, P, P, P, S,
                                ctypes.POINTER(S)], ctypes.c_int),
    "crdt_map_counter_ingest": ([P, P, P, P, P, ctypes.POINTER(MapCounterStates), ctypes.POINTER(MapDeferred), P],
                                ctypes.c_int),
    "crdt_map_counter_egress": ([P, ctypes.POINTER(MapCounterStates), ctypes.POINTER(MapDeferred), P, P, P, P, S,
                                 ctypes.POINTER(S)], ctypes.c_int),
    "crdt_map_orswot_ingest": ([P, P, P, P, P, P, ctypes.POINTER(MapOrswotStates), ctypes.POINTER(MapDeferred), P],
                               ctypes.c_int),
    "crdt_map_orswot_egress": ([P, ctypes.POINTER(MapOrswotStates), ctypes.POINTER(MapDeferred), P, P, P, P, P, S,
                                ctypes.POINTER(S)], ctypes.c_int),
    "crdt_orswot_forget_batch": ([P, P, S, P, S, S, S, S, S, P, S, P, P, S, P], ctypes.c_int),
    "crdt_map_forget_batch": ([P, ctypes.POINTER(MapStates), P, S, P, P, S, P], ctypes.c_int),
    "crdt_map_counter_forget_batch": ([P, ctypes.POINTER(MapCounterStates), P, S, P, P, S, P], ctypes.c_int),
    "crdt_map_orswot_forget_batch": ([P, ctypes.POINTER(MapOrswotStates), P, S, P, P, S, P], ctypes.c_int),
    "crdt_map_counter_apply_batch": ([P, ctypes.POINTER(MapCounterStates), P, P, P, S, ctypes.POINTER(MapCounterOps),
                                      P], ctypes.c_int),
    "crdt_map_orswot_apply_batch": ([P, ctypes.POINTER(MapOrswotStates), P, P, P, S, ctypes.POINTER(MapOrswotOps),
                                     P], ctypes.c_int),
    "crdt_map_apply_batch": ([P, ctypes.POINTER(MapStates), P, P, P, S, ctypes.POINTER(MapOps), P], ctypes.c_int),
    "crdt_orswot_merge_batch": ([P, ctypes.POINTER(OrswotStates), ctypes.POINTER(OrswotStates), P], ctypes.c_int),
    "crdt_map_counter_merge_batch": ([P, ctypes.POINTER(MapCounterStates), ctypes.POINTER(MapDeferred),
                                      ctypes.POINTER(MapCounterStates), ctypes.POINTER(MapDeferred), P], ctypes.c_int),
    "crdt_map_orswot_merge_batch": ([P, ctypes.POINTER(MapOrswotStates), ctypes.POINTER(MapDeferred),
                                     ctypes.POINTER(MapOrswotStates), ctypes.POINTER(MapDeferred), P], ctypes.c_int),
    "crdt_map_nested_merge_batch": ([P, ctypes.POINTER(MapNestedStates), ctypes.POINTER(MapDeferred),
                                     ctypes.POINTER(MapNestedStates), ctypes.POINTER(MapDeferred), P], ctypes.c_int),
    "crdt_map_merge_batch": ([P, ctypes.POINTER(MapStates), ctypes.POINTER(MapDeferred), ctypes.POINTER(MapStates),
                              ctypes.POINTER(MapDeferred), P], ctypes.c_int),
    "crdt_lwwreg_lub_many_sharded": ([P, P, P, S, S, S, U64, P, P, P], ctypes.c_int),
    "crdt_map_lub_many_sharded": ([P, ctypes.POINTER(MapBatch), S, S, ctypes.POINTER(MapOut)], ctypes.c_int),
    "crdt_map_lub_many_sharded_doff": ([P, ctypes.POINTER(MapBatch), P, S, S, S, ctypes.POINTER(MapOut)],
                                       ctypes.c_int),
    "crdt_map_counter_lub_many": ([P, ctypes.POINTER(MapCounterBatch), ctypes.POINTER(MapCounterOut)], ctypes.c_int),
    "crdt_map_orswot_lub_many": ([P, ctypes.POINTER(MapOrswotBatch), ctypes.POINTER(MapOrswotOut)], ctypes.c_int),
    "crdt_map_nested_lub_many": ([P, ctypes.POINTER(MapNestedBatch), ctypes.POINTER(MapNestedOut)], ctypes.c_int),
    "crdt_map_counter_lub_many_sharded": ([P, ctypes.POINTER(MapCounterBatch), S, S, ctypes.POINTER(MapCounterOut)],
                                          ctypes.c_int),
    "crdt_map_orswot_lub_many_sharded": ([P, ctypes.POINTER(MapOrswotBatch), S, S, ctypes.POINTER(MapOrswotOut)],
                                         ctypes.c_int),
    "crdt_map_nested_lub_many_sharded": ([P, ctypes.POINTER(MapNestedBatch), S, S, ctypes.POINTER(MapNestedOut)],
                                         ctypes.c_int),
    "crdt_vclock_ingest": ([P, P, P, S, P, S, P, S, P], ctypes.c_int),
    "crdt_pncounter_ingest": ([P, P, P, S, P, S, P, S, P], ctypes.c_int),
    "crdt_gset_ingest": ([P, P, P, S, P, S, P, S, P], ctypes.c_int),
    "crdt_lwwreg_ingest": ([P, P, P, S, P, P, P], ctypes.c_int),
    "crdt_orswot_ingest": ([P, P, P, S, P, S, P, S, P, P, P, P, P, S, ctypes.POINTER(S), P], ctypes.c_int),
    "crdt_vclock_egress": ([P, P, S, S, S, P, P, P, S, ctypes.POINTER(S)], ctypes.c_int),
    "crdt_pncounter_egress": ([P, P, S, S, S, P, P, P, S, ctypes.POINTER(S)], ctypes.c_int),
    "crdt_gset_egress": ([P, P, S, S, S, P, P, P, S, ctypes.POINTER(S)], ctypes.c_int),
    "crdt_lwwreg_egress": ([P, P, P, S, P], ctypes.c_int),
    "crdt_orswot_egress": ([P, P, P, S, S, S, P, P, P, P, P, P, P, P, S, ctypes.POINTER(S)], ctypes.c_int),
    "crdt_comm_unique_id": ([P], ctypes.c_int),
    "crdt_ctx_comm_init": ([P, P, ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "crdt_ctx_comm_destroy": ([P], ctypes.c_int),
    "crdt_ctx_comm_info": ([P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "crdt_mvreg_lub_many": ([P, ctypes.POINTER(MVRegBatch), ctypes.POINTER(MVRegOut)], ctypes.c_int),
    "crdt_mvreg_merge_batch": ([P, ctypes.POINTER(MVRegStates), ctypes.POINTER(MVRegStates), P], ctypes.c_int),
    "crdt_mvreg_apply_batch": ([P, ctypes.POINTER(MVRegStates), ctypes.POINTER(MVRegOps), P], ctypes.c_int),
    "crdt_ctx_comm_init_ops": ([P, ctypes.POINTER(CommOps), ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "crdt_ctx_comm_note": ([P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], ctypes.c_char_p),
    "crdt_orswot_lub_many_sharded": ([P, ctypes.POINTER(OrswotBatch), ctypes.POINTER(OrswotShardedOut)],
                                     ctypes.c_int),
    "crdt_orswot_lub_many_sharded_doff": ([P, ctypes.POINTER(OrswotBatch), P, S, ctypes.POINTER(OrswotShardedOut)],
                                          ctypes.c_int),
})
for _t in ("vclock", "gcounter", "pncounter", "gset"):
    _SIGS[f"crdt_{_t}_lub_many_sharded"] = ([P, P, S, S, S, S, S, P], ctypes.c_int)
for _t in ("vclock", "gcounter", "pncounter", "gset"):
    _SIGS[f"crdt_{_t}_lub_many"] = ([P, P, S, S, S, S, S, P, S, ctypes.c_uint], ctypes.c_int)
    _SIGS[f"crdt_{_t}_merge_batch"] = ([P, P, P, S, S, S, S], ctypes.c_int)

_lib = None


def load():
    """Load libcrdt_gpu.so (raises CrdtGpuUnavailable if it was never built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CrdtGpuUnavailable(
            f"{LIB_PATH} not found: build it with `make -C rust-crdt_amd` (or "
            "`python -c 'import __graft_entry__ as g; g.build()'`). There is no CPU fallback.")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime being present
        raise CrdtGpuUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, (argtypes, restype) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    if lib.crdt_abi_version() != CRDT_ABI_VERSION:  # a library built from another header revision
        raise CrdtGpuUnavailable(f"{LIB_PATH}: ABI revision {lib.crdt_abi_version()}, these bindings expect "
                                 f"{CRDT_ABI_VERSION} (include/crdt_gpu.h CRDT_ABI_VERSION)")
    _lib = lib
    return lib


def check(ctx_ptr, fn: str, rc: int) -> None:
    if rc != CRDT_OK:
        msg = load().crdt_last_error(ctx_ptr)
        raise CrdtGpuError(fn, rc, (msg or b"").decode(errors="replace"))
