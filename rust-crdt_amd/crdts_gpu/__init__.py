"""crdts_gpu — MI355X batched CvRDT merge for the `crdts` (rust-crdt) data model.

Host-side mirror of the reference crate's merge surface (`CvRDT::merge`, traits.rs:4-7;
`FunkyCvRDT::merge` for LWWReg, traits.rs:49-55) in batched form: for each type module,
`lub_many` folds many replicas and `merge_batch` runs many pairwise merges, on dense
structure-of-arrays states in HBM, through libcrdt_gpu.so (include/crdt_gpu.h).
There is no CPU fallback: without the HIP library every call raises CrdtGpuUnavailable.
"""
from ._abi import CrdtGpuError, CrdtGpuUnavailable, load as load_library  # noqa: F401
from .context import Context, synth_fill  # noqa: F401
from ._lattice import lub_many_multi  # noqa: F401
from . import apply, causal, gcounter, gset, host, intern, lwwreg, map, mvreg, orswot, pncounter, shard, synth, vclock, wire  # noqa: F401

__version__ = "0.1.0"
