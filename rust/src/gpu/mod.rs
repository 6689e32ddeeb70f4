//! Batched state merges on an MI355X through `libcrdt_gpu` (hand-written gfx950 HIP kernels
//! behind the C ABI of `include/crdt_gpu.h`).
//!
//! This is the `gpu` module a maintainer adds to the `crdts` crate (`src/gpu/`), together with
//! `build.rs` (the hipcc step) and `pub mod gpu;` in `src/lib.rs` behind a `gpu` feature.  It keeps
//! the crate's trait surface (`CvRDT::merge`, `traits.rs:4-7`; `FunkyCvRDT::merge` for `LWWReg`,
//! `traits.rs:49-55`) and adds the batched forms:
//!
//! * [`BatchCvRDT::lub_many`]: `let mut acc = T::new(); for r in replicas { acc.merge(r) }`
//!   (the fold of `test/orswot.rs:50-53`), computed on the GPU;
//! * [`BatchCvRDT::merge_batch`]: `for (s, o) in selves.iter_mut().zip(others) { s.merge(o) }`.
//!
//! States are interned to the dense structure-of-arrays layout the kernels read (actors, members
//! and set elements to dense indices; an absent actor is a 0 counter, exact because
//! `VClock::apply_dot` never stores 0, `vclock.rs:155-159`), merged on the GPU, and rebuilt.
//! The lattice types and `LWWReg` hand their host rows straight to the library through a second
//! ctx in `CRDT_MEM_HOST` mode (it streams them through HBM in chunks, overlapping PCIe with the
//! fold; `Orswot` and `Map` batches stream the same way, the value-typed Maps are staged whole).
//! [`DeviceBuf`] stays for callers that manage device
//! memory themselves.  Callers that keep replica states
//! resident in HBM use [`ffi`] directly on device buffers with [`GpuCtx::as_ptr`].
//!
//! Field access: `VClock::dots`, the `Orswot` fields and the `LWWReg` fields are already visible
//! to an in-crate module; the maintainer changes `GCounter::inner`, `PNCounter::{p, n}`,
//! `GSet::value`, the `Map` fields, `map::Entry` and `MVReg::vals` from private to `pub(crate)`
//! (visibility only, no behaviour change; `rust/lib.rs.patch`).
//!
//! Not built in the repository that ships it (its image has no Rust toolchain); the extern block
//! in [`ffi`] is generated from the header and checked against it by `tests/test_rust_shim.py`.
#![allow(unsafe_code)]

pub mod ffi;
mod hip;

use std::collections::{BTreeMap, BTreeSet, HashMap, HashSet};
use std::ffi::CStr;
use std::hash::Hash;
use std::os::raw::c_int;
use std::ptr;

use crate::error::Error as CrdtError;
use crate::orswot::Member;
use crate::traits::CvRDT;
use crate::vclock::{Actor, VClock};
use crate::map::Entry;
use crate::{GCounter, GSet, LWWReg, MVReg, Map, Orswot, PNCounter};

pub use hip::DeviceBuf;

/// A failed library or HIP call (status code and the library's message).
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct GpuError {
    /// `CRDT_E*` status (negative) or the HIP error code of a staging copy.
    pub code: i32,
    /// `crdt_last_error` text, or a description of the failed staging step.
    pub msg: String,
}

impl std::fmt::Display for GpuError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "libcrdt_gpu error {}: {}", self.code, self.msg)
    }
}

impl std::error::Error for GpuError {}

/// A `crdt_ctx`: one per host thread, bound to one HIP device (scratch and stream owned here).
pub struct GpuCtx {
    raw: *mut ffi::crdt_ctx,
    /// Same device, `CRDT_MEM_HOST` mode: host pointers, staged by the library.
    host: *mut ffi::crdt_ctx,
}

impl GpuCtx {
    /// `crdt_ctx_create(device)`.
    pub fn new(device: i32) -> Result<Self, GpuError> {
        // a library built from another header revision reads these structs differently
        let abi = unsafe { ffi::crdt_abi_version() };
        if abi != ffi::CRDT_ABI_VERSION {
            return Err(GpuError {
                code: ffi::CRDT_EUNSUPPORTED,
                msg: format!("libcrdt_gpu ABI revision {}, this binding expects {}", abi, ffi::CRDT_ABI_VERSION),
            });
        }
        let mut raw = ptr::null_mut();
        let rc = unsafe { ffi::crdt_ctx_create(device, &mut raw) };
        if rc != ffi::CRDT_OK {
            return Err(GpuError { code: rc, msg: last_error(ptr::null()) });
        }
        let mut host = ptr::null_mut();
        let rc = unsafe { ffi::crdt_ctx_create(device, &mut host) };
        if rc != ffi::CRDT_OK {
            unsafe { ffi::crdt_ctx_destroy(raw) };
            return Err(GpuError { code: rc, msg: last_error(ptr::null()) });
        }
        let ctx = GpuCtx { raw, host };
        ctx.check_host(unsafe { ffi::crdt_ctx_set_mem_kind(host, ffi::CRDT_MEM_HOST) })?;
        Ok(ctx)
    }

    /// Status of a call issued on the host-memory ctx.
    fn check_host(&self, rc: c_int) -> Result<(), GpuError> {
        if rc == ffi::CRDT_OK {
            Ok(())
        } else {
            Err(GpuError { code: rc, msg: last_error(self.host) })
        }
    }

    /// The raw handle, for calls through [`ffi`] on caller-owned device buffers.
    pub fn as_ptr(&self) -> *mut ffi::crdt_ctx {
        self.raw
    }

    /// Map a status code to `Result` (the library never throws across the ABI).
    pub fn check(&self, rc: c_int) -> Result<(), GpuError> {
        if rc == ffi::CRDT_OK {
            Ok(())
        } else {
            Err(GpuError { code: rc, msg: last_error(self.raw) })
        }
    }

    /// Block until the work issued through this ctx has finished.
    pub fn synchronize(&self) -> Result<(), GpuError> {
        self.check(unsafe { ffi::crdt_ctx_synchronize(self.raw) })
    }
}

impl Drop for GpuCtx {
    fn drop(&mut self) {
        unsafe {
            ffi::crdt_ctx_destroy(self.raw);
            ffi::crdt_ctx_destroy(self.host);
        }
    }
}

fn last_error(ctx: *const ffi::crdt_ctx) -> String {
    unsafe {
        let p = ffi::crdt_last_error(ctx);
        if p.is_null() {
            String::new()
        } else {
            CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    }
}

/// Batched extension of `CvRDT` (`traits.rs:4-7`); the single-pair `merge` is unchanged.
pub trait BatchCvRDT: CvRDT + Sized {
    /// `let mut acc = Self::new(); for r in replicas { acc.merge(r) }`, on the GPU.
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError>;
    /// `for (s, o) in selves.iter_mut().zip(others) { s.merge(o) }`, on the GPU, in place.
    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError>;
}

/// Capacity limits of the library this module binds (include/crdt_gpu.h; checked against the
/// header's stated limits by tests/test_rust_shim.py).  Past them a call returns `GpuError` with
/// `CRDT_EUNSUPPORTED` and leaves its inputs untouched.
/// Values per MVReg register (`crdt_map_lub_many`: V <= 16; `crdt_mvreg_*`: V <= 16;
/// `crdt_map_merge_batch` takes up to 32 per side, the smallest limit is the one checked here).
pub const MAP_MAX_VALUES: usize = 16;
/// Actors of the Map, MVReg and Orswot-apply kernels (A <= 1024).
pub const MAP_MAX_ACTORS: usize = 1024;
/// Deferred-remove slots of a pairwise merge, self + other: not bounded by the library (a pair
/// with more than 512 removes is forgotten in further passes), so only the address space limits it.
pub const MERGE_MAX_DEFERRED: usize = usize::MAX;

fn unsupported(msg: String) -> GpuError {
    GpuError { code: ffi::CRDT_EUNSUPPORTED, msg }
}

fn check_pairs(n_self: usize, n_other: usize) -> Result<(), GpuError> {
    if n_self != n_other {
        return Err(GpuError { code: ffi::CRDT_EINVAL,
                              msg: format!("merge_batch: {} selves but {} others", n_self, n_other) });
    }
    Ok(())
}

/// Dense indices for ids (actors, members, set elements): first-seen order.
struct Index<T: Ord + Clone> {
    pos: BTreeMap<T, usize>,
    ids: Vec<T>,
}

impl<T: Ord + Clone> Index<T> {
    fn new() -> Self {
        Index { pos: BTreeMap::new(), ids: Vec::new() }
    }
    fn intern(&mut self, id: &T) -> usize {
        if let Some(&i) = self.pos.get(id) {
            return i;
        }
        let i = self.ids.len();
        self.pos.insert(id.clone(), i);
        self.ids.push(id.clone());
        i
    }
    fn width(&self) -> usize {
        self.ids.len().max(1)
    }
}

/// Hash-keyed index for `Member: Clone + Hash + Eq` ids (no `Ord` bound in the crate).
struct HIndex<T: Clone + Hash + Eq> {
    pos: HashMap<T, usize>,
    ids: Vec<T>,
}

impl<T: Clone + Hash + Eq> HIndex<T> {
    fn new() -> Self {
        HIndex { pos: HashMap::new(), ids: Vec::new() }
    }
    fn intern(&mut self, id: &T) -> usize {
        if let Some(&i) = self.pos.get(id) {
            return i;
        }
        let i = self.ids.len();
        self.pos.insert(id.clone(), i);
        self.ids.push(id.clone());
        i
    }
    fn width(&self) -> usize {
        self.ids.len().max(1)
    }
}

fn clock_row<A: Actor>(c: &VClock<A>, idx: &Index<A>, row: &mut [u64]) {
    for (a, n) in c.dots.iter() {
        row[idx.pos[a]] = *n;
    }
}

fn row_clock<A: Actor>(row: &[u64], idx: &Index<A>) -> VClock<A> {
    let mut c = VClock::new();
    for (i, &n) in row.iter().enumerate() {
        if n != 0 && i < idx.ids.len() {
            c.dots.insert(idx.ids[i].clone(), n);
        }
    }
    c
}

/// Lattice lub / merge_batch of dense rows through one of the max / OR entry points.
enum Lattice {
    VClock,
    GCounter,
    PNCounter,
    GSet,
}

// Host rows go to the CRDT_MEM_HOST ctx as they are: the library stages them (no DeviceBuf).
fn lattice_lub(ctx: &GpuCtx, kind: Lattice, rows: &[u64], r: usize, w: usize) -> Result<Vec<u64>, GpuError> {
    let mut out = vec![0u64; w];
    let width = if let Lattice::PNCounter = kind { w / 2 } else { w };
    let rc = unsafe {
        let (i, o) = (rows.as_ptr(), out.as_mut_ptr());
        match kind {
            Lattice::VClock => ffi::crdt_vclock_lub_many(ctx.host, i, 1, r, width, w, r * w, o, w, 0),
            Lattice::GCounter => ffi::crdt_gcounter_lub_many(ctx.host, i, 1, r, width, w, r * w, o, w, 0),
            Lattice::PNCounter => ffi::crdt_pncounter_lub_many(ctx.host, i, 1, r, width, w, r * w, o, w, 0),
            Lattice::GSet => ffi::crdt_gset_lub_many(ctx.host, i, 1, r, width, w, r * w, o, w, 0),
        }
    };
    ctx.check_host(rc)?;
    Ok(out)
}

fn lattice_pairs(ctx: &GpuCtx, kind: Lattice, selves: &[u64], others: &[u64], n: usize, w: usize)
                 -> Result<Vec<u64>, GpuError> {
    let mut s = selves.to_vec();
    let width = if let Lattice::PNCounter = kind { w / 2 } else { w };
    let rc = unsafe {
        let (sp, op) = (s.as_mut_ptr(), others.as_ptr());
        match kind {
            Lattice::VClock => ffi::crdt_vclock_merge_batch(ctx.host, sp, op, n, width, w, w),
            Lattice::GCounter => ffi::crdt_gcounter_merge_batch(ctx.host, sp, op, n, width, w, w),
            Lattice::PNCounter => ffi::crdt_pncounter_merge_batch(ctx.host, sp, op, n, width, w, w),
            Lattice::GSet => ffi::crdt_gset_merge_batch(ctx.host, sp, op, n, width, w, w),
        }
    };
    ctx.check_host(rc)?;
    Ok(s)
}

// ---- VClock / GCounter: elementwise max (vclock.rs:130-136, gcounter.rs:44-48) ----------------
impl<A: Actor> BatchCvRDT for VClock<A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        let mut idx = Index::new();
        for r in &replicas {
            for a in r.dots.keys() {
                idx.intern(a);
            }
        }
        let (r, w) = (replicas.len(), idx.width());
        if r == 0 {
            return Ok(VClock::new());
        }
        let mut rows = vec![0u64; r * w];
        for (i, c) in replicas.iter().enumerate() {
            clock_row(c, &idx, &mut rows[i * w..(i + 1) * w]);
        }
        let out = lattice_lub(ctx, Lattice::VClock, &rows, r, w)?;
        Ok(row_clock(&out, &idx))
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        let n = selves.len();
        if n == 0 {
            return Ok(());
        }
        let mut idx = Index::new();
        for c in selves.iter().chain(others.iter()) {
            for a in c.dots.keys() {
                idx.intern(a);
            }
        }
        let w = idx.width();
        let (mut s, mut o) = (vec![0u64; n * w], vec![0u64; n * w]);
        for i in 0..n {
            clock_row(&selves[i], &idx, &mut s[i * w..(i + 1) * w]);
            clock_row(&others[i], &idx, &mut o[i * w..(i + 1) * w]);
        }
        let out = lattice_pairs(ctx, Lattice::VClock, &s, &o, n, w)?;
        for i in 0..n {
            selves[i] = row_clock(&out[i * w..(i + 1) * w], &idx);
        }
        Ok(())
    }
}

impl<A: Actor> BatchCvRDT for GCounter<A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        let inner = replicas.into_iter().map(|g| g.inner).collect();
        let mut out = GCounter::new();
        out.inner = <VClock<A> as BatchCvRDT>::lub_many(ctx, inner)?;
        Ok(out)
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        let mut s: Vec<VClock<A>> = selves.iter().map(|g| g.inner.clone()).collect();
        <VClock<A> as BatchCvRDT>::merge_batch(ctx, &mut s, others.into_iter().map(|g| g.inner).collect())?;
        for (g, c) in selves.iter_mut().zip(s) {
            g.inner = c;
        }
        Ok(())
    }
}

// ---- PNCounter: P and N maxima over rows P | N (pncounter.rs:70-75) ------------------------------
fn pn_rows<A: Actor>(states: &[&PNCounter<A>], idx: &Index<A>) -> Vec<u64> {
    let w = idx.width();
    let mut rows = vec![0u64; states.len() * 2 * w];
    for (i, s) in states.iter().enumerate() {
        let row = &mut rows[i * 2 * w..(i + 1) * 2 * w];
        clock_row(&s.p.inner, idx, &mut row[..w]);
        clock_row(&s.n.inner, idx, &mut row[w..]);
    }
    rows
}

fn pn_state<A: Actor>(row: &[u64], idx: &Index<A>) -> PNCounter<A> {
    let w = idx.width();
    let mut s = PNCounter::new();
    s.p.inner = row_clock(&row[..w], idx);
    s.n.inner = row_clock(&row[w..], idx);
    s
}

impl<A: Actor> BatchCvRDT for PNCounter<A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(PNCounter::new());
        }
        let mut idx = Index::new();
        for r in &replicas {
            for a in r.p.inner.dots.keys().chain(r.n.inner.dots.keys()) {
                idx.intern(a);
            }
        }
        let refs: Vec<&Self> = replicas.iter().collect();
        let rows = pn_rows(&refs, &idx);
        let out = lattice_lub(ctx, Lattice::PNCounter, &rows, replicas.len(), 2 * idx.width())?;
        Ok(pn_state(&out, &idx))
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        let n = selves.len();
        if n == 0 {
            return Ok(());
        }
        let mut idx = Index::new();
        for r in selves.iter().chain(others.iter()) {
            for a in r.p.inner.dots.keys().chain(r.n.inner.dots.keys()) {
                idx.intern(a);
            }
        }
        let w2 = 2 * idx.width();
        let s = pn_rows(&selves[..n].iter().collect::<Vec<_>>(), &idx);
        let o = pn_rows(&others[..n].iter().collect::<Vec<_>>(), &idx);
        let out = lattice_pairs(ctx, Lattice::PNCounter, &s, &o, n, w2)?;
        for i in 0..n {
            selves[i] = pn_state(&out[i * w2..(i + 1) * w2], &idx);
        }
        Ok(())
    }
}

// ---- GSet: bitmap union (gset.rs:38-40) ---------------------------------------------------------
fn set_row<T: Ord + Clone>(s: &BTreeSet<T>, idx: &Index<T>, row: &mut [u64]) {
    for x in s {
        let b = idx.pos[x];
        row[b / 64] |= 1u64 << (b % 64);
    }
}

fn row_set<T: Ord + Clone>(row: &[u64], idx: &Index<T>) -> BTreeSet<T> {
    let mut out = BTreeSet::new();
    for (w, &word) in row.iter().enumerate() {
        let mut x = word;
        while x != 0 {
            let b = w * 64 + x.trailing_zeros() as usize;
            x &= x - 1;
            if b < idx.ids.len() {
                out.insert(idx.ids[b].clone());
            }
        }
    }
    out
}

impl<T: Ord + Clone> BatchCvRDT for GSet<T> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(GSet::new());
        }
        let mut idx = Index::new();
        for r in &replicas {
            for x in &r.value {
                idx.intern(x);
            }
        }
        let w = (idx.width() + 63) / 64;
        let mut rows = vec![0u64; replicas.len() * w];
        for (i, r) in replicas.iter().enumerate() {
            set_row(&r.value, &idx, &mut rows[i * w..(i + 1) * w]);
        }
        let out = lattice_lub(ctx, Lattice::GSet, &rows, replicas.len(), w)?;
        let mut g = GSet::new();
        g.value = row_set(&out, &idx);
        Ok(g)
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        let n = selves.len();
        if n == 0 {
            return Ok(());
        }
        let mut idx = Index::new();
        for r in selves.iter().chain(others.iter()) {
            for x in &r.value {
                idx.intern(x);
            }
        }
        let w = (idx.width() + 63) / 64;
        let (mut s, mut o) = (vec![0u64; n * w], vec![0u64; n * w]);
        for i in 0..n {
            set_row(&selves[i].value, &idx, &mut s[i * w..(i + 1) * w]);
            set_row(&others[i].value, &idx, &mut o[i * w..(i + 1) * w]);
        }
        let out = lattice_pairs(ctx, Lattice::GSet, &s, &o, n, w)?;
        for i in 0..n {
            selves[i].value = row_set(&out[i * w..(i + 1) * w], &idx);
        }
        Ok(())
    }
}

// ---- LWWReg<V, u64>: FunkyCvRDT (lwwreg.rs:43-45 -> update :84-98) --------------------------------
/// Batched `FunkyCvRDT::merge` for `LWWReg<V, u64>` (values interned; equal values <=> equal ids).
pub trait BatchFunkyLww: Sized {
    /// The fold `acc = replicas[0]; for r in replicas[1..] { acc.merge(r) }` where an erroring
    /// merge leaves `acc` unchanged (as `update` does); returns the state and the index of the
    /// first merge that returned `Err(ConflictingMarker)`, if any.
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<(Self, Option<usize>), GpuError>;
    /// `selves[i].merge(others[i])` for every i: `Err(ConflictingMarker)` where the markers are
    /// equal and the values differ, that register then unchanged.
    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>)
                   -> Result<Vec<Result<(), CrdtError>>, GpuError>;
}

/// Order-preserving interning of markers: rank among the distinct markers, + 1 (`M: Ord` is all
/// `FunkyCvRDT for LWWReg<V, M>` asks, lwwreg.rs:30-46; equal markers <=> equal ids, and the
/// kernel's u64 compare orders ids exactly as `M::cmp` orders the markers).
fn marker_ids<'a, M: Ord + Clone + 'a, I: Iterator<Item = &'a M>>(markers: I) -> (Vec<u64>, BTreeMap<M, u64>) {
    let all: Vec<&M> = markers.collect();
    let set: BTreeSet<&M> = all.iter().cloned().collect();
    let rank: BTreeMap<M, u64> = set.into_iter().enumerate().map(|(i, m)| (m.clone(), i as u64 + 1)).collect();
    (all.iter().map(|m| rank[*m]).collect(), rank)
}

// ---- LWWReg<V, M>: FunkyCvRDT (lwwreg.rs:43-45 -> update :84-98) --------------------------------
impl<V: PartialEq + Clone, M: Ord + Clone> BatchFunkyLww for LWWReg<V, M> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<(Self, Option<usize>), GpuError> {
        let r = replicas.len();
        if r == 0 {
            return Err(GpuError { code: ffi::CRDT_EINVAL, msg: "LWWReg lub_many of no replica".into() });
        }
        let (markers, _) = marker_ids(replicas.iter().map(|x| &x.marker));
        // value ids only meet values under an EQUAL marker (the conflict test, lwwreg.rs:89-90), and
        // `V: PartialEq` is all there is: id = the first replica of the same marker class holding an
        // equal value (a linear scan within the class)
        let mut classes: HashMap<u64, Vec<usize>> = HashMap::new();
        let mut ids = Vec::with_capacity(r);
        for (i, x) in replicas.iter().enumerate() {
            let class = classes.entry(markers[i]).or_insert_with(Vec::new);
            let id = match class.iter().find(|&&j| replicas[j].val == x.val) {
                Some(&j) => j,
                None => {
                    class.push(i);
                    i
                }
            };
            ids.push(id as u64);
        }
        let (mut mk, mut vi, mut fc) = (0u64, 0u64, 0u64);
        ctx.check_host(unsafe {
            ffi::crdt_lwwreg_lub_many(ctx.host, markers.as_ptr(), ids.as_ptr(), 1, r, r, &mut mk, &mut vi, &mut fc, 0)
        })?;
        let win = &replicas[vi as usize];
        debug_assert_eq!(markers[vi as usize], mk);
        let state = LWWReg { val: win.val.clone(), marker: win.marker.clone() };
        Ok((state, if fc == u64::MAX { None } else { Some(fc as usize) }))
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>)
                   -> Result<Vec<Result<(), CrdtError>>, GpuError> {
        check_pairs(selves.len(), others.len())?;
        let n = selves.len();
        if n == 0 {
            return Ok(Vec::new());
        }
        let (ids, _) = marker_ids(selves.iter().map(|x| &x.marker).chain(others.iter().map(|x| &x.marker)));
        let (sm, om) = (ids[..n].to_vec(), ids[n..].to_vec());
        // per pair: self's value is id 0, other's is 0 when equal, else 1
        let sv = vec![0u64; n];
        let ov: Vec<u64> = (0..n).map(|i| if selves[i].val == others[i].val { 0 } else { 1 }).collect();
        let (mut m2, mut v2, mut c) = (sm, sv, vec![0u8; n]);
        ctx.check_host(unsafe {
            ffi::crdt_lwwreg_merge_batch(ctx.host, m2.as_mut_ptr(), v2.as_mut_ptr(), om.as_ptr(), ov.as_ptr(), n,
                                         c.as_mut_ptr())
        })?;
        let mut res = Vec::with_capacity(n);
        for (i, o) in others.into_iter().enumerate() {
            if c[i] != 0 {
                res.push(Err(CrdtError::ConflictingMarker));
            } else {
                if m2[i] != ids[i] || v2[i] != 0 {  // other won (a strictly larger marker)
                    selves[i] = o;
                }
                res.push(Ok(()));
            }
        }
        Ok(res)
    }
}

// ---- Orswot: dot-store join + deferred removes (orswot.rs:81-149, 230-250, 281-286) ---------------
struct OrswotDense<M: Member, A: Actor> {
    actors: Index<A>,
    members: HIndex<M>,
}

impl<M: Member, A: Actor> OrswotDense<M, A> {
    fn of<'a, I: Iterator<Item = &'a Orswot<M, A>>>(states: I) -> Self
    where
        M: 'a,
        A: 'a,
    {
        let mut d = OrswotDense { actors: Index::new(), members: HIndex::new() };
        for s in states {
            for a in s.clock.dots.keys() {
                d.actors.intern(a);
            }
            for (m, c) in s.entries.iter() {
                d.members.intern(m);
                for a in c.dots.keys() {
                    d.actors.intern(a);
                }
            }
            for (k, ms) in s.deferred.iter() {
                for a in k.dots.keys() {
                    d.actors.intern(a);
                }
                for m in ms {
                    d.members.intern(m);
                }
            }
        }
        d
    }

    /// (clock [A], entries [M][A], deferred rm rows [D][A], member bitmaps [D][Mw])
    fn ingest(&self, s: &Orswot<M, A>) -> (Vec<u64>, Vec<u64>, Vec<u64>, Vec<u64>) {
        let (a, m) = (self.actors.width(), self.members.width());
        let mw = (m + 63) / 64;
        let mut clock = vec![0u64; a];
        clock_row(&s.clock, &self.actors, &mut clock);
        let mut entries = vec![0u64; m * a];
        for (mem, c) in s.entries.iter() {
            let i = self.members.pos[mem];
            clock_row(c, &self.actors, &mut entries[i * a..(i + 1) * a]);
        }
        let (mut dcl, mut dmb) = (Vec::new(), Vec::new());
        for (k, ms) in s.deferred.iter() {
            let mut row = vec![0u64; a];
            clock_row(k, &self.actors, &mut row);
            let mut bits = vec![0u64; mw];
            for mem in ms {
                let b = self.members.pos[mem];
                bits[b / 64] |= 1u64 << (b % 64);
            }
            dcl.extend(row);
            dmb.extend(bits);
        }
        (clock, entries, dcl, dmb)
    }

    fn egress(&self, clock: &[u64], entries: &[u64], deferred: &[(Vec<u64>, Vec<u64>)]) -> Orswot<M, A> {
        let a = self.actors.width();
        let mut s = Orswot::new();
        s.clock = row_clock(clock, &self.actors);
        for (i, mem) in self.members.ids.iter().enumerate() {
            let row = &entries[i * a..(i + 1) * a];
            if row.iter().any(|&x| x != 0) {
                s.entries.insert(mem.clone(), row_clock(row, &self.actors));
            }
        }
        for (rm, bits) in deferred {
            let mut ms = HashSet::new();
            for (w, &word) in bits.iter().enumerate() {
                let mut x = word;
                while x != 0 {
                    let b = w * 64 + x.trailing_zeros() as usize;
                    x &= x - 1;
                    if b < self.members.ids.len() {
                        ms.insert(self.members.ids[b].clone());
                    }
                }
            }
            s.deferred.entry(row_clock(rm, &self.actors)).or_insert_with(HashSet::new).extend(ms);
        }
        s
    }
}

/// `lub_many` is the exact left fold `Orswot::new()` + `merge` of every replica for ANY states (a
/// replica with entry dots above its clock, e.g. deserialized, is folded in replica order by the
/// library, `include/crdt_gpu.h`); `merge_batch` is exact for any pair.
impl<M: Member, A: Actor> BatchCvRDT for Orswot<M, A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(Orswot::new());
        }
        let d = OrswotDense::of(replicas.iter());
        let (r, a, m) = (replicas.len(), d.actors.width(), d.members.width());
        let mw = (m + 63) / 64;
        let (mut clock, mut entries, mut dcl, mut dmb) = (Vec::new(), Vec::new(), Vec::new(), Vec::new());
        for s in &replicas {
            let (c, e, x, y) = d.ingest(s);
            clock.extend(c);
            entries.extend(e);
            dcl.extend(x);
            dmb.extend(y);
        }
        let nd = dcl.len() / a;
        let def_off: [usize; 2] = [0, nd];
        // host rows straight to the CRDT_MEM_HOST ctx: the library streams replica chunks through its
        // two device buffers (the join of chunk k overlaps the copy of chunk k+1)
        let (mut c, mut e, mut keep, mut mem) = (vec![0u64; a], vec![0u64; m * a], vec![0u8; nd], vec![0u64; nd * mw]);
        let batch = ffi::crdt_orswot_batch {
            G: 1, R: r, M: m, A: a,
            clock: clock.as_ptr(), clock_rstride: a, clock_gstride: r * a,
            entries: entries.as_ptr(), entry_mstride: a, entry_rstride: m * a, entry_gstride: r * m * a,
            def_off: def_off.as_ptr(), def_clock: dcl.as_ptr(), def_members: dmb.as_ptr(),
        };
        let mut out = ffi::crdt_orswot_out {
            clock: c.as_mut_ptr(), entries: e.as_mut_ptr(),
            def_keep: if nd > 0 { keep.as_mut_ptr() } else { ptr::null_mut() },
            def_members: if nd > 0 { mem.as_mut_ptr() } else { ptr::null_mut() },
        };
        ctx.check_host(unsafe { ffi::crdt_orswot_lub_many(ctx.host, &batch, &mut out) })?;
        let mut surv = Vec::new();
        for i in 0..nd {
            if keep[i] != 0 {
                surv.push((dcl[i * a..(i + 1) * a].to_vec(), mem[i * mw..(i + 1) * mw].to_vec()));
            }
        }
        Ok(d.egress(&c, &e, &surv))
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        let n = selves.len();
        if n == 0 {
            return Ok(());
        }
        let d = OrswotDense::of(selves[..n].iter().chain(others[..n].iter()));
        let (a, m) = (d.actors.width(), d.members.width());
        let mw = (m + 63) / 64;
        // self's slots hold the survivors of BOTH sides of its own pair: size them per pair
        let dcap_o = others[..n].iter().map(|s| s.deferred.len()).max().unwrap_or(0).max(1);
        let dcap_s = (0..n).map(|i| selves[i].deferred.len() + others[i].deferred.len()).max().unwrap_or(0).max(1);
        if dcap_s + dcap_o > MERGE_MAX_DEFERRED {
            return Err(unsupported(format!("Orswot merge_batch: {} + {} deferred slots > {}", dcap_s, dcap_o,
                                           MERGE_MAX_DEFERRED)));
        }
        // per-state deferred slots (the crdt_orswot_states layout)
        let side = |states: &[Self], dcap: usize| {
            let (mut c, mut e) = (Vec::with_capacity(n * a), Vec::with_capacity(n * m * a));
            let (mut dc, mut dm, mut cnt) = (vec![0u64; n * dcap * a], vec![0u64; n * dcap * mw], vec![0u32; n]);
            for (i, s) in states.iter().enumerate() {
                let (x, y, rows, bits) = d.ingest(s);
                c.extend(x);
                e.extend(y);
                let k = rows.len() / a;
                dc[i * dcap * a..i * dcap * a + k * a].copy_from_slice(&rows);
                dm[i * dcap * mw..i * dcap * mw + k * mw].copy_from_slice(&bits);
                cnt[i] = k as u32;
            }
            (c, e, dc, dm, cnt)
        };
        let (mut sc, mut se, mut sdc, mut sdm, mut scnt) = side(&selves[..n], dcap_s);
        let (mut oc, mut oe, mut odc, mut odm, mut ocnt) = side(&others[..n], dcap_o);
        let ss = ffi::crdt_orswot_states {
            N: n, M: m, A: a, Dcap: dcap_s,
            clock: sc.as_mut_ptr(), clock_stride: a, entries: se.as_mut_ptr(), entry_mstride: a, entry_sstride: m * a,
            def_clock: sdc.as_mut_ptr(), def_members: sdm.as_mut_ptr(), def_count: scnt.as_mut_ptr(),
        };
        let os = ffi::crdt_orswot_states {
            N: n, M: m, A: a, Dcap: dcap_o,
            clock: oc.as_mut_ptr(), clock_stride: a, entries: oe.as_mut_ptr(), entry_mstride: a, entry_sstride: m * a,
            def_clock: odc.as_mut_ptr(), def_members: odm.as_mut_ptr(), def_count: ocnt.as_mut_ptr(),
        };
        let mut stv = vec![0u32; n];
        // host arrays straight to the CRDT_MEM_HOST ctx: staged, merged in HBM, copied back into them
        ctx.check_host(unsafe { ffi::crdt_orswot_merge_batch(ctx.host, &ss, &os, stv.as_mut_ptr()) })?;
        let (c, e, dc, dm, cnt) = (&sc, &se, &sdc, &sdm, &scnt);
        // every status first: on an error no state of `selves` has been replaced
        if let Some(i) = (0..n).find(|&i| stv[i] != 0) {
            return Err(unsupported(format!("Orswot merge_batch: pair {} status {}", i, stv[i])));
        }
        for i in 0..n {
            let mut defs = Vec::new();
            for k in 0..cnt[i] as usize {
                let base = i * dcap_s + k;
                defs.push((dc[base * a..(base + 1) * a].to_vec(), dm[base * mw..(base + 1) * mw].to_vec()));
            }
            selves[i] = d.egress(&c[i * a..(i + 1) * a], &e[i * m * a..(i + 1) * m * a], &defs);
        }
        Ok(())
    }
}

// ---- Map<K, MVReg<V, A>, A>: exact per-key left fold (map.rs:140-220, mvreg.rs:112-128) ------------
// MVReg::merge compares value CLOCKS only (never the values), so every value instance gets a
// fresh u64 id into a per-call arena and comes back by clone; keys and actors are interned.
struct MapDense<K: Ord + Clone, A: Actor> {
    actors: Index<A>,
    keys: Index<K>,
    vmax: usize,
}

/// One state's dense rows (the crdt_map_states / crdt_map_deferred per-state layout).
struct MapRows {
    clock: Vec<u64>,    // [A]
    ec: Vec<u64>,       // [K][A]
    vclk: Vec<u64>,     // [K][V][A]
    vval: Vec<u64>,     // [K][V] arena ids
    def_clock: Vec<u64>, // [D][A]
    def_keys: Vec<u64>,  // [D][Kw]
}

impl<K: Ord + Clone, A: Actor> MapDense<K, A> {
    fn of<'a, V: Clone + 'a, I: Iterator<Item = &'a Map<K, MVReg<V, A>, A>>>(states: I) -> Self
    where
        K: 'a,
        A: 'a,
    {
        let mut d = MapDense { actors: Index::new(), keys: Index::new(), vmax: 1 };
        for s in states {
            for a in s.clock.dots.keys() {
                d.actors.intern(a);
            }
            for (k, e) in s.entries.iter() {
                d.keys.intern(k);
                for a in e.clock.dots.keys() {
                    d.actors.intern(a);
                }
                d.vmax = d.vmax.max(e.val.vals.len());
                for (c, _) in e.val.vals.iter() {
                    for a in c.dots.keys() {
                        d.actors.intern(a);
                    }
                }
            }
            for (rm, ks) in s.deferred.iter() {
                for a in rm.dots.keys() {
                    d.actors.intern(a);
                }
                for k in ks {
                    d.keys.intern(k);
                }
            }
        }
        d
    }

    fn ingest<V: Clone>(&self, s: &Map<K, MVReg<V, A>, A>, v: usize, arena: &mut Vec<V>) -> MapRows {
        let (a, k) = (self.actors.width(), self.keys.width());
        let kw = (k + 63) / 64;
        let mut r = MapRows {
            clock: vec![0u64; a],
            ec: vec![0u64; k * a],
            vclk: vec![0u64; k * v * a],
            vval: vec![0u64; k * v],
            def_clock: Vec::new(),
            def_keys: Vec::new(),
        };
        clock_row(&s.clock, &self.actors, &mut r.clock);
        for (key, e) in s.entries.iter() {
            let i = self.keys.pos[key];
            clock_row(&e.clock, &self.actors, &mut r.ec[i * a..(i + 1) * a]);
            for (slot, (c, val)) in e.val.vals.iter().enumerate().take(v) {
                let base = (i * v + slot) * a;
                clock_row(c, &self.actors, &mut r.vclk[base..base + a]);
                r.vval[i * v + slot] = arena.len() as u64;
                arena.push(val.clone());
            }
        }
        for (rm, ks) in s.deferred.iter() {
            let mut row = vec![0u64; a];
            clock_row(rm, &self.actors, &mut row);
            let mut bits = vec![0u64; kw];
            for key in ks {
                let b = self.keys.pos[key];
                bits[b / 64] |= 1u64 << (b % 64);
            }
            r.def_clock.extend(row);
            r.def_keys.extend(bits);
        }
        r
    }

    /// Rebuild a Map from one state's rows (value slot s of key k: vclk[(k*v + s)*a ..]).
    fn egress<V: Clone>(&self, clock: &[u64], ec: &[u64], vclk: &[u64], vval: &[u64], v: usize,
                        deferred: &[(Vec<u64>, Vec<u64>)], arena: &[V]) -> Map<K, MVReg<V, A>, A> {
        let a = self.actors.width();
        let mut m = Map::new();
        m.clock = row_clock(clock, &self.actors);
        for (i, key) in self.keys.ids.iter().enumerate() {
            let row = &ec[i * a..(i + 1) * a];
            if row.iter().all(|&x| x == 0) {
                continue;
            }
            let mut vals = Vec::new();
            for slot in 0..v {
                let base = (i * v + slot) * a;
                let vr = &vclk[base..base + a];
                if vr.iter().any(|&x| x != 0) {
                    vals.push((row_clock(vr, &self.actors), arena[vval[i * v + slot] as usize].clone()));
                }
            }
            m.entries.insert(key.clone(), Entry { clock: row_clock(row, &self.actors), val: MVReg { vals } });
        }
        for (rm, bits) in deferred {
            let mut ks = BTreeSet::new();
            for (w, &word) in bits.iter().enumerate() {
                let mut x = word;
                while x != 0 {
                    let b = w * 64 + x.trailing_zeros() as usize;
                    x &= x - 1;
                    if b < self.keys.ids.len() {
                        ks.insert(self.keys.ids[b].clone());
                    }
                }
            }
            m.deferred.entry(row_clock(rm, &self.actors)).or_insert_with(BTreeSet::new).extend(ks);
        }
        m
    }
}

impl<K: Ord + Clone, V: Clone, A: Actor> BatchCvRDT for Map<K, MVReg<V, A>, A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(Map::new());
        }
        let d = MapDense::of(replicas.iter());
        let (r, a, k, v) = (replicas.len(), d.actors.width(), d.keys.width(), d.vmax);
        let kw = (k + 63) / 64;
        if v > MAP_MAX_VALUES || a > MAP_MAX_ACTORS {
            return Err(unsupported(format!("Map lub_many: {} values per register / {} actors (limits {} / {})", v, a,
                                           MAP_MAX_VALUES, MAP_MAX_ACTORS)));
        }
        let mut arena = Vec::new();
        let (mut clock, mut ec, mut vclk, mut vval) = (Vec::new(), Vec::new(), Vec::new(), Vec::new());
        let (mut def_row, mut dcl, mut dks) = (Vec::new(), Vec::new(), Vec::new());
        for (i, s) in replicas.iter().enumerate() {
            let rows = d.ingest(s, v, &mut arena);
            clock.extend(rows.clock);
            ec.extend(rows.ec);
            vclk.extend(rows.vclk);
            vval.extend(rows.vval);
            for _ in 0..rows.def_clock.len() / a {
                def_row.push(i as u32);
            }
            dcl.extend(rows.def_clock);
            dks.extend(rows.def_keys);
        }
        let nd = def_row.len();
        let def_off: [usize; 2] = [0, nd];
        let batch = ffi::crdt_map_batch {
            G: 1, R: r, K: k, A: a, V: v,
            clock: clock.as_ptr(), clock_rstride: a, clock_gstride: r * a,
            ec: ec.as_ptr(), ec_rstride: k * a, ec_gstride: r * k * a,
            vclk: vclk.as_ptr(), vclk_rstride: k * v * a, vclk_gstride: r * k * v * a,
            vval: vval.as_ptr(), vval_rstride: k * v, vval_gstride: r * k * v,
            def_off: def_off.as_ptr(), def_row: def_row.as_ptr(), def_clock: dcl.as_ptr(), def_keys: dks.as_ptr(),
        };
        // Vout grows until the fold fits (flags bit 0 = some key folded to more values); the fold
        // state starts at the library's choice (4 values: the scanned fast path) and widens to 8,
        // then 16 values when a key overflows it (flags bit 2)
        let mut vout = 4usize;
        let mut vstate = 0usize;
        loop {
            let (mut oc, mut oec) = (vec![0u64; a], vec![0u64; k * a]);
            let (mut ovc, mut ovv) = (vec![0u64; k * vout * a], vec![0u64; k * vout]);
            let (mut flags, mut keep, mut okeys) = (vec![0u32; 1], vec![0u8; nd], vec![0u64; nd * kw]);
            let mut out = ffi::crdt_map_out {
                Vout: vout, Vstate: vstate,
                clock: oc.as_mut_ptr(), ec: oec.as_mut_ptr(), vclk: ovc.as_mut_ptr(), vval: ovv.as_mut_ptr(),
                nval: ptr::null_mut(), flags: flags.as_mut_ptr(),
                def_keep: if nd > 0 { keep.as_mut_ptr() } else { ptr::null_mut() },
                def_keys: if nd > 0 { okeys.as_mut_ptr() } else { ptr::null_mut() },
            };
            ctx.check_host(unsafe { ffi::crdt_map_lub_many(ctx.host, &batch, &mut out) })?;
            if flags[0] & 4 != 0 && vstate < 16 {
                vstate = if vstate < 8 { 8 } else { 16 };
                continue;
            }
            if flags[0] & 1 != 0 && vout < 64 {
                vout = (vout * 2).min(64);
                continue;
            }
            if flags[0] != 0 {
                return Err(GpuError { code: ffi::CRDT_EUNSUPPORTED, msg: format!("Map lub_many flags {}", flags[0]) });
            }
            let mut surv = Vec::new();
            for i in 0..nd {
                if keep[i] != 0 {
                    surv.push((dcl[i * a..(i + 1) * a].to_vec(), okeys[i * kw..(i + 1) * kw].to_vec()));
                }
            }
            return Ok(d.egress(&oc, &oec, &ovc, &ovv, vout, &surv, &arena));
        }
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        let n = selves.len();
        if n == 0 {
            return Ok(());
        }
        let d = MapDense::of(selves[..n].iter().chain(others[..n].iter()));
        let (a, k) = (d.actors.width(), d.keys.width());
        let kw = (k + 63) / 64;
        let nv = |s: &Self| s.entries.values().map(|e| e.val.vals.len()).max().unwrap_or(0);
        let vo = others[..n].iter().map(|s| nv(s)).max().unwrap_or(0).max(1);
        // a merged register holds at most its own values plus the other side's: per pair
        let vs = (0..n).map(|i| nv(&selves[i]) + nv(&others[i])).max().unwrap_or(0).max(1);
        let dcap_o = others[..n].iter().map(|s| s.deferred.len()).max().unwrap_or(0).max(1);
        let dcap_s = (0..n).map(|i| selves[i].deferred.len() + others[i].deferred.len()).max().unwrap_or(0).max(1);
        if vs > MAP_MAX_VALUES || a > MAP_MAX_ACTORS || dcap_s + dcap_o > MERGE_MAX_DEFERRED {
            return Err(unsupported(format!("Map merge_batch: {} values per register / {} actors / {} + {} deferred \
                                            slots (limits {} / {} / {})", vs, a, dcap_s, dcap_o, MAP_MAX_VALUES,
                                           MAP_MAX_ACTORS, MERGE_MAX_DEFERRED)));
        }
        let mut arena = Vec::new();
        let mut side = |states: &[Self], v: usize, dcap: usize| {
            let (mut c, mut ec, mut vc, mut vv) = (Vec::new(), Vec::new(), Vec::new(), Vec::new());
            let (mut dc, mut dk, mut cnt) = (vec![0u64; n * dcap * a], vec![0u64; n * dcap * kw], vec![0u32; n]);
            for (i, s) in states.iter().enumerate() {
                let rows = d.ingest(s, v, &mut arena);
                c.extend(rows.clock);
                ec.extend(rows.ec);
                vc.extend(rows.vclk);
                vv.extend(rows.vval);
                let nd = rows.def_clock.len() / a;
                dc[i * dcap * a..i * dcap * a + nd * a].copy_from_slice(&rows.def_clock);
                dk[i * dcap * kw..i * dcap * kw + nd * kw].copy_from_slice(&rows.def_keys);
                cnt[i] = nd as u32;
            }
            (c, ec, vc, vv, dc, dk, cnt)
        };
        let (mut sc, mut sec, mut svc, mut svv, mut sdc, mut sdk, mut scnt) = side(&selves[..n], vs, dcap_s);
        let (mut oc, mut oec, mut ovc, mut ovv, mut odc, mut odk, mut ocnt) = side(&others[..n], vo, dcap_o);
        let ss = ffi::crdt_map_states {
            N: n, K: k, A: a, V: vs,
            clock: sc.as_mut_ptr(), clock_stride: a, ec: sec.as_mut_ptr(), ec_stride: k * a,
            vclk: svc.as_mut_ptr(), vclk_stride: k * vs * a, vval: svv.as_mut_ptr(), vval_stride: k * vs,
        };
        let sd = ffi::crdt_map_deferred { clock: sdc.as_mut_ptr(), keys: sdk.as_mut_ptr(), count: scnt.as_mut_ptr(), Dcap: dcap_s };
        let os = ffi::crdt_map_states {
            N: n, K: k, A: a, V: vo,
            clock: oc.as_mut_ptr(), clock_stride: a, ec: oec.as_mut_ptr(), ec_stride: k * a,
            vclk: ovc.as_mut_ptr(), vclk_stride: k * vo * a, vval: ovv.as_mut_ptr(), vval_stride: k * vo,
        };
        let od = ffi::crdt_map_deferred { clock: odc.as_mut_ptr(), keys: odk.as_mut_ptr(), count: ocnt.as_mut_ptr(), Dcap: dcap_o };
        let mut stv = vec![0u32; n];
        ctx.check_host(unsafe { ffi::crdt_map_merge_batch(ctx.host, &ss, &sd, &os, &od, stv.as_mut_ptr()) })?;
        // every status first: on an error no state of `selves` has been replaced
        if let Some(i) = (0..n).find(|&i| stv[i] != 0) {
            return Err(unsupported(format!("Map merge_batch: pair {} status {}", i, stv[i])));
        }
        for i in 0..n {
            let mut defs = Vec::new();
            for j in 0..scnt[i] as usize {
                let base = i * dcap_s + j;
                defs.push((sdc[base * a..(base + 1) * a].to_vec(), sdk[base * kw..(base + 1) * kw].to_vec()));
            }
            selves[i] = d.egress(&sc[i * a..(i + 1) * a], &sec[i * k * a..(i + 1) * k * a],
                                 &svc[i * k * vs * a..(i + 1) * k * vs * a], &svv[i * k * vs..(i + 1) * k * vs], vs,
                                 &defs, &arena);
        }
        Ok(())
    }
}

// ---- Map<K, V, A> with counter, Orswot and nested-Map values (round 5) ----------------------------
// The library folds each key of these Maps in replica order (crdt_map_counter_lub_many,
// crdt_map_orswot_lub_many, crdt_map_nested_lub_many; host arrays through the CRDT_MEM_HOST ctx, staged
// whole).  `lub_many` is one group of R replicas; `merge_batch` is N groups of the two replicas
// [self_i, other_i]: Map::new().merge(s).merge(o) == s.merge(o) for every state a replica can hold (its
// deferred removes already applied to its entries and not covered by its own clock, map.rs:318-348).

/// A batch of groups, each a fold of its replicas: (clock, ec [K][A], the Map's deferred pool).
struct GroupPool {
    def_off: Vec<usize>,
    def_row: Vec<u32>,
    def_clock: Vec<u64>,
    def_keys: Vec<u64>,
}

fn key_bits<K: Ord + Clone>(ks: &BTreeSet<K>, idx: &Index<K>, kw: usize) -> Vec<u64> {
    let mut bits = vec![0u64; kw];
    for key in ks {
        let b = idx.pos[key];
        bits[b / 64] |= 1u64 << (b % 64);
    }
    bits
}

fn bit_keys<K: Ord + Clone>(bits: &[u64], idx: &Index<K>) -> BTreeSet<K> {
    let mut ks = BTreeSet::new();
    for (w, &word) in bits.iter().enumerate() {
        let mut x = word;
        while x != 0 {
            let b = w * 64 + x.trailing_zeros() as usize;
            x &= x - 1;
            if b < idx.ids.len() {
                ks.insert(idx.ids[b].clone());
            }
        }
    }
    ks
}

/// The Map-level interning shared by the value-typed Maps: actors and keys of the Map itself.
fn map_level_index<'a, K: Ord + Clone + 'a, V: crate::map::Val<A> + 'a, A: Actor + 'a>(
    states: &[&'a Map<K, V, A>], actors: &mut Index<A>, keys: &mut Index<K>) {
    for s in states {
        for a in s.clock.dots.keys() {
            actors.intern(a);
        }
        for (k, e) in s.entries.iter() {
            keys.intern(k);
            for a in e.clock.dots.keys() {
                actors.intern(a);
            }
        }
        for (rm, ks) in s.deferred.iter() {
            for a in rm.dots.keys() {
                actors.intern(a);
            }
            for k in ks {
                keys.intern(k);
            }
        }
    }
}

/// The Map's own deferred removes of every group, pooled in replica order (def_row local to its group).
fn group_pool<K: Ord + Clone, V: crate::map::Val<A>, A: Actor>(groups: &[Vec<&Map<K, V, A>>], actors: &Index<A>,
                                                               keys: &Index<K>) -> GroupPool {
    let (a, kw) = (actors.width(), (keys.width() + 63) / 64);
    let mut p = GroupPool { def_off: vec![0], def_row: Vec::new(), def_clock: Vec::new(), def_keys: Vec::new() };
    for g in groups {
        for (r, s) in g.iter().enumerate() {
            for (rm, ks) in s.deferred.iter() {
                let mut row = vec![0u64; a];
                clock_row(rm, actors, &mut row);
                p.def_row.push(r as u32);
                p.def_clock.extend(row);
                p.def_keys.extend(key_bits(ks, keys, kw));
            }
        }
        p.def_off.push(p.def_row.len());
    }
    p
}

/// The surviving removes of group g (def_keep / def_keys of the call) as the Map's deferred map.
fn group_survivors<K: Ord + Clone, A: Actor>(p: &GroupPool, g: usize, keep: &[u8], okeys: &[u64], actors: &Index<A>,
                                             keys: &Index<K>) -> HashMap<VClock<A>, BTreeSet<K>> {
    let (a, kw) = (actors.width(), (keys.width() + 63) / 64);
    let mut out: HashMap<VClock<A>, BTreeSet<K>> = HashMap::new();
    for d in p.def_off[g]..p.def_off[g + 1] {
        if keep[d] != 0 {
            let ks = bit_keys(&okeys[d * kw..(d + 1) * kw], keys);
            out.entry(row_clock(&p.def_clock[d * a..(d + 1) * a], actors)).or_insert_with(BTreeSet::new).extend(ks);
        }
    }
    out
}

fn pairs_as_groups<'a, T>(selves: &'a [T], others: &'a [T]) -> Vec<Vec<&'a T>> {
    selves.iter().zip(others.iter()).map(|(s, o)| vec![s, o]).collect()
}

/// GCounter (one row) / PNCounter (P | N rows) as the value rows of the counter Map fold.
trait CounterVal<A: Actor>: crate::map::Val<A> + Default + Sized {
    const W: usize;
    fn intern_actors(&self, idx: &mut Index<A>);
    fn rows(&self, idx: &Index<A>, out: &mut [u64]);
    fn from_rows(rows: &[u64], idx: &Index<A>) -> Self;
}

impl<A: Actor> CounterVal<A> for GCounter<A> {
    const W: usize = 1;
    fn intern_actors(&self, idx: &mut Index<A>) {
        for a in self.inner.dots.keys() {
            idx.intern(a);
        }
    }
    fn rows(&self, idx: &Index<A>, out: &mut [u64]) {
        clock_row(&self.inner, idx, out);
    }
    fn from_rows(rows: &[u64], idx: &Index<A>) -> Self {
        let mut g = GCounter::new();
        g.inner = row_clock(rows, idx);
        g
    }
}

impl<A: Actor> CounterVal<A> for PNCounter<A> {
    const W: usize = 2;
    fn intern_actors(&self, idx: &mut Index<A>) {
        for a in self.p.inner.dots.keys().chain(self.n.inner.dots.keys()) {
            idx.intern(a);
        }
    }
    fn rows(&self, idx: &Index<A>, out: &mut [u64]) {
        let a = idx.width();
        clock_row(&self.p.inner, idx, &mut out[..a]);
        clock_row(&self.n.inner, idx, &mut out[a..2 * a]);
    }
    fn from_rows(rows: &[u64], idx: &Index<A>) -> Self {
        let a = idx.width();
        let mut c = PNCounter::new();
        c.p.inner = row_clock(&rows[..a], idx);
        c.n.inner = row_clock(&rows[a..2 * a], idx);
        c
    }
}

/// Every group's fold of Map<K, counter> (crdt_map_counter_lub_many, G groups of equal R).
fn counter_map_folds<K: Ord + Clone, V: CounterVal<A>, A: Actor>(ctx: &GpuCtx, groups: &[Vec<&Map<K, V, A>>])
                                                                 -> Result<Vec<Map<K, V, A>>, GpuError> {
    let (g, r) = (groups.len(), groups[0].len());
    let (mut actors, mut keys) = (Index::new(), Index::new());
    let all: Vec<&Map<K, V, A>> = groups.iter().flat_map(|x| x.iter().copied()).collect();
    map_level_index(&all, &mut actors, &mut keys);
    for s in &all {
        for e in s.entries.values() {
            e.val.intern_actors(&mut actors);
        }
    }
    let (a, k, w) = (actors.width(), keys.width(), V::W);
    let kw = (k + 63) / 64;
    let (mut clock, mut ec, mut val) = (vec![0u64; g * r * a], vec![0u64; g * r * k * a], vec![0u64; g * r * k * w * a]);
    for (i, s) in all.iter().enumerate() {
        clock_row(&s.clock, &actors, &mut clock[i * a..(i + 1) * a]);
        for (key, e) in s.entries.iter() {
            let j = keys.pos[key];
            clock_row(&e.clock, &actors, &mut ec[(i * k + j) * a..(i * k + j + 1) * a]);
            e.val.rows(&actors, &mut val[(i * k + j) * w * a..(i * k + j + 1) * w * a]);
        }
    }
    let pool = group_pool(groups, &actors, &keys);
    let nd = pool.def_row.len();
    let batch = ffi::crdt_map_counter_batch {
        G: g, R: r, K: k, A: a, W: w,
        clock: clock.as_ptr(), clock_rstride: a, clock_gstride: r * a,
        ec: ec.as_ptr(), ec_rstride: k * a, ec_gstride: r * k * a,
        val: val.as_ptr(), val_rstride: k * w * a, val_gstride: r * k * w * a,
        def_off: if nd > 0 { pool.def_off.as_ptr() } else { ptr::null() },
        def_row: pool.def_row.as_ptr(), def_clock: pool.def_clock.as_ptr(), def_keys: pool.def_keys.as_ptr(),
    };
    let (mut oc, mut oec, mut ov) = (vec![0u64; g * a], vec![0u64; g * k * a], vec![0u64; g * k * w * a]);
    let (mut flags, mut keep, mut okeys) = (vec![0u32; g], vec![0u8; nd], vec![0u64; nd * kw]);
    let mut out = ffi::crdt_map_counter_out {
        clock: oc.as_mut_ptr(), ec: oec.as_mut_ptr(), val: ov.as_mut_ptr(), flags: flags.as_mut_ptr(),
        def_keep: if nd > 0 { keep.as_mut_ptr() } else { ptr::null_mut() },
        def_keys: if nd > 0 { okeys.as_mut_ptr() } else { ptr::null_mut() },
    };
    ctx.check_host(unsafe { ffi::crdt_map_counter_lub_many(ctx.host, &batch, &mut out) })?;
    if let Some(f) = flags.iter().find(|&&f| f != 0) {
        return Err(unsupported(format!("Map<K, counter> lub_many flags {}", f)));
    }
    let mut res = Vec::with_capacity(g);
    for gi in 0..g {
        let mut m: Map<K, V, A> = Map::new();
        m.clock = row_clock(&oc[gi * a..(gi + 1) * a], &actors);
        for (j, key) in keys.ids.iter().enumerate() {
            let row = &oec[(gi * k + j) * a..(gi * k + j + 1) * a];
            if row.iter().any(|&x| x != 0) {
                let v = V::from_rows(&ov[(gi * k + j) * w * a..(gi * k + j + 1) * w * a], &actors);
                m.entries.insert(key.clone(), Entry { clock: row_clock(row, &actors), val: v });
            }
        }
        m.deferred = group_survivors(&pool, gi, &keep, &okeys, &actors, &keys);
        res.push(m);
    }
    Ok(res)
}

impl<K: Ord + Clone, A: Actor> BatchCvRDT for Map<K, GCounter<A>, A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(Map::new());
        }
        Ok(counter_map_folds(ctx, &[replicas.iter().collect()])?.remove(0))
    }
    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        if selves.is_empty() {
            return Ok(());
        }
        let merged = counter_map_folds(ctx, &pairs_as_groups(selves, &others))?;
        for (s, m) in selves.iter_mut().zip(merged) {
            *s = m;
        }
        Ok(())
    }
}

impl<K: Ord + Clone, A: Actor> BatchCvRDT for Map<K, PNCounter<A>, A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(Map::new());
        }
        Ok(counter_map_folds(ctx, &[replicas.iter().collect()])?.remove(0))
    }
    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        if selves.is_empty() {
            return Ok(());
        }
        let merged = counter_map_folds(ctx, &pairs_as_groups(selves, &others))?;
        for (s, m) in selves.iter_mut().zip(merged) {
            *s = m;
        }
        Ok(())
    }
}

/// Limits of the Map<K, Orswot> fold (include/crdt_gpu.h: A <= 1,024, M <= 1,024, 16 nested removes;
/// past A = 64 or M = 32 the library runs its wide kernel).
pub const MAP_ORSWOT_MAX_ACTORS: usize = 1024;
pub const MAP_ORSWOT_MAX_MEMBERS: usize = 1024;

/// Every group's fold of Map<K, Orswot<M>> (crdt_map_orswot_lub_many, G groups of equal R).
fn orswot_map_folds<K: Ord + Clone, M: Member, A: Actor>(ctx: &GpuCtx, groups: &[Vec<&Map<K, Orswot<M, A>, A>>])
                                                         -> Result<Vec<Map<K, Orswot<M, A>, A>>, GpuError> {
    let (g, r) = (groups.len(), groups[0].len());
    let (mut actors, mut keys, mut mems) = (Index::new(), Index::new(), HIndex::new());
    let all: Vec<&Map<K, Orswot<M, A>, A>> = groups.iter().flat_map(|x| x.iter().copied()).collect();
    map_level_index(&all, &mut actors, &mut keys);
    for s in &all {
        for e in s.entries.values() {
            for x in e.val.clock.dots.keys() {
                actors.intern(x);
            }
            for (mem, c) in e.val.entries.iter() {
                mems.intern(mem);
                for x in c.dots.keys() {
                    actors.intern(x);
                }
            }
            for (rm, ms) in e.val.deferred.iter() {
                for x in rm.dots.keys() {
                    actors.intern(x);
                }
                for mem in ms {
                    mems.intern(mem);
                }
            }
        }
    }
    let (a, k, m) = (actors.width(), keys.width(), mems.width());
    if a > MAP_ORSWOT_MAX_ACTORS || m > MAP_ORSWOT_MAX_MEMBERS {
        return Err(unsupported(format!("Map<K, Orswot> lub_many: {} actors / {} members (limits {} / {})", a, m,
                                       MAP_ORSWOT_MAX_ACTORS, MAP_ORSWOT_MAX_MEMBERS)));
    }
    let kw = (k + 63) / 64;
    let mw = if m > 64 { (m + 63) / 64 } else { 1 }; // member-mask words
    let n = g * r * k;
    let (mut clock, mut ec, mut oc) = (vec![0u64; g * r * a], vec![0u64; n * a], vec![0u64; n * a]);
    let mut ent = vec![0u64; n * m * a];
    let (mut vd_off, mut vd_clock, mut vd_mem) = (vec![0u64], Vec::new(), Vec::new());
    for (i, s) in all.iter().enumerate() {
        clock_row(&s.clock, &actors, &mut clock[i * a..(i + 1) * a]);
        for j in 0..k {
            if let Some(e) = s.entries.get(&keys.ids[j]) {
                let b = i * k + j;
                clock_row(&e.clock, &actors, &mut ec[b * a..(b + 1) * a]);
                clock_row(&e.val.clock, &actors, &mut oc[b * a..(b + 1) * a]);
                for (mem, c) in e.val.entries.iter() {
                    let mi = mems.pos[mem];
                    clock_row(c, &actors, &mut ent[(b * m + mi) * a..(b * m + mi + 1) * a]);
                }
                for (rm, ms) in e.val.deferred.iter() {
                    let mut row = vec![0u64; a];
                    clock_row(rm, &actors, &mut row);
                    vd_clock.extend(row);
                    let mut words = vec![0u64; mw];
                    for x in ms {
                        let p = mems.pos[x];
                        words[p / 64] |= 1u64 << (p % 64);
                    }
                    vd_mem.extend(words);
                }
            }
            vd_off.push((vd_mem.len() / mw) as u64);
        }
    }
    let pool = group_pool(groups, &actors, &keys);
    let (nd, dv) = (pool.def_row.len(), vd_mem.len() / mw);
    // nested slots per key: the largest sum of one key's list lengths over its group (no fold result
    // holds more), at least the library's 16 (round 6: past 16 the library re-folds those keys exactly)
    let mut vdc = 16usize;
    for gi in 0..g {
        for j in 0..k {
            let mut t = 0usize;
            for ri in 0..r {
                let b = (gi * r + ri) * k + j;
                t += (vd_off[b + 1] - vd_off[b]) as usize;
            }
            vdc = vdc.max(t);
        }
    }
    let batch = ffi::crdt_map_orswot_batch {
        G: g, R: r, K: k, M: m, A: a,
        clock: clock.as_ptr(), ec: ec.as_ptr(), oc: oc.as_ptr(), ent: ent.as_ptr(),
        vd_off: vd_off.as_ptr(), vd_clock: vd_clock.as_ptr(), vd_mem: vd_mem.as_ptr(),
        def_off: if nd > 0 { pool.def_off.as_ptr() } else { ptr::null() },
        def_row: pool.def_row.as_ptr(), def_clock: pool.def_clock.as_ptr(), def_keys: pool.def_keys.as_ptr(),
        Dv: dv,
    };
    let (mut o_clock, mut o_ec, mut o_oc) = (vec![0u64; g * a], vec![0u64; g * k * a], vec![0u64; g * k * a]);
    let (mut o_ent, mut o_vdn) = (vec![0u64; g * k * m * a], vec![0u32; g * k]);
    let (mut o_vdc, mut o_vdm) = (vec![0u64; g * k * vdc * a], vec![0u64; g * k * vdc * mw]);
    let (mut flags, mut keep, mut okeys) = (vec![0u32; g], vec![0u8; nd], vec![0u64; nd * kw]);
    let mut out = ffi::crdt_map_orswot_out {
        clock: o_clock.as_mut_ptr(), ec: o_ec.as_mut_ptr(), oc: o_oc.as_mut_ptr(), ent: o_ent.as_mut_ptr(),
        vd_n: o_vdn.as_mut_ptr(), vd_clock: o_vdc.as_mut_ptr(), vd_mem: o_vdm.as_mut_ptr(), flags: flags.as_mut_ptr(),
        def_keep: if nd > 0 { keep.as_mut_ptr() } else { ptr::null_mut() },
        def_keys: if nd > 0 { okeys.as_mut_ptr() } else { ptr::null_mut() },
        Vd: vdc,
    };
    ctx.check_host(unsafe { ffi::crdt_map_orswot_lub_many(ctx.host, &batch, &mut out) })?;
    if let Some(f) = flags.iter().find(|&&f| f != 0) {
        return Err(unsupported(format!("Map<K, Orswot> lub_many flags {}", f)));
    }
    let mut res = Vec::with_capacity(g);
    for gi in 0..g {
        let mut mp: Map<K, Orswot<M, A>, A> = Map::new();
        mp.clock = row_clock(&o_clock[gi * a..(gi + 1) * a], &actors);
        for (j, key) in keys.ids.iter().enumerate() {
            let b = gi * k + j;
            let row = &o_ec[b * a..(b + 1) * a];
            if row.iter().all(|&x| x == 0) {
                continue;
            }
            let mut o = Orswot::new();
            o.clock = row_clock(&o_oc[b * a..(b + 1) * a], &actors);
            for (mi, mem) in mems.ids.iter().enumerate() {
                let er = &o_ent[(b * m + mi) * a..(b * m + mi + 1) * a];
                if er.iter().any(|&x| x != 0) {
                    o.entries.insert(mem.clone(), row_clock(er, &actors));
                }
            }
            for i in 0..o_vdn[b] as usize {
                let bits = &o_vdm[(b * vdc + i) * mw..(b * vdc + i + 1) * mw];
                let ms: HashSet<M> =
                    (0..m).filter(|&x| (bits[x / 64] >> (x % 64)) & 1 != 0).map(|x| mems.ids[x].clone()).collect();
                o.deferred.entry(row_clock(&o_vdc[(b * vdc + i) * a..(b * vdc + i + 1) * a], &actors))
                    .or_insert_with(HashSet::new).extend(ms);
            }
            mp.entries.insert(key.clone(), Entry { clock: row_clock(row, &actors), val: o });
        }
        mp.deferred = group_survivors(&pool, gi, &keep, &okeys, &actors, &keys);
        res.push(mp);
    }
    Ok(res)
}

impl<K: Ord + Clone, M: Member, A: Actor> BatchCvRDT for Map<K, Orswot<M, A>, A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(Map::new());
        }
        Ok(orswot_map_folds(ctx, &[replicas.iter().collect()])?.remove(0))
    }
    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        if selves.is_empty() {
            return Ok(());
        }
        let merged = orswot_map_folds(ctx, &pairs_as_groups(selves, &others))?;
        for (s, m) in selves.iter_mut().zip(merged) {
            *s = m;
        }
        Ok(())
    }
}

/// Limits of the nested Map fold (include/crdt_gpu.h: A <= 256, K2 <= 256 and V <= 64 values per register
/// since round 6).  Past 64 inner keys an inner key set is ceil(K2/64) mask words.
pub const MAP_NESTED_MAX_ACTORS: usize = 256;
pub const MAP_NESTED_MAX_INNER_KEYS: usize = 256;
pub const MAP_NESTED_MAX_VALUES: usize = 64;  // (round 6: past 8 the library's deep pass; was 8)

/// Every group's fold of Map<K, Map<K2, MVReg<V>>> (crdt_map_nested_lub_many, G groups of equal R) —
/// the type of the reference's own Map tests (test/map.rs:10).  Values travel as arena ids, as for
/// Map<K, MVReg> (MVReg::merge compares value clocks only).
fn nested_map_folds<K: Ord + Clone, K2: Ord + Clone, V: Clone, A: Actor>(
    ctx: &GpuCtx, groups: &[Vec<&Map<K, Map<K2, MVReg<V, A>, A>, A>>])
    -> Result<Vec<Map<K, Map<K2, MVReg<V, A>, A>, A>>, GpuError> {
    let (g, r) = (groups.len(), groups[0].len());
    let (mut actors, mut keys, mut ikeys) = (Index::new(), Index::new(), Index::new());
    let all: Vec<&Map<K, Map<K2, MVReg<V, A>, A>, A>> = groups.iter().flat_map(|x| x.iter().copied()).collect();
    map_level_index(&all, &mut actors, &mut keys);
    let mut vmax = 1usize;
    for s in &all {
        for e in s.entries.values() {
            let inner = [&e.val];
            map_level_index(&inner, &mut actors, &mut ikeys);
            for ie in e.val.entries.values() {
                vmax = vmax.max(ie.val.vals.len());
                for (c, _) in ie.val.vals.iter() {
                    for x in c.dots.keys() {
                        actors.intern(x);
                    }
                }
            }
        }
    }
    let (a, k, k2, v) = (actors.width(), keys.width(), ikeys.width(), vmax);
    if a > MAP_NESTED_MAX_ACTORS || k2 > MAP_NESTED_MAX_INNER_KEYS || v > MAP_NESTED_MAX_VALUES {
        return Err(unsupported(format!("nested Map lub_many: {} actors / {} inner keys / {} values (limits {} / {} / {})",
                                       a, k2, v, MAP_NESTED_MAX_ACTORS, MAP_NESTED_MAX_INNER_KEYS,
                                       MAP_NESTED_MAX_VALUES)));
    }
    let kw = (k + 63) / 64;
    let k2w = if k2 > 64 { (k2 + 63) / 64 } else { 1 };  // inner key-set mask words
    let n = g * r * k;
    let (mut clock, mut ec, mut ic) = (vec![0u64; g * r * a], vec![0u64; n * a], vec![0u64; n * a]);
    let (mut iec, mut ivc, mut ivv) = (vec![0u64; n * k2 * a], vec![0u64; n * k2 * v * a], vec![0u64; n * k2 * v]);
    let (mut id_off, mut id_clock, mut id_keys) = (vec![0u64], Vec::new(), Vec::new());
    let mut arena: Vec<V> = Vec::new();
    for (i, s) in all.iter().enumerate() {
        clock_row(&s.clock, &actors, &mut clock[i * a..(i + 1) * a]);
        for j in 0..k {
            if let Some(e) = s.entries.get(&keys.ids[j]) {
                let b = i * k + j;
                clock_row(&e.clock, &actors, &mut ec[b * a..(b + 1) * a]);
                clock_row(&e.val.clock, &actors, &mut ic[b * a..(b + 1) * a]);
                for (ik, ie) in e.val.entries.iter() {
                    let q = b * k2 + ikeys.pos[ik];
                    clock_row(&ie.clock, &actors, &mut iec[q * a..(q + 1) * a]);
                    mvreg_rows(&ie.val, &actors, v, &mut arena, &mut ivc[q * v * a..(q + 1) * v * a],
                               &mut ivv[q * v..(q + 1) * v]);
                }
                for (rm, ks) in e.val.deferred.iter() {
                    let mut row = vec![0u64; a];
                    clock_row(rm, &actors, &mut row);
                    id_clock.extend(row);
                    id_keys.extend(key_bits(ks, &ikeys, k2w));
                }
            }
            id_off.push((id_keys.len() / k2w) as u64);
        }
    }
    let pool = group_pool(groups, &actors, &keys);
    let (nd, di) = (pool.def_row.len(), id_keys.len() / k2w);
    // inner deferred slots per key: the largest sum of one key's inner list lengths over its group (no
    // fold result holds more), at least the library's 16 (round 6: past 16 those keys re-fold exactly)
    let mut idc = 16usize;
    for gi in 0..g {
        for j in 0..k {
            let mut t = 0usize;
            for ri in 0..r {
                let b = (gi * r + ri) * k + j;
                t += (id_off[b + 1] - id_off[b]) as usize;
            }
            idc = idc.max(t);
        }
    }
    let batch = ffi::crdt_map_nested_batch {
        G: g, R: r, K: k, K2: k2, V: v, A: a,
        clock: clock.as_ptr(), ec: ec.as_ptr(), ic: ic.as_ptr(), iec: iec.as_ptr(), ivc: ivc.as_ptr(), ivv: ivv.as_ptr(),
        id_off: id_off.as_ptr(), id_clock: id_clock.as_ptr(), id_keys: id_keys.as_ptr(), Di: di,
        def_off: if nd > 0 { pool.def_off.as_ptr() } else { ptr::null() },
        def_row: pool.def_row.as_ptr(), def_clock: pool.def_clock.as_ptr(), def_keys: pool.def_keys.as_ptr(),
    };
    let (mut o_clock, mut o_ec, mut o_ic) = (vec![0u64; g * a], vec![0u64; g * k * a], vec![0u64; g * k * a]);
    // MVReg slots per inner key in the result: every value the group's replicas hold for one register
    // fits (r * v), at least the library's 8, at most its 64 (past that the fold reports flags bit 6)
    let vs = (r * v).clamp(8, MAP_NESTED_MAX_VALUES);
    let (mut o_iec, mut o_ivc, mut o_ivv) = (vec![0u64; g * k * k2 * a], vec![0u64; g * k * k2 * vs * a],
                                             vec![0u64; g * k * k2 * vs]);
    let (mut o_nval, mut o_idn) = (vec![0u32; g * k * k2], vec![0u32; g * k]);
    let (mut o_idc, mut o_idk) = (vec![0u64; g * k * idc * a], vec![0u64; g * k * idc * k2w]);
    let (mut flags, mut keep, mut okeys) = (vec![0u32; g], vec![0u8; nd], vec![0u64; nd * kw]);
    let mut out = ffi::crdt_map_nested_out {
        clock: o_clock.as_mut_ptr(), ec: o_ec.as_mut_ptr(), ic: o_ic.as_mut_ptr(), iec: o_iec.as_mut_ptr(),
        ivc: o_ivc.as_mut_ptr(), ivv: o_ivv.as_mut_ptr(), nval: o_nval.as_mut_ptr(), id_n: o_idn.as_mut_ptr(),
        id_clock: o_idc.as_mut_ptr(), id_keys: o_idk.as_mut_ptr(), flags: flags.as_mut_ptr(),
        def_keep: if nd > 0 { keep.as_mut_ptr() } else { ptr::null_mut() },
        def_keys: if nd > 0 { okeys.as_mut_ptr() } else { ptr::null_mut() },
        Id: idc, Vs: vs,
    };
    ctx.check_host(unsafe { ffi::crdt_map_nested_lub_many(ctx.host, &batch, &mut out) })?;
    if let Some(f) = flags.iter().find(|&&f| f != 0) {
        return Err(unsupported(format!("nested Map lub_many flags {}", f)));
    }
    let mut res = Vec::with_capacity(g);
    for gi in 0..g {
        let mut mp: Map<K, Map<K2, MVReg<V, A>, A>, A> = Map::new();
        mp.clock = row_clock(&o_clock[gi * a..(gi + 1) * a], &actors);
        for (j, key) in keys.ids.iter().enumerate() {
            let b = gi * k + j;
            let row = &o_ec[b * a..(b + 1) * a];
            if row.iter().all(|&x| x == 0) {
                continue;
            }
            let mut inner: Map<K2, MVReg<V, A>, A> = Map::new();
            inner.clock = row_clock(&o_ic[b * a..(b + 1) * a], &actors);
            for (jj, ik) in ikeys.ids.iter().enumerate() {
                let q = b * k2 + jj;
                let ir = &o_iec[q * a..(q + 1) * a];
                if ir.iter().any(|&x| x != 0) {
                    let reg = mvreg_of(&o_ivc[q * vs * a..(q + 1) * vs * a], &o_ivv[q * vs..(q + 1) * vs],
                                       o_nval[q] as usize, &actors, &arena);
                    inner.entries.insert(ik.clone(), Entry { clock: row_clock(ir, &actors), val: reg });
                }
            }
            for i in 0..o_idn[b] as usize {
                let ks = bit_keys(&o_idk[(b * idc + i) * k2w..(b * idc + i + 1) * k2w], &ikeys);
                inner.deferred.entry(row_clock(&o_idc[(b * idc + i) * a..(b * idc + i + 1) * a], &actors))
                    .or_insert_with(BTreeSet::new).extend(ks);
            }
            mp.entries.insert(key.clone(), Entry { clock: row_clock(row, &actors), val: inner });
        }
        mp.deferred = group_survivors(&pool, gi, &keep, &okeys, &actors, &keys);
        res.push(mp);
    }
    Ok(res)
}

impl<K: Ord + Clone, K2: Ord + Clone, V: Clone, A: Actor> BatchCvRDT for Map<K, Map<K2, MVReg<V, A>, A>, A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(Map::new());
        }
        Ok(nested_map_folds(ctx, &[replicas.iter().collect()])?.remove(0))
    }
    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        if selves.is_empty() {
            return Ok(());
        }
        let merged = nested_map_folds(ctx, &pairs_as_groups(selves, &others))?;
        for (s, m) in selves.iter_mut().zip(merged) {
            *s = m;
        }
        Ok(())
    }
}

// ---- MVReg<V, A>: CvRDT::merge (mvreg.rs:112-128) on device buffers ------------------------------
// MVReg::merge compares value clocks only, so values travel as ids into a per-call arena (as for
// Map); the register's Vec order is kept slot for slot.
fn mvreg_rows<V: Clone, A: Actor>(r: &MVReg<V, A>, idx: &Index<A>, v: usize, arena: &mut Vec<V>, vclk: &mut [u64],
                                  vval: &mut [u64]) {
    let a = idx.width().max(1);
    for (slot, (c, val)) in r.vals.iter().enumerate().take(v) {
        clock_row(c, idx, &mut vclk[slot * a..(slot + 1) * a]);
        vval[slot] = arena.len() as u64;
        arena.push(val.clone());
    }
}

fn mvreg_of<V: Clone, A: Actor>(vclk: &[u64], vval: &[u64], slots: usize, idx: &Index<A>, arena: &[V]) -> MVReg<V, A> {
    let a = idx.width().max(1);
    let mut vals = Vec::new();
    for s in 0..slots {
        let row = &vclk[s * a..(s + 1) * a];
        if row.iter().any(|&x| x != 0) {
            vals.push((row_clock(row, idx), arena[vval[s] as usize].clone()));
        }
    }
    MVReg { vals }
}

impl<V: Clone, A: Actor> BatchCvRDT for MVReg<V, A> {
    fn lub_many(ctx: &GpuCtx, replicas: Vec<Self>) -> Result<Self, GpuError> {
        if replicas.is_empty() {
            return Ok(MVReg::new());
        }
        let mut idx = Index::new();
        for r in &replicas {
            for (c, _) in r.vals.iter() {
                for a in c.dots.keys() {
                    idx.intern(a);
                }
            }
        }
        let (n, a) = (replicas.len(), idx.width().max(1));
        let v = replicas.iter().map(|r| r.vals.len()).max().unwrap_or(0).max(1);
        if v > MAP_MAX_VALUES || a > MAP_MAX_ACTORS {
            return Err(unsupported(format!("MVReg lub_many: {} values per register / {} actors (limits {} / {})", v,
                                           a, MAP_MAX_VALUES, MAP_MAX_ACTORS)));
        }
        let mut arena = Vec::new();
        let (mut vclk, mut vval) = (vec![0u64; n * v * a], vec![0u64; n * v]);
        for (i, r) in replicas.iter().enumerate() {
            mvreg_rows(r, &idx, v, &mut arena, &mut vclk[i * v * a..(i + 1) * v * a], &mut vval[i * v..(i + 1) * v]);
        }
        let (dc, dv) = (DeviceBuf::from_host(&vclk)?, DeviceBuf::from_host(&vval)?);
        // the fold state holds 16 values; the output grows from 4 to 16 slots when it must
        let mut vout = 4usize;
        loop {
            let (oc, ov) = (DeviceBuf::<u64>::zeroed(vout * a)?, DeviceBuf::<u64>::zeroed(vout)?);
            let (nv, fl) = (DeviceBuf::<u32>::zeroed(1)?, DeviceBuf::<u32>::zeroed(1)?);
            let batch = ffi::crdt_mvreg_batch {
                G: 1, R: n, A: a, V: v,
                vclk: dc.as_ptr(), vclk_rstride: v * a, vclk_gstride: n * v * a,
                vval: dv.as_ptr(), vval_rstride: v, vval_gstride: n * v,
            };
            let mut out = ffi::crdt_mvreg_out {
                Vout: vout, Vstate: 16, vclk: oc.as_mut_ptr(), vval: ov.as_mut_ptr(), nval: nv.as_mut_ptr(),
                flags: fl.as_mut_ptr(),
            };
            ctx.check(unsafe { ffi::crdt_mvreg_lub_many(ctx.raw, &batch, &mut out) })?;
            let flags = fl.to_host()?[0];
            if flags & 1 != 0 && vout < 16 {
                vout = 16;
                continue;
            }
            if flags != 0 {
                return Err(unsupported(format!("MVReg lub_many: flags {} (more than 16 concurrent values)", flags)));
            }
            return Ok(mvreg_of(&oc.to_host()?, &ov.to_host()?, vout, &idx, &arena));
        }
    }

    fn merge_batch(ctx: &GpuCtx, selves: &mut [Self], others: Vec<Self>) -> Result<(), GpuError> {
        check_pairs(selves.len(), others.len())?;
        let n = selves.len();
        if n == 0 {
            return Ok(());
        }
        let mut idx = Index::new();
        for r in selves.iter().chain(others.iter()) {
            for (c, _) in r.vals.iter() {
                for a in c.dots.keys() {
                    idx.intern(a);
                }
            }
        }
        let a = idx.width().max(1);
        let vo = others.iter().map(|r| r.vals.len()).max().unwrap_or(0).max(1);
        // self's slots hold its kept values plus the other side's added ones: per pair
        let vs = (0..n).map(|i| selves[i].vals.len() + others[i].vals.len()).max().unwrap_or(0).max(1);
        if vs > MAP_MAX_VALUES || vo > MAP_MAX_VALUES || a > MAP_MAX_ACTORS {
            return Err(unsupported(format!("MVReg merge_batch: {} / {} values per register / {} actors (limits {} / {})",
                                           vs, vo, a, MAP_MAX_VALUES, MAP_MAX_ACTORS)));
        }
        let mut arena = Vec::new();
        let (mut sc, mut sv) = (vec![0u64; n * vs * a], vec![0u64; n * vs]);
        let (mut oc, mut ov) = (vec![0u64; n * vo * a], vec![0u64; n * vo]);
        for i in 0..n {
            mvreg_rows(&selves[i], &idx, vs, &mut arena, &mut sc[i * vs * a..(i + 1) * vs * a], &mut sv[i * vs..(i + 1) * vs]);
            mvreg_rows(&others[i], &idx, vo, &mut arena, &mut oc[i * vo * a..(i + 1) * vo * a], &mut ov[i * vo..(i + 1) * vo]);
        }
        let (dsc, dsv) = (DeviceBuf::from_host(&sc)?, DeviceBuf::from_host(&sv)?);
        let (doc, dov) = (DeviceBuf::from_host(&oc)?, DeviceBuf::from_host(&ov)?);
        let st = DeviceBuf::<u32>::zeroed(n)?;
        let ss = ffi::crdt_mvreg_states {
            N: n, A: a, V: vs, vclk: dsc.as_mut_ptr(), vclk_stride: vs * a, vval: dsv.as_mut_ptr(), vval_stride: vs,
        };
        let os = ffi::crdt_mvreg_states {
            N: n, A: a, V: vo, vclk: doc.as_mut_ptr(), vclk_stride: vo * a, vval: dov.as_mut_ptr(), vval_stride: vo,
        };
        ctx.check(unsafe { ffi::crdt_mvreg_merge_batch(ctx.raw, &ss, &os, st.as_mut_ptr()) })?;
        let stv = st.to_host()?;
        // every status first: on an error no register of `selves` has been replaced
        if let Some(i) = (0..n).find(|&i| stv[i] != 0) {
            return Err(unsupported(format!("MVReg merge_batch: pair {} status {}", i, stv[i])));
        }
        let (rc, rv) = (dsc.to_host()?, dsv.to_host()?);
        for i in 0..n {
            selves[i] = mvreg_of(&rc[i * vs * a..(i + 1) * vs * a], &rv[i * vs..(i + 1) * vs], vs, &idx, &arena);
        }
        Ok(())
    }
}
