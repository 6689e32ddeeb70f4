// build.rs of the `crdts` crate's `gpu` feature: the hipcc step.  Builds libcrdt_gpu.so for gfx950
// (`make -C <CRDT_GPU_DIR>`: hipcc --offload-arch=gfx950 of the HIP kernels and the C ABI, see
// rust-crdt_amd/Makefile) and links it, with the ROCm runtime, into the crate.  RCCL is bound by
// the library at run time (CRDT_RCCL_LIB, else the process's librccl.so.1, else /opt/rocm/lib).
//
//   CRDT_GPU_DIR   directory holding the Makefile and csrc/ (default: ../rust-crdt_amd)
//   ROCM_PATH      ROCm install (default: /opt/rocm)
//   CRDT_GPU_ARCH  offload arch (default: gfx950, MI355X)
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    if env::var_os("CARGO_FEATURE_GPU").is_none() {
        return; // the CPU-only crate builds exactly as before
    }
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let dir = env::var("CRDT_GPU_DIR")
        .map(PathBuf::from)
        .unwrap_or_else(|_| manifest.join("..").join("rust-crdt_amd"));
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    let arch = env::var("CRDT_GPU_ARCH").unwrap_or_else(|_| "gfx950".to_string());
    let jobs = env::var("NUM_JOBS").unwrap_or_else(|_| "8".to_string());
    let status = Command::new("make")
        .arg("-C")
        .arg(&dir)
        .arg(format!("-j{}", jobs))
        .arg(format!("ARCH={}", arch))
        .arg(format!("HIPCC={}/bin/hipcc", rocm))
        .arg("libcrdt_gpu.so")
        .status()
        .expect("failed to run make for libcrdt_gpu (hipcc)");
    assert!(status.success(), "building libcrdt_gpu.so with hipcc failed");
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=crdt_gpu");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}/lib", rocm);
    for f in ["csrc", "Makefile"] {
        println!("cargo:rerun-if-changed={}", dir.join(f).display());
    }
    println!("cargo:rerun-if-changed=../include/crdt_gpu.h");
}
