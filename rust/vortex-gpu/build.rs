//! Links the engine: $VORTEX_GPU_LIB_DIR (default: the directory holding libvortex_gpu.so in the
//! vortex_amd checkout, ../vortex_amd relative to this crate's original location).
use std::env;
use std::path::PathBuf;

fn main() {
    println!("cargo:rerun-if-env-changed=VORTEX_GPU_LIB_DIR");
    let dir = env::var("VORTEX_GPU_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap_or_default()).join("../../vortex_amd")
    });
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=vortex_gpu");
    // the engine's HIP runtime dependency resolves through its own RUNPATH; add ROCm's lib dir
    // for environments that need it at link time
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
}
