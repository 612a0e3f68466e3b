// Links libneptune_hip.so, built by `make -C neptune-core_amd` (hipcc, gfx950).  Set
// NEPTUNE_HIP_LIB_DIR to the directory holding it (neptune-core_amd/neptune_hip in this tree); the
// HIP runtime it needs (libamdhip64) comes from the ROCm install (ROCM_PATH, default /opt/rocm).
fn main() {
    let dir = std::env::var("NEPTUNE_HIP_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").expect("cargo sets CARGO_MANIFEST_DIR");
        format!("{here}/../../neptune_hip")
    });
    let rocm = std::env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-search=native={rocm}/lib");
    println!("cargo:rustc-link-lib=dylib=neptune_hip");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=NEPTUNE_HIP_LIB_DIR");
    println!("cargo:rerun-if-env-changed=ROCM_PATH");
    println!("cargo:rerun-if-changed={dir}/libneptune_hip.so");
}
