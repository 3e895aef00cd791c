//! Link libbackuwup_amd.so (HIP, gfx950), built in-tree by `python backuwup_amd/build.py`.
//! BACKUWUP_AMD_LIB_DIR overrides where it is looked for (default: ../../backuwup_amd, i.e. the
//! library next to the Python package of this repository).
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = match env::var("BACKUWUP_AMD_LIB_DIR") {
        Ok(d) => PathBuf::from(d),
        Err(_) => PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../backuwup_amd"),
    };
    println!("cargo:rerun-if-env-changed=BACKUWUP_AMD_LIB_DIR");
    println!("cargo:rerun-if-changed={}", dir.join("libbackuwup_amd.so").display());
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=backuwup_amd");
    // the library's own RUNPATH finds the ROCm runtime and RCCL; this finds the library itself
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
}
