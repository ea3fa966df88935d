//! Link librlnc_hip.so when the `hip` feature is on; nothing otherwise (the CPU build stays dependency-free).
//! RLNC_HIP_LIB_DIR = the directory holding librlnc_hip.so (in the librlnc_hip repository: `rlnc_amd/`).
fn main() {
    println!("cargo:rerun-if-env-changed=RLNC_HIP_LIB_DIR");
    if std::env::var_os("CARGO_FEATURE_HIP").is_none() {
        return;
    }
    let dir = std::env::var("RLNC_HIP_LIB_DIR").expect("RLNC_HIP_LIB_DIR must name the directory of librlnc_hip.so");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=rlnc_hip");
    // tests, benches and examples find the library at run time without LD_LIBRARY_PATH
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
}
