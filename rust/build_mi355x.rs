// Addition to hdfs-native's rust/build.rs (fn main), behind the `mi355x`
// feature: link the MI355X EC engine (hdfs-native_amd/lib/libhdfs_ec_amd.so,
// built by `make -C hdfs-native_amd`).  Not compiled in this repository
// (no cargo in the image).
//
//     #[cfg(feature = "mi355x")]
//     link_mi355x();

#[cfg(feature = "mi355x")]
fn link_mi355x() {
    let dir = std::env::var("HDFS_EC_AMD_LIB").unwrap_or_else(|_| "../hdfs-native_amd/lib".to_string());
    println!("cargo:rerun-if-env-changed=HDFS_EC_AMD_LIB");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=hdfs_ec_amd");
    // the engine links libamdhip64.so.7; let the loader find it at run time
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rustc-link-arg=-Wl,-rpath,/opt/rocm/lib");
}
