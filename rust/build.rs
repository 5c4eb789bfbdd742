// Links librtm.so, built in-tree by __graft_entry__.build() (2018rustraytracer_amd/).
fn main() {
    let dir = std::env::var("RTM_LIB_DIR").unwrap_or_else(|_| {
        let manifest = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{}/../2018rustraytracer_amd", manifest)
    });
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=rtm");
    println!("cargo:rerun-if-changed=../include/rtm.h");
}
