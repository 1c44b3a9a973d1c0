// Builds the MI355X library (../waffle_con_amd/csrc, hipcc --offload-arch=gfx950)
// into OUT_DIR and links it. ROCm's hipcc must be on PATH or at /opt/rocm/bin;
// HIPCC overrides. The device code targets gfx950 only.
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    let out = PathBuf::from(env::var("OUT_DIR").expect("OUT_DIR"));
    let root = PathBuf::from(env::var("CARGO_MANIFEST_DIR").expect("CARGO_MANIFEST_DIR"))
        .parent()
        .expect("the crate lives in <repo>/rust")
        .to_path_buf();
    let csrc = root.join("waffle_con_amd").join("csrc");
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".to_string());
    let jobs = env::var("NUM_JOBS").unwrap_or_else(|_| "8".to_string());
    let status = Command::new("make")
        .arg("-C")
        .arg(&csrc)
        .arg(format!("-j{}", jobs))
        .arg(format!("HIPCC={}", hipcc))
        .arg("ARCH=gfx950")
        .arg(format!("OUT={}", out.join("libwaffle_con.so").display()))
        .arg(format!("OBJ_DIR={}", out.join("obj").display()))
        .status()
        .expect("running make (hipcc from ROCm is required to build the MI355X backend)");
    assert!(status.success(), "building libwaffle_con.so for gfx950 failed");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=waffle_con");
    // the library is found next to the binary's rpath entry at run time
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
    println!("cargo:rerun-if-changed={}", csrc.display());
    println!("cargo:rerun-if-changed={}", root.join("include").join("waffle_con.h").display());
    println!("cargo:rerun-if-env-changed=HIPCC");
}
