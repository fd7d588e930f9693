// Builds libmysti_verify.so from the HIP/C++ sources with hipcc (gfx950 only) and links it.
// MYSTI_VERIFY_SRC: the mysticeti_amd/csrc directory (default: ../../mysticeti_amd/csrc).
// MYSTI_VERIFY_LIB_DIR: link a prebuilt library from this directory instead of compiling.
// Not built in the repository's image (no cargo); the compile line matches
// mysticeti_amd/build.py.
use std::env;
use std::path::PathBuf;
use std::process::Command;

const SOURCES: &[&str] = &[
    "kernels.hip", "batch.hip", "comb.hip", "ingest.hip", "blake2b_quad.hip", "blake2b_lane.hip", "block_walk.hip", "wal.hip", "engine.cpp",
    "block_codec.cpp",
];
// per-source flags (mysticeti_amd/build.py SOURCE_FLAGS)
const SOURCE_FLAGS: &[(&str, &[&str])] = &[
    ("batch.hip", &["-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
    ("blake2b_lane.hip", &["-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
    ("ingest.hip", &["-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
];

fn main() {
    println!("cargo:rerun-if-env-changed=MYSTI_VERIFY_LIB_DIR");
    println!("cargo:rerun-if-env-changed=MYSTI_VERIFY_SRC");
    println!("cargo:rerun-if-env-changed=HIPCC");
    if let Ok(dir) = env::var("MYSTI_VERIFY_LIB_DIR") {
        println!("cargo:rustc-link-search=native={dir}");
        println!("cargo:rustc-link-lib=dylib=mysti_verify");
        println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
        return;
    }
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let src = env::var("MYSTI_VERIFY_SRC")
        .map(PathBuf::from)
        .unwrap_or_else(|_| manifest.join("../../mysticeti_amd/csrc"));
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let mut objs = Vec::new();
    for s in SOURCES {
        let path = src.join(s);
        println!("cargo:rerun-if-changed={}", path.display());
        let obj = out.join(format!("{s}.o"));
        let mut cmd = Command::new(&hipcc);
        cmd.args(["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-function"]);
        for (name, flags) in SOURCE_FLAGS {
            if name == s {
                cmd.args(*flags);
            }
        }
        if !s.ends_with(".hip") {
            cmd.args(["-x", "hip"]);
        }
        cmd.arg("-c").arg(&path).arg("-o").arg(&obj);
        let st = cmd.status().expect("hipcc not found (set HIPCC)");
        assert!(st.success(), "hipcc failed on {s}");
        objs.push(obj);
    }
    let lib = out.join("libmysti_verify.so");
    let st = Command::new(&hipcc)
        .args(["--offload-arch=gfx950", "-shared", "-fPIC", "-o"])
        .arg(&lib)
        .args(&objs)
        .arg("-lpthread")
        .status()
        .expect("hipcc link");
    assert!(st.success(), "linking libmysti_verify.so failed");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=mysti_verify");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
}
