"""CPU: the Rust -sys crate (rust/mysti-verify-sys, the north star's "thin C-ABI FFI crate built
with hipcc from build.rs") matches include/mysti_verify.h and the product build.

cargo is not in this image, so the crate cannot be compiled here; this test holds its text to
the header instead: every prototype has an `extern "C"` item with the same parameter types and
return type, every #define has a constant of the same value, and build.rs compiles exactly the
sources mysticeti_amd/build.py compiles. A library linked from build.rs's source list must leave
no device-side launcher (namespace mvk) undefined. The crate replaces the verify of
/root/reference/mysticeti-core/src/crypto.rs:174-189 at net_sync.rs:352.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mysti_verify.h")
CRATE = os.path.join(ROOT, "rust", "mysti-verify-sys")
LIB_RS = os.path.join(CRATE, "src", "lib.rs")
BUILD_RS = os.path.join(CRATE, "build.rs")

# C parameter / return types of the header -> the Rust spelling the crate must use
C2RUST = {
    "mv_ctx*": "*mut mv_ctx",
    "const mv_ctx*": "*const mv_ctx",
    "mv_ctx**": "*mut *mut mv_ctx",
    "const mv_config*": "*const mv_config",
    "const uint8_t*": "*const u8",
    "uint8_t*": "*mut u8",
    "const uint32_t*": "*const u32",
    "uint32_t*": "*mut u32",
    "const uint64_t*": "*const u64",
    "uint64_t*": "*mut u64",
    "double*": "*mut f64",
    "void*": "*mut c_void",
    "void**": "*mut *mut c_void",
    "const char*": "*const c_char",
    "uint32_t": "u32",
    "uint64_t": "u64",
    "int64_t": "i64",
    "int64_t*": "*mut i64",
    "int": "i32",
    "mv_status": "i32",
}


def _norm(t: str) -> str:
    t = re.sub(r"\s+", " ", t.strip())
    t = re.sub(r"\s*\*", "*", t)
    return t


def header_prototypes():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    src = re.sub(r"^\s*#.*$", "", src, flags=re.M)
    src = src.replace('extern "C" {', "")
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(mv_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, params = _norm(m.group(1)), m.group(2), m.group(3)
        ps = []
        if params.strip() not in ("", "void"):
            for p in params.split(","):
                p = _norm(p)
                tm = re.match(r"(.*?)([A-Za-z_]\w*)$", p)
                ps.append(_norm(tm.group(1)))
        protos[name] = (ret, ps)
    return protos


def header_defines():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"#define\s+(MV_[A-Z0-9_]+)\s+\(?(-?\d+)u?\)?", src):
        out[m.group(1)] = int(m.group(2))
    return out


def rust_externs():
    src = open(LIB_RS).read()
    body = src[src.index('extern "C"'):]
    out = {}
    for m in re.finditer(r"pub fn (mv_[a-z0-9_]+)\s*\((.*?)\)\s*(->\s*([^;]+))?;", body, flags=re.S):
        name, params, ret = m.group(1), m.group(2), (m.group(4) or "").strip()
        ps = [re.sub(r"\s+", " ", p.split(":", 1)[1].strip()) for p in params.split(",") if p.strip()]
        out[name] = (ret, ps)
    return out


def rust_consts():
    src = open(LIB_RS).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"pub const (MV_[A-Z0-9_]+):\s*\w+\s*=\s*(-?\d+);", src)}


def test_every_prototype_has_a_matching_extern():
    protos, ext = header_prototypes(), rust_externs()
    assert len(protos) >= 29
    missing = sorted(set(protos) - set(ext))
    assert not missing, f"lib.rs lacks {missing}"
    extra = sorted(set(ext) - set(protos))
    assert not extra, f"lib.rs declares functions the header does not: {extra}"
    for name, (ret, ps) in protos.items():
        rret, rps = ext[name]
        want_ret = "" if ret == "void" else C2RUST[ret]
        assert rret == want_ret, (name, ret, rret)
        assert [C2RUST[p] for p in ps] == rps, (name, ps, rps)


def test_every_define_has_a_matching_const():
    defs, consts = header_defines(), rust_consts()
    assert "MV_NSTAGES" in defs and "MV_WAL_BAD_LENGTH" in defs and "MV_E_ALLOC" in defs
    for k, v in defs.items():
        assert k in consts, f"lib.rs lacks {k}"
        assert consts[k] == v, (k, v, consts[k])


def _sources_of(path, pattern):
    src = open(path).read()
    m = re.search(pattern, src, flags=re.S)
    return re.findall(r'"([\w.]+\.(?:hip|cpp))"', m.group(1))


def test_build_rs_compiles_the_product_sources():
    from mysticeti_amd import build as BP

    rs = _sources_of(BUILD_RS, r"const SOURCES: &\[&str\] = &\[(.*?)\];")
    assert rs == BP.SOURCES
    # per-source flags: build.rs's SOURCE_FLAGS table equals build.py's
    src = open(BUILD_RS).read()
    tab = re.search(r"const SOURCE_FLAGS: [^=]*= &\[(.*?)\];\n", src, re.S).group(1)
    got = {m.group(1): re.findall(r'"([^"]+)"', m.group(2)) for m in re.finditer(r'\("([^"]+)",\s*&\[(.*?)\]\)', tab)}
    assert got == BP.SOURCE_FLAGS


def test_library_from_build_rs_list_has_no_undefined_launchers():
    """Links the objects build.rs names (compiled with the product flags by build.py) into a
    library of its own and checks that no mvk:: launcher or mv_ entry point is undefined."""
    from mysticeti_amd import build as BP

    BP.build(verbose=False)
    rs = _sources_of(BUILD_RS, r"const SOURCES: &\[&str\] = &\[(.*?)\];")
    objs = [os.path.join(BP.OBJ, s + ".o") for s in rs]
    out_dir = os.path.join(BP.OBJ, "rust_list")
    os.makedirs(out_dir, exist_ok=True)
    lib = os.path.join(out_dir, "libmysti_verify.so")
    subprocess.run([BP.HIPCC, f"--offload-arch={BP.ARCH}", "-shared", "-fPIC", "-o", lib] + objs + ["-lpthread"],
                   check=True)
    und = subprocess.run(["nm", "-D", "-C", "--undefined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    bad = [l for l in und.splitlines() if "mvk::" in l or re.search(r"\bmv_", l)]
    assert not bad, bad
    defined = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                             check=True).stdout
    exported = set(re.findall(r"\bT (mv_[a-z0-9_]+)", defined))
    assert set(header_prototypes()) <= exported
