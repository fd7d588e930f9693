"""Builds libmysti_verify.so in-tree (hipcc, gfx950 only).

    python -m mysticeti_amd.build [--force]

Object files go to mysticeti_amd/_build/, the shared library to
mysticeti_amd/libmysti_verify.so (git-ignored; it travels with the gpurun snapshot).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libmysti_verify.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]
SOURCES = ["kernels.hip", "batch.hip", "comb.hip", "ingest.hip", "blake2b_quad.hip", "blake2b_lane.hip", "block_walk.hip", "wal.hip", "engine.cpp",
           "block_codec.cpp"]
# per-source compiler flags of the product build (rust/mysti-verify-sys/build.rs mirrors them):
# batch.hip under LLVM's max-ilp machine scheduler, config 2 +1.4% (294.4/294.7 -> 299.2/298.4 M
# sigs/s, interleaved A/B, profiles/r04/ab_ilp.txt)
SOURCE_FLAGS = {"batch.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
                "blake2b_lane.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
                "ingest.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}
HEADERS = ["asm_ops.h", "fe25519.h", "ge25519.h", "hash_dev.h", "scalar25519.h", "kernels.h", "block_codec.h", "tables.h", "carry32.h", "comb.h", "quad25519.h", "fe_q4.h", "fe_r16.h", "blake2b_quad.h", "block_verdict.h", "ingest_dev.h", "pt_r16.h"]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, force: bool, obj_dir: str = OBJ, defines=(), flags=()) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(obj_dir, src + ".o")
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(HERE, "..", "include", "mysti_verify.h")]
    if force or _newer(o, deps):
        lang = [] if src.endswith(".hip") else ["-x", "hip"]
        cmd = [HIPCC] + COMMON + SOURCE_FLAGS.get(src, []) + [f"-D{d}" for d in defines] + list(flags) + lang + \
            ["-c", s, "-o", o]
        subprocess.run(cmd, check=True)
    return o


def build(force: bool = False, verbose: bool = True, variant: str = "", defines=(), flags=(), only=()) -> str:
    """Builds the product library, or with `variant` an experiment build
    (mysticeti_amd/_build/<variant>/libmysti_verify.so, compiled with -D`defines` and the extra
    compiler `flags` -- on the sources in `only`, or all; load it with MV_LIB=<path>)."""
    obj_dir = os.path.join(OBJ, variant) if variant else OBJ
    lib = os.path.join(obj_dir, "libmysti_verify.so") if variant else LIB
    os.makedirs(obj_dir, exist_ok=True)
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, obj_dir, defines, flags if (not only or s in only) else ()),
                           SOURCES))
    if force or _newer(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs + ["-lpthread"]
        subprocess.run(cmd, check=True)
        if verbose:
            print("built", lib)
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--flag", dest="flags", action="append", default=[], help="extra compiler flag (variant builds)")
    ap.add_argument("--only", action="append", default=[], help="apply --flag to these sources only")
    a = ap.parse_args()
    build(force=a.force, variant=a.variant, defines=a.defines, flags=a.flags, only=a.only)
    sys.exit(0)
