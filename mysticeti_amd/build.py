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
SOURCES = ["kernels.hip", "engine.cpp", "block_codec.cpp"]
HEADERS = ["asm_ops.h", "fe25519.h", "ge25519.h", "hash_dev.h", "scalar25519.h", "kernels.h", "block_codec.h"]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, force: bool) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src + ".o")
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(HERE, "..", "include", "mysti_verify.h")]
    if force or _newer(o, deps):
        lang = [] if src.endswith(".hip") else ["-x", "hip"]
        cmd = [HIPCC] + COMMON + lang + ["-c", s, "-o", o]
        subprocess.run(cmd, check=True)
    return o


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _newer(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread"]
        subprocess.run(cmd, check=True)
        if verbose:
            print("built", LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(force=a.force)
    sys.exit(0)
