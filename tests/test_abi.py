"""CPU: the C-ABI library loads, exports every symbol include/mysti_verify.h declares,
and its host-only codec matches the oracle. No compute calls need a GPU here."""
import os
import re
import subprocess

import numpy as np
import pytest

import blocks as B
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mysti_verify.h")
LIB = os.path.join(ROOT, "mysticeti_amd", "libmysti_verify.so")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mv_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        from mysticeti_amd.build import build

        build()
    import mysticeti_amd as M

    return M.load_library()


def test_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mv_[a-z0-9_]+)", out))
    decl = declared_symbols()
    assert len(decl) >= 13
    missing = [s for s in decl if s not in exported]
    assert not missing, missing
    import mysticeti_amd as M

    assert set(M.EXPORTS) == set(decl)


def test_version(lib):
    import mysticeti_amd as M

    assert "gfx950" in M.version()


def test_create_without_gpu_fails_loudly(lib):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import mysticeti_amd as M

    with pytest.raises(M.MvError):
        M.Engine()


def test_host_preimage_matches_oracle(golden):
    import mysticeti_amd as M

    e = golden("block_edge.json")
    for c in e["cases"]:
        b = bytes.fromhex(c["bincode"])
        assert M.block_preimage(b) == O.block_preimage(b), c["note"]
    blks = B.gen_config4(O.sign, rounds=1, n_auth=10, n_inc=7, n_vr=5)
    for b in blks:
        assert M.block_preimage(b.bincode()) == b.preimage()


def test_host_preimage_rejects_garbage():
    import mysticeti_amd as M

    assert M.block_preimage(b"") is None
    assert M.block_preimage(bytes(10)) is None
    rng = np.random.default_rng(3)
    for _ in range(200):
        b = rng.integers(0, 256, size=int(rng.integers(0, 400)), dtype=np.uint8).tobytes()
        assert M.block_preimage(b) == O.block_preimage(b)
