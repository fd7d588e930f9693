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


@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_shard_plan_balances_ragged_bytes(lib, parts):
    """The multi-device split: contiguous shards covering every item once, each
    non-empty; every cut is the item boundary whose byte prefix is closest to its share of the
    total (so no shard exceeds the ideal share by more than the largest block)."""
    import mysticeti_amd as M

    rng = np.random.default_rng(parts)
    for n in (parts, parts + 1, 37, 1000):
        w = rng.integers(41, 20000, size=n).astype(np.uint64)
        w[rng.integers(0, n, size=max(1, n // 50))] = 2_000_000  # a few huge blocks
        cut = M.shard_plan(w, parts)
        assert cut[0] == 0 and cut[-1] == n and all(a < b for a, b in zip(cut, cut[1:]))
        share = float(w.sum()) / parts
        pre = np.concatenate([[0], np.cumsum(w.astype(np.float64))])
        for d in range(1, parts):
            c, target = cut[d], share * d
            lo, hi = cut[d - 1] + 1, n - (parts - d)  # non-empty shards on both sides
            best = min(range(lo, hi + 1), key=lambda k: abs(pre[k] - target))
            assert abs(pre[c] - target) <= abs(pre[best] - target) + 1e-6, (n, d, cut)
        sums = [int(w[a:b].sum()) for a, b in zip(cut, cut[1:])]
        assert max(sums) <= share + int(w.max()) + 1
    assert M.shard_plan([], 4) == [0, 0, 0, 0, 0]
    assert M.shard_plan([5, 5], 4)[-1] == 2
