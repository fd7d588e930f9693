import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # tests use the oracle as the checker


def pytest_sessionstart(session):
    # torch ships its own HIP runtime, and it must see the device before libmysti_verify.so's
    # runtime is loaded (a CPU test that loads the library first would leave torch -- and then
    # mv_create -- without devices): on a GPU box, initialise torch before any test runs
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: large-batch case")


@pytest.fixture(scope="session")
def engine():
    # torch ships its own HIP runtime: it must initialise the device before the
    # library's runtime does, or torch.cuda reports no devices (device-API tests
    # hand torch-allocated HBM to the library, as bench.py does)
    import torch

    torch.cuda.init()
    import mysticeti_amd as M

    eng = M.Engine(devices=(0,))
    yield eng
    eng.close()


@pytest.fixture(autouse=True)
def _fresh_batch_policy(request):
    """Every test starts the session engine's adaptive batch policy afresh (no guard or
    dense-failure route armed by an earlier test's bad signatures)."""
    if "engine" in request.fixturenames:
        request.getfixturevalue("engine").set_batch_groups(0)
    yield


@pytest.fixture
def opts(engine):
    """opts(name, value[, eng]): sets a runtime switch (mv_set_option; the library reads the
    environment only at mv_create) on the session engine or `eng` for one test, restored after."""
    saved = []

    def set_opt(name, value, eng=None):
        eng = eng or engine
        saved.append((eng, name, eng.get_option(name)))
        eng.set_option(name, int(value))

    yield set_opt
    for eng, name, old in reversed(saved):
        if eng.ctx:  # (an engine the test made and closed itself needs no restoring)
            eng.set_option(name, old)


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(ROOT, "tests", "golden")

    def load(name):
        with open(os.path.join(d, name)) as f:
            return json.load(f)

    return load
