"""Test configuration.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, the C
ABI library's exports, the C++ host driver and the multi-rank orchestration
over gloo. `-m gpu` runs on an MI355X and checks the HIP path against the
oracle through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


_GPU = None


def _gpu_available():
    # Asked once, before any test has loaded libphj_hip.so: torch carries its
    # own HIP/HSA runtime, which does not see the card if the system runtime
    # (the library's) opened it first.
    global _GPU
    if _GPU is None:
        try:
            import torch
            _GPU = torch.cuda.is_available()
        except Exception:
            _GPU = False
    return _GPU


def pytest_collection_modifyitems(config, items):
    if any(it.get_closest_marker("gpu") for it in items):
        _gpu_available()


@pytest.fixture(scope="session")
def ctx():
    """One HIP context for the whole GPU session (one process on the card)."""
    if not _gpu_available():
        pytest.fail("GPU test selected but no GPU is visible")
    import partitionedhashjoin_amd as phj
    c = phj.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def chunk_ctx(ctx):
    """A context that takes the chunked (histogram-free) pass 1 at every size
    (by default it starts at ~134M tuples; PHJ_P1_MIN_TILES, read at creation)."""
    import partitionedhashjoin_amd as phj
    old = os.environ.get("PHJ_P1_MIN_TILES")
    os.environ["PHJ_P1_MIN_TILES"] = "0"
    try:
        c = phj.Context(0)
    finally:
        if old is None:
            del os.environ["PHJ_P1_MIN_TILES"]
        else:
            os.environ["PHJ_P1_MIN_TILES"] = old
    yield c
    c.close()
