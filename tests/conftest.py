"""Shared pytest setup: the `gpu` marker, repo paths, and golden-vector loading."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "slatedb-go_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def ref_vectors():
    with open(os.path.join(REPO, "tests", "golden", "reference_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import binding
    binding.build()
    return binding


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """torch ships its own HIP runtime next to the system one libslatecodec links.  When the
    library's runtime opens the device first, torch's later init reports "No HIP GPUs are
    available"; torch first, then the library, works (bench.py's order).  GPU sessions that use
    torch device memory therefore initialise torch before any slate_ctx exists."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass
    yield


@pytest.fixture(scope="module", autouse=True)
def _free_contexts_between_modules():
    """Each GPU module makes its own contexts, and each context holds page-locked staging (the
    host-decode lanes' pieces, reader slots): collect the module's objects when it ends, so that
    one module's page-locked memory is released before the next one allocates its own (a context
    kept alive by a reference cycle until some later collection would otherwise hold it)."""
    yield
    import gc
    gc.collect()
