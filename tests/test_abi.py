"""CPU-side checks of the C-ABI library (no compute calls without a GPU)."""
import ctypes
import os

import pytest


def test_library_exports_every_header_symbol():
    import slatecodec as sc
    sc.build()
    L = ctypes.CDLL(sc.LIB_PATH)
    syms = sc.header_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sc.lib().slate_abi_version() == 1


def test_status_strings_match_oracle(oracle):
    import slatecodec as sc
    for code in list(range(0, 70)):
        o = oracle.status_string(code)
        if o != "unknown status":
            assert sc.status_string(code) == o, code


def test_no_device_fails_loudly():
    """Without a GPU the product refuses to run (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import slatecodec as sc
    with pytest.raises(sc.SlateError) as e:
        sc.Context(0)
    assert e.value.status == sc.E_NO_DEVICE


def test_kernel_code_object_is_gfx950():
    import slatecodec as sc
    blob = open(sc.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
