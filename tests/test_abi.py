"""CPU tests of the C ABI library: builds for gfx950, loads, exports every symbol include/pba.h declares."""
import ctypes
import os

import pytest

from helpers import engine_module

E = engine_module()


def test_library_builds_for_gfx950():
    E.build()
    assert os.path.exists(E.LIB_PATH)
    blob = open(E.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # embedded gfx950 code object


def test_every_header_function_is_exported():
    names = E.header_functions()
    assert len(names) >= 20
    L = ctypes.CDLL(E.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_test_build_exports_the_same_abi():
    """libpba_test.so (PBA_TEST_HOOKS: the hooks some GPU tests set) is the same ABI; the product library carries no
    hook names at all."""
    assert os.path.exists(E.TEST_LIB_PATH), "run __graft_entry__.build() (make test-lib)"
    L = ctypes.CDLL(E.TEST_LIB_PATH)
    missing = [n for n in E.header_functions() if not hasattr(L, n)]
    assert not missing, missing
    hooks = (b"PBA_TEST_PERTURB_DECISION", b"PBA_LM_HOST_DELAY_US", b"PBA_TEST_FORCE_DEGEN", b"PBA_LIN_LEGACY",
             b"PBA_TEST_ROW_WAVES64", b"PBA_TEST_PBLK_WALK")
    test_blob, prod_blob = open(E.TEST_LIB_PATH, "rb").read(), open(E.LIB_PATH, "rb").read()
    assert all(h in test_blob for h in hooks)
    assert not any(h in prod_blob for h in hooks)


def test_status_strings_and_version():
    L = E.lib()
    assert L.pba_version() >= 100
    for s in (0, -1, -2, -3, -4):
        assert L.pba_status_string(s)


def test_create_rejects_bad_options():
    L = E.lib()
    h = ctypes.c_void_p()
    opt = E.Options(0, 7, 0, 0.0)
    assert L.pba_create(ctypes.byref(opt), ctypes.byref(h)) == -1
    opt = E.Options(0, 0, 9, 0.0)
    assert L.pba_create(ctypes.byref(opt), ctypes.byref(h)) == -1
    assert L.pba_create(None, ctypes.byref(h)) == -1


def test_no_cpu_fallback_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    with pytest.raises(E.PbaError, match="device"):
        E.Engine(0, 0)
