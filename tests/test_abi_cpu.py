"""CPU tests of the C-ABI boundary: the library loads and exports every symbol
that include/huygens_hip.h declares; without a GPU it fails loudly (no CPU
fallback).  No compute call is made here."""
import ctypes as C
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    so = os.path.join(ROOT, "huygens_amd", "lib", "libhuygens_hip.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-j8", "-C", ROOT, "lib"], check=True)
    from huygens_amd import load
    return load()


def test_header_symbols_exported(lib):
    from huygens_amd import header_symbols
    syms = header_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    # and every one of them is bound in the Python mirror with a signature
    from huygens_amd._lib import _SIGS
    assert not [s for s in syms if s not in _SIGS]


def test_library_is_gfx950_code_object(lib):
    data = open(lib._name, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_no_gpu_fails_loudly(lib):
    if lib.hz_device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    h = C.c_void_p()
    rc = lib.hz_fb_create(2, 16, 0.1, 1.0, 0, C.byref(h))
    assert rc == -4  # HZ_E_NODEV
    assert b"no CPU fallback" in lib.hz_last_error()
    assert not h.value


def test_invalid_arguments_rejected_without_device(lib):
    h = C.c_void_p()
    assert lib.hz_fb_create(9, 16, 0.1, 1.0, 0, C.byref(h)) == -1
    assert lib.hz_fb_create(2, 0, 0.1, 1.0, 0, C.byref(h)) == -1
    assert lib.hz_fb_destroy(None) == 0
    assert lib.hz_fb_boost(None, 0, 1.0) == -1
