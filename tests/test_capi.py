"""The C-ABI library loads here (no GPU) and exports every symbol include/come.h declares;
argument validation fails with an error code + message before any device work."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from come_amd import _lib


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "come.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\s*\*?\s*(come_[a-z0-9_]+)\(",
                                 src, re.M)))


def test_header_declares_expected_entry_points():
    names = declared_symbols()
    assert set(names) == set(_lib.SYMBOLS), names


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert L.come_abi_version() == _lib.ABI_VERSION == 5


def test_library_is_the_build_of_the_sources_beside_it(monkeypatch):
    """libcome.so carries the SHA-256 of the sources it was built from; the binding compares it
    with the sources in the tree and refuses a stale library (the prebuilt .so that travels to the
    GPU box is therefore the committed sources' build)."""
    L = _lib.lib()
    assert L.come_source_sha256().decode() == _lib.source_sha256()
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "source_sha256", lambda: "0" * 64)
    with pytest.raises(_lib.ComeError, match="built from other sources"):
        _lib.lib()


def test_invalid_arguments_return_error_without_gpu():
    L = _lib.lib()
    p = ctypes.c_void_p(0)
    rc = L.come_sgns_o2(p, p, 0, 128, p, 1, 10, p, 5, 5, p, 10, 0.1, 1.0, 0, p)
    assert rc == -1 and b"V must be" in L.come_last_error()
    rc = L.come_sgns_o2(p, p, 10, 1000, p, 1, 10, p, 5, 5, p, 10, 0.1, 1.0, 0, p)
    assert rc == -1 and b"d must be" in L.come_last_error()
    rc = L.come_sgns_o1(p, 10, 8, p, 1, p, 50, p, 10, 0.1, 0, p)
    assert rc == -1 and b"negative" in L.come_last_error()
    rc = L.come_sgns_o2(p, p, 10, 8, p, 1, 10, p, 5, 0, p, 10, 0.1, 1.0, 7, p)
    assert rc == -1 and b"mode" in L.come_last_error()
    # empty batches are a no-op (no device access)
    assert L.come_sgns_o2(p, p, 10, 8, p, 0, 10, p, 5, 0, p, 10, 0.1, 1.0, 0, p) == 0
    assert L.come_sgns_o1(p, 10, 8, p, 0, p, 0, p, 10, 0.1, 0, p) == 0


def test_check_raises_with_message():
    L = _lib.lib()
    p = ctypes.c_void_p(0)
    with pytest.raises(_lib.ComeError, match="V must be"):
        _lib.check(L.come_sgns_o2(p, p, -1, 8, p, 1, 1, p, 1, 1, p, 1, 0.1, 1.0, 0, p), "o2")


def test_missing_library_fails_loudly(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libcome.so")
    with pytest.raises(_lib.ComeError, match="not found"):
        _lib.lib()


def test_launch_options_snapshot_and_per_call_struct():
    """come_set_option changes the process-wide snapshot that come_get_options returns; the
    ctypes LaunchOpts mirrors come_launch_opts field for field; unknown names are rejected."""
    L = _lib.lib()
    o = _lib.launch_opts()
    assert o.rows_per_wave == 16 and o.o1_rows_per_wave == 12 and o.gmm_cov_async == 4
    assert o.gmm_resp16 == 3
    assert o.o1_chunk == -1 and o.community_async == 3
    assert o.o2_update_count is None
    _lib.set_option("max_waves", 77)
    try:
        assert _lib.launch_opts().max_waves == 77
        assert _lib.launch_opts(max_waves=5).max_waves == 5  # per call, process value unchanged
        assert _lib.launch_opts().max_waves == 77
    finally:
        _lib.set_option("max_waves", 0)
    with pytest.raises(_lib.ComeError, match="unknown option"):
        _lib.set_option("no_such_knob", 1)
    with pytest.raises(ValueError):
        _lib.launch_opts(no_such_knob=1)
    assert ctypes.sizeof(_lib.LaunchOpts) == 16 * 4 + 8  # 16 ints, the pointer
    p = ctypes.c_void_p(0)
    rc = L.come_sgns_o2_ex(p, p, 0, 128, p, 1, 10, p, 5, 5, p, 10, 0.1, 1.0, 0, p,
                           ctypes.byref(o), p)
    assert rc == -1 and b"V must be" in L.come_last_error()


def test_abi2_flags_and_invalid_ring_in_hogwild():
    """ABI 2: COME_HOT_NONE is accepted as a mode flag; the LDS-ring kernel (o2_kernel=2) is
    sequential-only and a Hogwild request for it is refused before any device work (P = 0)."""
    L = _lib.lib()
    p = ctypes.c_void_p(16)
    assert L.come_sgns_o2(p, p, 10, 8, p, 0, 10, p, 5, 0, p, 10, 0.1, 1.0,
                          _lib.MODE_HOGWILD | _lib.HOT_NONE, p) == 0
    o = _lib.launch_opts(None, o2_kernel=2)
    rc = L.come_sgns_o2_ex(p, p, 10, 8, p, 0, 10, p, 5, 0, p, 10, 0.1, 1.0, _lib.MODE_HOGWILD,
                           None, ctypes.byref(o), p)
    assert rc == -1 and b"sequential" in L.come_last_error()
    o = _lib.launch_opts(None, o2_kernel=2)
    assert L.come_sgns_o2_ex(p, p, 10, 8, p, 0, 10, p, 5, 0, p, 10, 0.1, 1.0,
                             _lib.MODE_SEQUENTIAL, None, ctypes.byref(o), p) == 0
