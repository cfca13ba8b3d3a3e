"""CPU-side checks of the C-ABI boundary: the library loads and exports
every function include/reflow_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "reflow_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rf_[a-z0-9_]+)\s*\(", text)))


def test_header_parses():
    syms = declared_symbols()
    assert "rf_init" in syms and "rf_bloom_probe" in syms and "rf_graph_recompute" in syms


def test_library_exports_every_declared_symbol():
    from reflow_amd import capi
    L = capi.lib()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_binding_list_matches_header():
    from reflow_amd import capi
    assert sorted(capi.EXPORTS) == declared_symbols()


def test_version_and_error_without_device():
    from reflow_amd import capi
    L = capi.lib()
    assert L.rf_version().startswith(b"reflow-hip")
    # rf_init either succeeds (GPU present) or fails loudly -- never falls back
    h = ctypes.c_void_p()
    rc = L.rf_init(0, ctypes.byref(h))
    if rc == 0:
        L.rf_destroy(h)
    else:
        assert rc in (capi.RF_EDEVICE, capi.RF_EINVAL)
        assert len(L.rf_last_error()) > 0


def test_code_object_is_gfx950():
    so = os.path.join(ROOT, "reflow_amd", "libreflow_hip.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data


def test_graph_entry_points_refuse_null_arguments():
    """Entry points that need no device refuse bad arguments with RF_EINVAL
    before touching one (a binding's misuse fails loudly, never silently)."""
    from reflow_amd import capi
    L = capi.lib()
    assert L.rf_graph_adopt_slots(None, None) == capi.RF_EINVAL
    assert len(L.rf_last_error()) > 0
    assert L.rf_graph_stats_get(None, None) == capi.RF_EINVAL
    assert L.rf_graph_set_slots(None, None, None, 1) == capi.RF_EINVAL
