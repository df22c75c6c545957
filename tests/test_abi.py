"""CPU: libdts.so loads, exports every symbol include/dts.h declares, and
fails cleanly (no abort) without a device."""
import ctypes
import os
import re

import dtsffi as D

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "dts.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dts_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    L = D.lib()
    names = declared_functions()
    assert len(names) >= 19
    for n in names:
        assert hasattr(L, n), n
    assert sorted(D.EXPORTS) == names


def test_version_and_errors():
    L = D.lib()
    assert b"gfx950" in L.dts_version()
    assert L.dts_strerror(D.E_HIP) == b"HIP runtime error"
    assert L.dts_strerror(12345) == b"unknown error"


def test_null_and_bad_args_do_not_crash():
    L = D.lib()
    assert L.dts_ctx_create(0, None) == D.E_INVAL
    assert L.dts_graph_create(None, None, None) == D.E_INVAL
    assert L.dts_graph_wait(None) == D.E_INVAL
    assert L.dts_graph_submit(None, None, 0, None, None, None) == D.E_INVAL
    assert L.dts_graph_run_device(None, None, 0, None, None, None, None) == D.E_INVAL
    assert L.dts_qstat_finalize(0, 0, None, 0, None) == D.E_INVAL


def test_no_device_is_reported_not_fatal():
    if D.device_count() > 0:
        return
    h = ctypes.c_void_p()
    assert D.lib().dts_ctx_create(0, ctypes.byref(h)) == D.E_NODEV


def test_abi_version_matches_header():
    """DTS_ABI_VERSION in include/dts.h == the library's == the binding's, and the version
    string names it (the header stayed at 5 after the ABI-6 struct change)."""
    src = open(os.path.join(ROOT, "include", "dts.h")).read()
    hv = int(re.search(r"#define DTS_ABI_VERSION (\d+)", src).group(1))
    L = D.lib()
    assert L.dts_abi_version() == hv == D.ABI_VERSION
    assert f"abi {hv}".encode() in L.dts_version()


def test_struct_sizes_match_library():
    """sizeof() of every ABI struct as the library sees it == the ctypes layout, and every
    DTS_STRUCT_* id the header defines is answered (unknown ids -> DTS_E_INVAL)."""
    src = open(os.path.join(ROOT, "include", "dts.h")).read()
    ids = {int(v): n for n, v in re.findall(r"#define DTS_STRUCT_([A-Z_]+)\s+(\d+)", src)}
    assert sorted(ids) == sorted(D.STRUCT_IDS)
    L = D.lib()
    for which, cls in D.STRUCT_IDS.items():
        assert L.dts_abi_struct_size(which) == ctypes.sizeof(cls), (ids[which], cls.__name__)
    assert L.dts_abi_struct_size(99) == D.E_INVAL
    # the ABI-6 layout: dts_output_spec = 4 int32 + 2 double + 2 int32
    assert ctypes.sizeof(D.OutputSpec) == 40


def test_binding_refuses_abi_mismatch(monkeypatch):
    """dtsffi.abi_check raises on a library reporting another ABI version."""
    L = D.lib()

    class Fake:
        def dts_abi_version(self):
            return D.ABI_VERSION + 1

        def dts_abi_struct_size(self, which):
            return L.dts_abi_struct_size(which)
    import pytest
    with pytest.raises(RuntimeError, match="ABI"):
        D.abi_check(Fake())
