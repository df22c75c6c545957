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
