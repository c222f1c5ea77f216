"""CPU checks of the drop-in boundary: the gfx950 library loads and exports
every entry point include/contivcls.h declares (no compute calls here)."""
import os
import re

from vpp_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "contivcls.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(cls_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    L = _abi.lib()
    decl = declared_symbols()
    assert len(decl) >= 18
    for sym in decl:
        assert hasattr(L, sym), sym
    assert sorted(_abi.SYMBOLS) == decl


def test_abi_version():
    assert _abi.lib().cls_abi_version() == _abi.ABI_VERSION == 5


def test_engine_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    import pytest
    from vpp_amd.engine import Engine
    with pytest.raises(_abi.ClsError):
        Engine()


def test_library_is_gfx950_code_object():
    data = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_flag_values_match_header():
    text = open(os.path.join(ROOT, "include", "contivcls.h")).read()
    flags = {m.group(1): 1 << int(m.group(2))
             for m in re.finditer(r"CLS_F_(\w+)\s*=\s*1u\s*<<\s*(\d+)", text)}
    assert flags == {"DEVICE": _abi.F_DEVICE, "NO_VERDICT": _abi.F_NO_VERDICT, "ACCUMULATE": _abi.F_ACCUMULATE,
                     "FORCE_LINEAR": _abi.F_FORCE_LINEAR, "TIMING": _abi.F_TIMING, "CONN_CLS": _abi.F_CONN_CLS,
                     "COUNT": _abi.F_COUNT}


def test_timing_entry_points_refuse_null_engine():
    """cls_kernel_times / cls_kernel_starts / cls_kernel_times_reset /
    cls_last_kernel_ms: a null engine or count pointer is CLS_E_INVAL, no
    device call (the timing pair is stamped by the classify launch itself)."""
    import ctypes as C
    from vpp_amd import _abi
    L = _abi.lib()
    n = C.c_uint32(0)
    buf = (C.c_float * 4)()
    for fn in (L.cls_kernel_times, L.cls_kernel_starts):
        assert fn(None, buf, 4, C.byref(n)) == _abi.E_INVAL
        assert fn(None, None, 0, None) == _abi.E_INVAL
    assert L.cls_kernel_times_reset(None) == _abi.E_INVAL
    ms = C.c_float(0)
    assert L.cls_last_kernel_ms(None, C.byref(ms)) == _abi.E_INVAL


def test_compile_options_are_checked():
    """The compiler's option string (cls_compile_v4 / v16; the same keys as
    cls_engine_set_option): unknown keys and malformed values are refused."""
    import ctypes as C
    from aclgen import random_acl
    rules, _ = random_acl(1, 40, 0.0)
    cr = _abi.CRules(rules)
    need = C.c_uint64(0)
    f = _abi.lib().cls_compile_v4
    assert f(cr.ptr(), cr.n, None, 0, C.byref(need), None) == 0
    assert f(cr.ptr(), cr.n, None, 0, C.byref(need), b"orient=dst,list_mode_max=2,trie=0") == 0
    for bad in (b"bogus=1", b"orient=sideways", b"list_mode_max=two", b"trie"):
        assert f(cr.ptr(), cr.n, None, 0, C.byref(need), bad) == _abi.E_INVAL, bad


def test_library_never_reads_the_environment():
    """Tuning switches are engine options (cls_engine_set_option), not
    environment variables: no getenv in the library's sources."""
    import os
    import re
    d = os.path.join(os.path.dirname(_abi.__file__), "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".cpp", ".hpp", ".hip")):
            with open(os.path.join(d, f)) as fh:
                assert not re.search(r"\bgetenv\b|secure_getenv|environ\b", fh.read()), f
