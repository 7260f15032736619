"""The C-ABI boundary without a GPU: libaccord_deps.so loads, exports every function include/*.h declares,
and the product path refuses to run (loudly) when no device is present — there is no CPU fallback."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cassandra-accord_amd")
LIB = os.path.join(PKG, "libaccord_deps.so")


def _lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", PKG])
    return C.CDLL(LIB)


def declared_functions():
    names = []
    for h in os.listdir(os.path.join(ROOT, "include")):
        if h.endswith(".h"):
            src = open(os.path.join(ROOT, "include", h)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s+\**\s*(ad_[a-z0-9_]+)\s*\(", src, re.M):
                names.append(m.group(1))
    return sorted(set(n for n in names if not n.startswith(("ad_mix64", "ad_drop_hash", "ad_drop_threshold"))))


def test_header_declares_boundary():
    names = declared_functions()
    for must in ("ad_open", "ad_close", "ad_load_batch", "ad_preaccept_deps", "ad_fetch_deps", "ad_merge_deps",
                 "ad_merge_host", "ad_exec_levels", "ad_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = _lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, "declared in include/ but not exported: %s" % missing


def test_python_binding_covers_exports():
    import sys
    sys.path.insert(0, PKG)
    from accord_amd import engine
    assert set(engine.EXPORTED) >= set(declared_functions())


def test_open_without_device_fails_loudly():
    import sys
    sys.path.insert(0, PKG)
    from accord_amd import abi, engine
    if engine.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(engine.AccordDepsError):
        engine.DepsEngine(device=0)
    h = C.c_void_p()
    cfg = abi.AdConfig(3, 0)
    assert engine.lib().ad_open(0, C.byref(cfg), C.byref(h)) == abi.AD_ERR_DEVICE
    assert engine.lib().ad_open(0, C.byref(abi.AdConfig(0, 0)), C.byref(h)) == abi.AD_ERR_ARGUMENT
    assert engine.lib().ad_set_replica_model(None, C.byref(abi.AdReplicaModel(32, 0.1, 1))) == abi.AD_ERR_ARGUMENT
