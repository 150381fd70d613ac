"""CPU tests of the C-ABI boundary: libnas.so loads, exports exactly what
include/nas.h declares, and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re

import pytest

from kubernetesnetawarescheduler_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    with open(os.path.join(ROOT, "include", "nas.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nas_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ["nas_create", "nas_destroy", "nas_upload_snapshot", "nas_score_reference",
                 "nas_upload_latency", "nas_upload_pods", "nas_upload_capacity", "nas_place",
                 "nas_last_error", "nas_comm_init"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == declared()


def test_version():
    assert _lib.lib().nas_version() == 2


def test_create_fails_loudly_without_gpu():
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.nas_create(ctypes.byref(h), ctypes.byref(_lib.NasConfig(device=0)))
    if rc == 0:
        L.nas_destroy(h)
        pytest.skip("a GPU is visible here")
    assert rc == _lib.NAS_ERR_HIP
    assert not h.value


def test_engine_raises_without_gpu():
    from kubernetesnetawarescheduler_amd import Engine, NasError
    try:
        e = Engine(0)
    except NasError as err:
        assert err.code == _lib.NAS_ERR_HIP
        return
    e.close()
    pytest.skip("a GPU is visible here")


def test_null_context_is_an_argument_error():
    L = _lib.lib()
    assert L.nas_score(None) == _lib.NAS_ERR_ARG
    assert L.nas_get_timings(None, None) == _lib.NAS_ERR_ARG
    assert L.nas_last_error(None) == b"null context"


def test_missing_library_fails_loudly(monkeypatch):
    # no CPU fallback: without the built libnas.so every entry point raises
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setattr(_lib, "LIB_PATH", os.path.join(ROOT, "no_such_dir", "libnas.so"))
    with pytest.raises(_lib.NasError, match="not built"):
        _lib.lib()


def test_go_binding_uses_declared_abi():
    """scheduler/nas.go (the cgo binding for the reference's package main):
    every C.nas_* call and C.NAS_* constant it names is in include/nas.h, and
    the config field it sets exists (the Go toolchain is absent here)."""
    with open(os.path.join(ROOT, "scheduler", "nas.go")) as f:
        go = f.read()
    with open(os.path.join(ROOT, "include", "nas.h")) as f:
        hdr = f.read()
    funcs = set(re.findall(r"\bC\.(nas_[a-z0-9_]+)\(", go))
    assert funcs and funcs <= set(declared()), funcs - set(declared())
    L = _lib.lib()
    assert all(hasattr(L, n) for n in funcs)
    consts = set(re.findall(r"\bC\.(NAS_[A-Z0-9_]+)\b", go))
    defined = set(re.findall(r"#define\s+(NAS_[A-Z0-9_]+)", hdr))
    assert consts and consts <= defined, consts - defined
    assert set(re.findall(r"\bC\.(nas_[a-z_]+)\{", go)) <= {"nas_config"}
    assert re.search(r"int32_t\s+device\s*;", hdr)


def test_entries_carry_roctx_ranges():
    """Every C-ABI entry opens a roctx range (rocprofv3 --marker-trace)."""
    import shutil
    import subprocess
    if shutil.which("nm") is None:
        pytest.skip("needs nm")
    und = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "roctxRangePush" in und and "roctxRangePop" in und
    with open(os.path.join(ROOT, "kubernetesnetawarescheduler_amd", "csrc", "nas_api.hip")) as f:
        src = f.read()
    ranged = set(re.findall(r'NAS_RANGE\("(nas_[a-z0-9_]+)"\)', src))
    trivial = {"nas_version", "nas_last_error", "nas_get_timings", "nas_set_option",
               "nas_debug_counters"}
    assert set(declared()) - trivial <= ranged, set(declared()) - trivial - ranged
