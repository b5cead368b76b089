"""CPU tests of the drop-in boundary: libgpuverify.so builds, loads and exports
exactly the C-ABI include/gpuverify.h declares; without a GPU it fails loudly
(no silent CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

import gpuverify as gvm

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "gpuverify.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gv_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_the_python_binding_symbols():
    assert declared_symbols() == sorted(gvm.EXPORTED_SYMBOLS)


def _prototype_arity():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    arity = {}
    for name, args in re.findall(r"\b(gv_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", txt):
        a = args.strip()
        arity[name] = 0 if a in ("", "void") else a.count(",") + 1
    return arity


def _call_args(src, start):
    depth, i, n = 1, start, 1
    if src[start:].lstrip().startswith(")"):
        return 0
    while depth:
        c = src[i]
        depth += c == "("
        depth -= c == ")"
        n += c == "," and depth == 1
        i += 1
    return n


def test_go_binding_calls_declared_symbols_with_declared_arity():
    """go/crypto/gpuverify (source-only: no Go toolchain here) calls only
    functions include/gpuverify.h declares, each with its declared arity."""
    arity = _prototype_arity()
    src = open(os.path.join(REPO, "go", "crypto", "gpuverify", "gpuverify.go")).read()
    calls = [(m.group(1), _call_args(src, m.end())) for m in re.finditer(r"\bC\.(gv_\w+)\(", src)]
    assert len(calls) >= 8
    for name, n in calls:
        assert name in arity, name
        assert n == arity[name], (name, n, arity[name])


def test_library_exports_every_declared_symbol():
    if not os.path.exists(gvm.LIB_PATH):
        gvm.build()
    L = ctypes.CDLL(gvm.LIB_PATH)
    for sym in declared_symbols():
        assert hasattr(L, sym), sym
    out = subprocess.run(["nm", "-D", "--defined-only", gvm.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (gv_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", gvm.LIB_PATH],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(gvm.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_strerror_and_option_validation_without_gpu():
    L = gvm.load()
    assert L.gv_strerror(0) == b"ok"
    assert L.gv_strerror(-3) == b"HIP runtime error"
    assert L.gv_set_option(None, b"max_batch", 1024) == gvm.GV_EINVAL
    assert L.gv_verify_digests(None, 1, None, None, None, None) == gvm.GV_EINVAL


def test_open_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(gvm.GpuVerifyError):
        gvm.Verifier()


def test_libgvhost_exports_every_function_its_header_declares():
    """libgvhost.so (the host mirror) exports every gvh_* function
    cosmos-sdk-rootchain_amd/host/gvhost.h declares (incl. the IBC commit hook)."""
    import gvhost
    hdr = os.path.join(REPO, "cosmos-sdk-rootchain_amd", "host", "gvhost.h")
    txt = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(gvh_[a-z_0-9]+)\s*\(", txt)))
    assert "gvh_verify_commits" in names and len(names) >= 25
    L = gvhost.lib()
    for n in names:
        assert hasattr(L, n), n
