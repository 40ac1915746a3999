"""The C-ABI library loads and exports every symbol include/prgpu.h declares
(no compute call: runs without a GPU)."""
import ctypes
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    txt = (ROOT / "include" / "prgpu.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pr_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_all_declared_symbols():
    from proovread_amd import _abi
    lib = _abi.lib()
    syms = declared_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_ctx_create_fails_loudly_without_gpu():
    import pytest
    from proovread_amd import _abi
    n = ctypes.c_int(0)
    _abi.lib().pr_device_count(ctypes.byref(n))
    if n.value:
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="PR_ERR_HIP"):
        _abi.Context(0)
