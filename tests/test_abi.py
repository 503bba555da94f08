"""The C-ABI library loads and exports every symbol include/nts_hip.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import re
import subprocess

from conftest import ROOT


def header_symbols():
    text = (ROOT / "include" / "nts_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nts_hip_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_api():
    syms = header_symbols()
    from nts import _abi
    assert syms == sorted(_abi.EXPORTED)


def test_library_exports_every_header_symbol():
    from nts import _abi
    lib = _abi.lib()  # raises if the HIP library was not built
    for s in header_symbols():
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", str(_abi.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (nts_hip_\w+)", out))
    assert set(header_symbols()) <= exported
    assert lib.nts_hip_abi_version() == _abi.ABI_VERSION == 11


def test_library_is_gfx950_code_object():
    from nts import _abi
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", str(_abi.LIB_PATH)],
                         capture_output=True, text=True)
    blob = _abi.LIB_PATH.read_bytes()
    assert b"gfx950" in blob


def test_last_error_reports_invalid_arguments():
    from nts import _abi
    lib = _abi.lib()
    rc = lib.nts_hip_ctx_create(None, 0, None, 1)
    assert rc == 1  # NTS_ERR_INVALID, no GPU touched
    assert b"invalid argument" in lib.nts_hip_last_error()
