"""The C-ABI library loads and exports every symbol include/pixiu_amd.h declares
(no compute calls: CPU only)."""
import ctypes as C
import os
import re

import pytest

import pixiu_amd as px

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    hdr = open(os.path.join(ROOT, "include", "pixiu_amd.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(px_[a-z_]+)\s*\(", hdr)))


def test_header_matches_python_exports():
    assert declared() == sorted(px.EXPORTS)


def test_library_exports_every_symbol():
    lib = px.load_library()
    for name in declared():
        assert hasattr(lib, name), name


def test_strerror_and_bad_args():
    lib = px.load_library()
    assert lib.px_strerror(0) == b"ok"
    assert b"not found" in lib.px_strerror(8)
    # NULL contexts are rejected without touching a device
    assert lib.px_set_batch(None, 0, None, None, None, None, 0, None) == px.PX_EINVAL
    assert lib.px_stats_get(None, None) == px.PX_EINVAL


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(px.PxError):
        px.Store()


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setenv("PIXIU_AMD_LIB", str(tmp_path / "nope.so"))
    monkeypatch.setattr(px, "_LIB", None)
    with pytest.raises(ImportError):
        px.load_library()
