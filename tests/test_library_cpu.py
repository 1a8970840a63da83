"""The C-ABI library loads in a GPU-less process, exports every declared symbol,
and the product path refuses CPU tensors (no silent CPU fallback)."""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "plaincv_hip.h")).read()
    return sorted(set(re.findall(r"\b(pcv_\w+)\(", hdr)))


def test_library_exports_every_declared_symbol():
    from plaincv_amd import hip
    lib = hip.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(hip.SIGNATURES) | {"pcv_last_error_string"} == set(_declared())
    assert lib.pcv_muon_mat_size() == 13 * 8
    assert lib.pcv_chunk_size() == 16
    lib.pcv_last_error_string.restype = __import__("ctypes").c_char_p
    assert b"alignment" in lib.pcv_last_error_string(-2) or b"misaligned" in lib.pcv_last_error_string(-2)


def test_product_rejects_cpu_tensors():
    from plaincv_amd import kernels as K
    a = torch.zeros(8, 8, dtype=torch.bfloat16)
    out = torch.zeros(8, 8)
    with pytest.raises(ValueError):
        K.gemm(a, a, out)
    with pytest.raises(ValueError):
        K.layernorm_fwd(torch.zeros(4, 8), torch.ones(8), torch.zeros(8), torch.zeros(4, 8, dtype=torch.bfloat16),
                        torch.zeros(4), torch.zeros(4))


def test_gemm_shape_checks_before_launch():
    from plaincv_amd import kernels as K
    a = torch.zeros(8, 16, dtype=torch.bfloat16)
    b = torch.zeros(8, 4, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="contraction"):
        K.gemm(a, b, torch.zeros(8, 4))
    with pytest.raises(ValueError, match="bf16"):
        K.gemm(a.float(), torch.zeros(16, 4), torch.zeros(8, 4))


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    import importlib
    from plaincv_amd import hip
    monkeypatch.setattr(hip, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(hip, "_lib", None)
    with pytest.raises(hip.HipLibraryError):
        hip.load()
