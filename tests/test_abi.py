"""CPU checks of the C-ABI boundary: the library builds/loads and exports every symbol include/pso_amd.h declares
(no compute calls: there is no GPU here)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    h = open(os.path.join(ROOT, "include", "pso_amd.h")).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(pso_\w+)\(", h, flags=re.M)))


def test_header_declares_functions():
    names = _declared()
    assert "pso_gemm" in names and "pso_pair_loss_fwd" in names and "pso_attention_bwd" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    from pairwise_sample_optimization_amd import _lib
    l = _lib.lib()
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (pso_\w+)", out))
    for name in _declared():
        assert name in exported, name
        assert name in _lib.SIGNATURES, f"{name} not bound in _lib.SIGNATURES"
        getattr(l, name)
    assert l.pso_abi_version() == 1


def test_bound_signatures_match_header_arity():
    from pairwise_sample_optimization_amd import _lib
    h = open(os.path.join(ROOT, "include", "pso_amd.h")).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    for m in re.finditer(r"(pso_\w+)\(([^)]*)\);", h):
        name, args = m.group(1), m.group(2).strip()
        n = 0 if args in ("", "void") else len(args.split(","))
        assert len(_lib.SIGNATURES[name][1]) == n, (name, n, len(_lib.SIGNATURES[name][1]))


def test_no_cpu_fallback():
    import pytest
    import torch
    from pairwise_sample_optimization_amd import kernels, _lib
    a = torch.zeros(8, 8, dtype=torch.bfloat16)
    with pytest.raises(_lib.PsoLibError):
        kernels.gemm(a, a)
