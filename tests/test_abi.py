"""CPU checks of the C-ABI boundary: the library builds/loads and exports every symbol include/pso_amd.h declares
(no compute calls: there is no GPU here)."""
import os
import glob
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


def test_product_library_has_no_benchmark_knobs():
    """the benchmark knobs (include/pso_amd_knobs.h) and the measured-not-kept kernel forms live in the
    tools build only.  The product library exports none of the knob setters, reads no environment variable, and holds
    no g_* dispatch state; the tools build exports every knob the header declares."""
    from pairwise_sample_optimization_amd import _lib
    prod = os.path.join(os.path.dirname(_lib.__file__), "libpso_amd.so")
    knobs = os.path.join(os.path.dirname(_lib.__file__), "libpso_amd_knobs.so")
    h = open(os.path.join(ROOT, "include", "pso_amd_knobs.h")).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    knob_names = sorted(set(re.findall(r"^\s*\w+\s+\**(pso_\w+)\(", h, flags=re.M)))
    assert set(knob_names) == set(_lib.KNOB_SIGNATURES), knob_names
    exported = set(re.findall(r" T (pso_\w+)", subprocess.check_output(["nm", "-D", "--defined-only", prod]).decode()))
    assert not (exported & set(knob_names)), exported & set(knob_names)
    undefined = subprocess.check_output(["nm", "-D", "--undefined-only", prod]).decode()
    assert "getenv" not in undefined
    local = subprocess.check_output(["nm", "-C", prod]).decode()
    assert not re.search(r" [bBdD] g_(gemm|tn|attn|skip|mode|grid)", local)
    assert "attn_bwd_dkv_pp_kernel" not in local
    kexp = set(re.findall(r" T (pso_\w+)", subprocess.check_output(["nm", "-D", "--defined-only", knobs]).decode()))
    assert set(knob_names) <= kexp and set(_declared()) <= kexp
    for src in glob.glob(os.path.join(ROOT, "pairwise_sample_optimization_amd", "csrc", "*.hip")):
        txt = open(src).read()
        for m in re.finditer(r"^static (?:const )?(?:int|bool) g_\w+", txt, flags=re.M):
            # every mutable dispatch global sits inside an #ifdef PSO_BENCH_KNOBS block
            before = txt[:m.start()]
            assert before.rfind("#ifdef PSO_BENCH_KNOBS") > before.rfind("#endif"), (src, m.group(0))
