"""The knob-pinned kernel forms, run against the TOOLS build.

The product library libpso_amd.so has no benchmark knobs (include/pso_amd.h): its dispatch is the
automatic one and the measured-not-kept kernel forms are not compiled into it.  The tests that pin an alternative
form through a knob -- every forced GEMM tile / variant against its fp32 reference, the 8-phase / 256x160 / 256x320 /
conv forms on shapes the automatic dispatch would not send there, the attention forward / backward forms against the
default's bits -- therefore run in a child process on libpso_amd_knobs.so (the same sources compiled with
-DPSO_BENCH_KNOBS, include/pso_amd_knobs.h): `pytest -m "gpu and (knobs or knob_variants)"` with PSO_LIB=knobs.  The
default-form cases of the same tests also run in this (product-library) process."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(1500)
def test_knob_forms_in_tools_build(cuda, capsys):
    lib = os.path.join(ROOT, "pairwise_sample_optimization_amd", "libpso_amd_knobs.so")
    assert os.path.exists(lib), "libpso_amd_knobs.so not built (make -C pairwise_sample_optimization_amd/csrc)"
    env = dict(os.environ, PSO_LIB="knobs")
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "--timeout", "600",
           "--timeout-method", "thread", "-m", "gpu and (knobs or knob_variants)",
           os.path.join(ROOT, "tests", "test_gpu_kernels.py"), os.path.join(ROOT, "tests", "test_gpu_layers.py"),
           os.path.join(ROOT, "tests", "test_gpu_determinism.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=1400)
    tail = (r.stdout[-4000:] + r.stderr[-2000:])
    with capsys.disabled():  # the child's summary line belongs in the suite log
        print("\n[tools-build child] " + (r.stdout.strip().splitlines() or ["(no output)"])[-1], flush=True)
    out_dir = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out_dir):
        with open(os.path.join(out_dir, "knobs_child.log"), "w") as f:
            f.write(r.stdout + r.stderr)
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and " failed" not in r.stdout
