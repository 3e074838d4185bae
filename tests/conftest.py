import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


KNOBS = os.environ.get("PSO_LIB", "") == "knobs"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long CPU test")
    config.addinivalue_line("markers", "knobs: pins a kernel form through the benchmark knobs of the TOOLS build "
                                       "(libpso_amd_knobs.so): run by tests/test_knobs_build.py in a PSO_LIB=knobs "
                                       "child process; in the product-library process only its knob-free cases run")
    config.addinivalue_line("markers", "knob_variants: runs the default forms in every process and, in the tools-build "
                                       "child, the knob-pinned forms beside them (tests/test_knobs_build.py)")


def pytest_collection_modifyitems(config, items):
    """Knob-pinned cases need the tools build: in the product-library process (PSO_LIB unset) a `knobs` test runs only
    its knob-free parametrization (variant 0, when it has one) -- the rest runs in the knobs child process."""
    if KNOBS:
        return
    for it in items:
        if it.get_closest_marker("knobs") is None:
            continue
        cs = getattr(it, "callspec", None)
        if cs is not None and "variant" in cs.params and cs.params["variant"] == 0:
            continue
        it.add_marker(pytest.mark.skip(reason="benchmark-knob form: runs in the tools-build child process "
                                              "(tests/test_knobs_build.py)"))


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    return torch.device("cuda:0")

