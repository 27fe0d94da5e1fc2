import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the library honours its path-selecting test hooks (KC_NO_P3B, KC_SKM_POOL_CAP,
# ...) only with KC_TEST_HOOKS=1 (kc_device.h test_hook); the tests use them
os.environ["KC_TEST_HOOKS"] = "1"
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libkc_hip.so on the device)")
    config.addinivalue_line("markers", "slow: full-size configuration")


def load_pkg():
    if "kmer_counter_amd" in sys.modules:
        return sys.modules["kmer_counter_amd"]
    spec = importlib.util.spec_from_file_location("kmer_counter_amd",
                                                  os.path.join(ROOT, "kmer-counter_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["kmer_counter_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def kca():
    return load_pkg()


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session", autouse=True)
def _torch_gpu_first(request):
    """PyTorch ships its own HIP runtime (libamdhip64 under torch/lib) next to
    the system one libkc_hip.so links; in one process the GPU must be opened by
    PyTorch first, or its later torch.cuda init fails. GPU sessions that will
    mix the two (the key-space exchange tests) therefore open it up front."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
        except ImportError:
            return
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda:0")
