import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "host_policy: keeps the drop-in's default size policy "
                            "(tests/test_gpu_dropin.py)")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def gpu_present() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    return oracle.lib()


@pytest.fixture(scope="session")
def ref_lib():
    import oracle
    L = oracle.ref_lib("O2")
    if L is None:
        pytest.skip("oracle/_ref not built (reference sources absent on this machine)")
    return L
