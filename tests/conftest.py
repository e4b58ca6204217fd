import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libllmvox_hip.so")


def pytest_collection_finish(session):
    """tests/test_gpu_exit.py needs a child process started while this process has not yet touched the
    GPU (a process that has initialised the GPU must not fork + exec): it is started here, after
    collection, before the first test runs, when that test is selected and a GPU is present
    (device_count does not initialise the GPU on this image)."""
    if not any(it.nodeid.startswith("tests/test_gpu_exit.py") or "test_gpu_exit.py" in it.nodeid
               for it in session.items):
        return
    import subprocess
    import torch
    if torch.cuda.device_count() < 1:
        return
    session.config.lvx_exit_child = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "exit_child.py")],
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, cwd=ROOT)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
