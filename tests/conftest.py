import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKG = "starpu-inference-server_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libspi_hip.so on the device)")


@pytest.fixture(scope="session")
def spi():
    return importlib.import_module(PKG)


@pytest.fixture(scope="session")
def zoo():
    return importlib.import_module(PKG + ".zoo")


@pytest.fixture(scope="session")
def gpu(spi):
    if spi.lib.spi_device_count() < 1:
        pytest.skip("no HIP device")
    import torch
    return torch.device("cuda", 0)
