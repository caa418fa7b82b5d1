import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: CPU test that takes more than ~30 s")


def pytest_collection_modifyitems(session, config, items):
    # torch must see the GPU before libmigmres initialises HIP in this process (the loopback
    # tests create contexts without torch); afterwards torch.cuda.is_available() reports False
    if any(item.get_closest_marker("gpu") for item in items):
        try:
            import torch
            torch.cuda.is_available()
        except ImportError:
            pass
