import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "reference: needs /root/reference (container only)")


def pytest_collection_modifyitems(config, items):
    if not os.path.isdir("/root/reference"):
        skip = pytest.mark.skip(reason="reference tree not present on this machine")
        for it in items:
            if "reference" in it.keywords:
                it.add_marker(skip)
