import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    with open(os.path.join(ROOT, "tests", "golden", "frames.json")) as fh:
        meta = json.load(fh)
    blob = np.fromfile(os.path.join(ROOT, "tests", "golden", "frames.bin"), dtype=np.uint8)
    return meta, blob


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle

    oracle.build()
    return oracle
