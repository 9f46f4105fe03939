import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def ref_tables():
    import numpy as np

    return dict(np.load(os.path.join(GOLDEN, "reference_tables.npz")))


@pytest.fixture(scope="session")
def ref_pipeline():
    import numpy as np

    return dict(np.load(os.path.join(GOLDEN, "reference_pipeline.npz")))


@pytest.fixture(scope="session")
def oracle_vectors():
    import numpy as np

    return dict(np.load(os.path.join(GOLDEN, "oracle_vectors.npz")))
