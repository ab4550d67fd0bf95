import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


@pytest.fixture(scope="session")
def ref_vectors():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "ref_vectors.npz")))


def load_weights(tag):
    import numpy as np
    z = np.load(os.path.join(GOLDEN, "weights", tag + ".npz"))
    get = lambda k, n: [z["%s_%d" % (k, i)] for i in range(n)]
    out = {"actor": get("actor", 6), "critic": get("critic", 10)}
    if "target_0" in z:
        out["target"] = get("target", 10)
    return out
