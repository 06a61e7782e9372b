import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "diffpose-nw_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)

    return load


def record_delta(value, tol, tag=None):
    """Report an achieved parity delta against its bar and return ``value <= tol``.  Every call
    prints one ``DELTA {json}`` line (run pytest with -s or -rP to see it) and, when the
    environment names a file in DPK_DELTA_LOG, appends the same JSON there, so a GPU run leaves
    the achieved numbers beside the pass/fail (profiles/*_deltas.jsonl)."""
    import inspect
    import json

    if tag is None:
        fr = inspect.stack()[1]
        tag = f"{os.path.basename(fr.filename)}::{fr.function}:{fr.lineno}"
    rec = json.dumps({"tag": tag, "delta": float(value), "tol": float(tol), "pass": bool(value <= tol)})
    print("DELTA", rec)
    path = os.environ.get("DPK_DELTA_LOG")
    if path:
        with open(path, "a") as f:
            f.write(rec + "\n")
    return value <= tol
