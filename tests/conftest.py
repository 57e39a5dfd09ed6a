import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, "prov-gigapath-replication_amd")
for p in (ROOT, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden_meta():
    import json
    with open(os.path.join(GOLDEN, "golden_meta.json")) as f:
        return json.load(f)


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name)))


# ---------------------------------------------------------------------------------------------
# Parity record: every end-to-end golden comparison logs its measured worst max|d|/max|ref| and
# cosine per output kind, so the headroom against the tolerance is on record (printed in the
# terminal summary and written to gpurun_out/parity_metrics.json when that directory exists or
# can be created: the GPU box's scratch output, copied to profiles/ by hand).
PARITY = []


def record_parity(test, output, rel, cos, tol_rel, tol_cos, n_vectors=1):
    PARITY.append({"test": test, "output": output, "max_rel": float(rel), "min_cos": float(cos),
                   "tol_rel": float(tol_rel), "tol_cos": float(tol_cos), "vectors": int(n_vectors),
                   "headroom_rel": float(tol_rel / rel) if rel > 0 else None})


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if not PARITY:
        return
    import json
    tr = terminalreporter
    tr.write_sep("-", "parity vs reference goldens (worst vector per output)")
    for r in PARITY:
        tr.write_line("%-58s %-14s rel %.3e (tol %.0e)  cos %.7f (tol %.4f)  n=%d" % (
            r["test"][:58], r["output"], r["max_rel"], r["tol_rel"], r["min_cos"], r["tol_cos"], r["vectors"]))
    out = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_metrics.json"), "w") as f:
            json.dump(PARITY, f, indent=1)
    except OSError:
        pass
