import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


import pytest  # noqa: E402


@pytest.fixture(scope="session")
def config5():
    """BASELINE config 5 (2000 vars x 10 000 samples, seed 0) and the C oracle's stable skeleton on
    numpy's corrcoef to depth 4 (pc_oracle.c, every host core; about a minute), computed once per
    session for the full-size GPU parity tests."""
    import sys
    import time

    import numpy as np
    from oracle import cpc
    from rcaeval_amd import synth
    X = synth.gaussian_sem(2000, 10000, seed=0)
    Ch = np.corrcoef(X.T)
    t0 = time.perf_counter()
    print("oracle: config 5 to depth 4 ...", file=sys.stderr, flush=True)
    ref = cpc.skeleton(Ch, 10000, max_depth=4, want_union=True)
    print(f"oracle done in {time.perf_counter() - t0:.1f} s: tests {ref.tests}", file=sys.stderr, flush=True)
    return X, Ch, ref
