"""Debug: the smoke() case (n = 24, N = 600, FULL_P|RECORD) record keys, engine vs oracle, with the
small-graph kernel and with the level loop."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import cpc  # noqa: E402
from rcaeval_amd import synth  # noqa: E402
from rcaeval_amd.engine import get_engine  # noqa: E402


def keys(recs):
    return {(int(r["a"]), int(r["b"]), tuple(int(v) for v in r["s"][: r["d"]])): float(r["p"]) for r in recs}


eng = get_engine(0)
X = synth.gaussian_sem(24, 600, seed=3, w_low=0.3, w_high=0.9)
C = np.corrcoef(X.T)
ref = cpc.skeleton(C, 600, record_cap=1 << 16)
d = keys(ref.records)
print("ref levels", ref.levels, "tests", list(ref.tests), "records", len(d))
for small in [1, 0]:
    for flags in (2, 3):
        with eng.tuned(SMALL=small):      # the knob is read once per handle: set it on the handle
            out = eng.skeleton(C, 600, flags=flags, record_capacity=1 << 16)
        g = keys(out.records)
        byd = collections.Counter(len(k[2]) for k in g)
        byr = collections.Counter(len(k[2]) for k in d)
        print("SMALL", small, "driver", out.stats["driver"], "flags", flags, "levels", out.levels, "tests", out.stats["tests"], "records", len(g),
              "skeleton equal", bool(np.array_equal(out.removed_level, ref.removed_level)))
        print("   per depth gpu", sorted(byd.items()), "ref", sorted(byr.items()))
        print("   only ref", sorted(set(d) - set(g))[:8])
        print("   only gpu", sorted(set(g) - set(d))[:8])
