"""K1 alone at the headline shape (N = 10 000, n = 2 000), for rocprofv3 PMC passes: synthetic X
already on the device, `reps` calls of pcg_corr. usage: python tools/k1_run.py [reps]"""
import sys

import torch

sys.path.insert(0, ".")
from rcaeval_amd.engine import Engine  # noqa: E402
from rcaeval_amd import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
eng = Engine(0)
X = eng.to_device(synth.gaussian_sem(2000, 10000, seed=0, w_low=0.1, w_high=0.5))
for _ in range(reps):
    C = eng.corr(X)
torch.cuda.synchronize()
print("k1 ok", float(C[0, 1]))
