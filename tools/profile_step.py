"""Phase breakdown of one bench step (corr / device skeleton / result collection)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from rcaeval_amd import synth
from rcaeval_amd._lib import PcgStats, check
from rcaeval_amd.engine import get_engine

eng = get_engine(0)
X = synth.gaussian_sem(2000, 10000, seed=0)
Xd = eng.to_device(X)
torch.cuda.synchronize()
for it in range(3):
    t0 = time.perf_counter()
    C = eng.corr(Xd)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    n = 2000
    rl = torch.empty((n, n), dtype=torch.int8, device=eng.device)
    st = PcgStats()
    rc = eng.lib.pcg_skeleton(eng.h, ctypes.c_void_p(C.data_ptr()), n, n, 10000, 0.05, 4, 0,
                              ctypes.c_void_p(rl.data_ptr()), ctypes.byref(st))
    check(eng.h, rc, "skel")
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out = eng._collect(n, rl, st, 0.0)
    t3 = time.perf_counter()
    print(f"iter {it}: corr {1e3*(t1-t0):.2f} ms  skeleton-call {1e3*(t2-t1):.2f} ms  collect {1e3*(t3-t2):.2f} ms  "
          f"sum(level_ms) {sum(st.level_ms[:st.levels]):.2f}  rows {len(out.sep_xy)}", flush=True)
    print("   level_ms", [round(v, 3) for v in st.level_ms[:st.levels]], "kernel_ms",
          [round(v, 3) for v in st.kernel_ms[:st.levels]])
