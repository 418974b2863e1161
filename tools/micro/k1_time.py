"""Time pcg_corr (K1) of several libpcgpu builds on the 2000 x 10000 SEM: python k1_time.py a.so b.so ..."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from rcaeval_amd import synth  # noqa: E402

X = torch.from_numpy(synth.gaussian_sem(2000, 10000, seed=0)).cuda()
N, n = X.shape
ref = None
for path in sys.argv[1:]:
    lib = ctypes.CDLL(path)
    h = ctypes.c_void_p()
    assert lib.pcg_create(0, ctypes.byref(h)) == 0
    lib.pcg_set_stream(h, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    C = torch.empty((n, n), dtype=torch.float64, device="cuda")
    f = lambda: lib.pcg_corr(h, ctypes.c_void_p(X.data_ptr()), ctypes.c_int64(N), ctypes.c_int64(n), ctypes.c_int64(n),
                             ctypes.c_void_p(C.data_ptr()), ctypes.c_int64(n))
    for _ in range(3):
        assert f() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    c = C.cpu().numpy()
    if ref is None:
        ref = c
    print(f"{path}: {e0.elapsed_time(e1) / 20:.3f} ms/corr  max|dC| vs first = {np.abs(c - ref).max():.3g}", flush=True)
