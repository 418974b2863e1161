"""Time pcg_corr (K1) of the in-tree library under environment settings given on the command
line, each in a fresh child process (the knobs are read per call): python k1_env_time.py
"PCG_K1_I8=0" "PCG_K1_I8_KS=8" ... ; prints ms per call and max |C - numpy| of each."""
import os
import subprocess
import sys

CHILD = r'''
import ctypes, sys, numpy as np, torch
sys.path.insert(0, ".")
from rcaeval_amd import synth, _lib
X = synth.gaussian_sem(2000, 10000, seed=0)
ref = np.corrcoef(X.T)
Xd = torch.from_numpy(X).cuda()
N, n = X.shape
lib = _lib.load()
h = ctypes.c_void_p()
assert lib.pcg_create(0, ctypes.byref(h)) == 0
lib.pcg_set_stream(h, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
C = torch.empty((n, n), dtype=torch.float64, device="cuda")
f = lambda: lib.pcg_corr(h, ctypes.c_void_p(Xd.data_ptr()), N, n, n, ctypes.c_void_p(C.data_ptr()), n)
for _ in range(3):
    assert f() == 0
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    f()
e1.record()
torch.cuda.synchronize()
print("%.3f ms/corr  max|C - numpy| %.3g" % (e0.elapsed_time(e1) / 20, np.abs(C.cpu().numpy() - ref).max()))
'''


def main():
    for spec in sys.argv[1:]:
        env = dict(os.environ)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        print(f"{spec:40s} {out.stdout.strip() or out.stderr.strip()[-300:]}", flush=True)


if __name__ == "__main__":
    main()
