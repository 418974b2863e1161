"""Study for the fp32 screening sweep of k_level_lds_t (depth 4, config 5).

Samples depth-4 tests (x, y | S = T + {c}) of the 2000-var x 10k SEM on the graph at the
start of depth 4 (C oracle, depths 0..3), evaluates them
  (a) in fp64 from C (the reference-grade r^2), and
  (b) the way the fp32 sweep would: setup (L_T, L_T^-1, u_T, l_c, 1/lambda_c, u_c, c_xx) in
      fp64 from fp32(C), the per-y sweep in float32,
and reports the r^2 / threshold distribution, the fp32-vs-fp64 error against the a-priori
bound E_c = u * K * (1 + nu_c)^2 (nu_c = ||L_S^-1||_F), and the share of tests the bound
leaves undecided (the band the rare path recomputes in fp64).

    python tools/f32_screen_study.py [--nodes 24] [--per-node 40000]
"""
from __future__ import annotations

import argparse
import math
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from oracle import cpc  # noqa: E402  (study tool: the oracle is the checker here)
from rcaeval_amd import synth  # noqa: E402

U32 = 2.0 ** -24


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=24)
    ap.add_argument("--per-node", type=int, default=40000)
    ap.add_argument("--K", type=float, default=64.0)
    ap.add_argument("--n", type=int, default=2000)
    args = ap.parse_args()
    N = 10000
    t0 = time.time()
    X = synth.gaussian_sem(args.n, N, seed=0)
    C = cpc.corrcoef(X)
    sk = cpc.skeleton(C, N, max_depth=3, want_union=False)
    adj = sk.adj
    print(f"setup {time.time() - t0:.1f}s, edges at depth 4: {adj.sum() // 2}", flush=True)
    d = 4
    from scipy.stats import norm
    z = norm.ppf(1 - 0.05 / 2)
    thr = math.tanh(z / math.sqrt(N - d - 3)) ** 2
    rng = np.random.default_rng(1)
    deg = adj.sum(1)
    cand = np.nonzero((deg >= 6) & (deg <= 64))[0]
    xs = rng.choice(cand, size=min(args.nodes, len(cand)), replace=False)
    C32 = C.astype(np.float32).astype(np.float64)
    rows = []
    for x in xs:
        nb = np.nonzero(adj[x])[0]
        D = len(nb)
        B = args.per_node
        # random (y, T, c): T 3-subset, c < min(T) (local indices), y outside S
        loc = np.argsort(rng.random((B, D)), axis=1)[:, :5]
        S = np.sort(loc[:, :4], axis=1)
        yl = loc[:, 4]
        c = S[:, 0]
        T = S[:, 1:]
        gx = np.full(B, x)
        gy = nb[yl]
        gT = nb[T]
        gc = nb[c]
        rows.append((gx, gy, gT, gc))
    gx = np.concatenate([r[0] for r in rows])
    gy = np.concatenate([r[1] for r in rows])
    gT = np.concatenate([r[2] for r in rows])
    gc = np.concatenate([r[3] for r in rows])
    nt = len(gx)

    def partial(Cm, dtype_sweep):
        """T-group formulas: setup in fp64 from Cm, sweep in dtype_sweep."""
        CTT = Cm[gT[:, :, None], gT[:, None, :]]
        L = np.linalg.cholesky(CTT)
        Li = np.linalg.inv(L)
        uT = np.einsum("bij,bj->bi", Li, Cm[gT, gx[:, None]])
        lc = np.einsum("bij,bj->bi", Li, Cm[gT, gc[:, None]])
        lam2 = Cm[gc, gc] - (lc * lc).sum(1)
        rl = 1.0 / np.sqrt(lam2)
        uc = (Cm[gc, gx] - (lc * uT).sum(1)) * rl
        cxx = Cm[gx, gx] - (uT * uT).sum(1) - uc * uc
        # nu_c = ||L_S^-1||_F: [Li 0; -lc^T Li / lam, 1/lam]
        w = np.einsum("bi,bij->bj", lc, Li)
        nu = np.sqrt((Li * Li).sum((1, 2)) + ((w * w).sum(1) + 1.0) * rl * rl)
        f = dtype_sweep
        Lif, uTf, lcf, rlf, ucf = (a.astype(f) for a in (Li, uT, lc, rl, uc))
        mT = Cm[gT, gy[:, None]].astype(f)
        vT = np.einsum("bij,bj->bi", Lif, mT).astype(f)
        # the kernel's order: the k products accumulated onto -{A~_yy, A~_xy}
        ay_, ax_ = -Cm[gy, gy].astype(f), -Cm[gx, gy].astype(f)
        for i in range(vT.shape[1]):
            ay_ = (ay_ + vT[:, i] * vT[:, i]).astype(f)
            ax_ = (ax_ + uTf[:, i] * vT[:, i]).astype(f)
        byy, bxy = -ay_, -ax_
        sc = (Cm[gc, gy].astype(f) - (lcf * vT).sum(1, dtype=f)).astype(f)
        vc = (sc * rlf).astype(f)
        cyy = (byy - vc * vc).astype(f)
        cxy = (bxy - ucf * vc).astype(f)
        return cxx, cyy.astype(np.float64), cxy.astype(np.float64), nu, lam2

    cxx64, cyy64, cxy64, nu, lam2 = partial(C, np.float64)
    cxx32, cyy32, cxy32, nu32, _ = partial(C32, np.float32)
    r2 = cxy64 ** 2 / (cxx64 * cyy64)
    q = r2 / thr
    print(f"tests sampled {nt}; thr {thr:.4e}")
    print("r2/thr quantiles:", np.quantile(q, [0.001, 0.01, 0.05, 0.1, 0.25, 0.5]).round(3))
    print(f"indep share (r2 < thr): {np.mean(q < 1):.4e}")
    for b in (1e-3, 1e-2, 3e-2, 1e-1):
        print(f"  share with |r2/thr - 1| < {b:g}: {np.mean(np.abs(q - 1) < b):.3e}")
    E = U32 * args.K * (1.0 + nu) ** 2
    err = np.maximum.reduce([np.abs(cxy32 - cxy64), np.abs(cyy32 - cyy64), np.abs(cxx32 - cxx64)])
    ratio = err / E
    print(f"nu quantiles {np.quantile(nu, [0.5, 0.9, 0.99, 1.0]).round(3)}")
    print(f"max |err| / E_c = {ratio.max():.3e}  (99.99%: {np.quantile(ratio, 0.9999):.3e})")
    # decisions with the bound: dependent if (|cxy|-E)^2 > thr(cxx+E)(cyy+E); independent if
    # (|cxy|+E)^2 < thr(cxx-E)(cyy-E); otherwise band
    a = np.abs(cxy32)
    dep = (a > E) & ((a - E) ** 2 > thr * (1 + 1e-6) * (cxx32 + E) * (cyy32 + E))
    ind = ((a + E) ** 2 < thr * (1 - 1e-6) * (cxx32 - E) * (cyy32 - E)) & (cyy32 > E)
    band = ~(dep | ind)
    truth_dep = r2 > thr
    print(f"dep {dep.mean():.4f} ind {ind.mean():.4e} band {band.mean():.3e}")
    print(f"wrong dep: {(dep & ~truth_dep).sum()}  wrong ind: {(ind & truth_dep).sum()}")


if __name__ == "__main__":
    main()
