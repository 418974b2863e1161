"""The fp32 screen of k_level_lds_f (rcaeval_amd/csrc/skeleton.hip), emulated in numpy.

The kernel decides a depth-d test (x, y | S = T + {c}) in packed fp32 only when an a-priori
error bound makes the decision certain for the fp64 C; everything else is evaluated in fp64.
This test restates its arithmetic (setup in fp64 on A~ = fp32(C), sweep in float32, the
per-candidate constants, the one-compare dependence check and the rare path's independence
check) and checks on well-conditioned, near-collinear and random correlation matrices that no
test is decided "dependent" or "independent" unless the fp64 decision with the fp64 kernels'
band and conditioning guard (``decide`` in skeleton.hip) says the same. numpy's float32 ops
round once per operation (no FMA); the GPU's fused operations round less, inside the same bound.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

U32 = 2.0 ** -24
KE = 32.0      # = PCG_F32_KE (skeleton.hip)
TAU = 1e-4


def _thresholds(N, d, alpha=0.05):
    from scipy.stats import norm
    r2 = math.tanh(norm.ppf(1 - alpha / 2) / math.sqrt(N - d - 3)) ** 2
    return r2 * (1 - 1e-6), r2 * (1 + 1e-6), 0.5 * math.sqrt(r2)


def _chol(M):
    """Batched Cholesky as the kernels compute it: NaN (not an exception) past a bad pivot."""
    B, k, _ = M.shape
    L = np.zeros_like(M)
    with np.errstate(all="ignore"):
        for j in range(k):
            L[:, j, j] = np.sqrt(M[:, j, j] - (L[:, j, :j] ** 2).sum(1))
            for i in range(j + 1, k):
                L[:, i, j] = (M[:, i, j] - (L[:, i, :j] * L[:, j, :j]).sum(1)) / L[:, j, j]
    return L


def _lower_inv(L):
    """Inverse of a batch of lower-triangular factors (forward substitution, NaN-propagating)."""
    B, k, _ = L.shape
    Li = np.zeros_like(L)
    with np.errstate(all="ignore"):
        for j in range(k):
            Li[:, j, j] = 1.0 / L[:, j, j]
            for i in range(j + 1, k):
                Li[:, i, j] = -(L[:, i, j:i] * Li[:, j:i, j]).sum(1) / L[:, i, i]
    return Li


def _screen(C, x, y, T, c, N):
    """Tests (x, y | T + {c}) of one correlation matrix: see _screen_blocks."""
    idx = np.concatenate([x[:, None], y[:, None], c[:, None], T], axis=1)
    return _screen_blocks(C[idx[:, :, None], idx[:, None, :]], N)


def _screen_blocks(Cb, N):
    """Vectorised over (B, d+2, d+2) blocks ordered (x, y, c, T...): (dep32, ind32, dep64,
    ind64) as the kernel and decide() see them."""
    v = _sweep(Cb, N)
    return v["dep32"], v["ind32"], v["dep64"], v["ind64"]


def _sweep(Cb, N):
    """The kernel's arithmetic on (B, d+2, d+2) blocks ordered (x, y, c, T...) plus the fp64
    truth on C: a dict of the fp32 values (cxx, cyy, cxy as the sweep forms them), nu, E,
    the usability mask and both decisions."""
    B, m, _ = Cb.shape
    d = m - 2
    lo2, hi2, s = _thresholds(N, d)
    inv_s = 1.0 / s
    A = Cb.astype(np.float32).astype(np.float64)         # A~ (LDS)
    f = np.float32
    ar = np.arange(B)
    X, Y, Cc = 0, 1, 2
    Ti = np.arange(3, m)
    # --- setup in fp64 on A~ (kernel: T Cholesky, Li, u_T, candidate row, nu, E, constants)
    CTT = A[:, 3:, 3:]
    L = _chol(CTT)
    gT = np.min(np.diagonal(L, axis1=1, axis2=2) ** 2, axis=1)
    Li = _lower_inv(L)
    uT = np.einsum("bij,bj->bi", Li, A[:, Ti, X])
    liF = (Li * Li).sum((1, 2))
    lc = np.einsum("bij,bj->bi", Li, A[:, Ti, Cc])
    lam2 = A[:, Cc, Cc] - (lc * lc).sum(1)
    r = 1.0 / np.sqrt(lam2)
    u = (A[:, Cc, X] - (lc * uT).sum(1)) * r
    cxx = A[:, X, X] - (uT * uT).sum(1) - u * u
    w = np.einsum("bi,bij->bj", lc, Li)
    nu = np.sqrt(liF + ((w * w).sum(1) + 1.0) * r * r)
    E = KE * U32 * (1 + nu) ** 2
    te = E * inv_s
    g = np.minimum(gT, lam2) - E
    ok = (lam2 > 0) & (te <= 0.5) & (cxx - E > 0) & (g > 0)
    u8 = 8 * U32
    kg = TAU / np.where(g > 0, g, 1.0)
    hx = hi2 * (cxx + E)
    al = hx * (1 + 2 * te) * (1 + u8)
    be = (hx * E + E * s) * (1 + 2 * te) * (1 + u8)
    ga = (cxx - E) * (1 - te) * (1 - u8)
    ka = ((cxx - E) * E + kg + E * s + E * E) * (1 + u8)
    ok &= ga > al
    m_ = (0.5 * (al + ga)).astype(f)
    hh = (0.5 * (ga - al) - 2 * u8 * ga).astype(f)
    k1 = (0.5 * (be - ka)).astype(f)
    k2 = (0.5 * (be + ka) * (1 + u8)).astype(f)
    # --- the y sweep in float32
    Lif, uTf, lcf, rlf, ucf = Li.astype(f), uT.astype(f), lc.astype(f), r.astype(f), u.astype(f)
    mT = A[:, Ti, Y].astype(f)
    vT = np.einsum("bij,bj->bi", Lif, mT).astype(f)
    # the kernel accumulates onto -{A~_yy, A~_xy} (acc = -b after the k products, no separate
    # subtraction): the same order here, one rounding per step
    ay_, ax_ = -A[:, Y, Y].astype(f), -A[:, X, Y].astype(f)
    for i in range(vT.shape[1]):
        ay_ = (ay_ + vT[:, i] * vT[:, i]).astype(f)
        ax_ = (ax_ + uTf[:, i] * vT[:, i]).astype(f)
    byy, bxy = -ay_, -ax_
    sc = (A[:, Cc, Y].astype(f) - (lcf * vT).sum(1, dtype=f)).astype(f)
    vc = (sc * rlf).astype(f)
    cyy = (byy - vc * vc).astype(f)
    cxy = (bxy - ucf * vc).astype(f)
    wv = ((cxy * cxy - k1) - m_ * cyy).astype(f)
    h = (hh * cyy - k2).astype(f)
    dep32 = ok & (np.abs(wv) < h)
    # rare path: certain independence from the constants
    U8 = f(8 * U32)
    Alb = ((m_ + hh) * (f(1) - U8)).astype(f)
    Eub = ((k1 + k2) * f(inv_s) * (f(1) + U8)).astype(f)
    kgub = ((k2 - k1) * (f(1) + U8)).astype(f)
    ay = ((cyy - Eub) * (f(1) - U8)).astype(f)
    ax = ((np.abs(cxy) + Eub) * (f(1) + U8)).astype(f)
    lo2f = f(lo2 * (1 - 4 * U32))
    ind32 = ok & ~dep32 & (ay > 0) & (ax * ax * (f(1) + U8) < lo2f * Alb * ay) & \
        ((ax * ax + kgub) * (f(1) + U8) < Alb * ay)
    # --- fp64 truth on C (Cholesky of C_SS, S = {c} + T, and decide())
    Si = np.arange(2, m)
    LS = _chol(Cb[:, 2:, 2:])
    gmin = np.min(np.diagonal(LS, axis1=1, axis2=2) ** 2, axis=1)
    LSi = _lower_inv(LS)
    ux = np.einsum("bij,bj->bi", LSi, Cb[:, Si, X])
    vy = np.einsum("bij,bj->bi", LSi, Cb[:, Si, Y])
    cxx64 = Cb[:, X, X] - (ux * ux).sum(1)
    cyy64 = Cb[:, Y, Y] - (vy * vy).sum(1)
    cxy64 = Cb[:, X, Y] - (ux * vy).sum(1)
    den, num = cxx64 * cyy64, cxy64 * cxy64
    guard = (gmin > 0) & (den > 0) & (den - num > TAU / gmin)
    dep64 = guard & (num > hi2 * den)
    ind64 = guard & (num < lo2 * den)
    return {"dep32": dep32, "ind32": ind32, "dep64": dep64, "ind64": ind64, "ok": ok, "nu": nu,
            "cxx32": cxx.astype(f).astype(np.float64), "cyy32": cyy.astype(np.float64), "cxy32": cxy.astype(np.float64),
            "cxx64": cxx64, "cyy64": cyy64, "cxy64": cxy64}


def _tests(C, rng, count, d=4):
    n = len(C)
    idx = np.argsort(rng.random((count, n)), axis=1)[:, : d + 2]
    x, y = idx[:, 0], idx[:, 1]
    S = np.sort(idx[:, 2:], axis=1)
    return x, y, S[:, 1:], S[:, 0]


def _corr(X):
    return np.corrcoef(X, rowvar=False)


def _sem(n, N, rng, w=(0.1, 0.5)):
    X = rng.standard_normal((N, n))
    for j in range(1, n):
        par = rng.choice(j, size=min(j, 3), replace=False)
        X[:, j] += X[:, par] @ (rng.uniform(*w, size=len(par)) * rng.choice([-1, 1], size=len(par)))
    return X


@pytest.mark.parametrize("case", ["sem", "near_dup", "near_lincomb", "random"])
def test_screen32_never_wrong(case):
    rng = np.random.default_rng({"sem": 0, "near_dup": 1, "near_lincomb": 2, "random": 3}[case])
    N, n = 10000, 40
    X = _sem(n, N, rng)
    if case == "near_dup":                  # duplicated metrics with tiny noise
        for j in range(0, n, 5):
            X[:, j + 1] = X[:, j] + rng.standard_normal(N) * 10.0 ** rng.uniform(-7, -2)
    elif case == "near_lincomb":            # a column nearly a combination of others
        for j in range(3, n, 4):
            X[:, j] = X[:, j - 1] - 0.7 * X[:, j - 2] + 0.3 * X[:, j - 3] + rng.standard_normal(N) * 1e-4
    elif case == "random":
        X = rng.standard_normal((N, n)) @ rng.standard_normal((n, n)) * 0.3 + rng.standard_normal((N, n))
    C = _corr(X)
    x, y, T, c = _tests(C, rng, 60000)
    with np.errstate(all="ignore"):
        dep32, ind32, dep64, ind64 = _screen(C, x, y, T, c, N)
    assert not np.any(dep32 & ~dep64), "fp32 screen called a test dependent that fp64 does not"
    assert not np.any(ind32 & ~ind64), "fp32 screen called a test independent that fp64 does not"
    if case == "sem":
        # the screen decides nearly everything on well-conditioned data
        assert (dep32 | ind32).mean() > 0.995


def test_screen32_near_threshold():
    """Tests whose r^2 is placed at thr * (1 + delta), delta in [-3e-2, 3e-2] (C_xy moved so the
    partial correlation given S hits the target; c_xx, c_yy do not depend on C_xy): the screen
    never decides across the threshold, and it leaves only a narrow band to the fp64 path."""
    rng = np.random.default_rng(7)
    N, n, B = 10000, 30, 40000
    C = _corr(_sem(n, N, rng))
    x, y, T, c = _tests(C, rng, B)
    idx = np.concatenate([x[:, None], y[:, None], c[:, None], T], axis=1)
    Cb = C[idx[:, :, None], idx[:, None, :]].copy()
    _, hi2, _ = _thresholds(N, 4)
    thr = hi2 / (1 + 1e-6)
    LS = np.linalg.cholesky(Cb[:, 2:, 2:])
    LSi = np.linalg.inv(LS)
    ux = np.einsum("bij,bj->bi", LSi, Cb[:, 2:, 0])
    vy = np.einsum("bij,bj->bi", LSi, Cb[:, 2:, 1])
    cxx = Cb[:, 0, 0] - (ux * ux).sum(1)
    cyy = Cb[:, 1, 1] - (vy * vy).sum(1)
    delta = rng.uniform(-3e-2, 3e-2, B)
    rt = np.sqrt(thr * (1 + delta)) * rng.choice([-1.0, 1.0], B)
    cxy_new = (ux * vy).sum(1) + rt * np.sqrt(cxx * cyy)
    Cb[:, 0, 1] = Cb[:, 1, 0] = cxy_new
    dep32, ind32, dep64, ind64 = _screen_blocks(Cb, N)
    assert not np.any(dep32 & ~dep64)
    assert not np.any(ind32 & ~ind64)
    decided = dep32 | ind32
    assert decided[np.abs(delta) > 2e-2].mean() > 0.95


def _err_ratio(Cb, N=10000):
    """max over (c_xx, c_yy, c_xy) of |fp32 sweep value - fp64 value on C| / (K u (1 + nu)^2),
    K = KE = 32 (the derived bound, DESIGN.md "fp32 screen: error bound"; the kernel's E is
    2 KE u (1 + nu^2) >= this), per block; NaN where the candidate is unusable (ok false: the
    test never reaches the fp32 decision)."""
    with np.errstate(all="ignore"):
        v = _sweep(Cb, N)
        bound = KE * U32 * (1 + v["nu"]) ** 2
        err = np.maximum.reduce([np.abs(v["cxx32"] - v["cxx64"]), np.abs(v["cyy32"] - v["cyy64"]),
                                 np.abs(v["cxy32"] - v["cxy64"])])
        r = err / bound
    return np.where(v["ok"], r, np.nan)


def _blocks_from(Z, eps):
    """(B, 6, 6) correlation blocks Z Z^T + eps I (PSD), normalised to unit diagonal."""
    G = Z @ np.swapaxes(Z, 1, 2) + eps[:, None, None] * np.eye(Z.shape[1])
    s = 1.0 / np.sqrt(np.einsum("bii->bi", G))
    return G * s[:, :, None] * s[:, None, :]


def test_screen32_adversarial_error_ratio():
    """Adversarial search for the worst fp32-sweep error relative to the bound the screen
    relies on: blocks with near-collinear conditioning sets (nu up to the screen's cut-off,
    te = E / s <= 1/2), x and y nearly determined by S (small c_xx, c_yy), entries placed a
    half fp32 ulp from a rounding boundary; then a random hill-climb on the worst blocks. The
    derived bound needs K ~ 18; KE = 32. The worst ratio found must stay < 1/2."""
    rng = np.random.default_rng(2024)
    B, r = 512, 6
    worst = 0.0
    # starting population: factor models with a nearly collinear T / c block
    Z = rng.standard_normal((B, 6, r))
    lam = 10.0 ** rng.uniform(-4, -0.5, (B, 1))
    Z[:, 3, :] = Z[:, 2, :] + lam * rng.standard_normal((B, r))                  # T0 ~ c
    Z[:, 4, :] = Z[:, 3, :] * 0.5 + Z[:, 2, :] * 0.5 + lam * rng.standard_normal((B, r))
    Z[:, 0, :] = Z[:, 2, :] + 10.0 ** rng.uniform(-3, -1, (B, 1)) * rng.standard_normal((B, r))   # x ~ S
    Z[:, 1, :] = Z[:, 4, :] + 10.0 ** rng.uniform(-3, -1, (B, 1)) * rng.standard_normal((B, r))   # y ~ S
    eps = 10.0 ** rng.uniform(-6, -2, B)
    score = np.nan_to_num(_err_ratio(_blocks_from(Z, eps)), nan=-1.0)
    for it in range(300):
        step = 10.0 ** rng.uniform(-4, -1, (B, 1, 1))
        Zn = Z + step * rng.standard_normal(Z.shape)
        en = eps * 10.0 ** rng.uniform(-0.3, 0.3, B)
        Cn = _blocks_from(Zn, en)
        if it % 3 == 2:        # push entries to just below / above an fp32 rounding boundary
            f = Cn.astype(np.float32).astype(np.float64)
            ulp = np.spacing(np.abs(f).astype(np.float32)).astype(np.float64)
            Cn = f + np.sign(rng.standard_normal(Cn.shape)) * 0.4999 * ulp
            Cn = 0.5 * (Cn + np.swapaxes(Cn, 1, 2))
            np.einsum("bii->bi", Cn)[:] = 1.0
        sn = np.nan_to_num(_err_ratio(Cn), nan=-1.0)
        better = sn > score
        Z[better], eps[better], score[better] = Zn[better], en[better], sn[better]
        worst = max(worst, float(score.max()))
    print(f"worst |err| / (KE u (1 + nu)^2) found: {worst:.4f} (usable blocks: {(score >= 0).mean():.2f})")
    assert (score >= 0).mean() > 0.3, "search left the screen's usable region"
    assert worst < 0.5, worst
