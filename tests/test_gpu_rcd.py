"""GPU: RCD's discrete path — pcg_chisq_batch against oracle/chisq.py,
the device local_skeleton_discovery against the literal oracle, and rcd() end to end against the
same harness driven by the oracle skeleton. Parity with causal-learn 0.1.2.3 is unpinned."""
import numpy as np
import pytest

from oracle import chisq as och
from rcaeval_amd import synth

pytestmark = pytest.mark.gpu


def _rows(rng, n, count, dmax):
    rows, keys = [], []
    while len(rows) < count:
        d = int(rng.integers(0, dmax + 1))
        v = rng.choice(n, size=d + 2, replace=False)
        a, b = sorted(v[:2].tolist())
        S = sorted(v[2:].tolist())
        rows.append([a, b, d] + S + [-1] * (dmax - d))
        keys.append((a, b, S))
    return np.array(rows, np.int32), keys


@pytest.mark.parametrize("n,N,cmax,dmax,gsq", [(8, 1500, 5, 3, False), (12, 4000, 3, 4, False), (6, 800, 5, 2, True),
                                               (7, 3000, 6, 4, False), (9, 20000, 8, 4, False)])
def test_chisq_batch_matches_oracle(n, N, cmax, dmax, gsq):
    import torch
    from rcaeval_amd.engine import get_engine
    rng = np.random.default_rng(n * N)
    card = rng.integers(2, cmax + 1, n)
    codes = np.stack([rng.integers(0, c, N) for c in card], 1)
    codes[:, 1] = (codes[:, 0] + rng.integers(0, 2, N)) % card[1]          # some dependence
    eng = get_engine(0)
    data = torch.from_numpy(np.ascontiguousarray(codes.T.astype(np.int32))).to(eng.device)
    cd = torch.from_numpy(card.astype(np.int32)).to(eng.device)
    rows, keys = _rows(rng, n, 200, dmax)
    cells = max(int(np.prod(card[S + [a, b]])) for a, b, S in keys)
    stat, df, st = eng.chisq_batch(data, cd, N, n, rows, gsq, cells)
    assert (st == 0).all()
    for r, (a, b, S) in enumerate(keys):
        want, wdf = och.chisq_or_gsq_stat(codes[:, S + [a, b]].T, card[S + [a, b]], gsq)
        assert df[r] == wdf
        if gsq:   # the device log may differ from glibc's in the last bit
            assert abs(stat[r] - want) <= 1e-13 * abs(want), (r, stat[r], want)
        else:     # numpy's blocked pairwise order: bitwise
            assert stat[r] == want, (r, stat[r], want)


def test_chisq_batch_refuses_bad_rows():
    import torch
    from rcaeval_amd.engine import get_engine
    eng = get_engine(0)
    codes = np.random.default_rng(0).integers(0, 3, (500, 5))
    codes[7, 2] = 9                                                     # outside card[2] = 3
    data = torch.from_numpy(np.ascontiguousarray(codes.T.astype(np.int32))).to(eng.device)
    cd = torch.tensor([3, 3, 3, 3, 3], dtype=torch.int32, device=eng.device)
    rows = np.array([[0, 1, 1, 1, -1], [0, 1, 1, 7, -1], [0, 3, 1, 2, -1], [0, 1, 2, 3, 4]], np.int32)
    _, _, st = eng.chisq_batch(data, cd, 500, 5, rows, False, 243)
    assert list(st) == [3, 3, 3, 0]


def _discrete_frame(n, N, seed):
    rng = np.random.default_rng(seed)
    X = synth.gaussian_sem(n, N, seed=seed, w_low=0.5, w_high=1.0, edge_prob=0.3)
    bins = np.quantile(X, [0.2, 0.4, 0.6, 0.8], axis=0)
    codes = np.stack([np.searchsorted(bins[:, j], X[:, j]) for j in range(n)], 1)
    f = (rng.random(N) < 0.5).astype(int)
    codes[:, 0] = np.where(f == 1, (codes[:, 0] + 2) % 5, codes[:, 0])        # the F-node acts on node 0
    return np.concatenate([codes, f[:, None]], 1)


@pytest.mark.parametrize("n,N,seed,alpha", [(6, 1200, 1, 0.01), (10, 2000, 2, 0.05), (15, 3000, 3, 0.2)])
def test_local_skeleton_matches_oracle(n, N, seed, alpha):
    from rcaeval_amd.rcd import local_skeleton_discovery
    data = _discrete_frame(n, N, seed)
    np.random.seed(seed)
    got = local_skeleton_discovery(data, n, alpha)
    np.random.seed(seed)
    want = och.local_skeleton_discovery(data, n, alpha)
    np.testing.assert_array_equal(got.graph, want.graph)
    assert got.no_ci_tests == want.no_ci_tests
    for i in range(n + 1):
        for j in range(n + 1):
            assert got.sepset[i, j] == want.sepset[i, j]
            gp, wp = got.p_values[i, j], want.p_values[i, j]
            assert (gp is None) == (wp is None)
            if gp is not None:
                np.testing.assert_allclose(gp, wp, rtol=1e-12, atol=0)
    assert list(got.mi) == list(want.mi)


def _rcd_frame(m, rows, seed):
    df = synth.telemetry_frame(m, rows, n_constant=0, seed=seed)
    t0 = float(df["time"].iloc[rows // 2])
    col = df.columns[3]
    df.loc[df["time"] >= t0, col] = df.loc[df["time"] >= t0, col] * 3.0 + 5.0   # the root cause
    return df, t0


@pytest.mark.parametrize("m,rows,seed", [(12, 400, 0), (24, 600, 1)])
def test_rcd_end_to_end_matches_oracle_skeleton(m, rows, seed, monkeypatch):
    """rcd(): chunking, k-means bins, alpha sweep and neighbour ordering identical whether the
    skeletons run on the device or in the literal oracle (same global numpy RNG stream)."""
    import rcaeval_amd.rcd as R
    df, t0 = _rcd_frame(m, rows, seed)
    got = R.rcd(df.copy(), t0, seed=seed)["ranks"]

    def oracle_local(data, local_node, alpha, mi=(), labels=None, g_sq=False, device=None):
        return och.local_skeleton_discovery(data, local_node, alpha, mi=mi, labels=labels, G_sq=g_sq)

    monkeypatch.setattr(R, "local_skeleton_discovery", oracle_local)
    want = R.rcd(df.copy(), t0, seed=seed)["ranks"]
    assert got == want and len(got) > 0
