"""GPU parity: K1 correlation and K2/K3 skeleton vs the CPU oracle (C restatement).

Tolerances (north_star): p-values |dp| <= 1e-9 |p_ref| + 2^-51 (fisherz.p_close);
skeleton (removal depth of every pair) and sepset unions bit-identical; decisions may differ
only for tests with |p - alpha| < 1e-9, which the engine enumerates (near_alpha list).
"""
import numpy as np
import pytest

from oracle import cpc, fisherz
from rcaeval_amd import _lib, synth
from tests_support import assert_skeleton_matches, unions_from_engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from rcaeval_amd.engine import get_engine
    return get_engine(0)


def _key(r):
    return (int(r["a"]), int(r["b"]), tuple(int(v) for v in r["s"][: r["d"]]))


CASES = [  # (n, N, seed, w_low, w_high, edge_prob)
    (8, 300, 0, 0.3, 0.9, None),
    (20, 500, 1, 0.3, 0.9, None),
    (30, 2000, 2, 0.1, 0.5, None),
    (50, 600, 3, 0.3, 0.9, 0.1),
    (64, 1000, 4, 0.2, 0.8, 0.08),
    (65, 800, 5, 0.2, 0.8, 0.08),
    (130, 3000, 6, 0.1, 0.5, None),
]


@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES)
def test_corr_matches_numpy(eng, n, N, seed, wl, wh, ep):
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = eng.corr(X).cpu().numpy()
    ref = np.corrcoef(X.T)
    np.testing.assert_allclose(C, ref, rtol=0, atol=2e-14)


@pytest.mark.parametrize("n", [70, 300])
@pytest.mark.parametrize("kind", ["spikes", "scales", "constant", "nonfinite"])
def test_corr_hard_columns_match_numpy(eng, kind, n):
    """K1 on columns that stress a per-column fixed-point split: heavy-tailed spikes (max/rms ~
    100), scales from 1e-8 to 1e7 (memory bytes) plus a large offset, constant columns (numpy's
    0/0 NaN), and NaN / inf columns (NaN row and column). n = 70 runs the digit GEMMs, n = 300
    the CRT residue GEMMs."""
    rng = np.random.default_rng({"spikes": 1, "scales": 2, "constant": 3, "nonfinite": 4}[kind])
    N = 3000
    X = synth.gaussian_sem(n, N, seed=11, w_low=0.2, w_high=0.8)
    if kind == "spikes":
        for j in range(0, n, 3):
            X[rng.integers(0, N, 3), j] += rng.choice([-1, 1], 3) * 100 * X[:, j].std()
    elif kind == "scales":
        X *= 10.0 ** rng.uniform(-8, 7, n)
        X[:, 5] += 1e9
    elif kind == "constant":           # exactly summable: mean exact, variance 0, numpy's 0/0
        X[:, 3] = 0.0
        X[:, 7] = 2.5
    else:
        X[17, 4] = np.nan
        X[5, 8] = np.inf
    with np.errstate(invalid="ignore", divide="ignore"):
        ref = np.corrcoef(X.T)
    C = eng.corr(X).cpu().numpy()
    np.testing.assert_array_equal(np.isnan(C), np.isnan(ref))
    ok = ~np.isnan(ref)
    np.testing.assert_allclose(C[ok], ref[ok], rtol=0, atol=2e-14)


@pytest.mark.parametrize("n,N", [(256, 1000), (300, 1200), (513, 4097), (700, 33), (260, 40000), (2000, 10000)])
def test_corr_crt_matches_numpy(eng, n, N):
    """The CRT K1 (n >= 256: residue GEMMs, exact integer Gram of the b-bit truncated values,
    rounded once): ragged tiles (n = 300, 513, 700), a single k-block (N = 33), many slabs
    (N = 40000), the headline shape. Same tolerance as the digit path."""
    X = synth.gaussian_sem(n, N, seed=n + 7 * N, w_low=0.1, w_high=0.5)
    C = eng.corr(X).cpu().numpy()
    np.testing.assert_allclose(C, np.corrcoef(X.T), rtol=0, atol=2e-14)


@pytest.mark.parametrize("N", [778, 40000])
def test_corr_crt_extreme_magnitudes(eng, N):
    """The CRT rebuild at the top of its range: every centred value of a column has the same
    magnitude just below a power of two (balanced signs, so the mean is exactly 0 and |a| =
    trunc((1 - 2^-40) 2^b): the Gram entries reach (1 - 2^-39) N 4^b, the bound M / 2 is built
    for); three sign patterns shared by column groups: C is the +-1 pattern numpy gives (within its
    rounding) inside a group."""
    rng = np.random.default_rng(N)
    n = 300
    base = np.repeat([-1.0, 1.0], N // 2)
    sgn = np.stack([rng.permutation(base) for _ in range(3)], axis=1)
    grp = np.arange(n) % 3
    mag = (1.0 - 2.0 ** -40) * 2.0 ** rng.integers(-20, 20, n).astype(np.float64)
    X = np.ascontiguousarray(sgn[:, grp] * mag * np.where(np.arange(n) % 2, 1.0, -1.0))
    assert np.all(X.mean(axis=0) == 0.0)
    C = eng.corr(X).cpu().numpy()
    ref = np.corrcoef(X.T)
    np.testing.assert_allclose(C, ref, rtol=0, atol=2e-14)
    same = grp[:, None] == grp[None, :]
    assert np.all(np.abs(np.abs(C[same]) - 1.0) < 1e-14)


@pytest.mark.parametrize("n,N", [(300, 1200), (2000, 10000)])
def test_corr_crt_split_invariant(eng, n, N):
    """The CRT result is the correctly rounded exact Gram, so every split-K choice gives the same
    bits; a forced split-K that the rounding cannot reach takes the nearest reachable one (its
    plan signature says which ran); the digit path (PCG_TUNE_K1_CRT = 0) agrees to within
    its own truncation."""
    X = synth.gaussian_sem(n, N, seed=5, w_low=0.1, w_high=0.5)
    Xd = eng.to_device(X)
    C0 = eng.corr(Xd).cpu().numpy()

    def achievable(N):
        """split-K counts the plan's k-block rounding can reach (corr.hip crt_plan: TB k-blocks of
        32 rows rounded per slab to a multiple of CRT_KB = 4)"""
        TB = (N + 63) // 64 * 2
        out = []
        for ks in range(1, 17):
            kbk = -(-TB // ks)
            kbk = -(-kbk // 4) * 4
            if -(-TB // kbk) == ks:
                out.append(ks)
        return out
    reach = achievable(N)
    for ks in (1, 3, 7):
        with eng.tuned(K1_CRT_KS=ks):
            np.testing.assert_array_equal(eng.corr(Xd).cpu().numpy(), C0)
            # the plan takes the forced count, or the nearest count the rounding can reach
            got = (eng.k1_plan_signature(n, N) >> 32) & 0xFF
            assert got == min(reach, key=lambda r: (abs(r - ks), r)), (ks, got, reach)
    with eng.tuned(K1_CRT=0):
        Cd = eng.corr(Xd).cpu().numpy()
    np.testing.assert_allclose(Cd, C0, rtol=0, atol=1e-15)


@pytest.mark.parametrize("n,N", [(44, 7000), (3, 40000), (130, 8193), (200, 33), (64, 32 * 256 + 5)])
def test_corr_small_n_many_slabs(eng, n, N):
    """Small n splits K into up to 256 slabs of >= 32 rows (RQ2-shaped cases); ragged N and the
    single-slab tiny-N case included. Same tolerance as the numpy comparison above."""
    X = synth.gaussian_sem(n, N, seed=n + N, w_low=0.1, w_high=0.5)
    C = eng.corr(X).cpu().numpy()
    np.testing.assert_allclose(C, np.corrcoef(X.T), rtol=0, atol=2e-14)


@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES)
@pytest.mark.parametrize("flags", [0, _lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD])
@pytest.mark.parametrize("small", [1, 0])
def test_skeleton_matches_oracle(eng, n, N, seed, wl, wh, ep, flags, small):
    """Both drivers: n <= 64 runs the single-workgroup small-graph kernel (k_pc_small) unless
    PCG_TUNE_SMALL = 0 sends it through the level loop; larger n always take the level loop
    (pcg_stats.driver says which one produced the result)."""
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, N, record_cap=2_000_000)
    with eng.tuned(SMALL=small):
        out = eng.skeleton(C, N, flags=flags, record_capacity=2_000_000)
    assert out.stats["driver"] == ("small" if small and n <= 64 else "levels")
    assert_skeleton_matches(out, ref, n)
    if flags & _lib.PCG_FLAG_RECORD:
        d = {_key(r): r["p"] for r in ref.records}
        g = {_key(r): r["p"] for r in out.records}
        assert set(g) == set(d)
        keys = sorted(d)
        ok = fisherz.p_close([g[k] for k in keys], [d[k] for k in keys])
        assert ok.all(), [(keys[i], g[keys[i]], d[keys[i]]) for i in np.nonzero(~ok)[0][:5]]


@pytest.mark.parametrize("narrow", [4, 16])
@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES)
def test_wide_and_large_classes_match_oracle(eng, n, N, seed, wl, wh, ep, narrow):
    """Nodes above `narrow` neighbours leave the LDS-resident class: at the T-group depths they
    run the WIDE (128-bit mask) T-group kernel, elsewhere the staged kernels — the skeleton,
    the unions and the per-level test counts stay the oracle's."""
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, N)
    _lib.check(eng.h, eng.lib.pcg_set_narrow_degree(eng.h, narrow), "pcg_set_narrow_degree")
    try:
        with eng.tuned(SMALL=0):   # the level-loop kernels under test, also at n <= 64
            out = eng.skeleton(C, N)
    finally:
        eng.lib.pcg_set_narrow_degree(eng.h, 64)
    assert out.stats["driver"] == "levels"
    assert_skeleton_matches(out, ref, n)


@pytest.mark.parametrize("mask", [0, 0x1c])
@pytest.mark.parametrize("narrow", [64, 16])
@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES[2:])
def test_screen_precision_masks_match_oracle(eng, n, N, seed, wl, wh, ep, narrow, mask):
    """The fp32-screened T-group sweep (k_level_lds_f) against the all-fp64 one (mask 0) and
    with depth 2 screened too (0x1c), narrow and wide classes: identical skeletons, unions and
    per-level counts (PCG_TUNE_SCREEN_MASK)."""
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, N)
    _lib.check(eng.h, eng.lib.pcg_set_narrow_degree(eng.h, narrow), "pcg_set_narrow_degree")
    try:
        with eng.tuned(SMALL=0, SCREEN_MASK=mask):   # the level-loop kernels, also at n <= 64
            out = eng.skeleton(C, N)
    finally:
        eng.lib.pcg_set_narrow_degree(eng.h, 64)
    assert_skeleton_matches(out, ref, n)
    if mask == 0:
        assert sum(out.stats["screened"]) == 0


@pytest.mark.parametrize("blocks", [0, 0x10, 0x18])
@pytest.mark.parametrize("n,N,seed", [(300, 2000, 7), (700, 5000, 9)])
def test_node_images_match_oracle(eng, n, N, seed, blocks):
    """The fp32 sweep's staging choices (PCG_TUNE_NODE_BLOCKS): gathered from C (0), the fp32 LDS
    images built by k_node_blocks_t<true> and copied by LDS-DMA at depth 4 (0x10, the default) and
    at depths 3 and 4 (0x18); with depth 4 dispatched largest degree first. Removal depths,
    per-level counts and sepset unions equal the C oracle's at unlimited depth."""
    X = synth.gaussian_sem(n, N, seed=seed, w_low=0.1, w_high=0.5, edge_prob=8.0 / n)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, N)
    with eng.tuned(SMALL=0, NODE_BLOCKS=blocks):
        out = eng.skeleton(C, N)
    assert_skeleton_matches(out, ref, n)
    assert out.levels >= 5, out.levels


def _star(m, N, seed):
    """A common cause z (column 0) of m children: complete after depth 0, every child pair
    separated by {z} at depth 1 (~m^2/2 independent tests in the block of z)."""
    rng = np.random.default_rng(seed)
    z = rng.standard_normal(N)
    a = rng.uniform(0.5, 0.9, m)
    return np.column_stack([z, z[:, None] * a + rng.standard_normal((N, m))])


@pytest.mark.parametrize("l1z", [1, 0])
@pytest.mark.parametrize("case", ["star", "sem"])
def test_depth1_grouping_matches_oracle(eng, case, l1z):
    """Depth 1 grouped by conditioning node (k_level1_z, PCG_TUNE_L1Z = 1, the default) and the
    neighbour-pair kernel (0): equal skeletons, unions and per-level counts. The star's block
    of z holds ~1.3e4 mirror union bits (an independent (x, t | z) with z in adj(t) also marks
    the pair's other ordered side), past the kernel's 512-entry LDS list, so the inline search
    runs too."""
    if case == "star":   # (depth <= 2: the hub keeps its 160 edges, so deeper levels explode)
        X, N, md = _star(160, 3000, 11), 3000, 2
    else:
        N, md = 3000, -1
        X = synth.gaussian_sem(300, N, seed=12, w_low=0.2, w_high=0.6, edge_prob=0.05)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, N, max_depth=md)
    with eng.tuned(L1Z=l1z):
        out = eng.skeleton(C, N, max_depth=md)
    assert out.stats["driver"] == "levels"
    assert_skeleton_matches(out, ref, X.shape[1])
    if case == "star":
        assert out.stats["indep"][1] > 10000, out.stats["indep"]


def test_screen_list_overflow_reruns(eng):
    """A screen list too small for the fp32 sweep's undecided tests (config 5, depth <= 3:
    ~9e4 of them at depth 3) overflows, the level reports it with the capacity raised, and
    pcg_skeleton reruns: the result equals a run with room to spare."""
    X = synth.gaussian_sem(2000, 10000, seed=0)
    C = eng.corr(X)
    a = eng.skeleton(C, 10000, max_depth=3)
    assert a.stats["screened"][3] > 1000
    _lib.check(eng.h, eng.lib.pcg_set_screen_capacity(eng.h, 1000), "pcg_set_screen_capacity")
    b = eng.skeleton(C, 10000, max_depth=3)
    assert b.stats["screened"] == a.stats["screened"]
    assert b.stats["tests"] == a.stats["tests"] and b.stats["indep"] == a.stats["indep"]
    assert np.array_equal(b.removed_level, a.removed_level)


@pytest.mark.parametrize("noise", [1e-2, 1e-4, 1e-6, 1e-7])
@pytest.mark.parametrize("flags", [0, _lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD])
def test_near_collinear_columns_match_lu_oracle(eng, noise, flags):
    """Ill-conditioned sub-matrices (near-duplicate columns and a near linear combination, as
    RCAEval metric sets have them): the fast Cholesky paths must hand these tests to the exact
    LU path (conditioning guard, skeleton.hip decide) so that every decision and p-value is
    numpy.linalg.inv's (the C oracle's LU)."""
    rng = np.random.default_rng(11)
    X = synth.gaussian_sem(40, 800, seed=12, w_low=0.2, w_high=0.8, edge_prob=0.1)
    for j, i in ((5, 3), (17, 9), (30, 31), (22, 5)):
        X[:, j] = X[:, i] + noise * rng.standard_normal(len(X))
    X[:, 38] = X[:, 1] - 0.5 * X[:, 2] + noise * rng.standard_normal(len(X))
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, 800, record_cap=2_000_000)
    if ref.error:
        with pytest.raises(ValueError):
            eng.skeleton(C, 800, flags=flags, record_capacity=2_000_000)
        return
    out = eng.skeleton(C, 800, flags=flags, record_capacity=2_000_000)
    assert_skeleton_matches(out, ref, 40)
    if flags & _lib.PCG_FLAG_RECORD:
        d = {_key(r): r["p"] for r in ref.records}
        g = {_key(r): r["p"] for r in out.records}
        assert set(g) == set(d)
        keys = sorted(d)
        ok = fisherz.p_close([g[k] for k in keys], [d[k] for k in keys])
        assert ok.all(), [(keys[i], g[keys[i]], d[keys[i]]) for i in np.nonzero(~ok)[0][:5]]


def test_decide_and_fullp_agree_2000_depth2(eng):
    """Full-size (2000 vars) parity at depth <= 2 against the C oracle, threshold and full-p."""
    X = synth.gaussian_sem(2000, 10000, seed=0)
    C = eng.corr(X)
    Ch = C.cpu().numpy()
    ref = cpc.skeleton(Ch, 10000, max_depth=2, want_union=True)
    a = eng.skeleton(C, 10000, max_depth=2, flags=0)
    b = eng.skeleton(C, 10000, max_depth=2, flags=_lib.PCG_FLAG_FULL_P)
    for out in (a, b):
        assert_skeleton_matches(out, ref, 2000)


@pytest.mark.timeout(900)
def test_config5_full_depth4_matches_oracle(eng, config5):
    """BASELINE config 5 at full size and full depth: 2000 vars x 10 000 samples, seed 0,
    max_depth 4 — the benchmarked workload, whose depth 4 (83 % of the 4.9e9 unique tests) runs
    on the dominant k_level_lds_f<4> kernel (the fp32-screened sweep). Threshold-mode removal depth of every pair from
    pcg_pc_skeleton (K1 + skeleton in one call), per-level unique-test counts and sepset unions
    against the C oracle on np.corrcoef(X.T) (only pairs touched by an enumerated |p - alpha| < 1e-9 test are exempt); then the
    full-p kernels on the same graph, with recorded p of a fixed pair sample (1 in 4099 pairs,
    every depth) within 1e-9 relative (+2^-51) of the oracle's FisherZ."""
    import sys
    X, Ch, ref = config5
    # K1 + skeleton through the one C call (pcg_pc_skeleton); the oracle runs on numpy's
    # corrcoef, so the correlation kernel is inside the end-to-end comparison
    a, C = eng.corr_skeleton(X, max_depth=4, flags=0)
    assert np.abs(C.cpu().numpy() - Ch).max() <= 2e-14
    assert a.levels == 5 and sum(a.stats["tests"]) > 4.5e9
    b = eng.skeleton(C, 10000, max_depth=4, flags=_lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD,
                     record_capacity=4_000_000, record_sample=(4099, 17))
    print(f"near-alpha: oracle {len(ref.near_alpha)} / engine {len(a.near_alpha)}", file=sys.stderr, flush=True)
    flips = assert_skeleton_matches(a, ref, 2000)
    flips_b = assert_skeleton_matches(b, ref, 2000)
    # the fp32-screened sweep (default at depths 3-4) left only a small share to its fp64
    # screen; the all-fp64 T-group sweep gives the same skeleton
    assert 0 < a.stats["screened"][4] < 1e-3 * a.stats["tests"][4], a.stats["screened"]
    _lib.check(eng.h, eng.lib.pcg_set_screen_precision(eng.h, 0), "pcg_set_screen_precision")
    try:
        c = eng.skeleton(C, 10000, max_depth=4, flags=0)
    finally:
        eng.lib.pcg_set_screen_precision(eng.h, 1)
    assert sum(c.stats["screened"]) == 0
    assert_skeleton_matches(c, ref, 2000)
    print(f"near-alpha flips: threshold {flips}, full-p {flips_b}", file=sys.stderr, flush=True)
    rec = b.records
    per_depth = np.bincount(rec["d"], minlength=5)
    assert (per_depth[:5] > 100).all(), per_depth
    p_ref = np.empty(len(rec))
    for d in range(5):
        sel = np.nonzero(rec["d"] == d)[0]
        ab = np.ascontiguousarray(np.stack([rec["a"][sel], rec["b"][sel]], 1), dtype=np.int32)
        S = np.ascontiguousarray(rec["s"][sel, :max(d, 1)], dtype=np.int32)
        pr, err = cpc.fisherz_batch(Ch, 10000, ab, S, d)
        assert not err.any()
        p_ref[sel] = pr
    ok = fisherz.p_close(rec["p"], p_ref)
    assert ok.all(), [(rec[i], p_ref[i]) for i in np.nonzero(~ok)[0][:3]]


def test_constant_column_nan_is_dependent(eng):
    X = synth.gaussian_sem(12, 400, seed=7, w_low=0.3, w_high=0.9)
    X[:, 5] = 3.0                                   # constant -> NaN correlations -> p NaN
    with np.errstate(invalid="ignore", divide="ignore"):
        C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, 400)
    out = eng.skeleton(C, 400)
    np.testing.assert_array_equal(out.removed_level, ref.removed_level)
    assert (out.removed_level[5] == -1).sum() == 12   # NaN p never removes an edge (+ diagonal)


def test_duplicate_column_singular_raises(eng):
    X = synth.gaussian_sem(10, 300, seed=8, w_low=0.3, w_high=0.9)
    X[:, 3] = X[:, 2]
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, 300)
    if ref.error:
        with pytest.raises(ValueError):
            eng.skeleton(C, 300)


def test_tiny_sample_dof(eng):
    X = synth.gaussian_sem(6, 6, seed=9, w_low=0.3, w_high=0.9)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, 6)
    if ref.error:
        with pytest.raises(ValueError):
            eng.skeleton(C, 6)
    else:
        out = eng.skeleton(C, 6)
        np.testing.assert_array_equal(out.removed_level, ref.removed_level)


def test_max_depth_cap(eng):
    X = synth.gaussian_sem(40, 1000, seed=10, w_low=0.2, w_high=0.8, edge_prob=0.1)
    C = np.corrcoef(X.T)
    for md in (0, 1, 2):
        ref = cpc.skeleton(C, 1000, max_depth=md)
        out = eng.skeleton(C, 1000, max_depth=md)
        assert out.levels == ref.levels <= md + 1
        np.testing.assert_array_equal(out.removed_level, ref.removed_level)


@pytest.mark.parametrize("n,N,world", [(50, 600, 2), (130, 3000, 3), (300, 1200, 8), (700, 5000, 3),
                                       (2000, 10000, 8)])
def test_sharded_corr_bitwise_equals_single_gpu(eng, n, N, world):
    """K1 sharded over `world` ranks (each rank's packed share computed here in turn on one
    GPU, then concatenated rank-major as the all-gather would) is bitwise pcg_corr."""
    import torch
    X = synth.gaussian_sem(n, N, seed=n, w_low=0.1, w_high=0.5)
    Xd = eng.to_device(X)
    C1 = eng.corr(Xd)
    parts = [eng.corr_shard(Xd, r, world) for r in range(world)]
    Cw = eng.corr_shard_finish(torch.cat(parts), N, n, world)
    assert torch.equal(C1, Cw)
    if n <= 300:
        np.testing.assert_allclose(C1.cpu().numpy(), np.corrcoef(X.T), rtol=0, atol=2e-14)


def test_corr_shard_finish_refuses_exponents_of_another_call(eng):
    """The CRT finish reads the column exponents pcg_corr_shard left on the handle: a K1 call of
    another shape in between (or none at all) makes pcg_corr_shard_finish fail with
    PCG_ERR_INVALID instead of rebuilding C from foreign exponents."""
    import torch
    from rcaeval_amd import _lib
    n, N, world = 300, 1200, 2
    X = synth.gaussian_sem(n, N, seed=3, w_low=0.1, w_high=0.5)
    Xd = eng.to_device(X)
    parts = torch.cat([eng.corr_shard(Xd, r, world) for r in range(world)])
    eng.corr(eng.to_device(synth.gaussian_sem(400, 1500, seed=4)))
    with pytest.raises(_lib.PcgError) as e:
        eng.corr_shard_finish(parts, N, n, world)
    assert e.value.code == _lib.PCG_ERR_INVALID
    parts = torch.cat([eng.corr_shard(Xd, r, world) for r in range(world)])
    assert torch.equal(eng.corr_shard_finish(parts, N, n, world), eng.corr(Xd))


@pytest.mark.parametrize("n,N,max_depth", [(300, 1200, -1), (2000, 10000, 2)])
def test_native_sharded_single_rank_equals_single_gpu(eng, n, N, max_depth):
    """pcg_comm_init / pcg_corr_sharded / pcg_skeleton_sharded (the C-side RCCL driver) on a
    one-rank communicator: every collective runs; C is bitwise pcg_corr's, the skeleton,
    counters and sepset unions equal pcg_skeleton's."""
    import torch
    from rcaeval_amd._lib import check
    X = synth.gaussian_sem(n, N, seed=21)
    eng.comm_init(eng.comm_unique_id(), 0, 1)
    C1 = eng.corr(X)
    C2 = eng.corr_sharded(X)
    assert torch.equal(C1, C2)
    a = eng.skeleton(C1, N, max_depth=max_depth)
    b = eng.skeleton_sharded(C1, N, max_depth=max_depth)
    np.testing.assert_array_equal(a.removed_level, b.removed_level)
    assert a.stats["tests"] == b.stats["tests"] and a.stats["indep"] == b.stats["indep"]
    assert unions_from_engine(a) == unions_from_engine(b)
    check(eng.h, eng.lib.pcg_comm_destroy(eng.h), "pcg_comm_destroy")


@pytest.mark.parametrize("n", [2, 63, 64, 65, 130, 2000])
def test_packed_barrier_or_merges_ranks(eng, n):
    """pcg_level_pack / pcg_level_merge: the OR of three ranks' symmetric removal flags (and
    their status bytes) comes back byte-exact in both triangles; a rank that reports a local
    failure contributes no flags and sets status byte 3 (pcg_level_end -> PCG_ERR_PEER)."""
    import ctypes
    import torch
    lib, h = eng.lib, eng.h
    C = torch.eye(n, dtype=torch.float64, device=eng.device)
    rl = torch.empty((n, n), dtype=torch.int8, device=eng.device)
    rm = torch.zeros(n * n + _lib.PCG_RM_STATUS, dtype=torch.uint8, device=eng.device)
    _lib.check(h, lib.pcg_set_removal_buffer(h, ctypes.c_void_p(rm.data_ptr()), rm.numel()), "rm")
    try:
        _lib.check(h, lib.pcg_skeleton_init(h, ctypes.c_void_p(C.data_ptr()), n, n, 100, 0.05, 0,
                                            ctypes.c_void_p(rl.data_ptr())), "init")
        total = ctypes.c_int64()
        assert lib.pcg_level_begin(h, 0, ctypes.byref(total), None, None) == 0
        words = ctypes.c_int64()
        _lib.check(h, lib.pcg_level_packed_words(n, ctypes.byref(words)), "words")
        rng = np.random.default_rng(n)
        want = np.zeros((n, n), bool)
        parts = []
        for r in range(3):
            f = np.triu(rng.random((n, n)) < 0.1, 1)
            f |= f.T
            status = np.zeros(_lib.PCG_RM_STATUS, np.uint8)
            status[r % 3] = r == 2            # rank 2 raises the domain-error byte
            rm.copy_(torch.from_numpy(np.concatenate([f.reshape(-1).astype(np.uint8), status])))
            packed = torch.empty(words.value, dtype=torch.int64, device=eng.device)
            _lib.check(h, lib.pcg_level_pack(h, ctypes.c_void_p(packed.data_ptr()), 0), "pack")
            parts.append(packed)
            want |= f
        failed = torch.empty(words.value, dtype=torch.int64, device=eng.device)
        _lib.check(h, lib.pcg_level_pack(h, ctypes.c_void_p(failed.data_ptr()), 1), "pack failed rank")
        rm.fill_(7)
        g = torch.cat(parts)
        _lib.check(h, lib.pcg_level_merge(h, ctypes.c_void_p(g.data_ptr()), 3), "merge")
        eng.sync()
        got = rm[:n * n].cpu().numpy().reshape(n, n)
        np.testing.assert_array_equal(got, want.astype(np.uint8))
        st = rm[n * n:n * n + 8].cpu().numpy()
        assert list(st[:4]) == [0, 0, 1, 0]
        g2 = torch.cat(parts + [failed])
        _lib.check(h, lib.pcg_level_merge(h, ctypes.c_void_p(g2.data_ptr()), 4), "merge with failed rank")
        eng.sync()
        np.testing.assert_array_equal(rm[:n * n].cpu().numpy().reshape(n, n), want.astype(np.uint8))
        assert rm[n * n + 3].item() == 1
        assert lib.pcg_level_end(h, None) == _lib.PCG_ERR_PEER
    finally:
        lib.pcg_set_removal_buffer(h, None, 0)


@pytest.fixture(scope="module")
def n500():
    """n = 500 of the config-5 SEM family at unlimited depth, and the C oracle's run on it."""
    X = synth.gaussian_sem(500, 10000, seed=0)
    C = np.corrcoef(X.T)
    return C, cpc.skeleton(C, 10000, max_depth=-1)


@pytest.mark.parametrize("kernels", ["default", "per_lane_all", "wave_from_13"])
def test_full_depth_n500_matches_oracle(eng, n500, kernels):
    """The reference's default: no depth cap (SkeletonDiscovery.py:72). n = 500 of the config-5
    SEM family runs 19 levels — removal depths, per-level test counts and sepset unions equal the C
    oracle's for every deep-level kernel choice:
    * default: depths 13-16 on the per-lane k_level_lds<13..16>, 17-18 (levels of < 1e7 tests) on
      the one-wave-per-set k_level_wave;
    * per_lane_all: PCG_TUNE_LDS_SPILL_MIN = 0 puts depths 17 and 18 on the spilling per-lane
      instantiations k_level_lds<17>, <18> too (band tests decided by the wave in its LDS slot);
    * wave_from_13: PCG_TUNE_LDS_DEEP = 12, every depth beyond 12 on k_level_wave."""
    C, ref = n500
    knobs = {"default": {}, "per_lane_all": {"LDS_SPILL_MIN": 0}, "wave_from_13": {"LDS_DEEP": 12}}[kernels]
    with eng.tuned(**knobs):
        out = eng.skeleton(C, 10000)
    assert out.levels == ref.levels == 19
    assert out.stats["tests"][17] > 0 and out.stats["tests"][18] > 0
    assert_skeleton_matches(out, ref, 500)


@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES[:5])
@pytest.mark.parametrize("flags", [0, _lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD])
def test_wave_kernel_from_depth5_matches_oracle(eng, n, N, seed, wl, wh, ep, flags):
    """k_level_wave at every depth >= 5 (PCG_TUNE_WAVE_LO = 5): the deferred-list exact path and
    the FULL_P records of |S| <= 12 go through it too; skeleton, unions, counts and records as the
    oracle's."""
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, N, record_cap=2_000_000)
    with eng.tuned(SMALL=0, WAVE_LO=5):   # the level-loop kernels under test, also at n <= 64
        out = eng.skeleton(C, N, flags=flags, record_capacity=2_000_000)
    assert_skeleton_matches(out, ref, n)
    if flags & _lib.PCG_FLAG_RECORD:
        d = {_key(r): r["p"] for r in ref.records}
        g = {_key(r): r["p"] for r in out.records}
        assert set(g) == set(d)
        keys = sorted(d)
        assert fisherz.p_close([g[k] for k in keys], [d[k] for k in keys]).all()



def _engine_state(out):
    return (np.asarray(out.removed_level).copy(), list(out.stats["tests"]), list(out.stats["indep"]),
            unions_from_engine(out))


def test_deep_per_lane_kernel_equals_wave_kernels_n1000(eng):
    """Threshold-mode depths 13..20 on the per-lane k_level_lds (band tests decided by the wave in
    its LDS slot; depths 17..20 for levels of >= 1e7 tests) against the one-wave-per-set kernels
    (PCG_TUNE_LDS_DEEP = 12) on n = 1000 at unlimited depth (30 levels, 3.3e10 tests): removal
    depths, per-level counts and sepset unions identical. This is an engine-vs-engine check: the C
    oracle takes hours at n = 1000 and no n = 1000 golden exists. Both kernel families are pinned
    to the oracle, at every depth they run, by test_full_depth_n500_matches_oracle (n = 500 to
    depth 18, on the default, the per-lane-everywhere and the wave-from-13 kernel settings)."""
    X = synth.gaussian_sem(1000, 10000, seed=0)
    C = np.corrcoef(X.T)
    a = _engine_state(eng.skeleton(C, 10000))
    with eng.tuned(LDS_DEEP=12):
        b = _engine_state(eng.skeleton(C, 10000))
    assert len(a[1]) == len(b[1]) == 30
    np.testing.assert_array_equal(a[0], b[0])
    assert a[1] == b[1] and a[2] == b[2]
    assert a[3] == b[3]


@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES[:3])
def test_inline_export_equals_export_stream(eng, n, N, seed, wl, wh, ep):
    """Small graphs export their sepset unions on the handle's stream (PCG_TUNE_EXPORT_INLINE);
    the export stream (0) gives the same rows, and both match the oracle."""
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, N)
    with eng.tuned(SMALL=0):
        a = eng.skeleton(C, N)
    assert_skeleton_matches(a, ref, n)
    with eng.tuned(SMALL=0, EXPORT_INLINE=0):
        b = eng.skeleton(C, N)
    sa, sb = _engine_state(a), _engine_state(b)
    np.testing.assert_array_equal(sa[0], sb[0])
    assert sa[3] == sb[3]


def test_sepset_rows_in_engine_buffers_never_overwrite_live_results(eng):
    """pcg_set_sepset_buffers: from the second run of an n on, the sepset rows are exported straight
    into an engine-owned buffer and the result holds views of it (no copy after the call). A
    buffer that a live result, or any slice of it a caller kept, still views is never written
    again; the rows equal the copy path's and the oracle's."""
    from oracle import cpc
    from tests_support import unions_from_oracle
    n = 317                                      # an n no other test uses: its first run copies
    X1 = synth.gaussian_sem(n, 2000, seed=9)
    X2 = synth.gaussian_sem(n, 2000, seed=10)
    C1, C2 = eng.corr(X1), eng.corr(X2)
    a = eng.skeleton(C1, 2000)                  # the copy path (learns the row bound)
    b = eng.skeleton(C1, 2000)                  # rows in the engine's buffer
    assert b.sep_xy_dev._base is not None and a.sep_xy_dev._base is None
    # (rows are appended by atomics: their order differs run to run, the row sets do not)
    assert unions_from_engine(b) == unions_from_engine(a) and len(b.sep_xy) == len(a.sep_xy)
    bxy = b.sep_xy_dev.cpu().numpy().copy()
    bbits = b.sep_bits_dev.cpu().numpy().copy()
    c = eng.skeleton(C2, 2000)                  # b is alive: another buffer
    assert c.sep_xy_dev.data_ptr() != b.sep_xy_dev.data_ptr()
    np.testing.assert_array_equal(b.sep_xy_dev.cpu().numpy(), bxy)
    np.testing.assert_array_equal(b.sep_bits_dev.cpu().numpy(), bbits)
    kept = c.sep_bits_dev[:5]                   # a caller keeps a slice, drops the result
    kept_h = kept.cpu().numpy().copy()
    del c
    d = eng.skeleton(C1, 2000)
    np.testing.assert_array_equal(kept.cpu().numpy(), kept_h)
    assert unions_from_engine(d) == unions_from_engine(a)
    ref = cpc.skeleton(np.corrcoef(X1.T), 2000, want_union=True)
    assert unions_from_engine(d) == unions_from_oracle(ref, n)
    del kept, b
    e = eng.skeleton(C1, 2000)                  # nothing views the last buffer any more: reused
    assert e.sep_bits_dev._base is not None
    assert unions_from_engine(e) == unions_from_engine(a)
