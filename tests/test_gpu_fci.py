"""GPU: FCI on the engine against oracle/fci.py (the vendored FAS + FCI
restated literally, numpy/scipy FisherZ). Parity with causal-learn 0.1.3.3 is unpinned."""
import numpy as np
import pytest

from oracle import fci as ofci
from oracle import pagerank as opr
from rcaeval_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,N,seed,wl,wh,ep", [(12, 500, 1, .3, .9, .3), (30, 600, 3, .3, .9, .15),
                                                (50, 1000, 7, .2, .8, .06), (25, 300, 9, .1, .5, .3)])
def test_fci_pag_matches_oracle(n, N, seed, wl, wh, ep):
    from rcaeval_amd.fci import fci
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    want, sep, _ = ofci.fci(np.corrcoef(X.T), N)
    G, edges = fci(X)
    np.testing.assert_array_equal(G.graph, want)
    assert G.sep_sets == sep


@pytest.mark.parametrize("depth", [1, 2])
def test_fci_depth_cap_matches_oracle(depth):
    from rcaeval_amd.fci import fci
    X = synth.gaussian_sem(20, 800, seed=2, w_low=.2, w_high=.8, edge_prob=.2)
    want, _, _ = ofci.fci(np.corrcoef(X.T), 800, depth=depth)
    np.testing.assert_array_equal(fci(X, depth=depth)[0].graph, want)


@pytest.mark.parametrize("m,rows,seed", [(12, 200, 0), (46, 600, 4)])
def test_fci_pagerank_and_randomwalk_match_oracle_pipeline(m, rows, seed):
    """fci_pagerank: preprocess -> PAG -> page_rank pair rules (circle marks included) ->
    PageRank; fci_randomwalk: circle marks make random_walk raise -> @rca dummy ranks."""
    from rcaeval_amd.e2e import fci_pagerank, fci_randomwalk
    from rcaeval_amd.graph_heads.page_rank import page_rank_preprocess
    from rcaeval_amd.io.time_series import preprocess
    df = synth.telemetry_frame(m, rows, n_constant=2, seed=seed)
    out = fci_pagerank(df, 0, dataset="online-boutique")
    data = preprocess(df, dataset="online-boutique").ffill()
    names = data.columns.to_list()
    X = data.to_numpy().astype(float)
    g, _, _ = ofci.fci(np.corrcoef(X.T), X.shape[0])
    np.testing.assert_array_equal(out["adj"], g)
    scores = opr.pagerank(page_rank_preprocess(g).astype(float))
    ranked = sorted(zip(names, scores), key=lambda t: t[1], reverse=True)
    assert out["ranks"] == [n_ for n_, _ in ranked]
    rw = fci_randomwalk(df, 0, dataset="online-boutique")
    if (g == 2).any():
        assert rw["ranks"] == names and rw["adj"] == []          # ValueError in random_walk -> @rca
    else:
        np.testing.assert_array_equal(rw["adj"], g)
