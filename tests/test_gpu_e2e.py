"""GPU parity for the ranking heads and the drop-in RCA methods, plus the sharded path.

PageRank: bit-identical to the scikit-network restatement (golden).
Random walk: identical ranks and scores to the REFERENCE module's outputs (golden).
pc_pagerank / pc_randomwalk: identical rank lists to the oracle pipeline (numpy skeleton
restatement + Python orientation restatement + scipy PageRank + the reference glue).
"""
import json
import os
import socket
import sys

import numpy as np
import pytest

from rcaeval_amd import synth
from tests_support import assert_skeleton_matches

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_pagerank_bitwise_golden():
    from rcaeval_amd.graph_heads.page_rank import PageRank
    g = np.load(os.path.join(GOLD, "pagerank.npz"))
    for i in range(12):
        np.testing.assert_array_equal(PageRank().fit_transform(g[f"A{i}"]), g[f"s{i}"])


@pytest.mark.parametrize("m,n_iter", [(5, 10), (256, 10), (257, 10), (300, 10), (768, 12), (769, 12), (800, 30),
                                      (1100, 10)])
def test_pagerank_sizes_vs_oracle(m, n_iter):
    """Each layout of k_pagerank and its switch points: LDS vectors with a 256-thread block
    (m <= 256), LDS vectors with 1024 threads (m <= 768), global scratch (m > 768) — bitwise the
    scipy/numpy oracle, through both the dense and the CSR entry (pcg_pagerank_csr)."""
    from scipy import sparse
    from oracle import pagerank as opr
    from rcaeval_amd.graph_heads.page_rank import PageRank
    rng = np.random.default_rng(m)
    A = (rng.random((m, m)) < min(1.0, 6.0 / m)) * rng.random((m, m))
    A[rng.integers(0, m, size=max(1, m // 10))] = 0.0   # dangling nodes
    ref = opr.pagerank(A, n_iter=n_iter)
    np.testing.assert_array_equal(PageRank(n_iter=n_iter).fit_transform(A), ref)
    np.testing.assert_array_equal(PageRank(n_iter=n_iter).fit_transform(sparse.csr_matrix(A)), ref)


def test_pagerank_csr_refuses_understated_nnz_and_bad_columns():
    from scipy import sparse
    from rcaeval_amd._lib import PcgError
    from rcaeval_amd.engine import get_engine
    rng = np.random.default_rng(1)
    A = sparse.csr_matrix((rng.random((50, 50)) < 0.2) * 1.0)
    eng = get_engine(0)
    with pytest.raises(PcgError):
        eng.pagerank_csr(A.indptr, A.indices, A.data, 50, nnz=A.nnz // 2)
    bad = A.indices.copy()
    bad[3] = 77
    with pytest.raises(PcgError):
        eng.pagerank_csr(A.indptr, bad, A.data, 50)
    # the handle stays usable after a refusal
    np.testing.assert_array_equal(eng.pagerank_csr(A.indptr, A.indices, A.data, 50),
                                  eng.pagerank_dense(A.toarray()))


def test_pagerank_empty_input_raises():
    from rcaeval_amd.graph_heads.page_rank import PageRank
    with pytest.raises(ValueError):
        PageRank().fit_transform(np.zeros((4, 4)))


def test_random_walk_matches_reference_golden():
    from rcaeval_amd.graph_heads.random_walk import random_walk
    for c in json.load(open(os.path.join(GOLD, "random_walk.json"))):
        res = random_walk(np.array(c["adj"]), c["names"], num_loop=c["num_loop"])
        assert [r[0] for r in res] == c["ranks"]
        np.testing.assert_array_equal([r[1] for r in res], c["scores"])


def test_random_walk_serial_path_matches_numpy():
    """Non-uniform transition columns take the sequential kernel; compare with numpy's choice."""
    from oracle import random_walk as orw
    from rcaeval_amd.engine import get_engine
    rng = np.random.default_rng(5)
    P = rng.random((9, 9))
    P /= P.sum(0, keepdims=True)
    st = np.random.default_rng(0).bit_generator.state["state"]
    got = get_engine(0).random_walk_counts(P, 3, 500, st["state"], st["inc"])
    np.testing.assert_array_equal(got, orw.walk_counts(P, 3, 500))


def _oracle_pipeline(df, dataset, head, alpha=0.05, sli=None):
    """Reference-equivalent CPU pipeline built only from oracle restatements: C-restated skeleton
    (pc_oracle.c), Python-restated orientation, scipy PageRank, and the glue restated in the test
    (networkx DiGraph as pc_pagerank.py:20-29, the loop form of random_walk.py's transition
    matrix) — no product code besides the golden-pinned preprocess."""
    from oracle import cpc
    from oracle import orient as oor
    from oracle import pagerank as opr
    from oracle import random_walk as orw
    from rcaeval_amd.io.time_series import preprocess      # pinned by preprocess.npz (reference outputs)
    from tests_support import loop_transition_matrix, networkx_digraph_matrix
    data = preprocess(df, dataset=dataset)
    names = data.columns.to_list()
    X = data.to_numpy().astype(float)
    with np.errstate(invalid="ignore", divide="ignore"):
        C = np.corrcoef(X.T)
    r = cpc.skeleton(C, X.shape[0], alpha=alpha)
    n = C.shape[0]
    sep = np.empty((n, n), object)
    for a in range(n):
        for b in range(n):
            u = set()
            if a != b and r.removed_level[a, b] >= 1:
                for (p, q) in ((a, b), (b, a)):
                    bits = r.side_union[p, q]
                    u |= {j for j in range(n) if (int(bits[j >> 6]) >> (j & 63)) & 1}
            sep[a, b] = [tuple(u)]
    g = oor.orient(r.adj, sep)
    if head == "cloudranger":
        from rcaeval_amd.graph_heads.finalize import finalize_directed_adj
        from rcaeval_amd.graph_heads.relato_rank import relaToRank
        rank, _, _ = relaToRank(np.corrcoef(data.to_numpy().T), finalize_directed_adj(g).T, 10,
                                names.index(sli), beta=0.3, rho=0.2)
        return [names[k - 1] for k, _ in rank], g
    if head == "pagerank":
        M, _ = networkx_digraph_matrix(g)
        scores = opr.pagerank(M.T)
        ranked = sorted(zip(names, scores), key=lambda t: t[1], reverse=True)
        return [n_ for n_, _ in ranked], g
    uniq = list(dict.fromkeys(names))
    P = loop_transition_matrix(g, names, uniq)
    counts = orw.walk_counts(P, 0, len(names))
    ranked = sorted([(nm, counts[i] / len(names)) for i, nm in enumerate(uniq)], key=lambda t: t[1], reverse=True)
    return [n_ for n_, _ in ranked], g


@pytest.mark.parametrize("m,rows,seed", [(12, 200, 0), (38, 600, 1), (49, 600, 2)])
def test_pc_pagerank_matches_oracle_pipeline(m, rows, seed):
    from rcaeval_amd.e2e import pc_pagerank
    df = synth.telemetry_frame(m, rows, n_constant=2, seed=seed)
    out = pc_pagerank(df, 0, dataset="online-boutique")
    ranks, g = _oracle_pipeline(df, "online-boutique", "pagerank")
    assert out["ranks"] == ranks


@pytest.mark.parametrize("m,rows,seed", [(12, 200, 3), (46, 600, 4)])
def test_pc_randomwalk_matches_oracle_pipeline(m, rows, seed):
    from rcaeval_amd.e2e import pc_randomwalk
    from rcaeval_amd.graph_construction.pc import pc_default
    df = synth.telemetry_frame(m, rows, n_constant=2, seed=seed)
    out = pc_randomwalk(df, 0, dataset="online-boutique")
    ranks, g = _oracle_pipeline(df, "online-boutique", "randomwalk")
    assert out["ranks"] == ranks
    from rcaeval_amd.io.time_series import preprocess
    np.testing.assert_array_equal(pc_default(preprocess(df, dataset="online-boutique")), g)


def _glue_frame(case, tmp_path):
    """A glue.json case's input frame, as the generator built it (seeded synth -> CSV -> read)."""
    import pandas as pd
    sys.path.insert(0, GOLD)
    from make_glue_golden import frame, frame_digest
    m, rows, seed, nc, dataset, noise = case["case"]
    p = os.path.join(str(tmp_path), "case.csv")
    frame(m, rows, seed, nc, noise).to_csv(p, index=False)
    df = pd.read_csv(p)
    assert frame_digest(df) == case["input_digest"], "regenerated input frame differs from the golden's"
    return df, dataset


def _glue():
    return json.load(open(os.path.join(GOLD, "glue.json")))


@pytest.mark.parametrize("k", range(6))
def test_pc_pagerank_matches_reference_glue_golden(k, tmp_path):
    """pc_pagerank on the GPU == the REFERENCE pc_pagerank function executed under networkx 2.6.3
    with pc -> the oracle graph and PageRank -> the sknetwork restatement (glue.json): node
    names, the to_numpy_matrix matrix (isolated nodes dropped) and the misaligned rank list."""
    from rcaeval_amd.e2e import pc_pagerank
    from rcaeval_amd.graph_construction.pc import pc_default
    from rcaeval_amd.io.time_series import preprocess
    case = _glue()["pagerank"][k]
    df, dataset = _glue_frame(case, tmp_path)
    np.testing.assert_array_equal(pc_default(preprocess(df, dataset=dataset)), np.array(case["graph"]))
    out = pc_pagerank(df, 0, dataset=dataset)
    assert out["node_names"] == case["node_names"]
    np.testing.assert_array_equal(out["adj"], np.array(case["adj"]))
    assert out["ranks"] == case["ranks"]


@pytest.mark.parametrize("k", range(3))
def test_pc_randomwalk_matches_reference_glue_golden(k, tmp_path):
    """pc_randomwalk on the GPU == the REFERENCE pc_randomwalk + random_walk executed with
    pc_default -> the oracle graph (glue.json)."""
    from rcaeval_amd.e2e import pc_randomwalk
    case = _glue()["randomwalk"][k]
    df, dataset = _glue_frame(case, tmp_path)
    out = pc_randomwalk(df, 0, dataset=dataset)
    np.testing.assert_array_equal(out["adj"], np.array(case["graph"]))
    assert out["node_names"] == case["node_names"]
    assert out["ranks"] == case["ranks"]


def test_pc_pagerank_readme_path_dataset_none_keeps_time_and_constants():
    """dataset=None: preprocess is the identity, the time column and constant columns reach
    PC (NaN correlations -> dependent), as in the README example."""
    from rcaeval_amd.e2e import pc_pagerank
    df = synth.telemetry_frame(14, 300, n_constant=1, seed=9)
    out = pc_pagerank(df, 0)
    ranks, _ = _oracle_pipeline(df, None, "pagerank")
    assert out["ranks"] == ranks
    assert out["node_names"] == df.columns.to_list()


def test_deep_levels_constant_column_vs_c_oracle():
    """A constant column (NaN correlations, never separated) keeps PC running to depth n-2:
    depths > 12 run on the generic exact-path kernel."""
    from oracle import cpc
    from rcaeval_amd.engine import get_engine
    X = synth.gaussian_sem(17, 400, seed=31, w_low=0.3, w_high=0.9, edge_prob=0.2)
    X[:, 4] = 1.0
    with np.errstate(invalid="ignore", divide="ignore"):
        C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, 400)
    out = get_engine(0).skeleton(C, 400)
    assert out.levels == ref.levels and out.levels > 13
    assert out.stats["tests"] == ref.tests
    np.testing.assert_array_equal(out.removed_level, ref.removed_level)


@pytest.mark.parametrize("n,N,seed,prob", [(16, 600, 21, 0.25), (24, 300, 5, 0.35), (30, 2000, 8, 0.3)])
def test_causal_pc_sepset_and_p_values_surface(n, N, seed, prob):
    """cg.sepset element for element (tuples in the reference's set order, not as sets) and
    cg.p_values (every dependent p per visit, enumeration order) against oracle/skeleton.py."""
    from oracle import skeleton as osk
    from rcaeval_amd.causal import pc
    X = synth.gaussian_sem(n, N, seed=seed, w_low=0.3, w_high=0.9, edge_prob=prob)
    cg = pc(X)
    r = osk.skeleton_discovery(np.corrcoef(X.T), N)
    multi = 0
    for i in range(n):
        for j in range(n):
            if i == j:
                continue
            mine, ref = cg.sepset[i, j], r.sepset[i, j]
            assert len(mine) == len(ref)
            assert [tuple(map(int, t)) for t in mine] == [tuple(map(int, t)) for t in ref], (i, j)
            multi += any(len(t) > max(int(r.removed_level[i, j]), 0) for t in ref)
            pm, pr = cg.p_values[i, j], r.p_values[i, j]
            if pr is None:
                assert pm is None, (i, j)
                continue
            assert len(pm) == len(pr), (i, j)
            pm, pr = np.asarray(pm), np.asarray(pr)
            assert np.all(np.abs(pm - pr) <= 1e-9 * np.abs(pr) + 2.0 ** -51), (i, j)
    assert cg.no_ci_tests == sum(r.calls_per_level)
    assert multi > 0          # unions from several S: the insertion order is exercised


def test_sepset_order_matches_cpython_set_for_multi_s_unions():
    """A union assembled from several independent S (|union| > depth) keeps the reference's
    first-insertion order through CPython's set layout (members >= 8 collide in small tables)."""
    from oracle import skeleton as osk
    from rcaeval_amd.causal import pc
    X = synth.gaussian_sem(40, 400, seed=3, w_low=0.1, w_high=0.3, edge_prob=0.3)
    cg = pc(X)
    r = osk.skeleton_discovery(np.corrcoef(X.T), 400)
    seen = 0
    for i in range(40):
        for j in range(40):
            if i == j or r.sepset[i, j] is None:
                continue
            rl = int(r.removed_level[i, j])
            for t_m, t_r in zip(cg.sepset[i, j], r.sepset[i, j]):
                assert tuple(map(int, t_m)) == tuple(map(int, t_r)), (i, j)
                seen += rl > 0 and len(t_r) > rl
    assert seen > 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_worker(rank, world, port, X, q, max_depth=3):
    import torch
    import torch.distributed as dist
    from rcaeval_amd.dist import sharded_corr, sharded_skeleton
    from rcaeval_amd.engine import get_engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = get_engine(0)
    C = sharded_corr(eng, eng.to_device(X)) if world > 2 else eng.corr(X)
    out = sharded_skeleton(eng, C, X.shape[0], max_depth=max_depth)
    q.put((rank, out.removed_level.copy(), out.sep_xy.copy(), out.sep_bits.copy(), out.stats["tests"],
           [(int(r["a"]), int(r["b"])) for r in out.near_alpha]))
    dist.barrier()
    dist.destroy_process_group()
    torch.cuda.synchronize()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n,N,max_depth", [(2, 300, 3000, 3), (4, 700, 5000, 4), (8, 700, 5000, 5), (8, 300, 3000, -1)])
def test_sharded_skeleton_ranks_one_gpu(world, n, N, max_depth):
    """The torch.distributed driver (rcaeval_amd.dist, gloo on device tensors) with 2 / 4 / 8
    ranks sharing cuda:0 (K1 sharded too at 4 and 8): every rank's removal depths, per-level
    tests and sepset unions equal the single-GPU engine's and the C oracle's."""
    import multiprocessing as mp
    from types import SimpleNamespace

    from oracle import cpc
    from rcaeval_amd.engine import get_engine
    X = synth.gaussian_sem(n, N, seed=12)
    eng = get_engine(0)
    ref = eng.skeleton(eng.corr(X), N, max_depth=max_depth)
    oref = cpc.skeleton(np.corrcoef(X.T), N, max_depth=max_depth, want_union=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, X, q, max_depth)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=500) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0

    def unions(xy, bits):
        d = {}
        for (x, y), b in zip(xy, bits):
            d[(int(x), int(y))] = d.get((int(x), int(y)), 0) | int.from_bytes(b.tobytes(), "little")
        return d
    for rank, rl, xy, bits, tests, near in res:
        np.testing.assert_array_equal(rl, ref.removed_level)
        assert unions(xy, bits) == unions(ref.sep_xy, ref.sep_bits)
        assert tests == ref.stats["tests"]
        out = SimpleNamespace(removed_level=rl, sep_xy=xy, sep_bits=bits, stats={"tests": tests},
                              near_alpha=[{"a": a, "b": b} for a, b in near])
        assert_skeleton_matches(out, oref, n)


def _config5_sharded_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from rcaeval_amd.dist import sharded_corr, sharded_skeleton
    from rcaeval_amd.engine import get_engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = get_engine(0)
    X = synth.gaussian_sem(2000, 10000, seed=0)
    C = sharded_corr(eng, eng.to_device(X))          # K1 sharded: each rank its residue units
    out = sharded_skeleton(eng, C, 10000, max_depth=4)
    near = [(int(r["a"]), int(r["b"])) for r in out.near_alpha]
    q.put((rank, out.removed_level.copy(), out.sep_xy.copy(), out.sep_bits.copy(), out.stats["tests"], near,
           float(np.abs(C.cpu().numpy() - np.corrcoef(X.T)).max())))
    dist.barrier()
    dist.destroy_process_group()
    torch.cuda.synchronize()


@pytest.mark.timeout(900)
def test_config5_sharded_two_ranks_one_gpu_matches_oracle(config5):
    """North-star config 5 (2000 vars x 10 000 samples, depth 4) through the multi-GPU protocol at
    full size: 2 gloo ranks sharing cuda:0, K1 sharded by residue units (rcaeval_amd.dist
    .sharded_corr) and every depth's work list edge-sharded (pcg_level_split) with the packed
    removal-bit all-gather + OR merge at each level barrier. Every rank's removal depths,
    per-level unique-test counts (summed over ranks) and sepset unions equal the C oracle's on
    np.corrcoef(X.T) (near-alpha pairs exempt as in the single-GPU test). The protocol is verified
    at full size; its multi-GPU timing stays unmeasured on hardware (one GPU here)."""
    import multiprocessing as mp
    from types import SimpleNamespace
    _, _, ref = config5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config5_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=800) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, rl, xy, bits, tests, near, cerr in res:
        assert cerr <= 2e-14
        out = SimpleNamespace(removed_level=rl, sep_xy=xy, sep_bits=bits, stats={"tests": tests},
                              near_alpha=[{"a": a, "b": b} for a, b in near])
        assert_skeleton_matches(out, ref, 2000)
        assert sum(tests) > 4.5e9


def _rq2_worker(rank, world, port, root, out_dir, q):
    import torch.distributed as dist
    from rcaeval_amd import rq2
    from rcaeval_amd.engine import get_engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    get_engine(0)
    res = rq2.run(root, "pc_pagerank", "online-boutique", out_dir, rank=rank, world=world)
    q.put((rank, res["my_cases"], res.get("summary")))
    dist.destroy_process_group()


def test_rq2_two_ranks_deal_cases_one_gpu(tmp_path):
    """BASELINE config 2's dealing: rq2.run with rank r of 2 taking cases r, r + 2, ... of the
    sorted tree (two processes sharing cuda:0, gloo barrier); every case's rank list, whichever
    rank ran it, equals the CPU oracle pipeline, and rank 0 evaluates all of them."""
    import multiprocessing as mp
    from rcaeval_amd import rq2
    root = os.path.join(str(tmp_path), "data", "online-boutique")
    paths = synth.write_rq2_dataset(root, services=["cartservice", "adservice", "emailservice"],
                                    faults=("cpu", "delay"), cases=1, rows=1200)
    out_dir = os.path.join(str(tmp_path), "out")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rq2_worker, args=(r, 2, port, root, out_dir, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (mine, summ)) for r, mine, summ in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][0] + res[1][0] == len(paths) == 6 and res[0][0] == res[1][0] == 3
    assert set(res[0][1]) >= {"Avg@5-CPU", "Avg@5-DELAY"}
    for p in paths:
        c = rq2.load_case(p)
        ranks, _ = _oracle_pipeline(c["data"], "online-boutique", "pagerank")
        got = rq2.load_json(os.path.join(out_dir, "results", c["result_name"]))["0"]
        assert got == ranks


@pytest.mark.parametrize("world", [2, 3, 8])
def test_level_split_matches_split_by_work(world):
    """pcg_level_split (the C cut the sharded loop uses) == split_by_work over the chunk work
    prefix, at every depth of a real skeleton; the ranges tile [0, total)."""
    from rcaeval_amd.dist import GpuLevelBackend, split_by_work
    from rcaeval_amd.engine import get_engine
    eng = get_engine(0)
    X = synth.gaussian_sem(400, 2000, seed=21)
    C = eng.corr(X)
    be = GpuLevelBackend(eng, C, X.shape[0], 0.05, 0, world)
    try:
        for depth in range(4):
            total = be.begin(depth)
            if total is None:
                break
            prefix = be.prefix(total)
            cuts = [be.split(r, world) for r in range(world)]
            assert cuts == [split_by_work(prefix, r, world) for r in range(world)]
            assert cuts[0][0] == 0 and cuts[-1][1] == total
            assert all(cuts[r][1] == cuts[r + 1][0] for r in range(world - 1))
            be.run(0, total)
            be.end()
    finally:
        be.finish()


@pytest.mark.parametrize("dataset,services", [("online-boutique", ["cartservice", "adservice"]),
                                              ("sock-shop", ["carts", "orders"])])
def test_rq2_run_matches_oracle_per_case(tmp_path, dataset, services):
    """the RQ2 loop over an Online-Boutique- or Sock-Shop-shaped case tree
    (sock-shop: lat_50 / lat_99 dropped, lat_90 SLI, rq2.py:228-230,259-262); every case's rank
    list equals the CPU oracle pipeline on the same window."""
    from rcaeval_amd import rq2
    root = os.path.join(str(tmp_path), "data", dataset)
    paths = synth.write_rq2_dataset(root, services=services, faults=("cpu", "delay"), cases=1, rows=1200,
                                    flavor=dataset)
    out_dir = os.path.join(str(tmp_path), "out")
    res = rq2.run(root, "pc_pagerank", dataset, out_dir)
    assert res["cases"] == len(paths) == 4
    for p in paths:
        c = rq2.load_case(p)
        if dataset == "sock-shop":
            assert not any(col.endswith(("_lat_50", "_lat_99")) for col in c["data"].columns)
            assert c["sli"] == f"{c['service']}_lat_90"
        ranks, _ = _oracle_pipeline(c["data"], dataset, "pagerank")
        got = rq2.load_json(os.path.join(out_dir, "results", c["result_name"]))["0"]
        assert got == ranks
    assert set(res["summary"]) >= {"Avg@5-CPU", "Avg@5-DELAY"}


def _sem_frame(X, prefix):
    import pandas as pd
    df = pd.DataFrame(X, columns=[f"{prefix}{i}_lat" for i in range(X.shape[1])])
    df.insert(0, "time", np.arange(X.shape[0]))
    return df


@pytest.mark.parametrize("kind,seed", [("circa50", 5), ("circa50", 15), ("rcd50", 6)])
def test_pc_randomwalk_config3_50_node_sem(kind, seed):
    """BASELINE config 3: circa50 / rcd50-shaped 50-node SEMs (continuous, or discrete 0-5
    levels for RCD) through pc_randomwalk — rank lists and endpoint graph identical to the
    oracle pipeline."""
    from rcaeval_amd.e2e import pc_randomwalk
    if kind == "circa50":
        X = synth.gaussian_sem(50, 3000, seed=seed, w_low=0.3, w_high=0.9)
    else:
        X = synth.discrete_sem(50, 3000, seed=seed).astype(float)
    df = _sem_frame(X, "s")
    out = pc_randomwalk(df, 0, dataset=kind)
    ranks, g = _oracle_pipeline(df, kind, "randomwalk")
    assert out["ranks"] == ranks
    np.testing.assert_array_equal(out["adj"], g)


def test_pc_pagerank_config4_train_ticket_212():
    """BASELINE config 4: train-ticket-shaped frame (212 metrics x 600 rows, constant columns
    dropped by preprocess) through pc_pagerank — identical rank list and endpoint graph."""
    from rcaeval_amd.e2e import pc_pagerank
    df = synth.telemetry_frame(212, 600, n_constant=4, seed=11)
    out = pc_pagerank(df, 0, dataset="train-ticket")
    ranks, g = _oracle_pipeline(df, "train-ticket", "pagerank")
    assert out["ranks"] == ranks
    from rcaeval_amd.io.time_series import preprocess
    assert out["node_names"] == preprocess(df, dataset="train-ticket").columns.to_list()
    assert len(out["node_names"]) == g.shape[0]


@pytest.mark.parametrize("m,rows,seed", [(12, 200, 5), (38, 600, 6), (49, 600, 7)])
def test_cloudranger_matches_oracle_pipeline(m, rows, seed):
    """cloudranger.py:154-190: PC at alpha 0.1 on the engine + the second-order walk, under the
    same np.random seed as the oracle pipeline (C-restated skeleton, Python orientation)."""
    from rcaeval_amd.e2e import cloudranger
    df = synth.telemetry_frame(m, rows, n_constant=2, seed=seed)
    from rcaeval_amd.io.time_series import preprocess
    sli = preprocess(df, dataset="online-boutique").columns[seed % 5]
    np.random.seed(seed)
    out = cloudranger(df, 0, dataset="online-boutique", sli=sli)
    np.random.seed(seed)
    ranks, g = _oracle_pipeline(df, "online-boutique", "cloudranger", alpha=0.1, sli=sli)
    np.testing.assert_array_equal(out["adj"], g)
    assert out["ranks"] == ranks


@pytest.mark.parametrize("m,rows,seed", [(12, 600, 8), (38, 600, 9)])
def test_circa_matches_oracle_pipeline(m, rows, seed):
    """circa.py:15-41: stable PC on the engine + the RHT head; the oracle pipeline's endpoint
    matrix through the same head gives the same ranks."""
    from rcaeval_amd.e2e import circa
    from rcaeval_amd.graph_heads.rht import rht
    from rcaeval_amd.io.time_series import preprocess
    df = synth.telemetry_frame(m, rows, n_constant=2, seed=seed)
    inject = int(df["time"].iloc[0]) + 200
    np.random.seed(seed)
    out = circa(df.copy(), inject, dataset="online-boutique")
    _, g = _oracle_pipeline(df.copy(), "online-boutique", "pagerank")
    np.testing.assert_array_equal(out["adj"], g)
    data = preprocess(df.copy(), dataset="online-boutique")
    data["time"] = df["time"]
    np.random.seed(seed)
    want = [n for n, _ in sorted(rht(g, inject, data), key=lambda x: x[1], reverse=True)]
    assert out["ranks"] == want
    assert len(out["ranks"]) > 0


@pytest.mark.parametrize("method", ["circa", "cloudranger"])
def test_rq2_run_other_pc_methods(tmp_path, method):
    """rq2.py's loop with the other PC-based methods: every case's dumped
    ranks equal a direct call of the method on the same window, in the harness's case order
    and from the same np.random state (CloudRanger's walk and RHT's SLI draw use it)."""
    from rcaeval_amd import e2e, rq2
    root = os.path.join(str(tmp_path), "data", "online-boutique")
    synth.write_rq2_dataset(root, services=["cartservice", "adservice"], faults=("cpu", "delay"), cases=1, rows=1200)
    out_dir = os.path.join(str(tmp_path), "out")
    np.random.seed(4)
    res = rq2.run(root, method, "online-boutique", out_dir)
    assert res["cases"] == 4
    np.random.seed(4)
    for p in rq2.list_cases(root):
        c = rq2.load_case(p)
        want = getattr(e2e, method)(c["data"], c["inject_time"], dataset="online-boutique", sli=c["sli"],
                                    n_iter=c["num_node"])["ranks"]
        got = rq2.load_json(os.path.join(out_dir, "results", c["result_name"]))["0"]
        assert got == want and len(got) > 0


def _bg_frame(m, rows, seed):
    """Telemetry frame whose names the reference's with_bg patterns hit: frontend services,
    *_cpu / *_mem metrics and *_lat50 latencies."""
    svcs = ["frontend", "cart", "checkout", "frontend-web", "ad", "shipping", "pay", "email",
            "redis", "catalog", "currency", "reco", "user", "orders", "queue", "db", "cache"]
    df = synth.telemetry_frame(m, rows, n_constant=0, seed=seed, services=svcs)
    return df.rename(columns={c: c.replace("_latency", "_lat50") for c in df.columns})


@pytest.mark.parametrize("m,rows,seed", [(12, 300, 60), (30, 600, 61), (49, 800, 62)])
def test_pc_default_with_bg_matches_oracle(m, rows, seed):
    """pc_default(with_bg=True) (graph_construction/pc.py:6-9,19): banned pairs leave the GPU
    skeleton at depth 0, the knowledge-aware orientation runs in host C++; against the C-restated
    skeleton with the same banned pairs + the Python-restated orientation with the same masks.
    Parity unpinned [U] (no with_bg fixture in the reference, causal-learn not importable)."""
    from oracle import cpc
    from oracle import orient as oor
    from rcaeval_amd.background import banned_pairs
    from rcaeval_amd.causal import pc
    from rcaeval_amd.graph_construction.pc import background_knowledge, pc_default
    df = _bg_frame(m, rows, seed).drop(columns=["time"])
    names = df.columns.to_list()
    X = df.to_numpy().astype(float)
    F, R = background_knowledge.masks(names)
    B = banned_pairs(F)
    assert B.any() and F.sum() > B.sum()
    C = np.corrcoef(X.T)
    r = cpc.skeleton(C, X.shape[0], banned=B)
    n = len(names)
    sep = np.empty((n, n), object)
    for a in range(n):
        for b in range(n):
            u = set()
            if a != b and r.removed_level[a, b] >= 1:
                for (p_, q) in ((a, b), (b, a)):
                    bits = r.side_union[p_, q]
                    u |= {j for j in range(n) if (int(bits[j >> 6]) >> (j & 63)) & 1}
            sep[a, b] = [tuple(u)]
    want = oor.orient(r.adj, sep, knowledge=(F, R))
    got = pc_default(df, with_bg=True)
    np.testing.assert_array_equal(got, want)
    cg = pc(X, node_names=names, background_knowledge=background_knowledge)
    np.testing.assert_array_equal(cg.skeleton.removed_level, r.removed_level)
    assert list(cg.stats["calls"])[: r.levels] == r.calls and list(cg.stats["tests"])[: r.levels] == r.tests
    assert not np.array_equal(pc_default(df), got)          # the knowledge changed the graph


def test_causal_graph_release_drops_the_correlation():
    """pc() keeps the device C only for lazy p_values / sepset order; release() drops it."""
    from rcaeval_amd.causal import pc
    X = synth.gaussian_sem(10, 400, seed=3)
    cg = pc(X)
    g = cg.G.graph.copy()
    assert cg._run[0] is not None and not hasattr(cg.sepset._ci, "pvalues_status")   # tester not built yet
    cg.release()
    assert cg._run[0] is None and cg.sepset._ci is None
    np.testing.assert_array_equal(cg.G.graph, g)
    with pytest.raises(RuntimeError):
        cg.p_values
