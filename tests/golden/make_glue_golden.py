"""Golden vectors for the glue around the PC engine, produced by EXECUTING the reference's own
functions (run in the build container, where /root/reference exists):

  python tests/golden/make_glue_golden.py

Stage A (this interpreter) builds the inputs: seeded synthetic telemetry frames, and for each the
endpoint graph the oracle computes (oracle/cpc.py skeleton + oracle/orient.py UCSepset/Meek) on
the preprocessed frame; seeded RQ2 case trees (Online-Boutique-, Sock-Shop- and CIRCA-shaped).
Stage B runs under /opt/conda/bin/python3.9 (networkx 2.6.3, which still has
``to_numpy_matrix``): it reads the top-level functions ``pc_pagerank``
(RCAEval/e2e/pc_pagerank.py:12-40), ``pc_randomwalk`` (RCAEval/e2e/pc_randomwalk.py:10-30) and
``process`` (rq2.py:170-296) out of the reference files with ``ast`` and executes them with
``pc`` / ``pc_default`` bound to the oracle graph of that frame, ``PageRank`` bound to the
scikit-network restatement (oracle/pagerank.py), the REFERENCE ``preprocess`` and
``random_walk`` imported, and rq2's method slot bound to a recorder of the window it is given.
Only outputs are stored (tests/golden/glue.json): ranks, node names, the networkx matrix, and
sha256 digests of the inputs and of the rq2 window frame. The reference code itself is never
copied; the @rca decorator is not applied (its fallback is pinned separately).
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
PY39 = "/opt/conda/bin/python3.9"
sys.path.insert(0, ROOT)

# (m metrics, rows, seed, constant columns, dataset, noise columns): the noise columns are
# independent of everything, so they usually end up isolated (pc_pagerank.py:28 drops them and
# :33 zips the scores against the unfiltered names: misaligned ranks, reproduced on purpose)
PR_CASES = [(12, 200, 0, 2, "online-boutique", 0), (38, 600, 1, 2, "online-boutique", 0),
            (49, 600, 2, 2, "online-boutique", 0), (14, 300, 9, 1, None, 0),
            (20, 400, 21, 1, "online-boutique", 4), (30, 500, 22, 0, "sock-shop", 3)]
RW_CASES = [(12, 200, 3, 2, "online-boutique", 0), (46, 600, 4, 2, "online-boutique", 0),
            (16, 300, 23, 1, None, 2)]


def frame(m, rows, seed, n_constant, noise):
    """The seeded input frame of one case (tests rebuild it the same way)."""
    from rcaeval_amd import synth
    df = synth.telemetry_frame(m, rows, n_constant=n_constant, seed=seed)
    rng = np.random.default_rng(10_000 + seed)
    for k in range(noise):
        df.insert(len(df.columns) - 1, f"noise{k}_cpu", rng.standard_normal(rows))
    return df


def digest(a) -> str:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return hashlib.sha256(a.tobytes() + str(a.shape).encode()).hexdigest()


def frame_digest(df) -> str:
    return hashlib.sha256((digest(df.to_numpy(dtype=np.float64)) + "|" + ",".join(df.columns)).encode()).hexdigest()


def oracle_graph(df, dataset):
    from oracle import cpc
    from oracle import orient as oor
    from rcaeval_amd.io.time_series import preprocess
    data = preprocess(df, dataset=dataset)
    X = data.to_numpy().astype(float)
    with np.errstate(invalid="ignore", divide="ignore"):
        C = np.corrcoef(X.T)
    r = cpc.skeleton(C, X.shape[0])
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
    return oor.orient(r.adj, sep).astype(int), frame_digest(data)


RQ2_TREES = [("online-boutique", dict(faults=("cpu", "delay"), cases=1, rows=1200, seed=40)),
             ("sock-shop", dict(faults=("mem", "loss"), cases=1, rows=1100, seed=41))]


def write_trees(base):
    """Seeded RQ2 trees (tests rebuild them the same way) + one CIRCA-shaped 'rca_' case."""
    from rcaeval_amd import synth
    paths = []
    for dataset, kw in RQ2_TREES:
        root = os.path.join(base, "data", dataset)
        paths += synth.write_rq2_dataset(root, flavor=dataset, **kw)
    paths.append(write_rca_case(base))
    return sorted(paths)


def write_rca_case(base):
    """A synthetic 'rca_' case (rq2.py:185-201: root_cause.txt, inject_time.txt, fe_service.txt;
    columns get the SIM_ prefix, the index becomes the time column)."""
    import pandas as pd
    d = os.path.join(base, "data", "rca_circa", "10", "case_3")
    os.makedirs(d, exist_ok=True)
    rng = np.random.default_rng(42)
    X = rng.standard_normal((5000, 10)).cumsum(axis=0)
    X[rng.integers(0, 5000, 30), rng.integers(0, 10, 30)] = np.inf
    df = pd.DataFrame(X, columns=[str(i) for i in range(10)])
    df.to_csv(os.path.join(d, "data.csv"), index=False)
    for name, text in (("inject_time.txt", "2600"), ("root_cause.txt", "4"), ("fe_service.txt", "0")):
        with open(os.path.join(d, name), "w") as f:
            f.write(text + "\n")
    return os.path.join(d, "data.csv")


def stage_a(tmp):
    import pandas as pd
    spec = {"pagerank": [], "randomwalk": [], "rq2": []}
    for kind, cases in (("pagerank", PR_CASES), ("randomwalk", RW_CASES)):
        for i, (m, rows, seed, nc, dataset, noise) in enumerate(cases):
            csv = os.path.join(tmp, f"{kind}{i}.csv")
            frame(m, rows, seed, nc, noise).to_csv(csv, index=False)
            df = pd.read_csv(csv)           # the case as a harness reads it (tests do the same)
            g, dg = oracle_graph(df, dataset)
            np.save(os.path.join(tmp, f"{kind}{i}_graph.npy"), g)
            spec[kind].append({"case": [m, rows, seed, nc, dataset, noise], "csv": csv,
                               "graph": os.path.join(tmp, f"{kind}{i}_graph.npy"),
                               "input_digest": frame_digest(df), "preprocessed_digest": dg})
    for p in write_trees(tmp):
        spec["rq2"].append({"path": p, "rel": os.path.relpath(p, tmp),
                            "dataset": "synthetic" if "rca_" in p else p.split(os.sep + "data" + os.sep)[1].split(os.sep)[0]})
    with open(os.path.join(tmp, "spec.json"), "w") as f:
        json.dump(spec, f)
    return spec


def stage_b(tmp):
    """Runs under python3.9: the reference functions, executed (never stored)."""
    import argparse
    import ast
    import warnings

    import networkx as nx
    import pandas as pd
    warnings.simplefilter("ignore")
    sys.path.insert(0, REF)
    from RCAEval.graph_heads.random_walk import random_walk   # reference, imported
    from RCAEval.io.time_series import preprocess             # reference, imported

    from oracle import pagerank as opr                        # sknetwork restatement (test infra)

    def functions(path, names):
        tree = ast.parse(open(path).read())
        keep = []
        for node in tree.body:
            if isinstance(node, ast.FunctionDef) and node.name in names:
                node.decorator_list = []                      # @rca applied by the caller, not here
                keep.append(node)
        return keep

    spec = json.load(open(os.path.join(tmp, "spec.json")))
    out = {"pagerank": [], "randomwalk": [], "rq2": []}

    class _G:
        def __init__(self, g):
            self.graph = g

    class _CG:
        def __init__(self, g):
            self.G = _G(g)

    class PageRank:                                           # sknetwork 0.31.0 defaults [U]
        def fit_transform(self, A):
            return opr.pagerank(np.asarray(A, dtype=float))

    for kind, fname, src in (("pagerank", "pc_pagerank", "RCAEval/e2e/pc_pagerank.py"),
                             ("randomwalk", "pc_randomwalk", "RCAEval/e2e/pc_randomwalk.py")):
        body = functions(os.path.join(REF, src), {fname})
        for c in spec[kind]:
            g = np.load(c["graph"])
            ns = {"np": np, "nx": nx, "preprocess": preprocess, "random_walk": random_walk, "PageRank": PageRank}
            ns["pc"] = lambda X, _g=g: (_ for _ in ()).throw(AssertionError("shape")) if X.shape[1] != len(_g) \
                else _CG(_g)
            ns["pc_default"] = lambda data, _g=g: _g
            exec(compile(ast.Module(body=body, type_ignores=[]), src, "exec"), ns)
            df = pd.read_csv(c["csv"])
            assert frame_digest_py39(df) == c["input_digest"], "input frame differs between interpreters"
            res = ns[fname](df, 0, dataset=c["case"][4])
            out[kind].append({"case": c["case"], "input_digest": c["input_digest"],
                              "graph": np.asarray(g).tolist(), "node_names": res["node_names"], "ranks": res["ranks"],
                              "adj": np.asarray(res["adj"], dtype=float).tolist()})

    body = functions(os.path.join(REF, "rq2.py"), {"process"})
    for c in spec["rq2"]:
        seen = {}

        def capture(data, inject_time, **kw):
            seen.update(data=data, inject_time=inject_time, kw=kw)
            return {"ranks": ["captured"]}

        dumps = {}
        ns = {"np": np, "pd": pd, "os": os, "argparse": argparse, "json": json,
              "basename": os.path.basename, "dirname": os.path.dirname, "join": os.path.join,
              "datetime": __import__("datetime").datetime, "capture": capture, "result_path": os.path.join(tmp, "res"),
              "is_synthetic": "rca_" in c["path"],
              "args": argparse.Namespace(length=None, tdelta=0, method="capture", dataset=c["dataset"]),
              "dump_json": lambda filename, data: dumps.update({os.path.basename(filename): data})}
        exec(compile(ast.Module(body=body, type_ignores=[]), "rq2.py", "exec"), ns)
        ns["process"](c["path"])
        w = seen["data"]
        kw = seen["kw"]
        out["rq2"].append({"rel": c["rel"], "dataset": c["dataset"], "window_digest": frame_digest_py39(w),
                           "rows": int(w.shape[0]), "columns": list(w.columns), "inject_time": int(seen["inject_time"]),
                           "n_iter": int(kw["n_iter"]), "sli": kw["sli"], "result_file": list(dumps)[0],
                           "time_first_last": [float(w["time"].iloc[0]), float(w["time"].iloc[-1])]})
    with open(os.path.join(HERE, "glue.json"), "w") as f:
        json.dump(out, f)
    print("glue.json", {k: len(v) for k, v in out.items()})


def frame_digest_py39(df) -> str:
    """frame_digest for either interpreter (same bytes: float64 C-order values + column names)."""
    return frame_digest(df)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--stage-b":
        return stage_b(sys.argv[2])
    with tempfile.TemporaryDirectory() as tmp:
        stage_a(tmp)
        env = dict(os.environ, PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1")
        subprocess.check_call([PY39, os.path.abspath(__file__), "--stage-b", tmp], env=env)


if __name__ == "__main__":
    main()
