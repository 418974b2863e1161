"""Golden vectors for RCD's frame glue, produced by EXECUTING the reference's own functions
(run in the build container, where /root/reference exists):

  python tests/golden/make_rcd_glue_golden.py

The pure-pandas / numpy helpers of ``RCAEval/e2e/rcd.py`` (``drop_constant`` :31-32,
``preprocess_sock_shop`` :36-55, ``add_fnode_and_concat`` :64-67, ``_order_neighbors`` :211-222,
``_preprocess_for_fnode`` :230-235, ``_select_useful_cols`` :238-251, ``_match_columns`` :255-257,
``_scale_down_mem`` :260-268, ``_select_lat`` :271-272, ``_discretize`` :278-289,
``create_chunks`` :307-315) are read out of the reference file with ``ast`` and executed on seeded
synthetic frames (the module's matplotlib / causal-learn imports are not executed). Only outputs
are stored (tests/golden/rcd_glue.json): column lists, sha256 digests of the output frames,
chunk partitions and neighbour orders. The reference code itself is never copied.
"""
from __future__ import annotations

import ast
import hashlib
import json
import os
import warnings

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/RCAEval/e2e/rcd.py"
FUNCS = {"drop_constant", "preprocess_sock_shop", "_select_lat", "_scale_down_mem", "_select_useful_cols",
         "_match_columns", "add_fnode_and_concat", "create_chunks", "_order_neighbors", "_discretize",
         "_preprocess_for_fnode"}
NAMES = {"_rm_time", "_list_intersection", "F_NODE"}
KINDS = ("cpu", "mem", "lat_50", "lat_90", "lat_99", "xlat_90")


def case_frame(t: int) -> pd.DataFrame:
    """Seeded Sock-Shop-shaped frame of case t (tests rebuild it the same way)."""
    rng = np.random.default_rng(1000 + t)
    cols = ["time"] + [f"s{i}_{k}" for i in range(4) for k in KINDS]
    X = rng.standard_normal((40, len(cols))) * rng.uniform(0.1, 5, len(cols))
    mem = [c.endswith("_mem") for c in cols]
    X[:, mem] = np.abs(X[:, mem]) * 1e7
    df = pd.DataFrame(X, columns=cols)
    for j in rng.choice(len(cols), 4, replace=False):
        df.iloc[:, j] = 1.0
    return df


def case_pvalues(t: int):
    """Seeded object array of p-value lists (ragged, as cg.p_values rows are)."""
    rng = np.random.default_rng(2000 + t)
    p = np.empty(6, object)
    for i in range(6):
        p[i] = [float(v) for v in rng.random(int(rng.integers(1, 4)))]
    return p


def frame_digest(df) -> str:
    a = np.ascontiguousarray(df.to_numpy(dtype=np.float64))
    h = hashlib.sha256(a.tobytes() + str(a.shape).encode() + "|".join(map(str, df.columns)).encode())
    return h.hexdigest()


def reference_namespace():
    from sklearn.preprocessing import KBinsDiscretizer
    tree = ast.parse(open(REF).read())
    keep = [n for n in tree.body
            if (isinstance(n, ast.FunctionDef) and n.name in FUNCS)
            or (isinstance(n, ast.Assign) and isinstance(n.targets[0], ast.Name) and n.targets[0].id in NAMES)]
    ns = {"np": np, "pd": pd, "KBinsDiscretizer": KBinsDiscretizer, "print": lambda *a, **k: None}
    exec(compile(ast.Module(body=keep, type_ignores=[]), REF, "exec"), ns)
    return ns


def main():
    warnings.simplefilter("ignore")
    ref = reference_namespace()
    out = []
    for t in range(12):
        df = case_frame(t)
        n_df, a_df = df.iloc[:20].copy(), df.iloc[20:].copy()
        if t % 3 == 0:
            a_df = a_df.drop(columns=[df.columns[3]])
        rec = {"case": t}
        for su in (False, True):
            nn, aa = ref["preprocess_sock_shop"](n_df.copy(), a_df.copy(), 90, su)
            rec[f"sock_shop_{int(su)}"] = {"columns": list(nn.columns), "normal": frame_digest(nn),
                                          "anomalous": frame_digest(aa)}
        rec["drop_constant"] = list(ref["drop_constant"](df).columns)
        seed = 7 * t + 3
        np.random.seed(seed)
        rec["chunks"] = {"seed": seed, "gamma": 5, "chunks": [list(c) for c in ref["create_chunks"](df, 5)]}
        rec["order"] = ref["_order_neighbors"]([f"v{i}" for i in range(6)], case_pvalues(t))
        disc = ref["_preprocess_for_fnode"](df.iloc[:20, 1:7].copy(), df.iloc[20:, 1:7].copy(), 5)
        rec["discretized"] = {"columns": list(disc.columns), "digest": frame_digest(disc)}
        out.append(rec)
    with open(os.path.join(HERE, "rcd_glue.json"), "w") as f:
        json.dump(out, f)
    print("rcd_glue.json", len(out))


if __name__ == "__main__":
    main()
