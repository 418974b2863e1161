"""Column filters applied before PC — mirror of ``RCAEval/io/time_series.py``.

Behaviour follows the reference functions (file:line in each docstring); it is pinned by
golden vectors generated from the reference module (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np
import pandas as pd

_EXTRA_PREFIXES = ("main_", "PassthroughCluster_", "redis_", "rabbitmq", "queue", "session",
                   "istio-proxy")


def drop_constant(df: pd.DataFrame) -> pd.DataFrame:
    """Keep columns with any value differing from row 0 (``time_series.py:4-5``)."""
    keep = df.ne(df.iloc[0]).any(axis=0)
    return df.loc[:, keep]


def drop_near_constant(df: pd.DataFrame, threshold: float = 0.1) -> pd.DataFrame:
    """Keep columns whose share of values differing from row 0 exceeds ``threshold`` (``:8-9``)."""
    share = df.ne(df.iloc[0]).mean(axis=0)
    return df.loc[:, share > threshold]


def drop_time(df: pd.DataFrame) -> pd.DataFrame:
    """Drop ``time`` (else ``Time``) (``:12-17``)."""
    for name in ("time", "Time"):
        if name in df:
            return df.drop(columns=[name])
    return df


def drop_extra(df: pd.DataFrame) -> pd.DataFrame:
    """Drop ``time.1`` and infrastructure columns (``:20-39``)."""
    if "time.1" in df:
        df = df.drop(columns=["time.1"])
    doomed = [c for c in df.columns if "frontend-external" in c or c.startswith(_EXTRA_PREFIXES)]
    for c in doomed:
        df = df.drop(columns=[c])
    return df


def convert_mem_mb(df: pd.DataFrame) -> pd.DataFrame:
    """Divide every ``*_mem`` column by 1e6 (``:42-51``)."""
    def scale(col: pd.Series) -> pd.Series:
        return col / 1e6 if col.name.endswith("_mem") else col
    return df.apply(scale)


def select_useful_cols(data: pd.DataFrame) -> list:
    """Domain-knowledge column selection (``:65-84``)."""
    picked = []
    for c in data.columns:
        if "time" in c:
            picked.append(c)
        if c.endswith("_cpu") and data[c].std() > 1:
            picked.append(c)
        if c.endswith("_mem") and data[c].std() > 1:
            picked.append(c)
        if "lat50" in c and (data[c] * 1000).std() > 10:
            picked.append(c)
    return picked


def _drop_time_constant_mem(data: pd.DataFrame):
    """``convert_mem_mb(drop_constant(drop_time(data)))`` in one numpy pass for the frames RQ2
    hands over (str column names without duplicates, every non-time column float64); None when
    the frame is not of that kind (the pandas composition then runs). Same values bitwise: the
    same != row 0 test (NaN != NaN), the same IEEE division by 1e6, columns in the same order."""
    names = data.columns
    if len(data) == 0 or names.has_duplicates or not all(isinstance(c, str) for c in names):
        return None
    tn = "time" if "time" in names else ("Time" if "Time" in names else None)
    pos = [i for i, c in enumerate(names) if c != tn]
    dts = data.dtypes.to_numpy()
    if not pos or any(dts[i] != np.float64 for i in pos):
        return None
    v = data.iloc[:, pos].to_numpy()
    keep = np.flatnonzero((v != v[0]).any(axis=0))
    v = v[:, keep]                                               # a new array: safe to scale
    cols = names.take(pos).take(keep)
    mem = [i for i, c in enumerate(cols) if c.endswith("_mem")]
    if mem:
        v[:, mem] /= 1e6
    return pd.DataFrame(v, index=data.index, columns=cols)


def preprocess(data: pd.DataFrame, dataset=None, dk_select_useful: bool = False) -> pd.DataFrame:
    """``preprocess`` (``:96-111``): identity when ``dataset`` is None."""
    if dataset == "causalrca-sock-shop":
        return drop_time(data)
    if dataset is None:
        return data
    out = _drop_time_constant_mem(data)
    if out is None:
        out = convert_mem_mb(drop_constant(drop_time(data)))
    if dk_select_useful is True:
        out = drop_near_constant(drop_extra(out))
        out = out[select_useful_cols(out)]
    return out
