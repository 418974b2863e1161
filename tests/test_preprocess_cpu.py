"""CPU: preprocess's one-pass numpy path (io/time_series._drop_time_constant_mem) equals the
reference-shaped pandas composition convert_mem_mb(drop_constant(drop_time(df))) exactly —
values bitwise, dtypes, column order, index — on RQ2-shaped frames with NaN, constant columns,
single rows and a 'Time' column; frames outside its domain fall back to the pandas path."""
import numpy as np
import pandas as pd

from rcaeval_amd import synth
from rcaeval_amd.io import time_series as ts


def test_fast_path_equals_pandas_composition():
    rng = np.random.default_rng(0)
    for trial in range(150):
        m = int(rng.integers(3, 30))
        rows = int(rng.integers(1, 50))
        df = synth.telemetry_frame(m, rows, n_constant=int(rng.integers(0, 3)), seed=trial)
        if trial % 3 == 0:
            df.iloc[rng.integers(0, rows, 3), rng.integers(1, df.shape[1], 3)] = np.nan
        if trial % 5 == 0:
            df.iloc[:, 1] = df.iloc[0, 1]
        if trial % 7 == 0:
            df = df.rename(columns={"time": "Time"})
        fast = ts._drop_time_constant_mem(df)
        slow = ts.convert_mem_mb(ts.drop_constant(ts.drop_time(df)))
        assert fast is not None
        pd.testing.assert_frame_equal(fast, slow, check_exact=True)
        a, b = fast.to_numpy(), slow.to_numpy()
        assert np.array_equal(a.view(np.int64)[~np.isnan(b)], b.view(np.int64)[~np.isnan(b)])
        pd.testing.assert_frame_equal(ts.preprocess(df, dataset="online-boutique"), slow, check_exact=True)


def test_fast_path_declines_other_frames():
    df = synth.telemetry_frame(6, 20, n_constant=1, seed=1)
    assert ts._drop_time_constant_mem(df.iloc[:0]) is None                     # empty
    obj = df.copy()
    obj[obj.columns[2]] = obj[obj.columns[2]].astype(object)
    assert ts._drop_time_constant_mem(obj) is None                             # non-float column
    dup = df.copy()
    dup.columns = [df.columns[0]] + [df.columns[1]] * (df.shape[1] - 1)
    assert ts._drop_time_constant_mem(dup) is None                             # duplicate names
    for frame in (obj,):
        pd.testing.assert_frame_equal(ts.preprocess(frame, dataset="sock-shop"),
                                      ts.convert_mem_mb(ts.drop_constant(ts.drop_time(frame))))
