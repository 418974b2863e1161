"""RCA method plug-ins on the MI355X engine (mirror of ``RCAEval/e2e``).

``rca`` mirrors the reference wrapper (``RCAEval/e2e/__init__.py:21-31``): an exception
raised by the method returns the dummy ranking ``preprocess(data, dataset).columns`` — engine
run-time errors (``PcgError``: an overflowed list, a HIP error) included, with a warning, so an
RQ2 run records dummy ranks for that case like the reference would. Only ``EngineUnavailable``
(no GPU, library missing) propagates: there is no CPU path to degrade to, and a run without the
engine must fail loudly rather than score every case with dummy ranks.
"""
from __future__ import annotations

import functools
import warnings

from .._lib import EngineUnavailable, PcgError
from ..io.time_series import preprocess


def rca(func):
    """Tolerate method failures like the reference's ``@rca`` (``e2e/__init__.py:21-31``)."""
    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        try:
            return func(*args, **kwargs)
        except EngineUnavailable:
            raise
        except Exception as e:
            if isinstance(e, PcgError):
                warnings.warn(f"{func.__name__}: engine error, dummy ranks returned: {e}")
            data = preprocess(data=args[0], dataset=kwargs.get("dataset"), dk_select_useful=False)
            names = data.columns.to_list()
            return {"adj": [], "node_names": names, "ranks": names}
    return wrapper


from .circa import circa  # noqa: E402
from .cloudranger import cloudranger  # noqa: E402
from .pc_pagerank import pc_pagerank  # noqa: E402
from .fci_pagerank import fci_pagerank  # noqa: E402
from .pc_randomwalk import fci_randomwalk, pc_randomwalk  # noqa: E402

__all__ = ["rca", "circa", "cloudranger", "fci_pagerank", "fci_randomwalk", "pc_pagerank", "pc_randomwalk"]
