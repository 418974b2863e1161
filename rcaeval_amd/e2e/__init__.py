"""RCA method plug-ins on the MI355X engine (mirror of ``RCAEval/e2e``).

``rca`` mirrors the reference wrapper (``RCAEval/e2e/__init__.py:21-31``): an exception
raised by the method returns the dummy ranking ``preprocess(data, dataset).columns``.
Engine-availability failures (no GPU, library missing, HIP errors) are NOT swallowed —
there is no CPU fallback to degrade to, so they propagate.
"""
from __future__ import annotations

import functools

from .._lib import EngineUnavailable, PcgError
from ..io.time_series import preprocess


def rca(func):
    """Tolerate method failures like the reference's ``@rca`` (``e2e/__init__.py:21-31``)."""
    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        try:
            return func(*args, **kwargs)
        except (EngineUnavailable, PcgError):
            raise
        except Exception:
            data = preprocess(data=args[0], dataset=kwargs.get("dataset"), dk_select_useful=False)
            names = data.columns.to_list()
            return {"adj": [], "node_names": names, "ranks": names}
    return wrapper


from .circa import circa  # noqa: E402
from .cloudranger import cloudranger  # noqa: E402
from .pc_pagerank import pc_pagerank  # noqa: E402
from .pc_randomwalk import pc_randomwalk  # noqa: E402

__all__ = ["rca", "circa", "cloudranger", "pc_pagerank", "pc_randomwalk"]
