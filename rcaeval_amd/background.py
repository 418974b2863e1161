"""Background knowledge for the PC path: causal-learn ``BackgroundKnowledge`` [U] and its masks.

RCAEval builds one module-level instance (``RCAEval/graph_construction/pc.py:6-9``) and hands it
to ``pc`` when ``pc_default(..., with_bg=True)``. causal-learn (0.1.3.3, not vendored in the
reference) consults it in three places, which the engine reproduces from two n x n masks:

* skeleton, stable branch (``lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:86-106``): a pair
  forbidden in BOTH directions is queued for removal at depth 0 while its depth-0 test still
  runs (counts and p-values as without knowledge) — ``pcg_set_forbidden_pairs``;
* ``orient_by_background_knowledge`` before ``uc_sepset``, the collider skip in ``uc_sepset`` and
  the per-rule skip in ``meek`` — ``pcg_orient_bk`` (host C++).

Rule semantics follow the published class: a pattern rule matches ``re.match(pattern, name)``
(anchored at the start, not at the end); node rules compare node names; a tier map forbids
every edge from a later tier into an earlier one.
"""
from __future__ import annotations

import re

import numpy as np


def _name(node) -> str:
    return node.get_name() if hasattr(node, "get_name") else str(node)


class BackgroundKnowledge:
    """causal-learn ``BackgroundKnowledge`` [U]: same method names, chaining and type errors."""

    def __init__(self):
        self.forbidden_rules_specs = set()
        self.forbidden_pattern_rules_specs = set()
        self.required_rules_specs = set()
        self.required_pattern_rules_specs = set()
        self.tier_map: dict = {}
        self.tier_value_map: dict = {}

    # --- rules ---------------------------------------------------------------------------
    def add_forbidden_by_node(self, node1, node2):
        self.forbidden_rules_specs.add((_name(node1), _name(node2)))
        return self

    def add_required_by_node(self, node1, node2):
        self.required_rules_specs.add((_name(node1), _name(node2)))
        return self

    def add_forbidden_by_pattern(self, node_pattern1: str, node_pattern2: str):
        if type(node_pattern1) != str or type(node_pattern2) != str:
            raise TypeError("node_pattern must be type of str")
        self.forbidden_pattern_rules_specs.add((node_pattern1, node_pattern2))
        return self

    def add_required_by_pattern(self, node_pattern1: str, node_pattern2: str):
        if type(node_pattern1) != str or type(node_pattern2) != str:
            raise TypeError("node_pattern must be type of str")
        self.required_pattern_rules_specs.add((node_pattern1, node_pattern2))
        return self

    def add_node_to_tier(self, node, tier: int):
        if type(tier) != int:
            raise TypeError("tier must be type of int")
        if tier < 0:
            raise TypeError("tier must be a non-negative integer")
        self.tier_map[_name(node)] = tier
        self.tier_value_map.setdefault(tier, set()).add(_name(node))
        return self

    def remove_forbidden_by_node(self, node1, node2):
        self.forbidden_rules_specs.discard((_name(node1), _name(node2)))
        return self

    def remove_required_by_node(self, node1, node2):
        self.required_rules_specs.discard((_name(node1), _name(node2)))
        return self

    def remove_forbidden_by_pattern(self, node_pattern1: str, node_pattern2: str):
        self.forbidden_pattern_rules_specs.discard((node_pattern1, node_pattern2))
        return self

    def remove_required_by_pattern(self, node_pattern1: str, node_pattern2: str):
        self.required_pattern_rules_specs.discard((node_pattern1, node_pattern2))
        return self

    def remove_node_from_tier(self, node, tier: int):
        name = _name(node)
        if self.tier_map.get(name) == tier:
            del self.tier_map[name]
            self.tier_value_map[tier].discard(name)
        return self

    def is_in_which_tier(self, node) -> int:
        return self.tier_map.get(_name(node), -1)

    # --- queries (one pair) --------------------------------------------------------------
    def is_forbidden(self, node1, node2) -> bool:
        a, b = _name(node1), _name(node2)
        if (a, b) in self.forbidden_rules_specs:
            return True
        for p1, p2 in self.forbidden_pattern_rules_specs:
            if re.match(p1, a) is not None and re.match(p2, b) is not None:
                return True
        if a in self.tier_map and b in self.tier_map and self.tier_map[a] > self.tier_map[b]:
            return True
        return False

    def is_required(self, node1, node2) -> bool:
        a, b = _name(node1), _name(node2)
        if (a, b) in self.required_rules_specs:
            return True
        for p1, p2 in self.required_pattern_rules_specs:
            if re.match(p1, a) is not None and re.match(p2, b) is not None:
                return True
        return False

    # --- masks (all pairs at once) -------------------------------------------------------
    def masks(self, names) -> tuple[np.ndarray, np.ndarray]:
        """(forbidden, required) as n x n uint8, [i, j] = rule for names[i] -> names[j]; equal to
        ``is_forbidden`` / ``is_required`` pair by pair (each pattern is matched once per node)."""
        names = [_name(v) for v in names]
        n = len(names)
        index = {nm: i for i, nm in enumerate(names)}

        def build(node_rules, pattern_rules, tiers):
            M = np.zeros((n, n), bool)
            for a, b in node_rules:
                if a in index and b in index:
                    M[index[a], index[b]] = True
            cache: dict = {}

            def hits(p):
                if p not in cache:
                    cache[p] = np.array([re.match(p, nm) is not None for nm in names], bool)
                return cache[p]

            for p1, p2 in pattern_rules:
                M |= np.outer(hits(p1), hits(p2))
            if tiers:
                t = np.array([self.tier_map.get(nm, -1) for nm in names])
                has = t >= 0
                M |= np.outer(has, has) & (t[:, None] > t[None, :])
            return M.astype(np.uint8)

        return (build(self.forbidden_rules_specs, self.forbidden_pattern_rules_specs, True),
                build(self.required_rules_specs, self.required_pattern_rules_specs, False))


def banned_pairs(forbidden: np.ndarray) -> np.ndarray:
    """Pairs the stable skeleton removes at depth 0: forbidden both ways, off the diagonal."""
    B = (forbidden != 0) & (forbidden.T != 0)
    np.fill_diagonal(B, False)
    return B.astype(np.uint8)


__all__ = ["BackgroundKnowledge", "banned_pairs"]
