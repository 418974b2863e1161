"""Pure-Python replicas used by the CPU tests to pin the GPU kernels' arithmetic."""
import numpy as np


def pairwise_sum(a):
    """numpy's pairwise_sum (8 accumulators, 128-element leaves), as k_pagerank implements it."""
    n = len(a)
    if n < 8:
        r = 0.0
        for v in a:
            r += v
        return r
    if n <= 128:
        r = list(a[:8])
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += a[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return pairwise_sum(a[:n2]) + pairwise_sum(a[n2:])


def kernel_pagerank(A, d=0.85, n_iter=10, tol=1e-6):
    """Statement-by-statement replica of k_pagerank (rcaeval_amd/csrc/pagerank.hip)."""
    import numpy as np
    m = len(A)
    inv = [0.0] * m
    b = [0.0] * m
    for j in range(m):
        rs = 0.0
        for k in range(m):
            rs += abs(A[j][k])
        inv[j] = 1.0 / rs if rs != 0 else 0.0
        b[j] = (1.0 - d * (1.0 if rs != 0 else 0.0)) * (1.0 / m)
    cols = [[(j, d * (inv[j] * A[j][i])) for j in range(m) if A[j][i] != 0] for i in range(m)]
    s = list(b)
    for _ in range(n_iter):
        ss = pairwise_sum(s)
        s2 = []
        for i in range(m):
            acc = 0.0
            for j, v in cols[i]:
                acc += v * s[j]
            s2.append(acc + b[i] * ss)
        tot = pairwise_sum(s2)
        s2 = [v / tot for v in s2]
        diff = pairwise_sum([abs(x - y) for x, y in zip(s, s2)])
        if diff < tol:
            break
        s = s2
    fin = pairwise_sum(s)
    return np.array([v / fin for v in s])


def unions_from_oracle(ref, n):
    """Oracle side unions of removed ordered pairs, non-empty only: {(x, y): W-word tuple}."""
    import numpy as np
    W = (n + 63) // 64
    idx = np.argwhere(ref.removed_level > 0)
    if not len(idx):
        return {}
    rows = ref.side_union[idx[:, 0], idx[:, 1], :W]
    keep = rows.any(axis=1)
    return {(int(x), int(y)): tuple(int(b) for b in r) for (x, y), r in zip(idx[keep], rows[keep])}


def unions_from_engine(out):
    """Engine sepset-union rows (OR-ed per pair: an edge-sharded run may emit one per rank)."""
    rows = {}
    for (x, y), bits in zip(out.sep_xy, out.sep_bits):
        k = (int(x), int(y))
        v = tuple(int(b) for b in bits)
        rows[k] = tuple(a | b for a, b in zip(rows[k], v)) if k in rows else v
    return rows


def assert_skeleton_matches(out, ref, n, tests=True, unions=True):
    """Engine skeleton == oracle skeleton (removal depth of every pair, per-level unique-test
    counts, sepset unions), with the one exception north_star allows: a pair whose decision
    involves a test with |p - alpha| < 1e-9 (enumerated by either side) may differ. If such a
    pair's removal depth does differ, the graphs legitimately diverge after that depth, so
    everything is compared up to and including it. Returns the number of differing pairs."""
    import numpy as np
    near = {(int(r["a"]), int(r["b"])) for lst in (out.near_alpha, ref.near_alpha) for r in lst}
    rg, rr = np.asarray(out.removed_level), np.asarray(ref.removed_level)
    diff = np.argwhere(rg != rr)
    bad = [(int(x), int(y)) for x, y in diff if (min(x, y), max(x, y)) not in near]
    assert not bad, f"removal depth differs at {len(bad)} pairs outside near-alpha, e.g. " + str(
        [(p, int(rg[p]), int(rr[p])) for p in bad[:5]])
    if len(diff):   # a near-alpha flip: compare up to the first depth at which the graphs differ
        d0 = int(min(max(rg[x, y], rr[x, y]) for x, y in diff))
        rg = np.where((rg >= 0) & (rg <= d0), rg, -1)
        rr = np.where((rr >= 0) & (rr <= d0), rr, -1)
        iu = np.array([[min(x, y), max(x, y)] for x, y in diff])
        rg[iu[:, 0], iu[:, 1]] = rr[iu[:, 0], iu[:, 1]] = rg[iu[:, 1], iu[:, 0]] = rr[iu[:, 1], iu[:, 0]] = 0
        assert np.array_equal(rg, rr)
        levels = d0 + 1
    else:
        levels = len(ref.tests)
    if tests:
        assert list(out.stats["tests"][:levels]) == list(ref.tests[:levels])
    if unions:
        ug, ur = unions_from_engine(out), unions_from_oracle(ref, n)
        rl = np.asarray(ref.removed_level)
        keys = [k for k in set(ug) | set(ur)
                if (min(k), max(k)) not in near and 0 < rl[k] < levels]
        badu = [k for k in keys if ug.get(k) != ur.get(k)]
        assert not badu, f"sepset unions differ at {len(badu)} pairs, e.g. {badu[:5]}"
    return len(diff)


def loop_transition_matrix(adj, node_names, names, score_values=None, rho=0.5):
    """Statement-by-statement restatement of random_walk.py:267-296 + :156-178 (test only)."""
    m = len(adj)
    idx = {nm: i for i, nm in enumerate(names)}
    size = len(names)
    score = np.zeros(size) if score_values is None else np.asarray(score_values, float)
    edges = []
    for a in range(m):
        for b in range(m):
            ab, ba = int(adj[a, b]), int(adj[b, a])
            if ab == ba == 0:
                continue
            if (ab, ba) in ((-1, -1), (1, -1), (1, 0)):
                edges.append((b, a))
            elif (ab, ba) in ((-1, 1), (0, 1)):
                edges.append((a, b))
            elif (ab, ba) == (1, 1):
                edges += [(a, b), (b, a)]
            else:
                raise ValueError(f"Unexpected value: {adj[a, b]}, {adj[b, a]}")
    children = [set() for _ in range(size)]
    parents = [set() for _ in range(size)]
    for u, v in edges:                       # reversed: v -> u
        cu, cv = idx[node_names[u]], idx[node_names[v]]
        children[cv].add(cu)
        parents[cu].add(cv)
    M = np.zeros((size, size))
    for c in range(size):
        for ch in children[c]:
            M[ch, c] = rho * abs(score[ch])
        for pa in parents[c]:
            M[pa, c] = abs(score[pa])
        M[c, c] = max(abs(score[c]) - M[:, c].max(), 0)
        tot = M[:, c].sum()
        M[:, c] = M[:, c] / tot if tot > 0 else 1 / size
    return M


def networkx_digraph_matrix(adj):
    """pc_pagerank.py:20-29 written with networkx as the reference does (``to_numpy_array``: the
    values of networkx 2.5's ``to_numpy_matrix``, which 3.x removed; glue.json pins the 2.6.3
    call itself). Returns (matrix, sorted non-isolated nodes)."""
    import networkx as nx
    G = nx.DiGraph()
    for i in range(len(adj)):
        for j in range(len(adj)):
            if adj[i, j] == -1:
                G.add_edge(i, j)
            if adj[i, j] == 1:
                G.add_edge(j, i)
    nodes = sorted(G.nodes())
    return np.asarray(nx.to_numpy_array(G, nodelist=nodes)), nodes
