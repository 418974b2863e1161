"""Pure-Python replicas used by the CPU tests to pin the GPU kernels' arithmetic."""


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
