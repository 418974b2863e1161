"""CPU restatement of the CRT K1 arithmetic (corr.hip: crt_plan, k_residues, k_xtx_crt's epilogue,
k_crt_finish / crt_value), checked against the exact integer Gram in Python integers.

It pins the design choices the kernels rest on: the moduli count and bit width from N, offset-
binary residues through byte dot products with the offset folded into the accumulator, the
fp32 rint reduction (odd m, |s| < 2^19), the fp32 quotient estimate under the 0.01-bit margin, the
16-bit limb rebuild with signed carries, and the single rounding to fp64. Inputs include values
at the top of the range (|a| = 2^b - 1) and the largest N the plan allows per slab."""
import math

import numpy as np
import pytest

MODULI = [256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193, 191, 181, 179,
          173, 167, 163, 157, 151]
MAGIC = np.float32(12582912.0)


def plan(N, bmin=56):
    lm = 0.0
    for k, m in enumerate(MODULI, 1):
        lm += math.log2(m)
        b = math.floor((lm - math.log2(N) - 1.0 - 0.01) / 2.0)
        if b >= bmin:
            return k, min(b, 63)
    return None


def f32_fma(a, b, c):
    """fmaf: the exact a*b + c rounded once to fp32 (exact in fp64 for these operand sizes)."""
    return np.float32(np.float64(np.float32(a)) * np.float64(np.float32(b)) + np.float64(np.float32(c)))


def residue(a, m, b):
    """k_residues for one value: a + 2^b as (hi, lo) u32, byte dot products with the 2^(8q) mod m
    weights, the offset's residue subtracted in the accumulator, fp32 rint, the byte kept."""
    off = a + (1 << b)
    lo, hi = off & 0xFFFFFFFF, off >> 32
    if m == 256:
        return lo & 255
    wl = [pow(2, 8 * q, m) for q in range(4)]
    wh = [pow(2, 32 + 8 * q, m) for q in range(4)]
    s = sum(((lo >> (8 * q)) & 255) * wl[q] + ((hi >> (8 * q)) & 255) * wh[q] for q in range(4))
    s = (s - pow(2, b, m)) & 0xFFFFFFFF
    s = s - (1 << 32) if s >= 1 << 31 else s                    # the u32 accumulator read as int32
    assert abs(s) < 1 << 19
    x = np.float32(s)
    fi = np.float32(1.0) / np.float32(m)
    q = f32_fma(x, fi, MAGIC) - MAGIC                           # rint(s / m)
    r = int(f32_fma(q, np.float32(-m), x))
    assert -(m - 1) // 2 <= r <= (m - 1) // 2 and (s - r) % m == 0
    return r & 255


def rebuild(res_sums, k, b, ei=0, ej=0):
    """crt_value: z_i = r_i (M/m_i)^-1 mod m_i, S in 16-bit limbs, q from the fp32 sum, x = S - q M."""
    mods = MODULI[:k]
    M = math.prod(mods)
    L16 = 2 * (int(math.log2(M) // 32) + 1)
    acc, fs = [0] * L16, np.float32(0.0)
    for i, m in enumerate(mods):
        Mi = M // m
        y = pow(Mi % m, -1, m)
        z = (res_sums[i] * y) % m
        fs = f32_fma(z, np.float32(1.0) / np.float32(m), fs)
        for l in range(L16):
            acc[l] += z * ((Mi >> (16 * l)) & 0xFFFF)
    assert max(acc) < 1 << 29
    qq = math.floor(float(fs) + 0.5)
    carry, x = 0, 0
    for l in range(L16):
        v = carry + acc[l] - qq * ((M >> (16 * l)) & 0xFFFF)
        x |= (v & 0xFFFF) << (16 * l)
        carry = v >> 16
    if carry < 0:
        x -= 1 << (16 * L16)
    return x, math.ldexp(float(x), ei + ej - 2 * b) if x else 0.0


@pytest.mark.parametrize("N,top", [(1000, False), (10000, False), (10000, True), (130000, True)])
def test_crt_rebuild_is_the_exact_integer_gram(N, top):
    k, b = plan(N)
    M = math.prod(MODULI[:k])
    assert 56 <= b <= 63 and M > 2 * N * 4 ** b and (N != 10000 or (k, b) == (17, 59))
    rng = np.random.default_rng(N + top)
    cols = 2
    if top:     # |a| = 2^b - 1 with random signs: the Gram entries at (1 - 2^-b)^2 N 4^b
        A = [[int(sg) * ((1 << b) - 1) for sg in rng.choice([-1, 1], N)] for _ in range(cols)]
    else:
        A = [[int(v) for v in rng.integers(-(1 << 62), 1 << 62, N, dtype=np.int64) >> (63 - b)] for _ in range(cols)]
    for ca in range(cols):
        for cb in range(ca, cols):
            exact = sum(p * q for p, q in zip(A[ca], A[cb]))
            assert 2 * abs(exact) < M
            sums = []
            def bal(a, m):          # the balanced residue as k_residues stores it (its byte)
                r = a % m
                return (r - m if 2 * r > m else r) & 255
            for m in MODULI[:k]:
                # every value through the kernel's arithmetic at N = 1000; beyond, its result
                # (test_residue_matches_the_balanced_residue pins the two equal)
                ra = [residue(a, m, b) if N <= 1000 else bal(a, m) for a in A[ca]]
                rb = [residue(a, m, b) if N <= 1000 else bal(a, m) for a in A[cb]]
                # the GEMM: balanced int8 residues, exact int32 sums, reduced mod m to a byte
                sa = [r - 256 if r >= 128 else r for r in ra]
                sb = [r - 256 if r >= 128 else r for r in rb]
                sums.append(sum(p * q for p, q in zip(sa, sb)) % m)
            x, g = rebuild(sums, k, b)
            assert x == exact
            assert g == float(exact) * 2.0 ** (-2 * b)           # one rounding of the exact value


def test_residue_reduction_covers_every_accumulator_value():
    """The fp32 rint reduction is exact for every s the byte dot products can produce (|s| < 2^19)."""
    s = np.arange(-255, 8 * 255 * 255 + 1, dtype=np.int64)
    x = s.astype(np.float32)
    for m in MODULI[1:]:
        fi = np.float32(1.0) / np.float32(m)
        t = (x.astype(np.float64) * np.float64(fi) + np.float64(MAGIC)).astype(np.float32)
        q = (t - MAGIC).astype(np.float32)
        r = (x.astype(np.float64) - q.astype(np.float64) * m)
        assert np.all(np.abs(r) <= (m - 1) // 2)
        assert np.all((s - r.astype(np.int64)) % m == 0)


def test_residue_matches_the_balanced_residue():
    """k_residues' offset-binary byte-dot arithmetic equals the balanced residue (as a byte) for
    random values and the extremes +-(2^b - 1), 0, +-1, at every modulus and bit width."""
    rng = np.random.default_rng(5)
    for b in (56, 59, 63):
        vals = [0, 1, -1, (1 << b) - 1, -((1 << b) - 1)] + [int(v) >> (63 - b) for v in
                                                          rng.integers(-(1 << 62), 1 << 62, 200, dtype=np.int64)]
        for m in MODULI:
            for a in vals:
                r = a % m
                want = (r - m if 2 * r > m else r) & 255 if m != 256 else a & 255
                assert residue(a, m, b) == want, (a, m, b)
