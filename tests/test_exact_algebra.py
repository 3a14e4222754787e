"""CPU checks of the exact-integer GRM's algebra (csrc/grm_exact.hip), in Python integers:

* the weight grid: F = 52 − emin puts every kept weight's fp64 significand on the integers (W_j = w_j 2^F
  exactly), and the digit count S of xg_choose holds the largest W_j in S balanced base-128 digits,
* the digits: W = Σ_s 128^s ω_s with ω_s ∈ [−64, 63], so d·ω and d·2ω (d ∈ {0, 1, 2}) fit int8,
* the centring identity G_ik = 2^−F/n² [n² A_ik − n U_i − n U_k + C] against the standardised-genotype
  GRM of the reference (src/gwas.jl:112-126 before the 1/q; Z from oracle/oracle.py) — exactly, with
  fractions, on a small case,
* the v_perm selector encoding of the B operand (d = 2 → the 2ω byte, 1 → the ω byte, 0 → zero).
"""
import math
from fractions import Fraction

import numpy as np

import oracle


def weights(D):
    n = D.shape[0]
    Di = D.astype(np.int64)
    t = Di.sum(0)
    s2 = (Di * Di).sum(0)
    num = n * s2 - t * t
    keep = num > 0
    w = np.where(keep, (float(n) * (n - 1.0)) / np.where(keep, num, 1).astype(np.float64), 0.0)
    return t, w, keep


def digit_max(S):
    """The largest integer S balanced base-128 digits in [-64, 63] represent: 63 (128^S - 1) / 127."""
    return 63 * (128 ** S - 1) // 127


def choose(w):
    """xg_choose: (S, F, exact)."""
    kept = w[w > 0]
    emin = min(math.frexp(x)[1] - 1 for x in kept)  # ilogb
    wmax = float(kept.max())
    F = 52 - emin
    W = int(Fraction(wmax) * 2 ** F)  # exact: the largest weight on the 2^-F grid
    for S in (8, 9, 10):
        if W <= digit_max(S):
            return S, F, True
    S = 10
    return S, 7 * S - 3 - (math.frexp(wmax)[1] - 1), False


def to_int(x, F):
    m, e = math.frexp(x)
    M = int(math.ldexp(m, 53))
    sh = e - 53 + F
    return M << sh if sh >= 0 else (M + (1 << (-sh - 1))) >> (-sh)


def digits(W, S):
    out = []
    x = W
    for _ in range(S):
        r = x & 127
        if r >= 64:
            r -= 128
        out.append(r)
        x = (x - r) >> 7
    assert x == 0
    return out


def random_dosages(seed, n, p, lo=0.05, hi=0.5):
    rng = np.random.default_rng(seed)
    return rng.binomial(2, rng.uniform(lo, hi, p), size=(n, p)).astype(np.int8)


def test_grid_and_digits_are_exact():
    for seed, (n, p) in enumerate([(300, 500), (2000, 200), (50, 1000)]):
        D = random_dosages(seed, n, p)
        D[:, 0] = 0
        D[3, 0] = 1  # a single carrier: the widest weight range
        t, w, keep = weights(D)
        S, F, exact = choose(w)
        assert exact and 8 <= S <= 10
        for x in w[keep]:
            W = to_int(float(x), F)
            assert Fraction(W, 2 ** F) == Fraction(float(x))  # the weight itself, no rounding
            ds = digits(W, S)
            assert sum(d * 128 ** s for s, d in enumerate(ds)) == W
            assert all(-64 <= d <= 63 for d in ds)
            assert all(-128 <= k * d <= 127 for d in ds for k in (1, 2))


def test_centring_identity_equals_standardised_grm():
    n, p = 40, 60
    D = random_dosages(7, n, p)
    t, w, keep = weights(D)
    S, F, _ = choose(w)
    Wint = [to_int(float(x), F) if k else 0 for x, k in zip(w, keep)]
    Di = D.astype(object)
    A = [[sum(Wint[j] * int(Di[i, j]) * int(Di[k, j]) for j in range(p)) for k in range(n)] for i in range(n)]
    U = [sum(Wint[j] * int(t[j]) * int(Di[i, j]) for j in range(p)) for i in range(n)]
    C = sum(Wint[j] * int(t[j]) ** 2 for j in range(p))
    G_exact = [[Fraction(n * n * A[i][k] - n * U[i] - n * U[k] + C, n * n * 2 ** F) for k in range(n)] for i in range(n)]
    # the same sum with rational centring and the fp64 weights
    for i in range(0, n, 7):
        for k in range(0, n, 5):
            ref = sum(Fraction(float(w[j])) * (int(Di[i, j]) - Fraction(int(t[j]), n)) * (int(Di[k, j]) - Fraction(int(t[j]), n))
                      for j in range(p) if keep[j])
            assert G_exact[i][k] == ref
    # and the reference's standardised genotypes (fp64 oracle) to rounding
    X = D.astype(np.float64) / 2.0
    m, s, kp = oracle.colstats(X)
    Z = oracle.standardize(X, m, s, kp)
    Gz = Z @ Z.T
    Gf = np.array([[float(v) for v in row] for row in G_exact])
    assert np.abs(Gf - Gz).max() < 1e-12 * np.abs(Gz).max()


def test_perm_selector_encoding():
    """The St byte at locus k (b = k mod 4) selects, in v_perm(src0 = ω dword, src1 = 2ω dword, sel): bytes
    0-3 come from src1, 4-7 from src0, 12 is the constant zero."""
    rng = np.random.default_rng(3)
    for _ in range(200):
        om = rng.integers(-64, 64, 4)
        d = rng.integers(0, 3, 4)
        src0 = bytes((int(x) & 0xFF) for x in om)
        src1 = bytes(((2 * int(x)) & 0xFF) for x in om)
        pool = src1 + src0  # byte index 0..7
        out = []
        for b in range(4):
            sel = b if d[b] == 2 else (4 + b if d[b] == 1 else 12)
            out.append(0 if sel == 12 else pool[sel])
        got = [x - 256 if x > 127 else x for x in out]
        assert got == [int(d[b]) * int(om[b]) for b in range(4)]


def _perm(src0, src1, sel):
    """v_perm_b32 for selector bytes 0-7 and 12 (the only ones the exact GRM uses)."""
    pool = [(src1 >> (8 * k)) & 0xFF for k in range(4)] + [(src0 >> (8 * k)) & 0xFF for k in range(4)]
    out = 0
    for b in range(4):
        s = (sel >> (8 * b)) & 0xFF
        v = 0 if s == 12 else pool[s]
        out |= v << (8 * b)
    return out


def test_selector_dword_formula():
    """xg_transpose_u_kernel builds the four St selectors of a dword of dosages at once:
    h = v_perm(0, 0x0000040C, a) (12 / 4 / 0 for d = 0 / 1 / 2) plus b where d > 0."""
    for a_b in np.ndindex(3, 3, 3, 3):
        a = sum(d << (8 * b) for b, d in enumerate(a_b))
        h = _perm(0, 0x0000040C, a)
        m = (a | (a >> 1)) & 0x01010101
        sw = (h + ((m * 0xFF) & 0x03020100)) & 0xFFFFFFFF
        want = sum(((b if d == 2 else (4 + b if d == 1 else 12)) << (8 * b)) for b, d in enumerate(a_b))
        assert sw == want


def test_u_limbs():
    """U_i = Σ_j V_j d_ij in four 24-bit limbs of V_j (V_j < 2^89), 32-bit limb sums over 64 loci."""
    rng = np.random.default_rng(5)
    for _ in range(20):
        V = [int(x) for x in rng.integers(0, 2 ** 62, 64)]
        V = [v * int(rng.integers(1, 2 ** 26)) for v in V]  # up to ~2^88
        d = [int(x) for x in rng.integers(0, 3, 64)]
        limbs = [0, 0, 0, 0]
        for v, dd in zip(V, d):
            for l in range(4):
                limbs[l] += dd * ((v >> (24 * l)) & 0xFFFFFF)
        assert max(limbs) < 2 ** 31
        assert sum(x << (24 * l) for l, x in enumerate(limbs)) == sum(v * dd for v, dd in zip(V, d))


def test_digit_count_at_the_range_boundary_matches_exact_integers():
    """xg_choose (csrc/grm_exact.hip, via the host-only gbm_debug_xg_choose) picks S by an exact integer
    comparison of W_max = w_max 2^F with 63 (128^S - 1)/127: weights at, just below and just above each boundary
    (where the former 1e-12 double slack could round the wrong way) get the S the Python integers give, and W_max
    then fits S balanced digits."""
    import ctypes

    import gbm
    lib = gbm.load_library()
    for S in (8, 9):
        F = 52  # wmin = 1.0: emin = 0
        for target in (digit_max(S), digit_max(S) - 1, digit_max(S) + 1, digit_max(S) - 2 ** 5):
            w0 = float(Fraction(target, 2 ** F))
            for wmax in (np.nextafter(w0, 0.0), w0, np.nextafter(w0, np.inf)):
                Sc, Fc = ctypes.c_int(0), ctypes.c_int(0)
                ex = lib.gbm_debug_xg_choose(1.0, float(wmax), ctypes.byref(Sc), ctypes.byref(Fc))
                W = int(Fraction(float(wmax)) * 2 ** F)
                want = next(s for s in (8, 9, 10) if W <= digit_max(s))
                assert ex == 1 and Fc.value == F and Sc.value == want, (S, target, wmax, Sc.value, want)
                assert W <= digit_max(Sc.value)
                # the balanced digits of W rebuild it within S digits (the device kernel's loop)
                x, digits = W, []
                for _ in range(Sc.value):
                    r = x & 127
                    r = r - 128 if r >= 64 else r
                    digits.append(r)
                    x = (x - r) >> 7
                assert x == 0 and sum(d * 128 ** k for k, d in enumerate(digits)) == W


def test_digit_overflow_is_flagged_exactly_past_the_boundary():
    """xg_digits_kernel's range check (csrc/grm_exact.hip: after S balanced base-128 digits the remainder x must be
    0, else XgInfo bit 2 and gbm_dev_grm_exact_status fails the call): W = 63 (128^S - 1)/127 is the largest W that
    S digits hold (remainder 0, digits rebuild W), W + 1 is the first that leaves a remainder; for S = 8, 9, 10."""
    def remainder(W, S):
        x = W
        for _ in range(S):
            r = x & 127
            r = r - 128 if r >= 64 else r
            x = (x - r) >> 7
        return x

    for S in (8, 9, 10):
        top = digit_max(S)
        assert top == 63 * (128 ** S - 1) // 127
        assert remainder(top, S) == 0 and digits(top, S) == [63] * S
        assert remainder(top + 1, S) != 0
        assert remainder(top - 1, S) == 0
        # forcing S - 1 digits on a weight that needs S (GBM_XG_TEST_S, the GPU test's fault injection) is flagged
        assert remainder(digit_max(S - 1) + 1, S - 1) != 0
