#!/usr/bin/env python3
"""Numpy model of the "PC" (polyphase cascade) decimator: the interior of
log2(zoom) x scipy.signal.decimate(x, 2) (pypanadapter_spectrum.py:2096-2098) as
multistage FIR decimation plus all-pole recurrences at the OUTPUT rate.
Design tool, not used at run time.

H(z) = N(z) / D(z) is cheby1(8, .05, .4) (N = b0 (1 + z^-1)^8, D = prod of 4 sections).
Interior of K zero-phase stages (each followed by [::2]) = down-by-2^K of
prod_k |H(z^(2^k))|^2 (noble identity).  Every all-pole factor is moved to the output
rate w = z^(2^K) with the polyphase identity
    1 / D(z) = prod_{j=1}^{M-1} D(z W_M^j) / D_M(z^M),   D_M has the M-th powers of the poles,
and prod_{j=1}^{M-1} D(z W_M^j) = D(-z) D2(-z^2) D4(-z^4) ... splits into factors of
z, z^2, z^4, ..., so stage k's FIR gets the factors in z^(2^k):
    K = 3:  A(z) = N(z) D(-z)                      17 taps  -> zero-phase 33
            B(u) = N(u) D2(-u) D(-u)               25       -> 49   (u = z^2)
            C(v) = N(v) D4(-v) D2(-v) D(-v)        33       -> 65   (v = z^4)
            Q(w) = D8(w) D4(w) D2(w)               24 poles (radius <= 0.935^2 = 0.874)
    out = Q(w)^-1 Q(1/w)^-1 [ (CC')|2 (BB')|2 (AA')|2 x ]
The frame ends (odd extension, sosfilt_zi states) differ from this model only within a
few hundred output samples of each end; those come from the exact stage-wise path.
"""
import numpy as np
import scipy.signal as ss

SOS = ss.cheby1(8, 0.05, 0.4, output="sos")
B0 = SOS[0, 0]
A1, A2 = SOS[:, 4], SOS[:, 5]
N9 = B0 * np.array([1, 8, 28, 56, 70, 56, 28, 8, 1.0])


def neg(p):
    """p(z) -> p(-z) for a polynomial in z^-1."""
    return p * (-1.0) ** np.arange(len(p))


def conv(*ps):
    r = np.array([1.0])
    for p in ps:
        r = np.convolve(r, p)
    return r


def dpoly(a1, a2):
    return conv(*[np.array([1.0, a1[k], a2[k]]) for k in range(len(a1))])


def square_sections(a1, a2):
    """Sections of D2 (poles squared): (1 + a1 z^-1 + a2 z^-2)(1 - a1 z^-1 + a2 z^-2)
    = 1 + (2 a2 - a1^2) w^-1 + a2^2 w^-2."""
    return 2 * a2 - a1 ** 2, a2 ** 2


def stage_polys(K):
    """Per-stage FIR numerators (causal halves) and the output-rate all-pole sections."""
    secs = [(A1, A2)]                      # sections of D_{2^i}, i = 0..K
    for _ in range(K):
        secs.append(square_sections(*secs[-1]))
    polys = [dpoly(*s) for s in secs]      # D, D2, D4, D8 ...
    firs = []
    for k in range(K):
        # stage k (variable z^(2^k)) collects from every 1/D(z^(2^i)), i <= k, the
        # factor D_{2^(k-i)}(-.) ; plus N
        f = N9.copy()
        for i in range(k + 1):
            f = np.convolve(f, neg(polys[k - i]))
        firs.append(f)
    # output-rate denominators: from 1/D(z^(2^i)) -> D_{2^(K-i)}(w), i = 0..K-1
    q_secs = [secs[K - i] for i in range(K)]
    return firs, q_secs


def check_identity(K):
    firs, q_secs = stage_polys(K)
    w = np.linspace(0.01, np.pi - 0.01, 777)
    z = np.exp(1j * w)
    ev = lambda p, zz: np.polyval(p[::-1], 1 / zz)
    lhs = np.ones_like(z)
    for k in range(K):
        lhs *= ev(N9, z ** (2 ** k)) / ev(dpoly(A1, A2), z ** (2 ** k))
    rhs = np.ones_like(z)
    for k in range(K):
        rhs *= ev(firs[k], z ** (2 ** k))
    for a1, a2 in q_secs:
        rhs /= ev(dpoly(a1, a2), z ** (2 ** K))
    return np.abs(lhs - rhs).max()


def zp_fir(f):
    """Zero-phase FIR taps f(z) f(1/z), centred."""
    return np.convolve(f, f[::-1])


def pc_interior(x, K, dt=complex):
    """Interior model (frame ends not exact). Returns the output-rate sequence aligned
    with decimate^K(x) (index m <-> x index 2^K m)."""
    firs, q_secs = stage_polys(K)
    rdt = np.float32 if dt == np.complex64 else float
    y = x.astype(dt)
    for k in range(K):
        g = zp_fir(firs[k]).astype(rdt)
        c = (len(g) - 1) // 2
        full = np.convolve(y, g)                 # full[n] = sum_t g[t] y[n - t]
        # want out[m] = sum_t g[c + t] y[2m - t] = full[2m + c]
        y = full[c::2][: (len(y) + 1) // 2].astype(dt)
    sos = np.array([[1, 0, 0, 1, a1[j], a2[j]] for a1, a2 in q_secs for j in range(len(a1))])
    sos = sos.astype(rdt) if dt == np.complex64 else sos
    y = ss.sosfilt(sos, y)
    y = ss.sosfilt(sos, y[::-1])[::-1]
    return y.astype(dt)


def stats(K):
    firs, q_secs = stage_polys(K)
    out = []
    for k, f in enumerate(firs):
        g = zp_fir(f)
        out.append((k, len(g), g.sum(), np.abs(g).sum(), np.abs(g).max()))
    radii = []
    for a1, a2 in q_secs:
        radii += list(np.sqrt(np.abs(a2)))
    return out, radii


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for K in (1, 2, 3, 4):
        print(f"K={K} identity err {check_identity(K):.2e}")
        st, radii = stats(K)
        for k, n, s, sa, mx in st:
            print(f"  stage {k}: {n} taps  sum {s:.4g}  sum|g| {sa:.4g}  max {mx:.4g}  cancel {sa / abs(s):.3g}")
        print(f"  output-rate poles: {len(radii) * 2}, max radius {max(radii):.4f}")
    L = 299008
    x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)) / np.sqrt(2)
    n = np.arange(L)
    x += np.exp(2j * np.pi * 0.011 * n) + 0.1 * np.exp(-2j * np.pi * 0.027 * n)
    for K in (1, 2, 3):
        ref = x.copy()
        for _ in range(K):
            ref = ss.decimate(ref, 2)
        E = 400
        for dt in (complex, np.complex64):
            got = pc_interior(x, K, dt)
            err = np.abs(got[E:-E] - ref[E:-E]).max() / np.abs(ref).max()
            # edge reach: first index from the start where error < 1e-7 rel
            e = np.abs(got - ref) / np.abs(ref).max()
            bad = np.nonzero(e > (1e-6 if dt == np.complex64 else 1e-10))[0]
            lo = bad[bad < len(e) // 2].max() + 1 if (bad < len(e) // 2).any() else 0
            hi = len(e) - bad[bad >= len(e) // 2].min() if (bad >= len(e) // 2).any() else 0
            print(f"K={K} {np.dtype(dt).name}: interior max rel err {err:.2e}; edge reach {lo} / {hi} outputs")
