"""CPU checks of the PC decimator's host tables (pc_tables.cpp, no GPU needed):

* the FIR taps equal the polyphase factorisation rebuilt here from scipy's cheby1 sections;
* the LTI model those tables describe plus the library's shipped frame-end maps
  (pc_edge_maps.h, equal bit for bit to the fp64 builder's) reproduces
  3 x scipy.signal.decimate(x, 2) -- the reference's zoomfft at zoom 8
  (pypanadapter_spectrum.py:2096-2098) -- in float64, for every L mod 8.

The model is rebuilt here independently (numpy convolutions + scipy sosfilt of the same pole
moves) so this pins the tables the kernels read, not the library against itself."""
import ctypes

import numpy as np
import pytest
import scipy.signal as ss

SOS = ss.cheby1(8, 0.05, 0.4, output="sos")


def _lib():
    from pypanadapter_amd import _lib as L, build
    build.build()
    lib = L.load()
    f = lib.zfft__pc_tables
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    f.restype = ctypes.c_int
    return f


def _call(what, arg=0):
    f = _lib()
    buf = np.zeros(1 << 20, np.float32)
    n = f(what, arg, buf.ctypes.data, buf.size)
    assert n > 0, (what, arg, n)
    return buf[:n].astype(np.float64)


def _neg(p):
    p = p.copy()
    p[1::2] *= -1
    return p


def _conv(*ps):
    r = np.array([1.0])
    for p in ps:
        r = np.convolve(r, p)
    return r


def _secs():
    a1, a2 = SOS[:, 4].copy(), SOS[:, 5].copy()
    out = [(a1, a2)]
    for _ in range(3):
        a1, a2 = 2 * a2 - a1 ** 2, a2 ** 2
        out.append((a1, a2))
    return out


def _poly(a1, a2, idx):
    return _conv(*[np.array([1.0, a1[i], a2[i]]) for i in idx])


def _model():
    s = _secs()
    n9 = SOS[0, 0] * np.array([1, 8, 28, 56, 70, 56, 28, 8, 1.0])
    f0 = _conv(n9, _neg(_poly(*s[0], range(4))))
    f1 = _conv(n9, _neg(_poly(*s[1], range(4))), _neg(_poly(*s[0], range(4))))
    f2 = _conv(n9, _neg(_poly(*s[2], range(4))), _neg(_poly(*s[1], range(4))), _neg(_poly(*s[0], [0, 1])))
    g = [np.convolve(f, f[::-1]) for f in (f0, f1, f2)]
    own = [(s[0][0][i], s[0][1][i]) for i in (2, 3)]
    ap = [(s[3][0][i], s[3][1][i]) for i in range(4)] + [(s[2][0][i], s[2][1][i]) for i in range(4)] + \
         [(s[1][0][i], s[1][1][i]) for i in (0, 1)]
    return g, own, ap


def _run_model(x, g, own, ap):
    pad = 4096
    y = np.concatenate([np.zeros(pad), x, np.zeros(pad)])
    for r in range(3):
        if r == 2:
            so = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in own])
            y = ss.sosfilt(so, ss.sosfilt(so, y)[::-1])[::-1]
        c = (len(g[r]) - 1) // 2
        y = np.convolve(y, g[r])[c::2][:len(y) // 2]
    sa = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in ap])
    y = ss.sosfilt(sa, ss.sosfilt(sa, y)[::-1])[::-1]
    n3 = len(x)
    for _ in range(3):
        n3 = (n3 + 1) // 2
    return y[pad // 8:pad // 8 + n3]


def test_pc_fir_taps_match_polyphase_factorisation():
    g, _, _ = _model()
    taps = _call(0)
    want = np.concatenate(g)
    assert taps.size == want.size == 33 + 49 + 57
    np.testing.assert_allclose(taps, want, rtol=0, atol=4e-8 * np.abs(want).max())
    for k, gg in enumerate(g):  # zero phase: symmetric taps
        np.testing.assert_allclose(gg, gg[::-1], atol=1e-15)


def _edge_built(side, lm):
    """U (R x r), V (J x r) of the library's fp64 builder, run now."""
    v = _call(2 + side, lm)
    R, J, r = int(v[0]), int(v[1]), int(v[2])
    return v[3:3 + R * r].reshape(R, r), v[3 + R * r:3 + R * r + J * r].reshape(J, r)


def _edge_shipped(side, lm):
    """U, V of the constant map the plan uploads (pc_edge_maps.h, stored U then V^T)."""
    v = _call(4, 0 if side == 0 else 1 + lm)
    R, J, r = int(v[0]), int(v[1]), int(v[2])
    return v[3:3 + R * r].reshape(R, r), v[3 + R * r:3 + R * r + J * r].reshape(r, J).T


def _edge(side, lm):
    U, V = _edge_shipped(side, lm)
    return U @ V.T


@pytest.mark.parametrize("side,lm", [(0, 0)] + [(1, k) for k in range(8)])
def test_shipped_edge_maps_are_the_builders(side, lm):
    """pc_edge_maps.h (tools/gen_pc_edge.py) holds exactly what pc_edge_map builds today: the
    constants cannot drift from the sources they were generated from."""
    Ub, Vb = _edge_built(side, lm)
    Us, Vs = _edge_shipped(side, lm)
    assert Ub.shape == Us.shape and Vb.shape == Vs.shape
    np.testing.assert_array_equal(Us, Ub)
    np.testing.assert_array_equal(Vs, Vb)


@pytest.mark.parametrize("L", [16384, 16385, 16386, 16387, 20004, 20005, 20006, 20007])
def test_pc_model_plus_edge_maps_is_reference_decimate(L):
    g, own, ap = _model()
    rng = np.random.default_rng(L)
    x = rng.standard_normal(L) + 1j * rng.standard_normal(L)
    x += 3 * np.exp(2j * np.pi * 0.013 * np.arange(L))
    ref = x
    for _ in range(3):
        ref = ss.decimate(ref, 2)
    out = _run_model(x, g, own, ap)
    inner = np.abs(out - ref)[200:-200].max() / np.abs(ref).max()
    assert inner < 1e-12, inner        # the pole moves are exact in the interior
    CL, CR = _edge(0, L % 8), _edge(1, L % 8)
    out[:CL.shape[0]] += CL @ x[:CL.shape[1]]
    out[len(out) - CR.shape[0]:] += (CR @ x[::-1][:CR.shape[1]])[::-1]
    err = np.abs(out - ref).max() / np.abs(ref).max()
    assert err < 2e-7, err             # fp32 storage of the rank-~10 maps


# ---- zoom 4 (two stages; PcTab4, pc_walk_kernel<4>) ----

def _model4():
    s = _secs()
    n9 = SOS[0, 0] * np.array([1, 8, 28, 56, 70, 56, 28, 8, 1.0])
    f0 = _conv(n9, _neg(_poly(*s[0], range(4))))
    f1 = _conv(n9, _neg(_poly(*s[1], range(4))), _neg(_poly(*s[0], [0, 1])))
    g = [np.convolve(f, f[::-1]) for f in (f0, f1)]
    own = [(s[0][0][i], s[0][1][i]) for i in (2, 3)]
    ap = [(s[2][0][i], s[2][1][i]) for i in range(4)] + [(s[1][0][i], s[1][1][i]) for i in (0, 1)]
    return g, own, ap


def _run_model4(x, g, own, ap):
    pad = 4096
    y = np.concatenate([np.zeros(pad), x, np.zeros(pad)])
    for r in range(2):
        if r == 1:
            so = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in own])
            y = ss.sosfilt(so, ss.sosfilt(so, y)[::-1])[::-1]
        c = (len(g[r]) - 1) // 2
        y = np.convolve(y, g[r])[c::2][:len(y) // 2]
    sa = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in ap])
    y = ss.sosfilt(sa, ss.sosfilt(sa, y)[::-1])[::-1]
    n2 = (len(x) + 1) // 2
    n2 = (n2 + 1) // 2
    return y[pad // 4:pad // 4 + n2]


def _edge4(side, lm, shipped=False):
    if shipped:
        v = _call(14, 0 if side == 0 else 1 + lm)
        R, J, r = int(v[0]), int(v[1]), int(v[2])
        return v[3:3 + R * r].reshape(R, r), v[3 + R * r:3 + R * r + J * r].reshape(r, J).T
    v = _call(12 + side, lm)
    R, J, r = int(v[0]), int(v[1]), int(v[2])
    return v[3:3 + R * r].reshape(R, r), v[3 + R * r:3 + R * r + J * r].reshape(J, r)


def test_pc4_fir_taps_match_polyphase_factorisation():
    g, _, _ = _model4()
    taps = _call(5)
    want = np.concatenate(g)
    assert taps.size == want.size == 33 + 41
    np.testing.assert_allclose(taps, want, rtol=0, atol=4e-8 * np.abs(want).max())


@pytest.mark.parametrize("side,lm", [(0, 0)] + [(1, k) for k in range(4)])
def test_pc4_shipped_edge_maps_are_the_builders(side, lm):
    Ub, Vb = _edge4(side, lm)
    Us, Vs = _edge4(side, lm, shipped=True)
    assert Ub.shape == Us.shape and Vb.shape == Vs.shape
    np.testing.assert_array_equal(Us, Ub)
    np.testing.assert_array_equal(Vs, Vb)


@pytest.mark.parametrize("L", [16384, 16385, 16386, 16387, 20006, 262144 + 1])
def test_pc4_model_plus_edge_maps_is_reference_decimate(L):
    """Zoom 4 (cfg1): the two-stage model and its shipped frame-end maps give scipy's
    decimate(decimate(x, 2), 2) -- the reference's zoomfft at ratio 4 -- for every L mod 4."""
    g, own, ap = _model4()
    rng = np.random.default_rng(L + 4)
    x = rng.standard_normal(L) + 1j * rng.standard_normal(L)
    x += 3 * np.exp(2j * np.pi * 0.027 * np.arange(L))
    ref = ss.decimate(ss.decimate(x, 2), 2)
    out = _run_model4(x, g, own, ap)
    assert out.shape == ref.shape
    inner = np.abs(out - ref)[300:-300].max() / np.abs(ref).max()
    assert inner < 1e-12, inner
    UL, VL = _edge4(0, L % 4, shipped=True)
    UR, VR = _edge4(1, L % 4, shipped=True)
    CL, CR = UL @ VL.T, UR @ VR.T
    out[:CL.shape[0]] += CL @ x[:CL.shape[1]]
    out[len(out) - CR.shape[0]:] += (CR @ x[::-1][:CR.shape[1]])[::-1]
    err = np.abs(out - ref).max() / np.abs(ref).max()
    assert err < 2e-7, err


# ---- zoom 2 (one stage; PcTab2, pc_tail_kernel<2>: XA's factorisation as tiles) ----

def _model2():
    """v = x / D(z) (4 sections, causal), u = (M * v)|2 with M = N(z) N(1/z) D(-1/z) as the
    powers z^-8 .. z^16, out = u / D2(1/w) (4 sections, anticausal), sections slowest first."""
    s = _secs()
    n9 = SOS[0, 0] * np.array([1, 8, 28, 56, 70, 56, 28, 8, 1.0])
    dneg = _neg(_poly(*s[0], range(4)))           # D(-z): coefficient k of z^-k
    # Laurent product, as {power: coefficient}
    terms = {}
    for k, a in enumerate(n9):                      # N(z): z^-k
        for j, b in enumerate(n9):                  # N(1/z): z^+j
            for q, c in enumerate(dneg):            # D(-1/z): z^+q
                p = -k + j + q
                terms[p] = terms.get(p, 0.0) + a * b * c
    M = np.array([terms[p] for p in range(-8, 17)])
    own = sorted([(s[0][0][i], s[0][1][i]) for i in range(4)], key=lambda p: -p[1])
    ap = sorted([(s[1][0][i], s[1][1][i]) for i in range(4)], key=lambda p: -p[1])
    return M, own, ap


def _edge2(side, lm, shipped=False):
    if shipped:
        v = _call(17, 0 if side == 0 else 1 + lm)
        R, J, r = int(v[0]), int(v[1]), int(v[2])
        return v[3:3 + R * r].reshape(R, r), v[3 + R * r:3 + R * r + J * r].reshape(r, J).T
    v = _call(15 + side, lm)
    R, J, r = int(v[0]), int(v[1]), int(v[2])
    return v[3:3 + R * r].reshape(R, r), v[3 + R * r:3 + R * r + J * r].reshape(J, r)


def test_pc2_taps_and_sections():
    """Zoom 2's FIR is M = N(z) N(1/z) D(-1/z) (25 taps, z^-8 first), its input-rate sections
    the stage's four and its output-rate sections those squared (D2), slowest first."""
    M, own, ap = _model2()
    v = _call(6)
    assert v.size == 25 + 8 + 8
    np.testing.assert_allclose(v[:25], M, rtol=0, atol=6e-8 * np.abs(M).max())  # fp32 taps
    np.testing.assert_allclose(v[25:33].reshape(4, 2), np.array(own), rtol=1e-7)
    np.testing.assert_allclose(v[33:].reshape(4, 2), np.array(ap), rtol=1e-7)


@pytest.mark.parametrize("side,lm", [(0, 0), (1, 0), (1, 1)])
def test_pc2_shipped_edge_maps_are_the_builders(side, lm):
    Ub, Vb = _edge2(side, lm)
    Us, Vs = _edge2(side, lm, shipped=True)
    assert Ub.shape == Us.shape and Vb.shape == Vs.shape
    np.testing.assert_array_equal(Us, Ub)
    np.testing.assert_array_equal(Vs, Vb)


@pytest.mark.parametrize("L", [16384, 16385, 20006, 262144 + 1])
def test_pc2_model_plus_edge_maps_is_reference_decimate(L):
    """Zoom 2 (the UI's default fft_ratio, S:1497): the one-stage model -- D forward at the
    input rate, M, D2 backward at half rate -- and its shipped frame-end maps give scipy's
    decimate(x, 2) for both L mod 2."""
    M, own, ap = _model2()
    rng = np.random.default_rng(L + 2)
    x = rng.standard_normal(L) + 1j * rng.standard_normal(L)
    x += 3 * np.exp(2j * np.pi * 0.041 * np.arange(L))
    ref = ss.decimate(x, 2)
    pad = 4096
    y = np.concatenate([np.zeros(pad), x, np.zeros(pad)])
    so = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in own])
    v = ss.sosfilt(so, y)
    m = np.arange(len(y) // 2)
    u = np.zeros(len(m), complex)
    for i, c in enumerate(M):                  # u[m] = sum_p M_p v[2 m + p], p = i - 8
        idx = 2 * m + i - 8
        ok = (idx >= 0) & (idx < len(v))
        u[ok] += c * v[idx[ok]]
    sa = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in ap])
    out = ss.sosfilt(sa, u[::-1])[::-1][pad // 2:pad // 2 + (L + 1) // 2]
    assert out.shape == ref.shape
    inner = np.abs(out - ref)[300:-300].max() / np.abs(ref).max()
    assert inner < 1e-12, inner
    UL, VL = _edge2(0, L % 2, shipped=True)
    UR, VR = _edge2(1, L % 2, shipped=True)
    CL, CR = UL @ VL.T, UR @ VR.T
    out[:CL.shape[0]] += CL @ x[:CL.shape[1]]
    out[len(out) - CR.shape[0]:] += (CR @ x[::-1][:CR.shape[1]])[::-1]
    err = np.abs(out - ref).max() / np.abs(ref).max()
    assert err < 2e-7, err
