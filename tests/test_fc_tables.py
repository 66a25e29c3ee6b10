"""CPU checks of the FC decimator's host tables (pc_tables.cpp fc_build_row / fc_build_twiddles;
kernel fc_kernels.hip), no GPU needed:

* the zoom-8 model's input-rate response g (rebuilt here from scipy's cheby1 sections:
  |H(z)|^2 |H(z^2)|^2 |H(z^4)|^2) truncated at |k| <= 768, together with the shipped frame-end
  maps, reproduces 3 x scipy.signal.decimate(x, 2) (pypanadapter_spectrum.py:2096-2098) with the
  LO mixed in (S:2088-2094) to 7e-7 in float64 (measured 5.6e-7; at 1024 it would be 2e-7);
* the library's filter rows equal that g's modulated, folded spectrum built here;
* one block computed in numpy with the kernel's own index maps (passes A, B, C, the residue MAC
  with the library's row in the kernel's [4 k3 + r/2][t] order, the five inverse radix-4 stages)
  equals the direct overlap-save formula -- the index algebra of the kernel, pinned on CPU."""
import numpy as np
import pytest
import scipy.signal as ss

from test_pc_tables import _call, _edge

SOS = ss.cheby1(8, 0.05, 0.4, output="sos")
N, M, K, P = 8192, 1024, 768, 832      # fc_kernels.hip: kFcN, kFcN / 8, kFcK, kFcP


def _g():
    imp = np.zeros(6000)
    imp[0] = 1
    h = ss.sosfilt(SOS, imp)
    r = np.convolve(h, h[::-1])
    g = r
    for up in (2, 4):
        ru = np.zeros((len(r) - 1) * up + 1)
        ru[::up] = r
        g = np.convolve(g, ru)
    c = len(g) // 2
    return g[c - K:c + K + 1]


def _lo(L, ratio):
    return np.sqrt(2) * np.exp(-2j * np.pi * np.mod(np.arange(L) * ratio, 1.0))


def _c_table(ratio):
    """C[k][r] = W_N^(rk) sum_q G[k + M q] W_8^(rq) / (N sqrt 2), G = DFT of g e^(2 pi i ratio k)."""
    g = _g()
    k = np.arange(-K, K + 1)
    gc = np.zeros(N, complex)
    gc[k % N] = g * np.exp(2j * np.pi * np.mod(ratio * k, 1.0))
    G = np.fft.fft(gc)
    kk = np.arange(M)[:, None]
    r = np.arange(8)[None, :]
    S = sum(G[kk[:, 0] + M * q][:, None] * np.exp(-2j * np.pi * r * q / 8) for q in range(8))
    return S * np.exp(-2j * np.pi * r * kk / N) / (N * np.sqrt(2))


def _lib_row(arg):
    v = _call(19, arg)
    z = v[0::2] + 1j * v[1::2]                         # float2 index ((4 k3 + r/2) 256 + t) 2 + r%2
    C = np.zeros((M, 8), complex)
    for t in range(256):
        kp = (t >> 4) + 16 * (t & 15)
        for k3 in range(4):
            for r in range(8):
                C[kp + 256 * k3, r] = z[((4 * k3 + r // 2) * 256 + t) * 2 + (r & 1)]
    return C


def test_fc_twiddles():
    v = _call(18)
    w = v[0::2] + 1j * v[1::2]
    np.testing.assert_allclose(w, np.exp(-2j * np.pi * np.arange(M) / M), rtol=0, atol=1e-7)


@pytest.mark.parametrize("arg", [0, 437, 65536 + 437, 1048576 - 131072])
def test_fc_rows_are_the_modulated_folded_spectrum(arg):
    """arg / 2^20 = f_lo / fs: DC-ish, a small offset, +1/16 and -1/8 of fs."""
    got = _lib_row(arg)
    want = _c_table(arg / 2 ** 20)
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-7 * np.abs(want).max())


@pytest.mark.parametrize("L", [16384, 16387, 20005, 20006])
@pytest.mark.parametrize("ratio", [1.0 / 2.4e6, 150e3 / 2.4e6])
def test_fc_model_plus_edge_maps_is_reference_decimate(L, ratio):
    """The FC model (g truncated at 768, the LO as the filter's modulation and lo[8m] on the
    outputs) plus the shipped maps on the mixed input = decimate x 3 of the mixed input."""
    rng = np.random.default_rng(L)
    x = rng.standard_normal(L) + 1j * rng.standard_normal(L)
    x += 3 * np.exp(2j * np.pi * 0.013 * np.arange(L))
    lo = _lo(L, ratio)
    ref = x * lo
    for _ in range(3):
        ref = ss.decimate(ref, 2)
    g = _g() * np.exp(2j * np.pi * np.mod(ratio * np.arange(-K, K + 1), 1.0))
    n3 = len(ref)
    out = np.convolve(x, g)[K:K + L][::8][:n3] * lo[::8][:n3]
    CL, CR = _edge(0, L % 8), _edge(1, L % 8)
    xm = x * lo
    out[:CL.shape[0]] += CL @ xm[:CL.shape[1]]
    out[n3 - CR.shape[0]:] += (CR @ xm[::-1][:CR.shape[1]])[::-1]
    err = np.abs(out - ref).max() / np.abs(ref).max()
    assert err < 7e-7, err             # the truncation at 768 (5.6e-7 with the LO offset)


def test_fc_block_in_the_kernels_index_maps():
    """One block with the kernel's thread maps and the library's row: y[j] for j in [K/8, K/8 + P)
    equals the window's linear convolution with g', decimated by 8 (the kernel multiplies by
    lo[8m] afterwards; the row carries 1 / sqrt 2 for that)."""
    rng = np.random.default_rng(5)
    w = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    arg = 65536 + 437
    C = _lib_row(arg)
    W1 = lambda e: np.exp(-2j * np.pi * np.asarray(e) / M)
    d16 = np.exp(-2j * np.pi * np.outer(np.arange(16), np.arange(16)) / 16)
    d4 = np.exp(-2j * np.pi * np.outer(np.arange(4), np.arange(4)) / 4)
    big = {}
    for t in range(256):                 # pass A: pairs n = 2t + 512 i, residues 2 (t & 3), +1
        j0, r0 = t >> 2, 2 * (t & 3)
        for r in (r0, r0 + 1):
            v = np.array([w[2 * t + (r - r0) + 512 * i] for i in range(16)])
            o = (d16 @ v) * W1(j0 * np.arange(16))
            for k1 in range(16):
                big[(64 * k1 + j0, r)] = o[k1]
    for t in range(256):                 # pass B: k1 = t >> 4, j1 = (t >> 2) & 3, rp = t & 3
        k1, j1, rp = t >> 4, (t >> 2) & 3, t & 3
        for r in (2 * rp, 2 * rp + 1):
            v = np.array([big[(64 * k1 + j1 + 4 * i, r)] for i in range(16)])
            o = (d16 @ v) * W1(16 * j1 * np.arange(16))
            for k2 in range(16):
                big[(64 * k1 + j1 + 4 * k2, r)] = o[k2]
    small = np.zeros(M, complex)
    for t in range(256):                 # pass C + MAC + inverse stage 1: k' = (t >> 4) + 16 (t & 15)
        k1, k2 = t >> 4, t & 15
        kp = k1 + 16 * k2
        yf = np.zeros(4, complex)
        for r in range(8):
            a = d4 @ np.array([big[(64 * k1 + 4 * k2 + j, r)] for j in range(4)])
            yf += a * C[kp + 256 * np.arange(4), r]
        o = np.conj(d4) @ yf * np.conj(W1(kp * np.arange(4)))
        small[kp + 256 * np.arange(4)] = o
    for S, lowf in ((64, lambda t: t & 63), (16, lambda t: t & 15), (4, lambda t: t & 3)):
        new = small.copy()           # stages 2..4, each thread's fixed digits as in the kernel
        for t in range(256):
            if S == 64:
                i0 = (t & 63) + 256 * (t >> 6)
            elif S == 16:
                i0 = (t & 15) + 64 * ((t >> 4) & 3) + 256 * (t >> 6)
            else:
                i0 = (t & 3) + 16 * ((t >> 2) & 3) + 64 * ((t >> 4) & 3) + 256 * (t >> 6)
            idx = i0 + S * np.arange(4)
            new[idx] = np.conj(d4) @ small[idx] * np.conj(W1((M // (4 * S)) * lowf(t) * np.arange(4)))
        small = new
    y = np.zeros(M, complex)
    for t in range(256):                 # stage 5: t = b0 + 4 b1 + 16 b2 + 64 b3 -> j = t + 256 b4
        i0 = 4 * (t >> 6) + 16 * ((t >> 4) & 3) + 64 * ((t >> 2) & 3) + 256 * (t & 3)
        y[t + 256 * np.arange(4)] = np.conj(d4) @ small[i0 + np.arange(4)]
    g = _g() * np.exp(2j * np.pi * np.mod(arg / 2 ** 20 * np.arange(-K, K + 1), 1.0))
    direct = np.convolve(w, g)[K:K + N][::8] / np.sqrt(2)     # local index i = 8 j
    jv = np.arange(K // 8, K // 8 + P)
    err = np.abs(y[jv] - direct[jv]).max() / np.abs(direct[jv]).max()
    assert err < 1e-6, err               # the row's fp32 rounding
