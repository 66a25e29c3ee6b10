"""CPU checks of the FC decimator's host tables (pc_tables.cpp fc_build_row / fc_build_twiddles;
kernel fc_kernels.hip), no GPU needed, at zoom 8 and zoom 4:

* the zoom-Z model's input-rate response g (rebuilt here from scipy's cheby1 sections:
  |H(z)|^2 |H(z^2)|^2 (|H(z^4)|^2)) truncated at |k| <= K (768 / 512), together with the shipped
  frame-end maps, reproduces log2(Z) x scipy.signal.decimate(x, 2) (pypanadapter_spectrum.py:
  2096-2098) with the LO mixed in (S:2088-2094): to 7e-7 at zoom 8 (the truncation: 5.6e-7 with
  an LO offset, 2e-7 at K = 1024), 2e-7 at zoom 4;
* the library's filter rows equal that g's modulated, folded spectrum built here;
* one block computed in numpy with the kernel's own index maps (passes A, B, C, the residue MAC
  with the library's row in the kernel's order, the five inverse stages) equals the direct
  overlap-save formula -- the index algebra of the kernel, pinned on CPU."""
import numpy as np
import pytest
import scipy.signal as ss

from test_pc_tables import _call, _edge, _edge4

SOS = ss.cheby1(8, 0.05, 0.4, output="sos")
N = 8192
GEO = {8: dict(K=768, P=832), 4: dict(K=512, P=1792)}   # fc_kernels.hip Geo<Z> (kFcK, kFcP, kFc4K, kFc4P)
HOOK = {8: (18, 19), 4: (20, 21)}                        # zfft__pc_tables: twiddles, row


def _g(Z):
    imp = np.zeros(6000)
    imp[0] = 1
    h = ss.sosfilt(SOS, imp)
    r = np.convolve(h, h[::-1])
    g = r
    for up in (2, 4)[:int(np.log2(Z)) - 1]:
        ru = np.zeros((len(r) - 1) * up + 1)
        ru[::up] = r
        g = np.convolve(g, ru)
    c = len(g) // 2
    K = GEO[Z]["K"]
    return g[c - K:c + K + 1]


def _lo(L, ratio):
    return np.sqrt(2) * np.exp(-2j * np.pi * np.mod(np.arange(L) * ratio, 1.0))


def _c_table(Z, ratio):
    """C[k][r] = W_N^(rk) sum_q G[k + M q] W_Z^(rq) / (N sqrt 2), G = DFT of g e^(2 pi i ratio k)."""
    K, M = GEO[Z]["K"], N // Z
    k = np.arange(-K, K + 1)
    gc = np.zeros(N, complex)
    gc[k % N] = _g(Z) * np.exp(2j * np.pi * np.mod(ratio * k, 1.0))
    G = np.fft.fft(gc)
    kk = np.arange(M)[:, None]
    r = np.arange(Z)[None, :]
    S = sum(G[kk[:, 0] + M * q][:, None] * np.exp(-2j * np.pi * r * q / Z) for q in range(Z))
    return S * np.exp(-2j * np.pi * r * kk / N) / (N * np.sqrt(2))


def _lib_row(Z, arg):
    v = _call(HOOK[Z][1], arg)
    z = v[0::2] + 1j * v[1::2]          # float2 index (((Z / 2) k3 + r / 2) 256 + t) 2 + r % 2
    M = N // Z
    C = np.zeros((M, Z), complex)
    for t in range(256):
        kp = (t >> 4) + 16 * (t & 15)
        for k3 in range(M // 256):
            for r in range(Z):
                C[kp + 256 * k3, r] = z[(((Z // 2) * k3 + r // 2) * 256 + t) * 2 + (r & 1)]
    return C


@pytest.mark.parametrize("Z", [8, 4])
def test_fc_twiddles(Z):
    M = N // Z
    v = _call(HOOK[Z][0])
    w = v[0::2] + 1j * v[1::2]
    np.testing.assert_allclose(w, np.exp(-2j * np.pi * np.arange(M) / M), rtol=0, atol=1e-7)


@pytest.mark.parametrize("Z", [8, 4])
@pytest.mark.parametrize("arg", [0, 437, 65536 + 437, 1048576 - 131072])
def test_fc_rows_are_the_modulated_folded_spectrum(Z, arg):
    """arg / 2^20 = f_lo / fs: DC-ish, a small offset, +1/16 and -1/8 of fs."""
    got = _lib_row(Z, arg)
    want = _c_table(Z, arg / 2 ** 20)
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-7 * np.abs(want).max())


@pytest.mark.parametrize("Z,bound", [(8, 7e-7), (4, 2e-7)])
@pytest.mark.parametrize("L", [16384, 16387, 20005, 20006])
@pytest.mark.parametrize("ratio", [1.0 / 2.4e6, 150e3 / 2.4e6])
def test_fc_model_plus_edge_maps_is_reference_decimate(Z, bound, L, ratio):
    """The FC model (g truncated at K, the LO as the filter's modulation and lo[Z m] on the
    outputs) plus the shipped maps on the mixed input = decimate x log2(Z) of the mixed input."""
    K = GEO[Z]["K"]
    rng = np.random.default_rng(L)
    x = rng.standard_normal(L) + 1j * rng.standard_normal(L)
    x += 3 * np.exp(2j * np.pi * 0.013 * np.arange(L))
    lo = _lo(L, ratio)
    ref = x * lo
    for _ in range(int(np.log2(Z))):
        ref = ss.decimate(ref, 2)
    g = _g(Z) * np.exp(2j * np.pi * np.mod(ratio * np.arange(-K, K + 1), 1.0))
    nd = len(ref)
    out = np.convolve(x, g)[K:K + L][::Z][:nd] * lo[::Z][:nd]
    if Z == 8:
        CL, CR = _edge(0, L % 8), _edge(1, L % 8)
    else:
        (UL, VL), (UR, VR) = _edge4(0, 0, shipped=True), _edge4(1, L % 4, shipped=True)
        CL, CR = UL @ VL.T, UR @ VR.T
    xm = x * lo
    out[:CL.shape[0]] += CL @ xm[:CL.shape[1]]
    out[nd - CR.shape[0]:] += (CR @ xm[::-1][:CR.shape[1]])[::-1]
    err = np.abs(out - ref).max() / np.abs(ref).max()
    assert err < bound, err


@pytest.mark.parametrize("Z", [8, 4])
def test_fc_block_in_the_kernels_index_maps(Z):
    """One block with the kernel's thread maps and the library's row: y[j] for j in [K/Z, K/Z + P)
    equals the window's linear convolution with g', decimated by Z (the kernel multiplies by
    lo[Z m] afterwards; the row carries 1 / sqrt 2 for that)."""
    K, P = GEO[Z]["K"], GEO[Z]["P"]
    M, R1 = N // Z, N // Z // 256
    rng = np.random.default_rng(5)
    w = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    arg = 65536 + 437
    C = _lib_row(Z, arg)
    WM = lambda e: np.exp(-2j * np.pi * np.asarray(e) / M)
    dft = lambda R: np.exp(-2j * np.pi * np.outer(np.arange(R), np.arange(R)) / R)
    d16, d4, dR = dft(16), dft(4), dft(R1)
    big = {}
    for t in range(256):                 # pass A: pairs n = 2t + 512 i, residues 2t mod Z, +1
        j0, r0 = t >> (2 if Z == 8 else 1), (2 * t) % Z
        for r in (r0, r0 + 1):
            v = np.array([w[2 * t + (r - r0) + 512 * i] for i in range(16)])
            o = (d16 @ v) * WM(j0 * np.arange(16))
            for k1 in range(16):
                big[((M // 16) * k1 + j0, r)] = o[k1]
    for t in range(256):                 # pass B: k1 = t >> 4, j1, residue pair rp
        k1 = t >> 4
        j1, rp = ((t >> 2) & 3, t & 3) if Z == 8 else ((t >> 1) & 7, t & 1)
        for r in (2 * rp, 2 * rp + 1):
            v = np.array([big[((M // 16) * k1 + j1 + (M // 256) * i, r)] for i in range(16)])
            o = (d16 @ v) * WM(16 * j1 * np.arange(16))
            for k2 in range(16):
                big[((M // 16) * k1 + j1 + (M // 256) * k2, r)] = o[k2]
    small = np.zeros(M, complex)
    for t in range(256):                 # pass C + MAC + inverse stage 1: k' = (t >> 4) + 16 (t & 15)
        k1, k2 = t >> 4, t & 15
        kp = k1 + 16 * k2
        yf = np.zeros(R1, complex)
        for r in range(Z):
            a = dR @ np.array([big[((M // 16) * k1 + R1 * k2 + j, r)] for j in range(R1)])
            yf += a * C[kp + 256 * np.arange(R1), r]
        small[kp + 256 * np.arange(R1)] = np.conj(dR) @ yf * np.conj(WM(kp * np.arange(R1)))
    for S, lowf in ((64, lambda u: u & 63), (16, lambda u: u & 15), (4, lambda u: u & 3)):
        new = small.copy()           # stages 2..4, each butterfly's fixed digits as in the kernel
        for u in range(M // 4):
            if S == 64:
                i0 = (u & 63) + 256 * (u >> 6)
            elif S == 16:
                i0 = (u & 15) + 64 * ((u >> 4) & 3) + 256 * (u >> 6)
            else:
                i0 = (u & 3) + 16 * ((u >> 2) & 3) + 64 * ((u >> 4) & 3) + 256 * (u >> 6)
            idx = i0 + S * np.arange(4)
            new[idx] = np.conj(d4) @ small[idx] * np.conj(WM((M // (4 * S)) * lowf(u) * np.arange(4)))
        small = new
    y = np.zeros(M, complex)
    for u in range(M // 4):              # stage 5: u = b0 + R1 (b1 + 4 b2 + 16 b3) -> j = u + (M/4) b4
        b0, r = u % R1, u // R1
        i0 = 4 * ((r >> 4) & 3) + 16 * ((r >> 2) & 3) + 64 * (r & 3) + 256 * b0
        y[u + (M // 4) * np.arange(4)] = np.conj(d4) @ small[i0 + np.arange(4)]
    g = _g(Z) * np.exp(2j * np.pi * np.mod(arg / 2 ** 20 * np.arange(-K, K + 1), 1.0))
    direct = np.convolve(w, g)[K:K + N][::Z] / np.sqrt(2)     # local index i = Z j
    jv = np.arange(K // Z, K // Z + P)
    err = np.abs(y[jv] - direct[jv]).max() / np.abs(direct[jv]).max()
    assert err < 1e-6, err               # the row's fp32 rounding


@pytest.mark.parametrize("Z", [8, 4])
def test_fc_inverse_stages_2_to_4_are_wave_local(Z):
    """fc_kernels.hip drops the workgroup barriers between inverse stages 2, 3 and 4 (stage_sync):
    every slot a wave's butterflies read or write there has b0 = i >> 8 equal to (t >> 6) + 4 h,
    and each stage's slots of one wave are the same set -- no slot crosses waves until stage 5."""
    M = N // Z
    NB = M // 1024
    bases = ((lambda u: (u & 63) + 256 * (u >> 6), 64),
             (lambda u: (u & 15) + 64 * ((u >> 4) & 3) + 256 * (u >> 6), 16),
             (lambda u: (u & 3) + 16 * ((u >> 2) & 3) + 64 * ((u >> 4) & 3) + 256 * (u >> 6), 4))
    for w in range(4):
        sets = []
        for base, S in bases:
            slots = set()
            for t in range(64 * w, 64 * w + 64):
                for h in range(NB):
                    for a in range(4):
                        i = base(t) + 1024 * h + S * a        # ps(i) + 1088 h = ps(i + 1024 h)
                        assert i >> 8 == (t >> 6) + 4 * h
                        slots.add(i)
            sets.append(slots)
        assert sets[0] == sets[1] == sets[2]
        assert len(sets[0]) == 256 * NB
