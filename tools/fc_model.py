#!/usr/bin/env python3
"""Numpy model of a fast-convolution (overlap-save FFT) form of the zoom-8 decimator
(design tool, not used at run time).

The interior of three scipy.signal.decimate(x, 2) (pypanadapter_spectrum.py:2096-2098) is the
zero-phase LTI filter G(z) = |H(z)|^2 |H(z^2)|^2 |H(z^4)|^2 on the zero-extended frame, then
[::8].  G's impulse response g is two-sided and decays with the slowest pole
(r = .935 at rate 1/4); truncated at |k| <= K it is an FIR of 2K + 1 taps at the input rate.

Overlap-save with an N-point FFT: a block reads N input samples x[8 m0 - K ...], takes X = FFT(x),
multiplies by G_N = FFT(g circularly placed), and the decimated outputs are
    y[m0 + j] = (1/N) sum_{k < N/8} W_{N/8}^{-kj} sum_{q < 8} (X G_N)[k + q N/8]
(K a multiple of 8): the ↓8 is an 8-fold alias sum in frequency followed by an N/8-point
inverse FFT.  Valid outputs per block P = (N - 2K) / 8.

Prints the tail of g against K, the VALU estimate per input sample, and the fp32 error of the
form (scipy.fft in single precision) against the fp64 model and against decimate x 3.
"""
import numpy as np
import scipy.fft as sf
import scipy.signal as ss

SOS = ss.cheby1(8, 0.05, 0.4, output="sos")


def g_full(n=6000):
    """g = autocorrelation of h at rates 1, 2, 4 convolved (centre at index len // 2)."""
    imp = np.zeros(n)
    imp[0] = 1
    h = ss.sosfilt(SOS, imp)
    r = np.convolve(h, h[::-1])              # |H(z)|^2, centre n - 1
    g = r
    for up in (2, 4):
        ru = np.zeros((len(r) - 1) * up + 1)
        ru[::up] = r
        g = np.convolve(g, ru)
    c = len(g) // 2
    return g, c


def taps(K, gg=None):
    g, c = gg if gg is not None else g_full()
    return g[c - K:c + K + 1]


def fc_decimate(x, gk, N, dt=np.complex64):
    """Overlap-save FFT decimation by 8 with the fold; returns outputs m = 0 .. ceil(L/8) - 1."""
    K = (len(gk) - 1) // 2
    assert K % 8 == 0 and N % 8 == 0
    L = len(x)
    nout = -(-L // 8)
    P = (N - 2 * K) // 8
    gc = np.zeros(N, dtype=complex)
    gc[:K + 1] = gk[K:]
    gc[N - K:] = gk[:K]
    GN = sf.fft(gc).astype(dt)
    xp = np.concatenate([np.zeros(K, dtype=dt), x.astype(dt), np.zeros(N + 8 * P, dtype=dt)])
    out = np.zeros(nout, dtype=dt)
    for m0 in range(0, nout, P):
        blk = xp[8 * m0:8 * m0 + N]
        Y = sf.fft(blk) * GN
        Yf = Y.reshape(8, N // 8).sum(axis=0)
        y = sf.ifft(Yf) / 8                  # ifft's 1/(N/8) times 1/8 = 1/N
        # local index i = 8 j + K  ->  j = 0 .. P-1 after shifting by K / 8
        yj = np.roll(y, -(K // 8))[:P]
        n = min(P, nout - m0)
        out[m0:m0 + n] = yj[:n]
    return out


def model_fp64(x, gk):
    K = (len(gk) - 1) // 2
    y = np.convolve(x, gk)[K:K + len(x)]
    return y[::8]


def valu_estimate(N, K):
    """Lane-instructions per input sample: 1.75 per point per radix-2 stage (radix-4 butterflies
    with packed complex arithmetic), the stages that resolve the low log2(N/8) bits of k at full
    length, the H multiply and fold at 2 per point, the N/8 inverse at 1/8 length, x N / (8 P)."""
    lg = int(np.log2(N))
    per_point = 1.75 * (lg - 3) + 2 + 1.75 * (lg - 3) / 8
    P = (N - 2 * K) // 8
    return per_point * N / (8 * P) + 3.3


def main():
    gg = g_full()
    g, c = gg
    s = np.abs(g).sum()
    print("sum|g| %.4f, g[0] %.4f" % (s, g[c]))
    for K in (512, 768, 1024, 1280, 1536, 2048):
        tail = np.abs(g[c + K + 1:]).sum() * 2 / s
        print(f"K {K:5d}: tail sum / sum|g| {tail:.2e};  VALU/sample N=8192 "
              f"{valu_estimate(8192, K):.1f}  N=16384 {valu_estimate(16384, K):.1f}")
    rng = np.random.default_rng(7)
    L = 299008
    x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)) / np.sqrt(2)
    x += np.exp(2j * np.pi * 0.011 * np.arange(L)) + 1e-3 * np.exp(2j * np.pi * 0.3 * np.arange(L))
    ex = x
    for _ in range(3):
        ex = ss.decimate(ex, 2)
    ref_full = model_fp64(x, taps(2048, gg))
    for K in (768, 1024, 1280):
        gk = taps(K, gg)
        for N in (8192, 16384):
            got = fc_decimate(x, gk, N)
            e = np.abs(got - ref_full) / np.abs(ref_full).max()
            ee = np.abs(got - ex) / np.abs(ex).max()
            mid = slice(400, len(ex) - 400)
            print(f"K {K} N {N}: fp32 vs fp64 model (K=2048) max {e.max():.2e} rms {np.sqrt((e**2).mean()):.1e};"
                  f" vs decimate x3 interior max {ee[mid].max():.2e}")


if __name__ == "__main__":
    main()


# ------------------------------------------------------------------ the kernel's block, index-exact
# One block: the window w[n], n < 8192 (input x[8 m0 - K + n]); residues r = n mod 8, a_r[m] = w[8m + r].
# Forward, per residue (1024-point DIF): m = j0 + 64 i; pass A radix 16 over i -> k1, twiddle W1024^(j0 k1);
# j0 = j1 + 4 i2; pass B radix 16 over i2 -> k2, twiddle W64^(j1 k2); pass C radix 4 over j1 -> k3;
# A_r[k1 + 16 k2 + 256 k3].  Fold + filter: Yf[k] = sum_r A_r[k] C[k][r].  Inverse (1024-point, DIF in k):
# k = k' + 256 a4 ... five radix-4 stages, output y[j], j = b0 + 4 b1 + 16 b2 + 64 b3 + 256 b4.
W = lambda n, e: np.exp(-2j * np.pi * np.asarray(e) / n)


def c_table(gk, N=8192):
    """C[k][r] = (1/N) W_N^(r k) sum_q G[k + (N/8) q] W_8^(r q), G = FFT_N(g circular)."""
    K = (len(gk) - 1) // 2
    gc = np.zeros(N, dtype=complex)
    gc[:K + 1] = gk[K:]
    gc[N - K:] = gk[:K]
    G = np.fft.fft(gc)
    M = N // 8
    k = np.arange(M)[:, None]
    r = np.arange(8)[None, :]
    S = np.zeros((M, 8), dtype=complex)
    for q in range(8):
        S += G[k[:, 0] + M * q][:, None] * W(8, r * q)
    return S * W(N, r * k) / N


def block_model(w, C):
    a = w.reshape(1024, 8).T                       # a[r][m]
    # pass A
    P1 = np.zeros((8, 16, 64), dtype=complex)      # [r][k1][j0]
    i = np.arange(16)
    for j0 in range(64):
        v = a[:, j0 + 64 * i]                      # [r][i]
        b = v @ W(16, np.outer(i, i))              # dft16 over i -> k1
        P1[:, :, j0] = b * W(1024, j0 * i)[None, :]
    # pass B
    P2 = np.zeros((8, 16, 16, 4), dtype=complex)   # [r][k1][k2][j1]
    for j1 in range(4):
        v = P1[:, :, j1 + 4 * i]                   # [r][k1][i2]
        c = v @ W(16, np.outer(i, i))
        P2[:, :, :, j1] = c * W(64, j1 * i)[None, None, :]
    # pass C + MAC
    A = np.einsum('rabj,jk->rabk', P2, W(4, np.outer(np.arange(4), np.arange(4))))   # [r][k1][k2][k3]
    kk = (np.arange(16)[:, None, None] + 16 * np.arange(16)[None, :, None] + 256 * np.arange(4)[None, None, :])
    Yf = np.einsum('rabk,abkr->abk', A, C[kk])     # [k1][k2][k3]
    # inverse: k' = k1 + 16 k2 -> flat array Yk[k] (k = k' + 256 a4)
    Y = np.zeros(1024, dtype=complex)
    Y[kk.ravel()] = Yf.ravel()
    # stage s over digit a_(5-s) with stride S, output digit b_(s-1); twiddle W_(4S)^(-b klow)
    pos = Y.copy()                                 # position = digits, in place
    for S in (256, 64, 16, 4, 1):
        new = pos.copy()
        for base in range(1024):
            if (base // S) % 4:
                continue
            klow = base % S
            v = pos[base + S * np.arange(4)]
            o = v @ np.conj(W(4, np.outer(np.arange(4), np.arange(4))))
            if S > 1:
                o = o * np.conj(W(4 * S, np.arange(4) * klow))
            new[base + S * np.arange(4)] = o
        pos = new
    # position p = b4 + 4 b3 + 16 b2 + 64 b1 + 256 b0  ->  j = digit reverse
    p = np.arange(1024)
    d = [(p >> (2 * s)) & 3 for s in range(5)]     # d0 = b4, d1 = b3, d2 = b2, d3 = b1, d4 = b0
    j = d[4] + 4 * d[3] + 16 * d[2] + 64 * d[1] + 256 * d[0]
    y = np.zeros(1024, dtype=complex)
    y[j] = pos
    return y


def check_block():
    rng = np.random.default_rng(3)
    gg = g_full()
    gk = taps(1024, gg)
    w = rng.standard_normal(8192) + 1j * rng.standard_normal(8192)
    C = c_table(gk)
    y = block_model(w, C)
    # direct: y_loc[j] = (1/N) sum_k (FFT(w) G)[k] W^(-8 j k)
    K = 1024
    gc = np.zeros(8192, dtype=complex)
    gc[:K + 1] = gk[K:]
    gc[8192 - K:] = gk[:K]
    full = np.fft.ifft(np.fft.fft(w) * np.fft.fft(gc))
    ref = full[::8]
    print("block model vs direct: max |d| %.2e (|ref| max %.2e)" % (np.abs(y - ref).max(), np.abs(ref).max()))


if __name__ == "__main__" and __import__("sys").argv[1:] == ["block"]:
    check_block()
