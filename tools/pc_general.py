#!/usr/bin/env python3
"""Design numbers of the PC decimator for other zooms (groundwork for DESIGN.md §8 item 3;
not used at run time).  For log2(zoom) = K stages of scipy.signal.decimate(x, 2)
(pypanadapter_spectrum.py:2096-2098) the PC form moves every all-pole factor of stages
0 .. K-2 down to the output rate (polyphase identity, tools/pc_proto.py) and keeps the last
stage's two slowest sections at its own rate, as the zoom-8 kernels do (K = 3, pc_tables.cpp):

    rate 2^-k (k < K):  y_{k+1} = (g_k * y_k)|2,  g_k = f_k f_k'
    rate 2^-(K-1):      the last stage's sections 2, 3, zero phase, before g_{K-1}
    rate 2^-K:          the moved poles as zero-phase sections (radius <= 0.935^2)

Prints per K: FIR lengths, multiply-adds per input sample (FIRs + the recurrences priced as
block-parallel passes at 4 per sample and section), the output-rate sections' radii, and the
fp32 error of the interior against float64 decimate^K (frame ends excluded: the zoom-8 form
restores them with low-rank maps)."""
import numpy as np
import scipy.signal as ss

from pc_proto import A1, A2, N9, conv, neg, square_sections

OWN = [2, 3]


def design(K):
    secs = [(A1, A2)]
    for _ in range(K):
        secs.append(square_sections(*secs[-1]))
    poly = lambda s, idx: conv(*[np.array([1.0, s[0][i], s[1][i]]) for i in idx]) if idx else np.array([1.0])
    firs = []
    for k in range(K):
        f = N9.copy()
        for i in range(k + 1):  # 1 / D(z^(2^i)) moved to rate 2^-(k+1) contributes D_{2^(k-i)}(-.)
            idx = [0, 1, 2, 3] if (k < K - 1 or i < k) else [j for j in range(4) if j not in OWN]
            f = np.convolve(f, neg(poly(secs[k - i], idx)))
        firs.append(f)
    g = [np.convolve(f, f[::-1]) for f in firs]
    own = [(secs[0][0][i], secs[0][1][i]) for i in OWN]
    ap = []
    for i in range(K - 1):
        ap += [(secs[K - i][0][j], secs[K - i][1][j]) for j in range(4)]
    ap += [(secs[1][0][j], secs[1][1][j]) for j in range(4) if j not in OWN]
    ap.sort(key=lambda s: -s[1])
    return g, own, ap


def run(x, g, own, ap, dt):
    rdt = np.float32 if dt == np.complex64 else np.float64
    K = len(g)
    y = x.astype(dt)
    for k in range(K):
        if k == K - 1:
            so = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in own], rdt)
            y = ss.sosfilt(so, ss.sosfilt(so, y)[::-1])[::-1].astype(dt)
        c = (len(g[k]) - 1) // 2
        y = np.convolve(y, g[k].astype(rdt))[c::2][:len(y) // 2].astype(dt)
    sa = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in ap], rdt)
    return ss.sosfilt(sa, ss.sosfilt(sa, y)[::-1])[::-1]


def main():
    rng = np.random.default_rng(11)
    for K in (1, 2, 3, 4):
        g, own, ap = design(K)
        macs = sum(len(gk) / 2 ** (k + 1) for k, gk in enumerate(g))
        rec = 4 * 2 * len(own) / 2 ** (K - 1) + 4 * 2 * len(ap) / 2 ** K
        L = 8192 * 2 ** K
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)) / np.sqrt(2)
        x += 3 * np.exp(2j * np.pi * 0.3 / 2 ** K * np.arange(L))
        ref = x
        for _ in range(K):
            ref = ss.decimate(ref, 2)
        pad = 4096 * 2 ** K  // 2 ** K * 2 ** K
        xp = np.concatenate([np.zeros(pad), x, np.zeros(pad)])
        err = {}
        for dt in (np.complex128, np.complex64):
            out = run(xp, g, own, ap, dt)[pad // 2 ** K:pad // 2 ** K + len(ref)]
            e = np.abs(out - ref)[600:-600].max() / np.abs(ref).max()
            err[np.dtype(dt).name] = float(e)
        print(f"zoom {2 ** K}: FIR taps {[len(gk) for gk in g]}, FIR MACs/input sample {macs:.2f}, "
              f"recurrence MACs/input sample {rec:.2f}, output-rate sections {len(ap)} "
              f"(radius <= {max(np.sqrt(a2) for _, a2 in ap):.3f}), interior error {err}")


if __name__ == "__main__":
    main()
