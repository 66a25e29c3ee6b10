#!/usr/bin/env python3
"""Why PC's fp32 error is 5-6e-6 of the peak rather than the 2.4-3.8e-6 of tools/pc_model.py
(CPU only, numpy).  The model computes its FIRs with np.dot (blocked /
pairwise sums); the kernels sum the taps of FIR alpha (33) and beta (49) one by one in tap
order.  On the zf_n512_z8 fixture (tests/golden/zoomfft.npz, LO 1 Hz, mixed in float64 and
cast to complex64) this prints the model's max error relative to the peak with the two FIRs
summed as: np.dot, in tap order (the kernels), in two sums (even / odd taps), and with
symmetric tap pairs added first.  Measured: 3.75e-6 / 5.63e-6 / 4.47e-6 / 3.92e-6, against
the GPU's 5.3e-6 (tiles) and 6.07e-6 (walk) on the same input (tools/dbg/pc_fixture_error.py).
usage: (from tools/) python3 dbg/pc_fir_order.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pc_model as pm  # noqa: E402

C64 = np.complex64


def f32(a):
    return a.astype(C64)


def fir(g, xs, nout, mode):
    G = len(g)
    sl = lambda t: xs[t: t + 2 * nout: 2][:nout]  # noqa: E731
    if mode == "dot":
        return np.array([np.dot(g, xs[2 * i:2 * i + G]) for i in range(nout)], C64)
    if mode == "order":
        acc = np.zeros(nout, C64)
        for t in range(G):
            acc = f32(acc + f32(np.float32(g[t]) * sl(t)))
        return acc
    if mode == "two":
        a, b = np.zeros(nout, C64), np.zeros(nout, C64)
        for t in range(G):
            if t % 2 == 0:
                a = f32(a + f32(np.float32(g[t]) * sl(t)))
            else:
                b = f32(b + f32(np.float32(g[t]) * sl(t)))
        return f32(a + b)
    acc = np.zeros(nout, C64)  # "pairs"
    for t in range(G // 2):
        acc = f32(acc + f32(np.float32(g[t]) * f32(sl(t) + sl(G - 1 - t))))
    return f32(acc + f32(np.float32(g[G // 2]) * sl(G // 2)))


def k1(xin, mode):
    n2 = pm.y2_len(len(xin))
    out = np.zeros(n2, C64)
    g0, g1 = pm.G[0].astype(np.float32), pm.G[1].astype(np.float32)
    for tau in range(-(-n2 // pm.K1_Q)):
        qs = pm.Q0 + pm.K1_Q * tau
        xs = 4 * qs - 64
        xt = np.zeros(4128 + 64, C64)
        lo, hi = max(xs, 0), min(xs + 4128, len(xin))
        if hi > lo:
            xt[lo - xs:hi - xs] = xin[lo:hi]
        y1 = np.concatenate([fir(g0, xt, 2031, mode), np.zeros(64, C64)])
        nq = min(pm.K1_Q, n2 - (qs - pm.Q0))
        out[qs - pm.Q0:qs - pm.Q0 + nq] = fir(g1, y1, pm.K1_Q, mode)[:nq]
    return out


def main():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    zf = np.load(os.path.join(root, "tests", "golden", "zoomfft.npz"))
    x = zf["zf_n512_z8/x"].astype(np.complex128)
    L = len(x)
    xm = x * np.sqrt(2) * np.exp(-2j * np.pi * 1.0 * np.arange(L) / 2.4e6)
    ex = pm.exact(xm)
    CL, CR = pm.edge_matrices(L)
    x32 = xm.astype(C64)
    for mode in ("dot", "order", "two", "pairs"):
        n3 = pm.stage_len(L)
        out = pm.k2(k1(x32, mode), n3, C64).astype(complex)
        R, J = CL.shape
        out[:R] += CL @ x32[:J]
        out[n3 - R:] += (CR @ x32[::-1][:J])[::-1]
        e = np.abs(out - ex) / np.abs(ex).max()
        print(f"FIRs alpha, beta summed {mode:6s}: max {e.max():.2e}, rms {np.sqrt((e ** 2).mean()):.2e}")


if __name__ == "__main__":
    main()
