#!/usr/bin/env python3
"""Block-level numpy model of the PC (polyphase cascade) decimator kernels for zoom 8
(design tool for pypanadapter_amd/csrc/pc_kernels.hip; not used at run time).

Model (tools/pc_proto.py): interior of 3 x scipy.signal.decimate(x, 2)
(pypanadapter_spectrum.py:2096-2098) =
    y1 = (g0 * x)|2          g0 = f0 f0',  f0 = N D(-z)                       33 taps
    y2 = (g1 * y1)|2         g1 = f1 f1',  f1 = N D2(-u) D(-u)                49 taps
    z2 = S(v) S(1/v) y2      S = the two slowest sections of D at their own rate (v = z^4)
    u3 = (g2 * z2)|2         g2 = f2 f2',  f2 = N D4(-v) D2(-v) Dfast(-v)      57 taps
    out = A(w) A(1/w) u3     A = D8 D4 D2fast: 10 sections at the output rate, radius <= .765
The model is the LTI cascade on the zero-extended frame; scipy's edge rules (odd extension,
sosfilt_zi states) differ from it only near the frame ends, by a linear map of the first /
last J input samples onto the first / last R outputs (edge matrices, computed here from
impulses: exact - model).  All pole moves keep fp32 conditioning (the slowest pole of the
last stage stays at its own rate; moving it to the output rate amplified fp32 rounding to
~1e-3).

Kernel structure modelled here:
  K1 tiles: 992 y2 outputs per tile from 4128 input samples (FIR alpha then beta).
  K2 tiles: 2048 outputs per tile from a 5376-sample y2 span (own-rate sections over
        256 thread blocks of 21 with block scans and cross-wave steps; FIR gamma; the
        10-section cascade on 4 waves, each a quarter of the tile with 64-sample halos
        over 64 lane blocks of 10), edges by the matrices.
  (KW, the walk kernel, runs the same arithmetic with tiles in frame order: the causal
  own-rate sections carry state instead of the left halo -- same values to fp32 rounding.)
"""
import numpy as np
import scipy.signal as ss

from pc_proto import A1, A2, N9, conv, dpoly, neg, square_sections

K = 3
SECS = [(A1, A2)]
for _ in range(K):
    SECS.append(square_sections(*SECS[-1]))


def sec_poly(a1, a2, idx):
    return conv(*[np.array([1.0, a1[i], a2[i]]) for i in idx])


OWN = [2, 3]         # the two slowest sections of D stay at rate 1/4 (fp32 error 2e-6 vs
FAST = [0, 1]        # 1.3e-5 with only the slowest: tools/pc_model.py variants)
F0 = conv(N9, neg(dpoly(*SECS[0])))
F1 = conv(N9, neg(dpoly(*SECS[1])), neg(dpoly(*SECS[0])))
F2 = conv(N9, neg(dpoly(*SECS[2])), neg(dpoly(*SECS[1])), neg(sec_poly(*SECS[0], FAST)))
G = [np.convolve(f, f[::-1]) for f in (F0, F1, F2)]
OWN_SEC = [(SECS[0][0][i], SECS[0][1][i]) for i in OWN]
AP_SECS = ([(SECS[3][0][i], SECS[3][1][i]) for i in range(4)] +
           [(SECS[2][0][i], SECS[2][1][i]) for i in range(4)] +
           [(SECS[1][0][i], SECS[1][1][i]) for i in FAST])
AP_SECS.sort(key=lambda s: -s[1])      # slowest first


# ---------------------------------------------------------------- section block tables
class SecTab:
    """y[t] = x[t] - a1 y[t-1] - a2 y[t-2]; state s = (y[t-1], y[t-2]).  Real modal basis
    (rotation-scaling block), scan powers for blocks of B, zero-input responses."""

    def __init__(self, a1, a2, B, levels, eps=1e-10):
        self.a1, self.a2, self.B = a1, a2, B
        A = np.array([[-a1, -a2], [1.0, 0.0]])
        w, V = np.linalg.eig(A)
        k = int(np.argmax(w.imag))
        T = np.stack([V[:, k].real, V[:, k].imag], axis=1)
        self.T, self.Ti = T, np.linalg.inv(T)
        self.Bd = self.Ti @ A @ T
        self.r = abs(w[k])
        self.A = A
        self.levels = levels
        self.pw = [np.linalg.matrix_power(self.Bd, B * (1 << d)) for d in range(max(levels, 1))]
        # zero-input response of output t (t = 0 first output of the block) to the entering
        # modal state m: y[t] = e0 . A^(t+1) T m
        self.ct = np.array([(np.linalg.matrix_power(A, t + 1) @ T)[0] for t in range(B)])
        mag = np.abs(self.ct).max(axis=1)
        keep = np.nonzero(mag > eps * max(mag.max(), 1e-300))[0]
        self.dcut = int(keep.max()) + 1 if len(keep) else 0

    def lane_pow(self, n):
        return np.linalg.matrix_power(self.Bd, self.B * n)


def run_zero(X, a1, a2, dt):
    """zero-state run over the last axis of X (blocks x B); returns Y and exit states."""
    Y = np.empty_like(X)
    y1 = np.zeros(X.shape[0], dt)
    y2 = np.zeros(X.shape[0], dt)
    for t in range(X.shape[1]):
        y = (X[:, t] - a1 * y1 - a2 * y2).astype(dt)
        y2, y1 = y1, y
        Y[:, t] = y
    return Y, np.stack([y1, y2], axis=1)


def block_section(X, tab, wave=64, dt=complex):
    """One section, causal, over blocks X (nblk x B): zero-state runs, modal scan
    (tab.levels Kogge-Stone levels inside each wave of `wave` blocks, then one cross-wave
    step from the previous wave's last block), corrections for t < dcut.  Block 0 enters
    from a zero state."""
    f32 = dt == np.complex64
    cast = (lambda a: np.asarray(a, np.float32)) if f32 else (lambda a: a)
    a1, a2 = (np.float32(tab.a1), np.float32(tab.a2)) if f32 else (tab.a1, tab.a2)
    Y, E = run_zero(X, a1, a2, dt)
    Ti = cast(tab.Ti)
    M = (E @ Ti.T).astype(dt)                       # modal exit states (nblk x 2)
    n = M.shape[0]
    for d in range(tab.levels):
        sh = 1 << d
        P = cast(tab.pw[d])
        prev = np.zeros_like(M)
        for i in range(n):
            if (i % wave) >= sh:
                prev[i] = M[i - sh]
        M = (M + prev @ P.T).astype(dt)
    # cross-wave: block i of wave w adds Bd^(B (i+1)) M[last block of wave w-1]
    Mx = M.copy()
    for i in range(n):
        w, li = divmod(i, wave)
        if w > 0:
            P = cast(tab.lane_pow(li + 1))
            Mx[i] = (M[i] + P @ M[w * wave - 1]).astype(dt)
    ent = np.zeros_like(Mx)
    ent[1:] = Mx[:-1]
    ct = cast(tab.ct[:tab.dcut])
    Y[:, :tab.dcut] = (Y[:, :tab.dcut] + ent @ ct.T).astype(dt)
    return Y


# ---------------------------------------------------------------- kernel models
Q0 = -16           # first y2 index (support of the model)
K1_Q = 992         # y2 outputs per K1 tile
K2_M = 2048        # outputs per K2 tile
K2_SPAN = 5376     # y2 samples per K2 tile (256 x 21)
K2_LEFT = 560      # span starts at 2 m0 - K2_LEFT
AP_HALO = 64
AP_BLK = 10
U3_BASE = 128      # u3 index k <-> output m0 - 128 + k


def stage_len(L, k=K):
    for _ in range(k):
        L = (L + 1) // 2
    return L


def y2_len(L):
    m_hi = (L + 15) // 2
    q1 = (m_hi + 24) // 2 + 1
    return q1 - Q0


def k1(x, dt=complex):
    """x: mixed frame (complex).  Returns y2 buffer (index q - Q0)."""
    rdt = np.float32 if dt == np.complex64 else float
    L = len(x)
    n2 = y2_len(L)
    out = np.zeros(n2, dt)
    g0, g1 = G[0].astype(rdt), G[1].astype(rdt)
    ntile = -(-n2 // K1_Q)
    for tau in range(ntile):
        qs = Q0 + K1_Q * tau
        xs = 4 * qs - 64
        xt = np.zeros(4128, dt)
        lo, hi = max(xs, 0), min(xs + 4128, L)
        if hi > lo:
            xt[lo - xs:hi - xs] = x[lo:hi]
        # y1[ms + i], ms = 2 qs - 24, i in [0, 2048): x local 2i + 16 + t
        y1 = np.array([np.dot(g0, xt[2 * i:2 * i + 33]) for i in range(2031)], dt)
        for k in range(K1_Q):
            q = qs + k
            if q - Q0 >= n2:
                break
            out[q - Q0] = np.dot(g1, y1[2 * k:2 * k + 49])
    return out


OWN_TABS = [SecTab(a1, a2, B=21, levels=0) for a1, a2 in OWN_SEC]
AP_TABS = [SecTab(a1, a2, B=AP_BLK, levels=0) for a1, a2 in AP_SECS]
for _t in AP_TABS + OWN_TABS:   # scan depth from the block decay: (r^B)^reach < 1e-9
    reach = 1
    while (_t.r ** _t.B) ** reach > 1e-9:
        reach += 1
    _t.levels = int(np.ceil(np.log2(reach))) if reach > 1 else 0
    _t.pw = [np.linalg.matrix_power(_t.Bd, _t.B * (1 << d)) for d in range(max(_t.levels, 1))]


def k2(y2, n3, dt=complex):
    rdt = np.float32 if dt == np.complex64 else float
    out = np.zeros(n3, dt)
    g2 = G[2].astype(rdt)
    for m0 in range(0, n3, K2_M):
        qs = 2 * m0 - K2_LEFT
        span = np.zeros(K2_SPAN, dt)
        lo, hi = max(qs - Q0, 0), min(qs - Q0 + K2_SPAN, len(y2))
        if hi > lo:
            span[lo - (qs - Q0):hi - (qs - Q0)] = y2[lo:hi]
        X = span.reshape(256, 21)
        for tab in OWN_TABS:                                       # causal
            X = block_section(X, tab, dt=dt)
        X = X[::-1, ::-1].copy()
        for tab in OWN_TABS:                                       # anticausal
            X = block_section(X, tab, dt=dt)
        z2 = X[::-1, ::-1].reshape(-1)
        # u3[m0 - 128 + k], k in [0, 2304): z2 local 2k + 304 + t, t in [-28, 28]
        h = (len(g2) - 1) // 2
        c0 = K2_LEFT - 2 * U3_BASE
        u3 = np.array([np.dot(g2, z2[2 * k + c0 - h:2 * k + c0 + h + 1]) for k in range(2304)], dt)
        v = np.zeros(K2_M, dt)
        for q in range(4):     # wave q: outputs [512 q, + 512) from u3 [32 + 512 q, + 704)
            k0 = U3_BASE - AP_HALO + (K2_M // 4) * q
            V = u3[k0:k0 + 64 * AP_BLK].reshape(64, AP_BLK)
            for tab in AP_TABS:
                V = block_section(V, tab, dt=dt)
            V = V[::-1, ::-1].copy()
            for tab in AP_TABS:
                V = block_section(V, tab, dt=dt)
            V = V[::-1, ::-1].reshape(-1)
            v[(K2_M // 4) * q:(K2_M // 4) * (q + 1)] = V[AP_HALO:AP_HALO + K2_M // 4]
        n = min(K2_M, n3 - m0)
        out[m0:m0 + n] = v[:n]
    return out


def model_fp64(x):
    """The LTI model itself (convolutions + sosfilt), for the edge matrices."""
    L = len(x)
    pad = 4096
    y = np.concatenate([np.zeros(pad), x, np.zeros(pad)])
    for r in range(3):
        if r == 2:
            s = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in OWN_SEC])
            y = ss.sosfilt(s, y)
            y = ss.sosfilt(s, y[::-1])[::-1]
        g = G[r]
        c = (len(g) - 1) // 2
        y = np.convolve(y, g)[c::2][:len(y) // 2]
    s = np.array([[1, 0, 0, 1, a1, a2] for a1, a2 in AP_SECS])
    y = ss.sosfilt(s, y)
    y = ss.sosfilt(s, y[::-1])[::-1]
    m0 = pad // 8
    return y[m0:m0 + stage_len(L)]


def exact(x):
    for _ in range(K):
        x = ss.decimate(x, 2)
    return x


def edge_matrices(L, J=1536, R=192):
    """Left: out[m] += sum_j CL[m, j] x[j]; right: out[n3-1-m] += sum_j CR[m, j] x[L-1-j]."""
    Lc = 8192 + (L % 8)
    CL = np.zeros((R, J))
    CR = np.zeros((R, J))
    for j in range(J):
        e = np.zeros(Lc)
        e[j] = 1
        CL[:, j] = (exact(e) - model_fp64(e))[:R]
        e = np.zeros(Lc)
        e[Lc - 1 - j] = 1
        CR[:, j] = (exact(e) - model_fp64(e))[::-1][:R]
    return CL, CR


def pc_decimate(x, CL, CR, dt=complex):
    y2 = k1(x, dt)
    n3 = stage_len(len(x))
    out = k2(y2, n3, dt).astype(complex)
    R, J = CL.shape
    out[:R] += CL @ x[:J]
    out[n3 - R:] += (CR @ x[::-1][:J])[::-1]
    return out


if __name__ == "__main__":
    rng = np.random.default_rng(7)
    print("taps", [len(g) for g in G], "own r", [t.r for t in OWN_TABS], "levels", [t.levels for t in OWN_TABS],
          "dcut", [t.dcut for t in OWN_TABS])
    print("AP radii", np.round([t.r for t in AP_TABS], 3), "levels", [t.levels for t in AP_TABS],
          "dcut", [t.dcut for t in AP_TABS])
    for L in (20000, 20003):
        CL, CR = edge_matrices(L)
        nzl = np.abs(CL) > 1e-10
        print("edge support rows", np.nonzero(nzl.any(1))[0].max() + 1, "cols", np.nonzero(nzl.any(0))[0].max() + 1)
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)) / np.sqrt(2)
        x += np.exp(2j * np.pi * 0.011 * np.arange(L))
        ref = exact(x)
        for dt in (complex, np.complex64):
            got = pc_decimate(x.astype(dt) if dt == np.complex64 else x, CL, CR, dt)
            e = np.abs(got - ref) / np.abs(ref).max()
            print(L, np.dtype(dt).name, f"max rel err {e.max():.2e} (edges {max(e[:200].max(), e[-200:].max()):.2e})")
