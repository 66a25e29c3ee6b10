#!/usr/bin/env python3
"""Numpy model of the "XA" zero-phase decimation stage (design tool for
pypanadapter_amd/csrc/xa_kernels.hip; not used at run time).

scipy.signal.decimate(x, 2) = sosfiltfilt(cheby1(8, .05, .4)) then [::2]
(_signaltools.py:4718-4828 / 4831-4989, called by pypanadapter_spectrum.py:2096-2098).
The cascade is H(z) = N(z) / D(z), N = b0 (1 + z^-1)^8, D = prod_k (1 + a1k z^-1 + a2k z^-2).
Since D(z) D(-z) = D2(z^2) (D2_k(w) = 1 + (2 a2k - a1k^2) w^-1 + a2k^2 w^-2), the zero-phase
stage followed by [::2] factors exactly as

    v = (1 / D(z)) ext                       forward all-pole cascade, full rate, causal
    h_j = sum_k M_k v_(j-8+k), j odd          25-tap FIR M = N(z) N(1/z) D(-1/z), kept j only
    g = (1 / D2(1/w)) h                      backward all-pole cascade on the kept (odd) j only

with scipy's edge rules carried over exactly: odd extension by 27, forward pre-history
= the steady state of constant ext[0] (sosfilt_zi * ext[0]); backward post-history = the
steady state of constant f[e-1] (f = N v is formed explicitly only near the frame end).
That costs 8 + 12.5 + 4 multiply-adds per input sample instead of the DF2T cascade's 2 x 17.

Parallel schedule (one wave per frame, tiles of 64 lanes x B samples, lane i owns
sub-block i): both all-pole passes run from a zero state per lane, then a modal
Kogge-Stone scan over lanes gives every lane its entering state (per-mode depth from the
pole radius), and outputs get Cm[t] . m_in.  The FIR window (8 back, 16 ahead) is moved
one 16-sample step back so a lane needs only its own and the previous lane's v.  The
backward pass of a tile starts from a provisional zero state at its top; its bottom exit
state is exact and is the top state of the tile below (one-tile lag), whose top K kept
outputs get the decaying correction Cm2full[d] . q (d = distance from the top).
The HIP kernel applies the per-lane corrections as a second pass instead (it reruns each
lane's sub-block from the exact entering state T . m_in, streaming the FIR), which is the
same linear map; only the one-tile-lag correction of the held outputs is kept as modelled.

Prints the fp64 model error (schedule exactness) and an fp32 emulation error vs scipy."""
import numpy as np
import scipy.signal as ss

SOS = ss.cheby1(8, 0.05, 0.4, output="sos")
A1, A2, B0 = SOS[:, 4], SOS[:, 5], SOS[0, 0]
PAD = 27
LANES = 64
N9 = B0 * np.array([1, 8, 28, 56, 70, 56, 28, 8, 1.0])
_dneg = np.array([1.0])
for _k in range(4):
    _dneg = np.convolve(_dneg, [1.0, -A1[_k], A2[_k]])
MP = np.convolve(N9, _dneg)            # taps on f_(j+k), k = 0..16 (anti-causal part)
M = np.convolve(MP, N9[::-1])          # taps on v_(j-8+k), k = 0..24
C1, C2 = 2 * A2 - A1 ** 2, A2 ** 2     # half-rate all-pole sections (w = z^2)


def ap_step(s, u, a1, a2):
    """One sample through the all-pole cascade.  s = (y_k[t-1], y_k[t-2]) per section,
    flattened (s[2k], s[2k+1]).  Returns new s, output."""
    s = s.copy()
    x = u
    for k in range(4):
        y = x - a1[k] * s[2 * k] - a2[k] * s[2 * k + 1]
        s[2 * k + 1] = s[2 * k]
        s[2 * k] = y
        x = y
    return s, x


def state_space(a1, a2):
    A = np.zeros((8, 8))
    C = np.zeros(8)
    for i in range(8):
        e = np.zeros(8)
        e[i] = 1
        s2, y = ap_step(e, 0.0, a1, a2)
        A[:, i] = s2
        C[i] = y
    return A, C


def modal(A):
    """Real modal basis T (columns Re v, Im v per pole pair, slowest last)."""
    w, V = np.linalg.eig(A)
    pairs = sorted([k for k in range(8) if w[k].imag > 0], key=lambda k: abs(w[k]))
    T = np.zeros((8, 8))
    for j, k in enumerate(pairs):
        v = V[:, k] / np.linalg.norm(V[:, k])
        T[:, 2 * j], T[:, 2 * j + 1] = v.real, v.imag
    Ti = np.linalg.inv(T)
    Bd = Ti @ A @ T
    radius = np.array([abs(w[k]) for k in pairs])
    return T, Ti, Bd, radius


class Pass:
    """Tables of one all-pole cascade (forward: a1, a2 at full rate; backward: c1, c2)."""

    def __init__(self, a1, a2, steps, eps=1e-9):
        self.a1, self.a2 = a1, a2
        self.A, self.C = state_space(a1, a2)
        self.T, self.Ti, self.Bd, self.radius = modal(self.A)
        self.steps = steps                  # samples per lane sub-block
        self.levels = [max(1, int(np.ceil(np.log2(np.log(eps) / (steps * np.log(r))))))
                       for r in self.radius]
        self.levels = [min(lv, 6) for lv in self.levels]
        self.cm = np.array([self.C @ np.linalg.matrix_power(self.A, t) @ self.T
                            for t in range(steps)])          # (steps, 8)

    def bpow(self, p):
        Mx = np.linalg.matrix_power(self.Bd, p)
        return np.array([[Mx[2 * j, 2 * j], Mx[2 * j, 2 * j + 1]] for j in range(4)])

    def cm_far(self, d):
        return self.C @ np.linalg.matrix_power(self.A, d) @ self.T

    def steady(self, c):
        """State for constant input c forever (all-pole cascade: y_k = y_(k-1) / D_k(1))."""
        s = np.zeros(8, dtype=np.result_type(c, complex))
        x = c
        for k in range(4):
            x = x / (1 + self.a1[k] + self.a2[k])
            s[2 * k] = s[2 * k + 1] = x
        return s


def apply_modal(cs, m):
    out = np.empty_like(m)
    for j in range(4):
        c, s = cs[j]
        a, b = m[..., 2 * j], m[..., 2 * j + 1]
        out[..., 2 * j] = c * a + s * b
        out[..., 2 * j + 1] = -s * a + c * b
    return out


def tile_pass(P, U, m_in, dt):
    """U: (LANES, steps) inputs in processing order; m_in: modal state entering lane 0.
    Returns corrected outputs (LANES, steps) and modal state after lane 63."""
    L, S = U.shape
    Y = np.empty_like(U)
    Z = np.zeros((L, 8), dt)
    a1 = P.a1.astype(np.float32) if dt == np.complex64 else P.a1
    a2 = P.a2.astype(np.float32) if dt == np.complex64 else P.a2
    for t in range(S):                                  # zero-state run, all lanes at once
        x = U[:, t]
        for k in range(4):
            y = (x - a1[k] * Z[:, 2 * k] - a2[k] * Z[:, 2 * k + 1]).astype(dt)
            Z[:, 2 * k + 1] = Z[:, 2 * k]
            Z[:, 2 * k] = y
            x = y
        Y[:, t] = x
    cast = (lambda a: a.astype(dt))
    f32 = dt == np.complex64
    Ti = P.Ti.astype(np.float32) if f32 else P.Ti
    Mz = cast(Z @ Ti.T)
    Mz[0] = Mz[0] + cast(apply_modal(P.bpow(S), m_in[None, :]))[0]
    Vs = Mz.copy()
    for j in range(4):
        for d in range(P.levels[j]):
            sh = 1 << d
            cs = P.bpow(S * sh)[j]
            if f32:
                cs = cs.astype(np.float32)
            a, b = Vs[:, 2 * j].copy(), Vs[:, 2 * j + 1].copy()
            pa, pb = np.zeros_like(a), np.zeros_like(b)
            pa[sh:], pb[sh:] = a[:-sh], b[:-sh]
            Vs[:, 2 * j] = cast(a + cs[0] * pa + cs[1] * pb)
            Vs[:, 2 * j + 1] = cast(b - cs[1] * pa + cs[0] * pb)
    Min = np.vstack([m_in[None, :].astype(dt), Vs[:-1]])
    cm = P.cm.astype(np.float32) if f32 else P.cm
    return cast(Y + Min @ cm.T), Vs[-1]


def xa_stage(x, B=32, K=192, f32=False):
    """One decimate(x, 2) by the XA schedule.  B: samples per lane (forward), K: kept
    outputs of the held tile that get the one-tile-lag correction."""
    dt = np.complex64 if f32 else complex
    T = LANES * B
    fwd = Pass(A1, A2, B)
    bwd = Pass(C1, C2, B // 2)
    Mt = M.astype(np.float32) if f32 else M
    MPt = MP.astype(np.float32) if f32 else MP
    N9t = N9.astype(np.float32) if f32 else N9
    x = x.astype(dt)
    n = len(x)
    e = n + 2 * PAD
    ext = np.concatenate([2 * x[0] - x[PAD:0:-1], x, 2 * x[-1] - x[-2:-PAD - 2:-1]]).astype(dt)
    nt = (e + 16 + T - 1) // T           # forward tiles; FIR/backward tile tau covers [tau T-16, tau T+T-16)
    # forward (exact per tile): v over [0, nt T)
    m = fwd.Ti @ fwd.steady(ext[0])
    v = np.empty(nt * T, dt)
    for tau in range(nt):
        u = np.zeros(T, dt)
        seg = ext[tau * T:(tau + 1) * T]
        u[:len(seg)] = seg
        vv, m = tile_pass(fwd, u.reshape(LANES, B), m.astype(dt), dt)
        v[tau * T:(tau + 1) * T] = vv.reshape(-1)
    vss = fwd.steady(ext[0])[6]          # v pre-history (last section steady value)
    # f near the end (explicit), clamped beyond e-1
    vp = np.concatenate([np.full(8, vss, dt), v[:e]])
    fe = np.array([np.dot(N9t, vp[s + 8 - np.arange(9)]) for s in range(e - 17, e)], dt)
    f_tail = np.concatenate([fe, np.full(17, fe[-1], dt)])   # f_(e-17) ... f_(e+16)
    h_ss = fe[-1] * (MP.sum().astype(np.float32) if f32 else MP.sum())

    def h_at(j):
        if j + 16 <= e - 1:
            w = np.array([v[j - 8 + k] if j - 8 + k >= 0 else vss for k in range(25)], dt)
            return np.dot(Mt, w)
        if j > e - 1:
            return h_ss
        return np.dot(MPt, f_tail[j - (e - 17):j - (e - 17) + 17])

    n_out = (n + 1) // 2
    out = np.zeros(n_out, dt)
    held = None
    for tau in range(nt):
        base = tau * T - 16                       # FIR/backward tile [base, base + T)
        js = base + 1 + 2 * np.arange(T // 2)     # odd positions, ascending
        h = np.array([h_at(j) if j >= PAD - 24 else 0 for j in js], dt)
        last = tau == nt - 1
        # backward: descending order; lanes in reverse (lane 0 = top sub-block)
        Hd = h[::-1].reshape(LANES, B // 2)
        top = bwd.Ti @ bwd.steady(h_ss) if last else np.zeros(8, complex)
        g, q = tile_pass(bwd, Hd, top.astype(dt), dt)
        g = g.reshape(-1)[::-1]                   # ascending, uncorrected for the top state
        if held is not None:
            hb, hg = held                          # held tile: corrections from its top down
            for d in range(min(K, len(hg))):
                hg[len(hg) - 1 - d] += bwd.cm_far(d) @ q
            ms = (hb + 1 - PAD) // 2 + np.arange(len(hg))
            ok = (ms >= 0) & (ms < n_out)
            out[ms[ok]] = hg[ok]
        held = (base, g.astype(complex))
        if last:
            ms = (base + 1 - PAD) // 2 + np.arange(len(g))
            ok = (ms >= 0) & (ms < n_out)
            out[ms[ok]] = g[ok]
    return out


if __name__ == "__main__":
    fwd, bwd = Pass(A1, A2, 32), Pass(C1, C2, 16)
    print("fwd radii", np.round(fwd.radius, 4), "levels", fwd.levels, "cond(T)", f"{np.linalg.cond(fwd.T):.1f}")
    print("bwd radii", np.round(bwd.radius, 4), "levels", bwd.levels, "cond(T)", f"{np.linalg.cond(bwd.T):.1f}")
    rng = np.random.default_rng(3)
    for n in (100, 5000, 9000, 20011):
        x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        x += 4 * np.exp(2j * np.pi * 0.013 * np.arange(n))
        ref = ss.sosfiltfilt(SOS, x)[::2]
        for f32 in (False, True):
            got = xa_stage(x.astype(np.complex64) if f32 else x, f32=f32)
            print(n, "fp32" if f32 else "fp64", "max rel err",
                  f"{np.abs(got - ref).max() / np.abs(ref).max():.2e}")
