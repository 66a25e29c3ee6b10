#!/usr/bin/env python3
"""Numpy model of the exact-tile (XT) zero-phase decimation stage in MODAL state coordinates
(design tool for pypanadapter_amd/csrc/xt_kernels.hip; not used at run time).

Per tile of 64 lanes x 16 samples and per pass direction:
  1. every lane runs the DF2T cascade (scipy _sosfilt order) from a zero state over its
     16 samples -> provisional outputs y0[t] and end state z (DF2T coordinates);
  2. m = Ti z: the end state in the real modal basis of A (4 rotation-scaling 2x2 blocks,
     one per pole pair), where a step of 16 samples is a per-mode complex multiply;
  3. Kogge-Stone inclusive scan over lanes, per mode only as many levels as its pole radius
     needs (|lambda|^(16 * 2^levels) < ~1e-9): radii .587 .682 .808 .935 -> 2 2 3 5 levels;
  4. corrections y[t] += Cm[t] . m_in, Cm[t] = C A^t T (the entering state's response).
The backward pass runs the same on the reversed tile with a provisional top state 0; the
exact top state arrives with the next tile (its bottom exit state) and is applied to the
held kept outputs with the per-lane powers Lambda^(16 j) (one-tile lag).

Prints fp64-schedule error, fp32 emulation error and plain fp32 sosfiltfilt error, all
relative to scipy's fp64 sosfiltfilt()[::2]."""
import numpy as np
import scipy.signal as ss

sos = ss.cheby1(8, 0.05, 0.4, output="sos")
zi = ss.sosfilt_zi(sos).reshape(8)
LANES, B = 64, 16
TILE = LANES * B
PAD = 27


def step(s, u, sosm=sos, dt=complex):
    s = s.copy()
    x = u
    for k in range(4):
        b0, b1, b2, _, a1, a2 = sosm[k]
        y = dt(b0 * x + s[2 * k])
        s[2 * k] = dt(b1 * x - a1 * y + s[2 * k + 1])
        s[2 * k + 1] = dt(b2 * x - a2 * y)
        x = y
    return s, x


A = np.zeros((8, 8))
C = np.zeros(8)
for i in range(8):
    e = np.zeros(8)
    e[i] = 1
    s2, y = step(e, 0.0, dt=float)
    A[:, i] = s2
    C[i] = y

# real modal basis: columns (Re v, Im v) of one eigenvector per conjugate pair
w, V = np.linalg.eig(A)
pairs = [k for k in range(8) if w[k].imag > 0]
pairs.sort(key=lambda k: abs(w[k]))
T = np.zeros((8, 8))
for j, k in enumerate(pairs):
    v = V[:, k] / np.linalg.norm(V[:, k])
    T[:, 2 * j], T[:, 2 * j + 1] = v.real, v.imag
Ti = np.linalg.inv(T)
Bd = Ti @ A @ T
radius = np.array([abs(w[k]) for k in pairs])
LEVELS = [int(np.ceil(np.log2(np.log(1e-9) / (B * np.log(r))))) for r in radius]
Cm = np.array([C @ np.linalg.matrix_power(A, t) @ T for t in range(B)])   # (B, 8)


def block_pow(p):
    """(c, s) per mode of the 2x2 block of Bd^p: [[c, s], [-s, c]]."""
    M = np.linalg.matrix_power(Bd, p)
    return np.array([[M[2 * j, 2 * j], M[2 * j, 2 * j + 1]] for j in range(4)])


def apply_modal(cs, m):
    """m (..., 8) complex modal state times block diag [[c, s], [-s, c]]."""
    out = np.empty_like(m)
    for j in range(4):
        c, s = cs[j]
        a, b = m[..., 2 * j], m[..., 2 * j + 1]
        out[..., 2 * j] = c * a + s * b
        out[..., 2 * j + 1] = -s * a + c * b
    return out


def tile_pass(u, m_in, f32):
    """One direction over a tile (ascending): -> outputs (TILE,), exit modal state."""
    dt = np.complex64 if f32 else complex
    cast = (lambda a: a.astype(np.complex64)) if f32 else (lambda a: a)
    sosm = sos.astype(np.float32) if f32 else sos
    U = u.reshape(LANES, B).astype(dt)
    Y0 = np.empty_like(U)
    Z = np.empty((LANES, 8), dt)
    for i in range(LANES):
        s = np.zeros(8, dt)
        for t in range(B):
            s, Y0[i, t] = step(s, U[i, t], sosm, dt)
        Z[i] = s
    Tif = Ti.astype(np.float32) if f32 else Ti
    Mz = cast(Z @ Tif.T)                                  # modal end states
    Mz[0] = Mz[0] + cast(apply_modal(block_pow(B), m_in[None, :]))[0]
    Vs = Mz.copy()
    for j in range(4):                                     # per-mode truncated scan
        for d in range(LEVELS[j]):
            sh = 1 << d
            cs = block_pow(B * sh)[j]
            if f32:
                cs = cs.astype(np.float32)
            a, b = Vs[:, 2 * j].copy(), Vs[:, 2 * j + 1].copy()
            pa, pb = np.zeros_like(a), np.zeros_like(b)
            pa[sh:], pb[sh:] = a[:-sh], b[:-sh]
            Vs[:, 2 * j] = cast(a + cs[0] * pa + cs[1] * pb)
            Vs[:, 2 * j + 1] = cast(b - cs[1] * pa + cs[0] * pb)
    Min = np.vstack([m_in[None, :].astype(dt), Vs[:-1]])   # state entering each lane
    Cmf = Cm.astype(np.float32) if f32 else Cm
    Y = cast(Y0 + Min @ Cmf.T)
    return Y.reshape(-1), Vs[-1]


def xt_stage(x, f32):
    n = len(x)
    e = n + 2 * PAD
    ext = np.concatenate([2 * x[0] - x[PAD:0:-1], x, 2 * x[-1] - x[-2:-PAD - 2:-1]])
    nt = (e + TILE - 1) // TILE
    m = Ti @ (zi * ext[0])
    yf = np.empty(nt * TILE, complex)
    for t in range(nt):
        u = np.zeros(TILE, complex)
        seg = ext[t * TILE:(t + 1) * TILE]
        u[:len(seg)] = seg
        yf[t * TILE:(t + 1) * TILE], m = tile_pass(u, m, f32)
    yf = yf[:e]
    out = np.empty(e, complex)
    held = None
    for t in range(nt):
        lo, hi = t * TILE, min((t + 1) * TILE, e)
        u = np.full(TILE, yf[e - 1], complex)    # constant tail beyond e-1: steady state
        u[:hi - lo] = yf[lo:hi]
        top = Ti @ (zi * yf[e - 1]) if t == nt - 1 else np.zeros(8, complex)
        yb, m_bot = tile_pass(u[::-1], top, f32)
        yb = yb[::-1].copy()
        if held is not None:                    # lag: exact top state of the held tile
            plo, phi, ph = held
            Yh = ph.reshape(LANES, B)            # reversed-lane order j, step t
            corr = np.array([[Cm[tt] @ apply_modal(block_pow(B * j), m_bot[None, :])[0]
                              for tt in range(B)] for j in range(LANES)])
            out[plo:phi] = (Yh + corr).reshape(-1)[::-1][:phi - plo]
        held = (lo, hi, yb[::-1].copy())
        if t == nt - 1:
            out[lo:hi] = yb[:hi - lo]
    return out[PAD:PAD + n][::2]


if __name__ == "__main__":
    print("pole radii", np.round(radius, 4), "levels", LEVELS, "cond(T)", f"{np.linalg.cond(T):.1f}")
    off = Bd.copy()
    for j in range(4):
        off[2 * j:2 * j + 2, 2 * j:2 * j + 2] = 0
    print("off-block residue", f"{np.abs(off).max():.1e}")
    rng = np.random.default_rng(3)
    x = rng.standard_normal(9000) + 1j * rng.standard_normal(9000)
    ref = ss.sosfiltfilt(sos, x)[::2]
    for f32 in (False, True):
        got = xt_stage(x.astype(np.complex64) if f32 else x, f32)
        print("fp32" if f32 else "fp64", "max rel err", f"{np.abs(got - ref).max() / np.abs(ref).max():.2e}")
    r32 = ss.sosfiltfilt(sos.astype(np.complex64), x.astype(np.complex64))[::2]
    print("plain fp32 sosfiltfilt", f"{np.abs(r32 - ref).max() / np.abs(ref).max():.2e}")
