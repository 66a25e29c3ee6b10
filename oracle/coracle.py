"""ctypes front-end of the float64 C oracle (oracle/zfft_oracle.c).

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may use it as the checker; the product (pypanadapter_amd) never imports it.

The window array follows scipy.signal.get_window(window, nperseg) (periodic), exactly as
`welch` builds it (_spectral_py.py `_triage_segments`); nperseg = min(N, L_d) reproduces
welch's short-input branch.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_DIR, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _DIR], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        lib.oracle_zoomfft.restype = ctypes.c_int64
        lib.oracle_zoomfft.argtypes = [P, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_int, ctypes.c_int, P, P, P]
        lib.oracle_welch_row.restype = ctypes.c_int
        lib.oracle_welch_row.argtypes = [P, ctypes.c_int64, ctypes.c_double, ctypes.c_int,
                                         ctypes.c_int, P, ctypes.c_int, P]
        lib.oracle_waterfall_init.argtypes = [P, ctypes.c_int, P]
        lib.oracle_waterfall_push.argtypes = [P, ctypes.c_int, P, ctypes.c_int, P]
        lib.oracle_waterfall_read.argtypes = [P, ctypes.c_int, ctypes.c_int64, P]
        _lib = lib
    return _lib


def decim_filter():
    """(sos (4,6), zi (4,2)) float64, pinned by tools/gen_coeffs.py."""
    with open(os.path.join(_DIR, "cheby1_q2.json")) as fh:
        d = json.load(fh)
    sos = np.array([[float.fromhex(v) for v in r] for r in d["sos_hex"]], np.float64)
    zi = np.array([[float.fromhex(v) for v in r] for r in d["zi_hex"]], np.float64)
    return sos, zi


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def stage_lengths(L: int, zoom: int):
    n = [L]
    z = zoom
    while z > 1:
        n.append((n[-1] + 1) // 2)
        z //= 2
    return n


def zoomfft(x: np.ndarray, ratio: int, fs: float, f_lo: float = 1.0, mix: bool = True) -> np.ndarray:
    """S:2088-2100 -> complex128 decimated signal."""
    lib = _load()
    x = np.ascontiguousarray(x, dtype=np.complex64)
    sos, zi = decim_filter()
    sos = np.ascontiguousarray(sos)
    zi = np.ascontiguousarray(zi)
    out = np.empty(max(len(x), 1), dtype=np.complex128)
    n = lib.oracle_zoomfft(_ptr(x), len(x), fs, f_lo, int(ratio), int(bool(mix)), _ptr(sos),
                           _ptr(zi), _ptr(out))
    if n < 0:
        raise ValueError(f"oracle_zoomfft failed ({n}): input too short or bad ratio")
    return out[:n].copy()


def window(window, nperseg: int) -> np.ndarray:
    import scipy.signal as ss
    return np.asarray(ss.get_window(window, nperseg), dtype=np.float64)


def welch_row(x: np.ndarray, fs: float, n_fft: int, n_win: int, win="hamming") -> np.ndarray:
    """S:2111-2119 -> float64 dB row: the slice [N//2 - W//2, N//2 + W//2), 2 (W//2) long."""
    lib = _load()
    x = np.ascontiguousarray(x, dtype=np.complex128)
    nperseg = min(n_fft, len(x))
    w = win if isinstance(win, np.ndarray) else window(win, nperseg)
    w = np.ascontiguousarray(w, dtype=np.float64)
    assert len(w) == nperseg
    row = np.empty(n_win & ~1, dtype=np.float64)
    rc = lib.oracle_welch_row(_ptr(x), len(x), fs, n_fft, n_win, _ptr(w), nperseg, _ptr(row))
    if rc:
        raise ValueError(f"oracle_welch_row failed ({rc})")
    return row


def psd_row(chunk: np.ndarray, fs: float, n_fft: int, zoom: int, n_win: int,
            win="hamming", f_lo: float = 1.0) -> np.ndarray:
    """The row `update(chunk)` hands to waterfall.image_update (S:2102-2122)."""
    x = zoomfft(chunk, zoom, fs, f_lo, mix=zoom > 1)
    return welch_row(x, fs, n_fft, n_win, win)


class WaterfallRing:
    """Ring-offset restatement of Waterfall.init_image/image_update (S:1625-1664)."""

    def __init__(self):
        self.W = 0

    def image_update(self, psd: np.ndarray, scroll: int) -> None:
        lib = _load()
        W = int(psd.size)
        if W != self.W:
            self.W = W
            self.init_image()
        buf = np.ascontiguousarray(psd, dtype=np.float64)
        lib.oracle_waterfall_push(_ptr(self.ring), W, _ptr(self.off), int(scroll), _ptr(buf))
        psd[...] = buf  # the reference stamps the grid into the caller's row in place

    def init_image(self) -> None:
        lib = _load()
        self.ring = np.empty((self.W // 4, self.W), dtype=np.float64)
        self.off = np.zeros(1, dtype=np.int64)
        lib.oracle_waterfall_init(_ptr(self.ring), self.W, _ptr(self.off))

    @property
    def img_array(self) -> np.ndarray:
        lib = _load()
        img = np.empty_like(self.ring)
        lib.oracle_waterfall_read(_ptr(self.ring), self.W, int(self.off[0]), _ptr(img))
        return img
