"""numpy/scipy library-call restatement of the reference's DSP path.

TEST INFRASTRUCTURE ONLY (checker + bench.py cpu_baseline leg).  It makes the same
library calls the reference makes, with two generalisations the build's ABI needs:

  * LO on integer n with a per-stream f_lo (reference: float arange, f_demod = 1 Hz,
    pypanadapter_spectrum.py:2090-2094 / pypanadapter_thread.py:1526-1530);
  * the crop width W is an argument (S uses self.N_WIN, S:2114; T uses 2*int(0.5*N/z),
    T:1542-1543).

Everything else is the reference's code path verbatim in behaviour:
  zoomfft   S:2088-2100   decimate(x, 2) log2(ratio) times
  update    S:2108-2119   welch(..., window, nperseg=N, nfft=N) -> fftshift -> crop -> 20*log10
  Waterfall S:1625-1664   -500 init, grid stamps, img[-1]=psd, np.roll(img, -scroll, 0), ticks
"""
from __future__ import annotations

import warnings

import numpy as np
import scipy.signal


def local_oscillator(L: int, fs: float, f_lo: float = 1.0) -> np.ndarray:
    n = np.arange(L)
    turns = np.mod(n * (f_lo / fs), 1.0)
    return 2 ** .5 * np.exp(-2j * np.pi * turns)


def zoomfft(x: np.ndarray, ratio: int, fs: float, f_lo: float = 1.0) -> np.ndarray:
    x_mix = x * local_oscillator(len(x), fs, f_lo)
    for _ in range(int(np.log2(ratio))):
        x_mix = scipy.signal.decimate(x_mix, 2)
    return x_mix


def psd_row(chunk: np.ndarray, fs: float, n_fft: int, zoom: int, n_win: int,
            window="hamming", f_lo: float = 1.0) -> np.ndarray:
    if zoom > 1:
        chunk = zoomfft(chunk, zoom, fs, f_lo)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # "Input data is complex, switching to return_onesided=False"
        _, spec = scipy.signal.welch(chunk, fs, window=window, nperseg=n_fft, nfft=n_fft)
    spec = np.fft.fftshift(spec)[n_fft // 2 - n_win // 2:n_fft // 2 + n_win // 2]
    return 20 * np.log10(abs(spec))


class Waterfall:
    """Literal restatement of the reference's image model (full-image np.roll per line)."""

    def __init__(self):
        self.fftwidth = 0

    def init_image(self):
        self.img_array = -500 * np.ones((self.fftwidth // 4, self.fftwidth))
        self.img_array[:, 0] = 0
        self.img_array[:, self.fftwidth - 1] = 0

    def image_update(self, psd: np.ndarray, scroll: int) -> None:
        w = np.size(psd)
        if w != self.fftwidth:
            self.fftwidth = w
            self.init_image()
        for x in (0, w // 2, w - 1):
            psd[x] = 0
        self.img_array[-1:] = psd
        self.img_array = np.roll(self.img_array, -scroll, 0)
        for i, x in enumerate(range(0, w - 1, w // 10)):
            if i != 5 and i != 10:
                if scroll > 0:
                    self.img_array[5:15, x] = 0
                else:
                    self.img_array[-10:-2, x] = 0
