"""Drop-in facade for the reference's DSP call sites.

The reference computes each waterfall line inline (pypanadapter_spectrum.py:2102-2119):

    if AppState.fft_ratio > 1:
        chunk = self.zoomfft(chunk, AppState.fft_ratio)
    sample_freq, spec = scipy.signal.welch(chunk, fs, window=AppState.fft_tapering,
                                           nperseg=AppState.fft_size, nfft=AppState.fft_size)
    spec = np.fft.fftshift(spec)[N//2 - self.N_WIN//2 : N//2 + self.N_WIN//2]
    psd = 20 * np.log10(abs(spec))
    self.waterfall.image_update(psd)

With this module those lines become `psd = psd_row(chunk, ...)` and `Waterfall` keeps its
`image_update(psd)` / `img_array` surface, backed by the device ring.  Like the
reference, `AppState` fields may change between frames: `PlanCache` re-creates the plan
whenever (N, zoom, W, window, fs, f_lo) change (S:1753-1757, 2079-2086, 1358-1363).
"""
from __future__ import annotations

import threading

import numpy as np

from .engine import ZoomFFT

_tls = threading.local()  # a plan is not re-entrant: one cache per calling thread


def _key(window):
    if isinstance(window, np.ndarray):
        return ("array", window.tobytes())
    return window if isinstance(window, str) else tuple(window)


class PlanCache:
    """Plan keyed on the AppState fields the reference re-reads every frame."""

    def __init__(self, device: int = 0):
        self.device = device
        self._key = None
        self.plan: ZoomFFT | None = None

    def get(self, fs, n_fft, zoom, n_win, window="hamming", f_lo=1.0,
            in_dtype="complex64") -> ZoomFFT:
        key = (float(fs), int(n_fft), int(zoom), int(n_win), _key(window), float(f_lo), in_dtype)
        if key != self._key:
            if self.plan is not None:
                self.plan.close()
            self.plan = ZoomFFT(n_fft, zoom, fs, n_win=n_win, window=window, f_lo=f_lo,
                                device=self.device, in_dtype=in_dtype)
            self._key = key
        return self.plan


def _cache(device: int, purpose: str = "rows") -> PlanCache:
    """Per thread, device and purpose: zoomfft and psd_row keep separate plans, so code
    alternating the two does not rebuild a plan on every call."""
    caches = getattr(_tls, "caches", None)
    if caches is None:
        caches = _tls.caches = {}
    key = (device, purpose)
    if key not in caches:
        caches[key] = PlanCache(device)
    return caches[key]


def zoomfft(x, ratio: int, fs: float, f_lo: float = 1.0, device: int = 0) -> np.ndarray:
    """ApplicationDisplay.zoomfft (S:2088-2100): LO mix + log2(ratio) x decimate(x, 2)."""
    plan = _cache(device, "zoomfft").get(fs, 32, int(ratio), 2, "hamming", f_lo)
    return plan.decimate(x)


def psd_row(chunk, fs: float, fft_size: int, fft_ratio: int, n_win: int | None = None,
            window="hamming", f_lo: float = 1.0, device: int = 0) -> np.ndarray:
    """The row ApplicationDisplay.update hands to waterfall.image_update (S:2102-2119).

    Returns a fresh, writable float64 array (the reference's dtype), length n_win
    (default N / zoom, i.e. N_WIN after fft_change, S:1757).  A real chunk (AudioPan,
    S:712-713) runs as real input: mixed to complex by the LO when zooming, and through
    welch's one-sided branch at zoom 1, whose row is the reference's shorter slice.
    """
    n_win = int(fft_size) // int(fft_ratio) if n_win is None else int(n_win)
    real = not np.iscomplexobj(chunk)
    plan = _cache(device).get(fs, fft_size, fft_ratio, n_win, window, f_lo,
                              "f32" if real else "complex64")
    return plan.rows(chunk).astype(np.float64)


def thread_psd_row(chunk, fs: float, fft_size: int, fft_ratio: int, window="hamming",
                   f_lo: float = 1.0, device: int = 0):
    """PSD.update of the threaded variant (pypanadapter_thread.py:1513-1548): skips chunks
    shorter than fft_size (T:1522-1523) and crops W = 2*int(0.5*N/zoom) (T:1542)."""
    if len(chunk) < fft_size:
        return None
    n_win = 2 * int(0.5 * fft_size / fft_ratio)
    return psd_row(chunk, fs, fft_size, fft_ratio, n_win, window, f_lo, device)


class Waterfall:
    """Waterfall.init_image / image_update / img_array (S:1625-1664) on the device ring.

    `image_update(psd)` stamps the grid into the caller's row in place (as S:1646-1648
    does; the reference then plots that same stamped row, S:2130), writes it as the new
    line, rolls by `scroll` and stamps the tick marks.  `img_array` materialises the
    image in the reference's row order (float64, like the reference's array).

    The device ring holds float32 (half the HBM and PCIe of float64 per line; the GPU
    rows are float32 anyway).  A float64 row from the reference's own pipeline (its psd is
    float64, S:2106) is stored as its float32 rounding, so `img_array` equals the
    reference's image exactly for float32-representable rows and within half a float32 ulp
    (<= 7.6e-6 dB for |dB| < 256) otherwise; the grid stamps (0) and the -500 fill are exact.
    Pinned by tests/test_gpu_parity.py::test_waterfall_float64_rows_are_held_as_float32.

    `image_update` stages the row on the host; the device push happens with the next read of
    the image (`img_array`, `render`, `autolevel`), together with that read in one round trip
    (zfft_waterfall_push_read64 / _push_render: one kernel, one copy, one wait per line), or
    when H rows are pending.  The image returned is the same as with a push per call.

    Buffer reuse: `img_array` and `render()` return one of two page-locked arrays this
    Waterfall owns and uses in turn, so an array stays valid until the read after next (what
    pyqtgraph's setImage per line needs: it copies or draws at once).  A caller that keeps
    images (recording, diffing, handing them to another thread) copies them, or passes its
    own array as `out=` to `render` / `image(out=...)`.  Like the reference's class, one
    Waterfall is for one thread.
    """

    def __init__(self, scroll: int = 1, device: int = 0, fs: float = 2.4e6):
        self.scroll = int(scroll)
        self.device = device
        self.fs = fs
        self.fftwidth = 0
        self._plan: ZoomFFT | None = None
        self._cmap = "Default"
        self._levels = (-220.0, -120.0)  # Waterfall.__init__ (S:1593-1598)
        self._pending: list[np.ndarray] = []  # rows image_update staged for the next read

    def _ensure(self, width: int):
        if width != self.fftwidth or self._plan is None:
            self._pending = []  # a new width re-inits the image (S:1632-1636)
            if self._plan is not None:
                self._plan.close()
            n_fft = 1 << max(5, (width - 1).bit_length())
            self._plan = ZoomFFT(n_fft, 1, self.fs, n_win=width, scroll=self.scroll,
                                 device=self.device)
            self._plan.waterfall_colormap(self._cmap)
            self._plan.waterfall_levels(*self._levels)
            self.fftwidth = width

    def init_image(self):
        self._pending = []
        if self._plan is not None:
            self._plan.waterfall_reset(self.scroll)

    def _take_pending(self):
        n = len(self._pending)
        rows = None if n == 0 else self._pending[0] if n == 1 else np.stack(self._pending)
        self._pending = []
        return rows

    def flush(self) -> None:
        """Push the staged rows to the device ring now (no image read)."""
        if self._plan is not None and self._pending:
            for r in np.atleast_2d(self._take_pending()):
                self._plan.waterfall_push(r)

    def close(self):
        """Release the device ring (the reference's image is garbage-collected)."""
        self._pending = []
        if self._plan is not None:
            self._plan.close()
            self._plan = None
            self.fftwidth = 0

    def set_scroll(self, scroll: int):
        """ApplicationDisplay.on_invertscroll_clicked (S:2074-2077): new direction + init."""
        self.scroll = int(scroll)
        self.init_image()

    def image_update(self, psd: np.ndarray) -> None:
        width = int(np.size(psd))
        self._ensure(width)
        for x in (0, width // 2, width - 1):
            psd[x] = 0
        self._pending.append(np.array(psd, dtype=np.float32).reshape(width))
        if len(self._pending) >= max(1, width // 4):  # H rows: the oldest would scroll out
            self.flush()

    def image(self, out: np.ndarray | None = None) -> np.ndarray:
        """The float64 (H, W) image in the reference's row order, staged rows pushed first."""
        if self._plan is None:
            raise AttributeError("img_array is created by the first image_update")
        return self._plan.waterfall_push_emit(self._take_pending(), True, out)

    @property
    def img_array(self) -> np.ndarray:
        return self.image()

    # ---- rendering: Waterfall.lookuptable / newlevel / autolevel, and the
    #      RGBA image pyqtgraph's ImageItem draws from img_array (S:1579-1623, 1667-1685)
    Colors = ("Default", "Matrix", "Red Green", "Tropical")

    def _need_plan(self):
        if self._plan is None:
            raise AttributeError("the waterfall image is created by the first image_update")
        return self._plan

    def lookuptable(self, choice: str) -> None:
        self._cmap = choice if choice in self.Colors else "Default"  # S:1613-1614
        if self._plan is not None:
            self._plan.waterfall_colormap(self._cmap)

    def newlevel(self, low: float, high: float):
        self._levels = (float(low), float(high))
        if self._plan is not None:
            self._plan.waterfall_levels(low, high)
        return low, high

    def autolevel(self):
        """Levels from the 2nd / 98th percentiles of the pixels below 0 (what S:1676
        computes; the reference stores them in unused attributes, so its button is a no-op)."""
        plan = self._need_plan()
        self.flush()
        self._levels = plan.waterfall_autolevel()
        return self._levels

    @property
    def levels(self):
        return self._plan.waterfall_levels() if self._plan is not None else self._levels

    def render(self, out: np.ndarray | None = None) -> np.ndarray:
        """RGBA uint8 (H, W, 4) in img_array's row order, staged rows pushed first (one
        round trip); see the class docstring for the reuse of the returned array."""
        return self._need_plan().waterfall_push_emit(self._take_pending(), False, out)


class Data:
    """pypanadapter_thread.py's `Data` (T:1400-1483) on the pinned double-buffered IQRing
    (SURVEY §8f-1), same calls: the reader thread's `add(chunk)` (T:2191) and the PSD
    worker's `get_data_start(); size = real_size; chunk = data[:size]; get_data_end()`
    (T:1516-1520).  `get_data_start` drains the ring, so `data[:real_size]` stays intact
    while the reader keeps adding (the reference hands out a view it keeps overwriting).
    `new_complex` takes complex64 (or, with `in_dtype="cu8"`, the RTL-SDR's raw interleaved
    uint8 I,Q bytes), `new_real` real float32 samples (AudioPan).  `fft_size` stands for
    AppState.fft_size, the target setter's lower bound (T:1477).  The NewtRap pacing
    (`delay_time`, the sleep in add) is out of scope; `target` keeps the reference's rules.
    Pinned by tests/golden/ring.npz, sequences of the reference's own class."""

    def __init__(self, chunk_size: int = 8196 * 2, in_dtype: str = "complex64",
                 fft_size: int = 2048):
        self.chunk_size = int(chunk_size)
        self.max_size = self.chunk_size * 16          # T:1406
        self.target_size = self.max_size * .9         # T:1407
        self.in_dtype = in_dtype
        self.fft_size = int(fft_size)
        self._ring = None
        self.data = None
        self.real = False
        self.real_size = 0
        self.total_size = 0

    def _new(self, in_dtype: str, real: bool):
        from .engine import IQRing
        if self._ring is not None:
            self._ring.close()
        self._ring = IQRing(self.chunk_size, in_dtype)
        self.real = real
        self.data, self.real_size, self.total_size = None, 0, 0
        return self

    def new_complex(self):
        """T:1419-1423 (new_common: empty buffer, counts 0)."""
        return self._new("complex64" if self.in_dtype == "f32" else self.in_dtype, False)

    def new_real(self):
        """T:1413-1417: real samples (AudioPan's float32 stream)."""
        return self._new("f32", True)

    def add(self, chunk):
        """T:1433-1457 without the pacing sleep: fold back at max_size, then the target clip
        np.clip(target_size, 8192, max_size) (T:1445) before the write."""
        self.target_size = np.clip(self.target_size, 8192, self.max_size)
        self._ring.add(chunk)

    def get_data_start(self):
        frame, total = self._ring.take()
        self.data = frame
        self.real_size = len(frame) if self._ring.in_dtype in ("complex64", "f32") else len(frame) // 2
        self.total_size = total

    def get_data_end(self):
        pass  # the counts were reset by the drain in get_data_start

    def process(self, plan):
        """get_data_start + PSD.update's DSP in one call (zfft_ring_process)."""
        return self._ring.process(plan)

    @property
    def size(self):
        """Data.size: where the next chunk goes (T:1426, 1449)."""
        return self._ring.state()[0]

    @property
    def target(self):
        return self.target_size

    @target.setter
    def target(self, t):
        if t >= self.fft_size and t <= self.max_size:  # T:1474-1479
            self.target_size = t

    @property
    def maxsize(self):
        return self.max_size
