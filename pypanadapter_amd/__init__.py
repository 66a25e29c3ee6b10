"""pypanadapter_amd -- MI355X-native Zoom-FFT spectrum/waterfall engine.

Drop-in for alfille/pypanadapter's IQ -> waterfall-line hot path
(pypanadapter_spectrum.py:2088-2130, pypanadapter_thread.py:1513-1549,
Waterfall S:1625-1664).  The compute runs in libzfft.so (hand-written gfx950 HIP
kernels behind the C-ABI in include/zfft.h); this package is the ctypes host side.
"""
from .engine import IQRing, ZoomFFT, colormap_lut, device_count, native_window, pinned_empty  # noqa: F401
from .panadapter import Data, PlanCache, Waterfall, psd_row, thread_psd_row, zoomfft  # noqa: F401

__all__ = ["ZoomFFT", "Waterfall", "PlanCache", "psd_row", "thread_psd_row", "zoomfft",
           "device_count", "native_window", "IQRing", "Data", "colormap_lut", "pinned_empty"]
