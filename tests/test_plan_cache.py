"""Plan reuse of the module-level facade (panadapter.zoomfft / psd_row): the reference
re-reads AppState every frame (S:2088-2119), the facade rebuilds a plan only when a key
field changes -- and zoomfft and psd_row keep separate plans.  CPU-only: ZoomFFT is
replaced by a recorder, no device call is made."""
import threading

import numpy as np

from pypanadapter_amd import panadapter


class _Rec:
    made = []

    def __init__(self, n_fft, zoom, fs, **kw):
        self.key = (n_fft, zoom, fs, kw.get("n_win"), kw.get("in_dtype"))
        self.closed = False
        _Rec.made.append(self)

    def close(self):
        self.closed = True

    def decimate(self, x):
        return np.zeros(len(x) // self.key[1], np.complex64)

    def rows(self, chunk):
        return np.zeros(self.key[3], np.float32)


def test_zoomfft_and_psd_row_keep_separate_plans(monkeypatch):
    monkeypatch.setattr(panadapter, "ZoomFFT", _Rec)
    monkeypatch.setattr(panadapter, "_tls", threading.local())
    _Rec.made = []
    x = np.zeros(4096 * 8, np.complex64)
    for _ in range(3):
        panadapter.zoomfft(x, 8, 2.4e6)
        row = panadapter.psd_row(x, 2.4e6, 4096, 8)
        assert row.dtype == np.float64 and len(row) == 512
    assert len(_Rec.made) == 2 and not any(p.closed for p in _Rec.made)
    # a changed key field rebuilds only that purpose's plan
    panadapter.psd_row(x, 2.4e6, 4096, 4)
    assert len(_Rec.made) == 3 and _Rec.made[1].closed and not _Rec.made[0].closed
