#!/usr/bin/env python3
"""Debug helper (GPU box): where the XA decimated IQ departs from the C oracle (64-output
blocks above 1e-3 relative error), for a few frame lengths and zooms."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypanadapter_amd import ZoomFFT  # noqa: E402
from oracle import coracle  # noqa: E402

coracle.build()
rng = np.random.default_rng(5)
for z, L in ((4, 20000), (4, 70001), (8, 70001), (4, 299008)):
    x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
    with ZoomFFT(4096, z, 2.4e6) as plan:
        plan.set_path(3)
        d = plan.decimate(x)
    ref = coracle.zoomfft(x, z, 2.4e6)
    err = np.abs(d - ref) / np.abs(ref).max()
    bad = np.nonzero(err > 1e-3)[0]
    print(f"z={z} L={L} len={len(d)} max={err.max():.3e} nbad={len(bad)}",
          f"first={bad[:1]} last={bad[-1:]}" if len(bad) else "")
    if len(bad):
        blk = 64
        prof = err[: len(err) // blk * blk].reshape(-1, blk).max(1)
        idx = np.nonzero(prof > 1e-3)[0]
        print("  bad 64-blocks:", idx[:40], "of", len(prof))
