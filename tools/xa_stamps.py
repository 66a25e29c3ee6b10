#!/usr/bin/env python3
"""Per-phase cycle shares of the XA stage kernel from a -DXA_STAMPS=1 build
(tools/build_variants.py stamps=XA_STAMPS=1 (adds ZFFT_DIAG); run with ZFFT_LIB_PATH=<that lib>).
Diagnostic only: read the SHARES, not the run time of this build."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypanadapter_amd import ZoomFFT, _lib  # noqa: E402

SEGS = ["load+transpose", "fwd pass 1+modal", "fwd scan", "fwd pass 2+FIR+P", "frame-end v",
        "frame-end f/h", "bwd pass 1+modal", "bwd scan+pass 2", "finish_held", "flush"]


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    L = 299008
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((F, L, 2), dtype=np.float32) * 0.7).view(np.complex64)[..., 0]
    lib = _lib.load()
    buf = (ctypes.c_ulonglong * 11)()
    with ZoomFFT(4096, 8, 2.4e6) as plan:
        plan.set_path(3)
        plan.rows(x[:64])
        lib.zfft_debug_xa_stamps(buf)
        plan.rows(x)
        rc = lib.zfft_debug_xa_stamps(buf)
    assert rc == 0, rc
    v = np.array(list(buf), dtype=np.float64)
    tiles = v[10]
    tot = v[:10].sum()
    print(f"frames {F}  tiles (all stages) {tiles:.0f}  cycles/tile {tot / tiles:.0f}")
    for name, c in zip(SEGS, v[:10]):
        print(f"  {name:16s} {c / tiles:8.0f} cyc/tile  {100 * c / tot:5.1f} %")


if __name__ == "__main__":
    main()
