#!/usr/bin/env python3
"""Per-phase cycle shares of the FC kernel (path 6) from a -DFC_STAMPS=1 build of
fc_kernels.hip with tools/patches/fc_stamps_r06.patch applied (run with ZFFT_LIB_PATH=<that lib>).
Diagnostic only: read the SHARES (s_memtime cycles per wave and block, each barrier's wait in the
phase it ends), not the run time of this build.  usage: fc_stamps.py [frames]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypanadapter_amd import ZoomFFT, _lib  # noqa: E402

SEGS = ["window in (prefetch wait, convert) + next prefetch issued", "pass A (DFT16 x2, twiddles, LDS) + barrier",
        "pass B + barrier", "pass C (C loads, DFT, MAC, inverse stage 1) + barrier",
        "inverse stages 2-4 + barrier", "stage 5 + x lo + stores"]


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = 299008
    import torch
    import bench
    dev = torch.device("cuda:0")
    x = bench.make_frames(torch, F, L, bench.CONFIGS["cfg2"], dev, 0)
    lib = _lib.load()
    buf = (ctypes.c_ulonglong * (len(SEGS) + 1))()
    with ZoomFFT(4096, 8, 2.4e6) as plan:
        plan.set_path(6)
        rows = torch.empty((F, 512), dtype=torch.float32, device=dev)
        for _ in range(3):
            plan.process_device(x.data_ptr(), L, F, rows.data_ptr())
        torch.cuda.synchronize()
        lib.zfft_debug_fc_stamps(buf)
        plan.process_device(x.data_ptr(), L, F, rows.data_ptr())
        torch.cuda.synchronize()
        rc = lib.zfft_debug_fc_stamps(buf)
    assert rc == 0, rc
    v = np.array(list(buf), dtype=np.float64)
    n = len(SEGS)
    wave_blocks = v[n]
    tot = v[:n].sum()
    print(f"frames {F}  wave-blocks {wave_blocks:.0f}  cycles per wave and block {tot / wave_blocks:.0f}")
    for name, c in zip(SEGS, v[:n]):
        print(f"  {name:60s} {c / wave_blocks:8.0f} cyc  {100 * c / tot:5.1f} %")


if __name__ == "__main__":
    main()
