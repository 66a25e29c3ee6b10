#!/usr/bin/env python3
"""Per-phase cycle shares of the PC walk kernel (path 5) from a -DPC_STAMPS=1 build
(tools/build_variants.py stamps=PC_STAMPS=1 (adds ZFFT_DIAG); run with ZFFT_LIB_PATH=<that lib>).
Diagnostic only: read the SHARES (cycles per wave and tile, barrier waits included in the phase
that ends with the barrier), not the run time of this build.  usage: pc_stamps.py [frames]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypanadapter_amd import ZoomFFT, _lib  # noqa: E402

SEGS = ["barrier after x to LDS (4 sub)", "FIR alpha (4 sub)", "y1 to LDS (4 sub)", "FIR beta+z (4 sub)",
        "own-rate causal", "own-rate anticausal", "FIR gamma", "output-rate sections",
        "out staging+stores", "x wait+LO mix+x to LDS (4 sub)"]


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
        plan.set_path(5)
        rows = torch.empty((F, 512), dtype=torch.float32, device=dev)
        for _ in range(3):
            plan.process_device(x.data_ptr(), L, F, rows.data_ptr())
        torch.cuda.synchronize()
        lib.zfft_debug_pc_stamps(buf)
        plan.process_device(x.data_ptr(), L, F, rows.data_ptr())
        torch.cuda.synchronize()
        rc = lib.zfft_debug_pc_stamps(buf)
    assert rc == 0, rc
    v = np.array(list(buf), dtype=np.float64)
    n = len(SEGS)
    wave_tiles = v[n]  # every wave's lane 0 adds its tile count
    tot = v[:n].sum()
    print(f"frames {F}  wave tiles {v[n]:.0f}  cycles per wave and tile {tot / wave_tiles:.0f}")
    for name, c in zip(SEGS, v[:n]):
        print(f"  {name:24s} {c / wave_tiles:8.0f} cyc  {100 * c / tot:5.1f} %")


if __name__ == "__main__":
    main()
