"""Single cfg2 frame per call: device time of the whole chain vs the path-1 block size
(plan.tune(block, warm)), HIP events via plan.timings()."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import time  # noqa: E402

from pypanadapter_amd import ZoomFFT, synth  # noqa: E402

N, z, fs = 4096, 8, 2.4e6
for L in (N * 73, N * 256):
    x = synth.make_iq(L, fs, 4242, n_fft=N, zoom=z, n_win=N // z)
    for block in (0, 64, 128, 256, 512):
        with ZoomFFT(N, z, fs, n_win=N // z) as plan:
            if block:
                plan.tune(block, 192)
            for _ in range(20):
                plan.rows(x)
            plan.set_timing(True)
            dev = 0.0
            t0 = time.perf_counter()
            for _ in range(40):
                plan.rows(x)
                dev += sum(plan.timings()) / 40
            wall = (time.perf_counter() - t0) / 40 * 1e3
        print(f"L={L} block={block or 'auto'} device_ms={dev:.4f} wall_ms={wall:.4f}", flush=True)
