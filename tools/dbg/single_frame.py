"""Kernel breakdown of the reference's use: one cfg2 frame per call (psd_row through
zfft_process).  Run under rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pypanadapter_amd import ZoomFFT, synth  # noqa: E402

N, z, fs = 4096, 8, 2.4e6
x = synth.make_iq(N * 73, fs, 4242, n_fft=N, zoom=z, n_win=N // z)
with ZoomFFT(N, z, fs, n_win=N // z) as plan:
    for _ in range(50):
        plan.rows(x)
    plan.set_timing(True)
    acc = {}
    for _ in range(20):
        plan.rows(x)
        for i, (nm, ms) in enumerate(zip(plan.launch_names(), plan.timings())):
            acc[f"{i}:{nm}"] = acc.get(f"{i}:{nm}", 0.0) + ms / 20
    print({k: round(v, 4) for k, v in acc.items()})
