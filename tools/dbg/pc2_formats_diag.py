"""Zoom-2 row errors of the PC tiles (4), XA (3) and the blocked passes (1) on the complex32
per-frame-LO case of tests/test_gpu_pc.py::test_pc2_input_formats_and_lo."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import row_errors  # noqa: E402
from oracle import coracle  # noqa: E402
from pypanadapter_amd import ZoomFFT, synth  # noqa: E402

F, L, N = 3, 131072 + 1, 2048
f_lo = [1.0, 150e3 + 1.0, -300e3 + 1.0]
x = np.stack([synth.make_iq(L, 2.4e6, 8900 + f, n_fft=N, zoom=2, n_win=1024, f_lo=f_lo[f]) for f in range(F)])
for fmt in ("complex64", "complex32"):
    if fmt == "complex32":
        arr = np.ascontiguousarray(x).view(np.float32).astype(np.float16)
        v = arr.astype(np.float64)
        vals = v[..., 0::2] + 1j * v[..., 1::2]
    else:
        arr, vals = x, x.astype(np.complex128)
    for path in (4, 3, 1):
        with ZoomFFT(N, 2, 2.4e6, n_win=1024, in_dtype=fmt, flip=True) as plan:
            plan.set_path(path)
            plan.set_lo_frames(f_lo, 1)
            rows = plan.rows(arr)
        errs = [row_errors(rows[f], coracle.psd_row(vals[f, ::-1], 2.4e6, N, 2, 1024, f_lo=f_lo[f])) for f in range(F)]
        print(fmt, "path", path, " ".join(f"f{f}: ddB {e[0]:.2e} damp {e[1]:.2e}" for f, e in enumerate(errs)))
