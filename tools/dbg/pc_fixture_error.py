#!/usr/bin/env python3
"""Where the zoomfft fixtures' PC error comes from (GPU diagnostic, not a
test).  For each tests/golden/zoomfft.npz case with >= 16384 samples, the decimated IQ's max
error relative to the output peak against the fixture (the reference's own zoomfft output):
  mix   the engine as shipped (LO mixed on the device: lo[n0] lo[2t+j] / sqrt 2 in fp32)
  pre   the LO applied in float64 on the host and cast to complex64, the engine at f_lo = 0
        (its LO table is then sqrt 2: one more fp32 rounding, no composite)
for paths 4 (tiles) and 5 (walk), and the error's position (interior or within 200 of an end).
usage: pc_fixture_error.py [out.json]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pypanadapter_amd import ZoomFFT  # noqa: E402


def main():
    zf = np.load(os.path.join(ROOT, "tests", "golden", "zoomfft.npz"))
    out = {}
    for nm in sorted({k.split("/")[0] for k in zf.files}):
        n_fft, n_avg, ratio, seed = (int(v) for v in zf[nm + "/meta"])
        x, ref = zf[nm + "/x"], zf[nm + "/y"]
        if x.size < 16384 or ratio == 1:
            continue
        n = np.arange(x.size)
        pre = (x.astype(np.complex128) * np.exp(-2j * np.pi * 1.0 * n / 2.4e6)).astype(np.complex64)
        for path in (4, 5):
            for kind, xin, flo in (("mix", x, 1.0), ("pre", pre, 0.0)):
                with ZoomFFT(max(32, n_fft), ratio, 2.4e6, f_lo=flo) as plan:
                    plan.set_path(path)
                    y = plan.decimate(xin)
                e = np.abs(y - ref) / np.abs(ref).max()
                i = int(e.argmax())
                key = f"{nm}/path{path}/{kind}"
                out[key] = {"max": float(e.max()), "at": i, "of": int(e.size),
                            "edge": bool(i < 200 or i >= e.size - 200),
                            "interior_max": float(e[200:-200].max()) if e.size > 400 else None}
                print(key, out[key])
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
