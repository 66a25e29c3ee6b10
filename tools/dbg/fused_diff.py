"""Debug: XA stage-wise vs fused decimation at given lengths; saves arrays for offline study."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pypanadapter_amd import ZoomFFT
out = {}
for z, L in [(8, 4173), (4, 112), (8, 299008), (2, 5000)]:
    rng = np.random.default_rng(700 + z)
    x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
    out[f"x_{z}_{L}"] = x
    for fuse in (1, 2, 3):
        with ZoomFFT(32, z, 2.4e6) as plan:
            plan.set_path(3)
            plan.set_fuse(fuse)
            out[f"d{fuse}_{z}_{L}"] = plan.decimate(x)
            if fuse == 1 and z >= 4:  # intermediate stages, stage-wise
                for zz in (2, 4):
                    if zz < z:
                        with ZoomFFT(32, zz, 2.4e6) as p2:
                            p2.set_path(3)
                            out[f"s{zz}_{z}_{L}"] = p2.decimate(x)
os.makedirs("gpurun_out/dbg", exist_ok=True)
np.savez("gpurun_out/dbg/fused_diff.npz", **out)
print("saved", len(out))
