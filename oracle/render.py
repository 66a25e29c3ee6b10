"""Waterfall rendering oracle -- TEST INFRASTRUCTURE ONLY.

numpy restatement of what the reference's Waterfall hands to pyqtgraph
(pypanadapter_spectrum.py:1579-1623, 1667-1685) and what pyqtgraph draws from it:

* lookuptable(choice)  -> pg.ColorMap(pos, color).getLookupTable(0.0, 1.0, 256): the stops
  of Waterfall.Colors interpolated per channel (np.interp) at np.linspace(0, 1, 256),
  truncated to uint8; opaque maps have no alpha column (ImageItem draws alpha 255).
  'Default' holds the stop value 2020 in a uint8 array (S:1581): numpy < 2 wrapped it to
  2020 % 256 = 228, numpy 2 raises OverflowError -- the restatement uses the wrapped value.
* setLevels([min, max]) + setImage(img.T, autoLevels=False) -> makeARGB: rescaleData
  (v - min) * (256 / (max - min)), clipped to [0, 255], astype(uint8), then the LUT row.
* autolevel -> np.percentile(img[img < 0], [2, 98]) (S:1676; the reference then assigns
  the result to unused attributes, so its levels never change -- the build applies them).

pyqtgraph is not installed in this image and is not vendored by the reference, so these
restatements are from its published algorithm: parity with pyqtgraph itself is unpinned
(the tests pin the device path to this restatement bit for bit).
"""
from __future__ import annotations

import numpy as np

COLORS = {
    "Default": ([0, .4, 1.], [[0, 0, 90, 255], [200, 2020 % 256, 0, 255], [255, 0, 0, 255]]),
    "Matrix": ([0., 1.], [[0, 0, 0, 255], [0, 255, 0, 255]]),
    "Red Green": ([0., 0.5, 1.], [[0, 0, 0, 255], [0, 255, 0, 255], [255, 0, 0, 255]]),
    "Tropical": ([0., .2, .4, .6, .8, 1.], [[68, 40, 153, 255], [222, 68, 252, 255],
                                            [252, 38, 99, 255], [252, 181, 38, 255],
                                            [86, 235, 49, 255], [3, 71, 7, 255]]),
}


def lookup_table(choice: str) -> np.ndarray:
    """256 x 4 uint8 (alpha 255): Waterfall.lookuptable (S:1611-1623)."""
    if choice not in COLORS:
        choice = "Default"
    pos, col = COLORS[choice]
    pos = np.array(pos, dtype=np.float64)
    col = np.array(col, dtype=np.float64)
    x = np.linspace(0.0, 1.0, 256)
    lut = np.empty((256, 4), dtype=np.uint8)
    for ch in range(3):
        lut[:, ch] = np.interp(x, pos, col[:, ch]).astype(np.uint8)
    lut[:, 3] = 255
    return lut


def render(img: np.ndarray, lut: np.ndarray, levels) -> np.ndarray:
    """makeARGB(img, lut, levels) as RGBA (H, W, 4), rows as given."""
    lo, hi = float(levels[0]), float(levels[1])
    if lo == hi:
        hi = np.nextafter(hi, 2 * hi)
    rng = hi - lo
    rng = 1.0 if rng == 0 else rng
    d = np.asarray(img, dtype=np.float64) - lo
    d *= 256 / rng
    idx = np.clip(d, 0, 255).astype(np.uint8)
    return lut[idx]


def autolevel(img: np.ndarray):
    """S:1676 as intended: (2nd, 98th) percentiles of the pixels below 0."""
    a = np.asarray(img, dtype=np.float64)
    lo, hi = np.percentile(a[a < 0], [2, 98])
    return float(lo), float(hi)
