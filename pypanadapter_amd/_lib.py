"""ctypes binding of libzfft.so (include/zfft.h).

ctypes releases the GIL for the duration of each call, so a QThreadPool worker
(pypanadapter_thread.py:1485-1549) can run the engine while the GUI thread paints.
There is no CPU fallback: if the library is missing the import of the engine fails.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os

from .build import LIB_PATH

ZFFT_OK = 0
ZFFT_EINVAL = -1
ZFFT_ESHORT = -2
ZFFT_EHIP = -3
ZFFT_ENOMEM = -4
ZFFT_ENODEV = -5
ZFFT_EUNSUPPORTED = -6
ZFFT_EINTERNAL = -7

WINDOW_KINDS = {
    "hamming": 0, "hann": 1, "blackman": 2, "blackmanharris": 3, "nuttall": 4, "flattop": 5,
    "barthann": 6, "bartlett": 7, "triang": 8, "bohman": 9, "parzen": 10, "boxcar": 11,
    "kaiser": 12, "gaussian": 13, "general_gaussian": 14, "tukey": 15, "exponential": 16,
    "chebwin": 17, "dpss": 18,
}
# scipy.signal.get_window aliases (scipy/signal/windows/_windows.py `_win_equiv`)
WINDOW_ALIASES = {
    "hamm": "hamming", "ham": "hamming", "han": "hann", "black": "blackman",
    "blk": "blackman", "blackharr": "blackmanharris", "bkh": "blackmanharris", "nutl": "nuttall",
    "nut": "nuttall", "flat": "flattop", "flt": "flattop", "brthan": "barthann", "bth": "barthann",
    "bman": "bohman", "bmn": "bohman",
    "bart": "bartlett", "brt": "bartlett", "triangle": "triang", "tri": "triang", "parz": "parzen",
    "par": "parzen", "box": "boxcar", "ones": "boxcar", "rect": "boxcar", "rectangular": "boxcar",
    "ksr": "kaiser", "gauss": "gaussian", "gss": "gaussian", "general gaussian": "general_gaussian",
    "general gauss": "general_gaussian", "general_gauss": "general_gaussian", "ggs": "general_gaussian",
    "tuk": "tukey", "poisson": "exponential", "cheb": "chebwin",
}
WIN_ARRAY = 100


class zfft_config(ctypes.Structure):
    _fields_ = [
        ("n_fft", ctypes.c_int32), ("zoom", ctypes.c_int32), ("n_win", ctypes.c_int32),
        ("window_kind", ctypes.c_int32), ("fs", ctypes.c_double), ("f_lo", ctypes.c_double),
        ("window_param", ctypes.c_double * 2), ("scroll", ctypes.c_int32),
        ("in_dtype", ctypes.c_int32), ("device", ctypes.c_int32), ("flip_input", ctypes.c_int32),
    ]


EXPORTS = [
    "zfft_plan_create", "zfft_plan_destroy", "zfft_process", "zfft_process_device",
    "zfft_decimate", "zfft_decimated_length", "zfft_waterfall_push", "zfft_waterfall_push_device",
    "zfft_waterfall_read", "zfft_waterfall_reset", "zfft_waterfall_shape", "zfft_window_values",
    "zfft_plan_tune", "zfft_plan_timing", "zfft_plan_timings", "zfft_plan_timing_names",
    "zfft_plan_path", "zfft_plan_welch", "zfft_plan_set_lo_frames", "zfft_last_error",
    "zfft_plan_config", "zfft_plan_row_length", "zfft_ring_create", "zfft_ring_destroy", "zfft_ring_add",
    "zfft_ring_state", "zfft_ring_take", "zfft_ring_process",
    "zfft_colormap_lut", "zfft_waterfall_colormap", "zfft_waterfall_levels",
    "zfft_waterfall_get_levels", "zfft_waterfall_autolevel", "zfft_waterfall_render",
    "zfft_waterfall_render_device", "zfft_waterfall_push_render", "zfft_waterfall_push_read64",
    "zfft_host_alloc", "zfft_host_free",
    "zfft_device_count", "zfft_version",
]

_lib = None


class ZfftError(RuntimeError):
    pass


def _share_hip_runtime_with_torch() -> None:
    """PyTorch-ROCm ships its own libamdhip64.so (file name without the .7 suffix but the
    same SONAME, libamdhip64.so.7).  If libzfft.so loads first, the dynamic linker maps
    /opt/rocm's runtime under that SONAME and torch later maps its own file too: two HIP
    runtimes in one process, and torch then reports "No HIP GPUs are available".  When
    torch is installed, pre-load its runtime globally so libzfft.so binds to that one."""
    if os.environ.get("ZFFT_HIP_RUNTIME", "") == "system":
        return
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if not spec or not spec.submodule_search_locations:
        return
    hip = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(hip):
        ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)


def load(path: str = ""):
    """Load libzfft.so; raises OSError (loudly) when it has not been built.  ZFFT_LIB_PATH
    selects another in-tree build of the same library (A/B of build variants)."""
    global _lib
    path = path or os.environ.get("ZFFT_LIB_PATH") or LIB_PATH
    if _lib is not None:
        return _lib
    _share_hip_runtime_with_torch()
    if not os.path.exists(path):
        raise OSError(f"libzfft.so not built at {path}: run `python -m pypanadapter_amd.build` "
                      "(there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    P, I32, I64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    cfgp = ctypes.POINTER(zfft_config)
    sig = {
        "zfft_plan_create": (ctypes.c_int, [cfgp, P, ctypes.POINTER(P)]),
        "zfft_plan_destroy": (ctypes.c_int, [P]),
        "zfft_process": (ctypes.c_int, [P, P, I64, I32, P]),
        "zfft_process_device": (ctypes.c_int, [P, P, I64, I32, P, P]),
        "zfft_decimate": (ctypes.c_int, [P, P, I64, P, ctypes.POINTER(I64)]),
        "zfft_decimated_length": (I64, [I64, I32]),
        "zfft_waterfall_push": (ctypes.c_int, [P, P]),
        "zfft_waterfall_push_device": (ctypes.c_int, [P, P, I32, P]),
        "zfft_waterfall_read": (ctypes.c_int, [P, P]),
        "zfft_waterfall_reset": (ctypes.c_int, [P, I32]),
        "zfft_waterfall_shape": (ctypes.c_int, [P, ctypes.POINTER(I32), ctypes.POINTER(I32)]),
        "zfft_window_values": (ctypes.c_int, [I32, P, I32, P]),
        "zfft_plan_tune": (ctypes.c_int, [P, I32, I32]),
        "zfft_plan_timing": (ctypes.c_int, [P, I32]),
        "zfft_plan_timings": (ctypes.c_int, [P, P, I32, ctypes.POINTER(I32)]),
        "zfft_plan_timing_names": (ctypes.c_char_p, [P]),
        "zfft_plan_path": (ctypes.c_int, [P, I32]),
        "zfft_plan_welch": (ctypes.c_int, [P, I32]),
        "zfft_plan_set_lo_frames": (ctypes.c_int, [P, P, I32, I32]),
        "zfft_last_error": (ctypes.c_char_p, []),
        "zfft_plan_config": (ctypes.c_int, [P, cfgp]),
        "zfft_plan_row_length": (ctypes.c_int, [P]),
        "zfft_ring_create": (ctypes.c_int, [I64, I32, ctypes.POINTER(P)]),
        "zfft_ring_destroy": (ctypes.c_int, [P]),
        "zfft_ring_add": (ctypes.c_int, [P, P, I64]),
        "zfft_ring_state": (ctypes.c_int, [P, ctypes.POINTER(I64), ctypes.POINTER(I64),
                                            ctypes.POINTER(I64)]),
        "zfft_ring_take": (ctypes.c_int, [P, ctypes.POINTER(P), ctypes.POINTER(I64),
                                           ctypes.POINTER(I64)]),
        "zfft_ring_process": (ctypes.c_int, [P, P, P, ctypes.POINTER(I32)]),
        "zfft_colormap_lut": (ctypes.c_int, [ctypes.c_char_p, P]),
        "zfft_waterfall_colormap": (ctypes.c_int, [P, ctypes.c_char_p]),
        "zfft_waterfall_levels": (ctypes.c_int, [P, D, D]),
        "zfft_waterfall_get_levels": (ctypes.c_int, [P, ctypes.POINTER(D), ctypes.POINTER(D)]),
        "zfft_waterfall_autolevel": (ctypes.c_int, [P, ctypes.POINTER(D), ctypes.POINTER(D)]),
        "zfft_waterfall_render": (ctypes.c_int, [P, P]),
        "zfft_waterfall_render_device": (ctypes.c_int, [P, P, P]),
        "zfft_waterfall_push_render": (ctypes.c_int, [P, P, I32, P]),
        "zfft_waterfall_push_read64": (ctypes.c_int, [P, P, I32, P]),
        "zfft_host_alloc": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(P)]),
        "zfft_host_free": (ctypes.c_int, [P]),
        "zfft_device_count": (ctypes.c_int, []),
        "zfft_version": (ctypes.c_int, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    """Map a negative ZFFT_E* code to the exception the reference path would raise."""
    if rc == ZFFT_OK:
        return
    msg = (_lib.zfft_last_error() or b"").decode(errors="replace") if _lib else ""
    text = f"{what}: {msg} (code {rc})"
    if rc in (ZFFT_EINVAL, ZFFT_ESHORT):
        raise ValueError(text)  # scipy raises ValueError for these (e.g. padlen)
    if rc == ZFFT_EUNSUPPORTED:
        raise NotImplementedError(text)
    raise ZfftError(text)
