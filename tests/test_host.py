"""CPU-only checks of the product's host side: the C-ABI library loads and exports what
include/zfft.h declares, config validation, native windows vs scipy.get_window, the pinned
filter constants.  No compute call reaches a GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_functions():
    text = open(os.path.join(ROOT, "include", "zfft.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(zfft_[a-z_0-9]+)\s*\(",
                                 text, re.M)))


def test_library_exports_every_declared_symbol(zfft_lib):
    from pypanadapter_amd import _lib
    declared = header_functions()
    assert len(declared) >= 15
    assert sorted(_lib.EXPORTS) == declared
    for name in declared:
        assert hasattr(zfft_lib, name), name
    assert zfft_lib.zfft_version() == 1


def test_decimated_length(zfft_lib):
    from oracle.coracle import stage_lengths
    for L in (28, 64, 100003, 299008, 1048576):
        for z in (1, 2, 8, 512):
            assert zfft_lib.zfft_decimated_length(L, z) == stage_lengths(L, z)[-1]
    assert zfft_lib.zfft_decimated_length(100, 3) == -1


def _cfg(**kw):
    from pypanadapter_amd._lib import zfft_config
    c = zfft_config()
    c.n_fft, c.zoom, c.n_win, c.window_kind = 4096, 8, 512, 0
    c.fs, c.f_lo, c.scroll = 2.4e6, 1.0, 1
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.mark.parametrize("bad", [dict(n_fft=1000), dict(n_fft=16), dict(zoom=3), dict(zoom=1024),
                                 dict(n_win=1), dict(n_win=8192), dict(n_win=0), dict(fs=0.0),
                                 dict(scroll=0), dict(window_kind=99), dict(window_kind=100),
                                 dict(in_dtype=4), dict(in_dtype=-1), dict(flip_input=2)])
def test_config_validation(zfft_lib, bad):
    plan = ctypes.c_void_p()
    rc = zfft_lib.zfft_plan_create(ctypes.byref(_cfg(**bad)), None, ctypes.byref(plan))
    assert rc == -1, (bad, rc)
    assert zfft_lib.zfft_last_error()
    assert not plan.value


def test_nodev_is_loud(zfft_lib):
    plan = ctypes.c_void_p()
    if zfft_lib.zfft_device_count() == 0:  # CPU container: no GPU -> ENODEV, loudly
        rc = zfft_lib.zfft_plan_create(ctypes.byref(_cfg()), None, ctypes.byref(plan))
        assert rc == -5
        from pypanadapter_amd import ZoomFFT
        with pytest.raises(RuntimeError):
            ZoomFFT(4096, 8, 2.4e6)


WINDOWS = ["hamming", "hann", "blackman", "blackmanharris", "nuttall", "flattop", "barthann",
           "bartlett", "triang", "bohman", "parzen", "boxcar", ("kaiser", 14), ("gaussian", 7),
           ("general_gaussian", 1.5, 7), ("tukey", 0.3), ("tukey", 0.0), ("tukey", 1.0),
           ("kaiser", 0.5), "han", "rect", "bmn", ("general gaussian", 2, 5), "tukey",
           ("exponential", 3), "exponential", ("exponential", 3, 2.5), "poisson"]
# windows computed through a solver / DFT, compared with scipy's LAPACK / pocketfft results
# to 5e-9 of the window maximum (fp32 rounding is 6e-8): the taper list's dpss and chebwin.
# dpss is conditioning-limited: at M=32768, NW=0.7 the top two eigenvalues of the
# tridiagonal differ by 6e-9 relative, so any fp64 eigenvector is only good to ~1e-9.
SOLVED = [("dpss", 3), ("dpss", 1.5), ("dpss", 0.7), ("chebwin", 100), ("cheb", 50)]


@pytest.mark.parametrize("win", WINDOWS, ids=str)
@pytest.mark.parametrize("M", [1, 2, 3, 7, 64, 584, 1000, 4096])
def test_native_windows_match_scipy(zfft_lib, win, M):
    import scipy.signal as ss
    from pypanadapter_amd import native_window
    ref = ss.get_window(win, M)
    got = native_window(win, M)
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("win", SOLVED, ids=str)
@pytest.mark.parametrize("M", [7, 64, 584, 1000, 4096, 32768])
def test_native_solved_windows_match_scipy(zfft_lib, win, M):
    import scipy.signal as ss
    from pypanadapter_amd import native_window
    ref = ss.get_window(win, M)
    got = native_window(win, M)
    np.testing.assert_allclose(got, ref, rtol=0, atol=5e-9)


@pytest.mark.parametrize("M", [65536, 4097])
def test_native_chebwin_long(zfft_lib, M):
    """chebwin's DFT runs at any length (Bluestein); cfg5 uses nperseg = 65536, whose
    extended length 65537 is prime (pocketfft takes Bluestein there too).  Agreement to
    2e-8 of the maximum: under the fp32 rounding (6e-8) the kernels see."""
    import scipy.signal as ss
    from pypanadapter_amd import native_window
    np.testing.assert_allclose(native_window(("chebwin", 100), M),
                               ss.get_window(("chebwin", 100), M), rtol=0, atol=2e-8)


def test_window_refusals_follow_scipy(zfft_lib):
    """Windows get_window refuses are refused (ValueError), not silently defaulted."""
    import scipy.signal as ss
    from pypanadapter_amd import native_window
    from pypanadapter_amd.engine import _window_spec
    for win, M in [("kaiser", 64), ("gaussian", 64), ("chebwin", 64), ("dpss", 64),
                   (("dpss", 40), 64), (("general_gaussian", 1.5), 64)]:
        with pytest.raises((ValueError, TypeError)):  # general_gaussian without sig: TypeError
            ss.get_window(win, M)
        with pytest.raises(ValueError):
            native_window(win, M)
    with pytest.raises(ValueError):  # slepian: unknown to scipy 1.15 as well
        _window_spec(("slepian", 0.3))
    kind, _, arr = _window_spec(np.hanning(16))
    assert kind == 100 and arr.dtype == np.float32


def test_filter_constants_pinned_to_scipy():
    import json
    import scipy.signal as ss
    from oracle.coracle import decim_filter
    sos, zi = decim_filter()
    np.testing.assert_array_equal(sos, ss.cheby1(8, 0.05, 0.8 / 2, output="sos"))
    np.testing.assert_array_equal(zi, ss.sosfilt_zi(sos))
    hdr = open(os.path.join(ROOT, "pypanadapter_amd", "csrc", "cheby1_q2.h")).read()
    vals = [float.fromhex(v) for v in re.findall(r"-?0x[0-9a-f.]+p[+-]\d+", hdr)]
    np.testing.assert_array_equal(np.array(vals[:24]).reshape(4, 6), sos)
    np.testing.assert_array_equal(np.array(vals[24:32]).reshape(4, 2), zi)
    _ = json


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "pypanadapter_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", text).replace("_oracle_", ""), f
