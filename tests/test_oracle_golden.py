"""Pin the oracle: both CPU restatements against rows produced by the reference itself.

Golden vectors come from running pypanadapter_spectrum.py / pypanadapter_thread.py in
the build container (tools/gen_golden.py).  The float64 C oracle must reproduce every
zoom>1 row to ~1e-9 dB; zoom==1 rows are computed by the reference in float32
(welch on the complex64 chunk), so there the float64 oracle sits within the fp32 gate.
"""
import numpy as np
import pytest

from conftest import (assert_row_close, case_input, golden_cases, golden_rows, window_of)

CASES = golden_cases()["cases"]


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_c_oracle_matches_reference_rows(c, oracle_lib):
    x = case_input(c)
    row = oracle_lib.psd_row(x, c["fs"], c["n_fft"], c["zoom"], c["n_win"], window_of(c["window"]),
                             c["f_lo"])
    ref = golden_rows()[c["name"]]
    tol = 1e-8 if c["zoom"] > 1 else 1e-3
    assert_row_close(row, ref, c["name"], db_tol=tol, amp_tol=1e-9 if c["zoom"] > 1 else 1e-5)


@pytest.mark.parametrize("c", [c for c in CASES if c["n_samples"] <= 300000][:12],
                         ids=lambda c: c["name"])
def test_scipy_path_matches_reference_rows(c):
    from oracle import scipy_path
    x = case_input(c)
    row = scipy_path.psd_row(x, c["fs"], c["n_fft"], c["zoom"], c["n_win"], window_of(c["window"]),
                             c["f_lo"])
    assert_row_close(row, golden_rows()[c["name"]], c["name"], db_tol=1e-9, amp_tol=1e-12)


def test_thread_and_spectrum_variants_agree():
    rows = golden_rows()
    assert np.array_equal(rows["cfg2"], rows["T_cfg2"])  # bit-identical


def test_zoomfft_fixtures(oracle_lib):
    import os
    from conftest import GOLDEN
    zf = np.load(os.path.join(GOLDEN, "zoomfft.npz"))
    names = sorted({k.split("/")[0] for k in zf.files})
    for nm in names:
        n_fft, n_avg, ratio, seed = zf[nm + "/meta"]
        y = oracle_lib.zoomfft(zf[nm + "/x"], int(ratio), 2.4e6, 1.0, mix=True)
        ref = zf[nm + "/y"]
        assert y.shape == ref.shape
        np.testing.assert_allclose(y, ref, rtol=0, atol=1e-12 * np.abs(ref).max())


def test_known_answers(oracle_lib):
    rows = golden_rows()
    # a tone at decimated bin k lands at row index k + W/2 (SURVEY §4 KAT)
    assert int(np.argmax(rows["kat_tone_bin37"])) == 37 + 128
    # unit-variance complex white noise at zoom 1: linear mean of the PSD = 1/fs
    p = 10 ** (rows["kat_noise_z1"] / 20.0)
    assert abs(10 * np.log10(p.mean()) - 10 * np.log10(1 / 2.4e6)) < 0.1


def test_short_input_and_minimal_lengths(oracle_lib):
    with pytest.raises(ValueError):  # stage 0 needs > 27 samples (sosfiltfilt padlen)
        oracle_lib.zoomfft(np.zeros(27, np.complex64), 2, 2.4e6)
    y = oracle_lib.zoomfft(np.ones(28, np.complex64), 2, 2.4e6)
    assert y.shape == (14,)


def _waterfall_golden():
    import json
    import os
    from conftest import GOLDEN
    wf = np.load(os.path.join(GOLDEN, "waterfall.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "cases.json")))["waterfall"]
    return wf, meta


@pytest.mark.parametrize("impl", ["ring", "roll"])
def test_waterfall_sequences(impl, oracle_lib):
    from oracle import scipy_path
    wf, meta = _waterfall_golden()
    for m in meta:
        scroll = m["scroll"]
        w = oracle_lib.WaterfallRing() if impl == "ring" else scipy_path.Waterfall()
        for k, width in enumerate(m["widths"]):
            if k in m["invert_at"]:
                scroll = -scroll
                if getattr(w, "fftwidth", getattr(w, "W", 0)):
                    w.init_image()
            row = wf[f"{m['name']}/row{k}"].astype(np.float64)
            w.image_update(row, scroll)
            np.testing.assert_array_equal(row.astype(np.float32), wf[f"{m['name']}/stamped{k}"])
            if (k + 1) in m["snaps"]:
                np.testing.assert_array_equal(w.img_array.astype(np.float32),
                                              wf[f"{m['name']}/img{k + 1}"], err_msg=m["name"])


def test_oracle_odd_width_is_the_reference_slice(oracle_lib):
    """fftshift(P)[N//2 - W//2 : N//2 + W//2] for odd W has W - 1 entries (S:2114); the C
    oracle and the library-call restatement agree on it."""
    from oracle import scipy_path
    from pypanadapter_amd import synth
    x = synth.make_iq(32768, 2.4e6, 5, n_fft=1024, zoom=4, n_win=256)
    for W in (255, 97, 1024):
        a = oracle_lib.psd_row(x, 2.4e6, 1024, 4, W)
        b = scipy_path.psd_row(x, 2.4e6, 1024, 4, W)
        assert a.shape == b.shape == (W & ~1,)
        np.testing.assert_allclose(a, b, atol=1e-7)
