"""GPU parity: the HIP path through the C-ABI against the reference's golden rows and the
float64 oracle.  Gate (conftest.py): |ddB| <= 1e-3 within 100 dB of the row
peak and |d amp| <= 1e-5 x peak amplitude; waterfall images bit-exact given the rows."""
import json
import os
import threading

import numpy as np
import pytest

from conftest import (GOLDEN, assert_row_close, case_input, check_rel, golden_cases, golden_rows,
                      row_errors, window_of)

pytestmark = pytest.mark.gpu
CASES = golden_cases()["cases"]


@pytest.fixture(scope="module", autouse=True)
def _gpu(zfft_lib):
    from pypanadapter_amd import device_count
    assert device_count() >= 1, "GPU tests need a HIP device"


def _plan_for(c, **kw):
    from pypanadapter_amd import ZoomFFT
    w = window_of(c["window"])  # every taper-list window is generated natively
    return ZoomFFT(c["n_fft"], c["zoom"], c["fs"], n_win=c["n_win"], window=w, f_lo=c["f_lo"], **kw)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_golden_rows(c):
    x = case_input(c)
    with _plan_for(c) as plan:
        row = plan.rows(x)
    assert row.shape == (c["n_win"],) and row.dtype == np.float32
    assert_row_close(row, golden_rows()[c["name"]], c["name"])


@pytest.mark.parametrize("path", [1, 3])
def test_golden_rows_every_schedule(path):
    """Every decimator schedule reproduces the reference rows (zoom > 1 cases)."""
    for c in CASES:
        if c["zoom"] == 1:
            continue
        x = case_input(c)
        with _plan_for(c) as plan:
            plan.set_path(path)
            row = plan.rows(x)
        assert_row_close(row, golden_rows()[c["name"]], f"{c['name']} path={path}")


def test_golden_rows_four_step_welch():
    """The four-step Welch (N1 x 256) reproduces the reference rows wherever it applies
    (n_fft >= 4096), including the short-input branch; the one-workgroup kernel refuses
    n_fft > 16384 loudly."""
    big = [c for c in CASES if c["n_fft"] >= 4096]
    assert any(c["n_fft"] > 16384 for c in big)
    for c in big:
        x = case_input(c)
        with _plan_for(c) as plan:
            plan.set_welch(2)
            row = plan.rows(x)
            if c["n_fft"] > 16384:
                with pytest.raises(NotImplementedError):
                    plan.set_welch(1)
        assert_row_close(row, golden_rows()[c["name"]], f"{c['name']} four-step")


def test_array_windows_reproduce_golden_rows():
    """ZFFT_WIN_ARRAY (any scipy window handed over as values) gives the same rows."""
    import scipy.signal as ss
    from pypanadapter_amd import ZoomFFT
    for c in CASES:
        if not c["name"].startswith("win_"):
            continue
        w = ss.get_window(window_of(c["window"]), c["n_fft"])
        n_dec = c["n_samples"]
        for _ in range(c["zoom"].bit_length() - 1):
            n_dec = (n_dec + 1) // 2
        with ZoomFFT(c["n_fft"], c["zoom"], c["fs"], n_win=c["n_win"], window=w) as plan:
            if n_dec < c["n_fft"]:
                # short-input branch: scipy.signal.welch raises for an array window longer
                # than the decimated frame (_spectral_py.py _triage_segments); so do we
                with pytest.raises(ValueError, match="longer than input"):
                    plan.rows(case_input(c))
                continue
            row = plan.rows(case_input(c))
        assert_row_close(row, golden_rows()[c["name"]], f"{c['name']} as array")


def test_zoomfft_fixtures():
    from pypanadapter_amd import ZoomFFT
    zf = np.load(os.path.join(GOLDEN, "zoomfft.npz"))
    for nm in sorted({k.split("/")[0] for k in zf.files}):
        n_fft, n_avg, ratio, seed = (int(v) for v in zf[nm + "/meta"])
        ref = zf[nm + "/y"]
        # path 1 (exact sosfiltfilt order) at 2e-6; the automatic schedule (path 0: PC's tiles
        # for one frame from 16384 samples on) and the walk (path 5, automatic from 4096
        # frames) at 6.5e-6, the documented default tolerance (include/zfft.h): measured
        # 1.3-5.3e-6 for the tiles and 6.07e-6 for the walk on zf_n512_z8 (the tolerance ledger,
        # profiles/r06h; DESIGN §3.5: the FIR taps summed in order)
        for path in (1, 0, 5):
            if path == 5 and (ratio not in (4, 8) or zf[nm + "/x"].size < 16384):
                continue
            with ZoomFFT(max(32, n_fft), ratio, 2.4e6) as plan:
                plan.set_path(path)
                y = plan.decimate(zf[nm + "/x"])
            assert y.shape == ref.shape and y.dtype == np.complex64
            tol = 6.5e-6 if (path in (0, 5) and ratio > 1 and zf[nm + "/x"].size >= 16384) else 2e-6
            check_rel(y, ref, tol, f"zoomfft/{nm}/path{path}")


def test_waterfall_sequences():
    from pypanadapter_amd import ZoomFFT
    wf = np.load(os.path.join(GOLDEN, "waterfall.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "cases.json")))["waterfall"]
    for m in meta:
        scroll, plan, width = m["scroll"], None, None
        for k, w in enumerate(m["widths"]):
            if w != width:
                if plan:
                    plan.close()
                plan = ZoomFFT(4096 if w <= 4096 else 16384, 1, 2.4e6, n_win=w, scroll=scroll)
                width = w
            if k in m["invert_at"]:
                scroll = -scroll
                plan.waterfall_reset(scroll)
            plan.waterfall_push(wf[f"{m['name']}/row{k}"])
            if (k + 1) in m["snaps"]:
                np.testing.assert_array_equal(plan.waterfall_image(), wf[f"{m['name']}/img{k + 1}"],
                                              err_msg=f"{m['name']} after {k + 1}")
        plan.close()


def test_waterfall_facade_stamps_row_in_place():
    from pypanadapter_amd import Waterfall
    wf = np.load(os.path.join(GOLDEN, "waterfall.npz"))
    w = Waterfall(scroll=1)
    for k in range(40):
        row = wf[f"w64_up/row{k}"].astype(np.float64)
        w.image_update(row)
        np.testing.assert_array_equal(row.astype(np.float32), wf[f"w64_up/stamped{k}"])
    np.testing.assert_array_equal(w.img_array.astype(np.float32), wf["w64_up/img40"])
    assert w.img_array.dtype == np.float64


def test_waterfall_float64_rows_are_held_as_float32():
    """The device ring is float32: the reference's float64 rows (its psd is
    float64, S:2106) come back from img_array as float64 of their float32 rounding, so
    img_array equals the reference's image exactly where the dB values are float32-exact and
    within half a float32 ulp (|dB| < 256: 7.6e-6 dB) elsewhere.  Stamps (0) and the -500 fill
    are exact either way."""
    from oracle.scipy_path import Waterfall as RefWaterfall
    from pypanadapter_amd import Waterfall
    rng = np.random.default_rng(64)
    w, ref = Waterfall(scroll=1), RefWaterfall()
    for k in range(20):
        row = rng.uniform(-200.0, -110.0, 256)           # float64, not float32-representable
        assert np.any(row.astype(np.float32).astype(np.float64) != row)
        w.image_update(row.copy())
        ref.image_update(row.copy(), 1)
    got = w.img_array
    assert got.dtype == np.float64
    np.testing.assert_array_equal(got, ref.img_array.astype(np.float32).astype(np.float64))
    assert np.abs(got - ref.img_array).max() <= 2.0 ** -16
    assert np.any(got != ref.img_array)                   # documented, not hidden
    w.close()


@pytest.mark.parametrize("W", [64, 512])
@pytest.mark.parametrize("scroll", [1, -1])
def test_waterfall_batch_push_matches_sequence(W, scroll):
    """zfft_waterfall_push_device of K rows at once (the parallel row + surviving-stamp
    launches) equals K reference image_update calls in order, for K < H, K = H and K > H,
    from a ring already offset by single pushes."""
    import torch
    from oracle.scipy_path import Waterfall as RefWaterfall
    from pypanadapter_amd import ZoomFFT
    H = W // 4
    rng = np.random.default_rng(W + scroll)
    with ZoomFFT(4096, 1, 2.4e6, n_win=W, scroll=scroll) as plan:
        ref = RefWaterfall()
        for k in range(3):
            row = rng.uniform(-200, -100, W).astype(np.float32)
            plan.waterfall_push(row)
            ref.image_update(row.astype(np.float64), scroll)
        for K in (5, H, H + 7):
            rows = rng.uniform(-200, -100, (K, W)).astype(np.float32)
            d = torch.from_numpy(rows).cuda()
            plan.waterfall_push_device(d.data_ptr(), K, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            for r in rows:
                ref.image_update(r.astype(np.float64), scroll)
            np.testing.assert_array_equal(plan.waterfall_image(), ref.img_array.astype(np.float32),
                                          err_msg=f"W={W} scroll={scroll} K={K}")


@pytest.mark.parametrize("W", [64, 512])
@pytest.mark.parametrize("scroll", [1, -1])
def test_waterfall_push_emit_matches_separate_calls(W, scroll):
    """zfft_waterfall_push_render / _push_read64 (rows pushed and the image read in one
    round trip; one fused kernel for a single row) give bit for bit what zfft_waterfall_push
    then zfft_waterfall_render / zfft_waterfall_read give, for 0, 1, 3, H and H + 2 rows per
    call, across a scroll inversion, with NaN pixels and non-default levels."""
    from pypanadapter_amd import ZoomFFT
    H = W // 4
    rng = np.random.default_rng(3 * W + scroll)
    kw = dict(n_win=W, scroll=scroll)
    with ZoomFFT(4096, 1, 2.4e6, **kw) as a, ZoomFFT(4096, 1, 2.4e6, **kw) as b:
        for p in (a, b):
            p.waterfall_colormap("Tropical")
            p.waterfall_levels(-190.0, -115.0)
        sc = scroll
        for step, K in enumerate([1, 1, 0, 3, 1, H, 1, H + 2, 1, 1]):
            if step == 6:  # the reference's scroll inversion (S:2074-2077) mid-sequence
                sc = -sc
                a.waterfall_reset(sc)
                b.waterfall_reset(sc)
            rows = rng.uniform(-200, -100, (K, W)).astype(np.float32)
            if K:
                rows[0, 5] = np.nan
            for r in rows:
                b.waterfall_push(r)
            f64 = step % 2 == 1
            got = a.waterfall_push_emit(rows if K else None, f64, out=None).copy()
            want = b.waterfall_image().astype(np.float64) if f64 else b.waterfall_render().copy()
            np.testing.assert_array_equal(got, want, err_msg=f"W={W} scroll={scroll} step={step} K={K}")
        np.testing.assert_array_equal(a.waterfall_image(), b.waterfall_image())


def test_waterfall_facade_deferred_reads_follow_the_reference():
    """The facade stages image_update rows and pushes them with the next image read: reading
    img_array / render after every line, after every few lines and across a width change (a
    new image) follows the reference's image_update sequence exactly; autolevel sees the
    staged rows."""
    from oracle import render as rr
    from oracle.scipy_path import Waterfall as RefWaterfall
    from pypanadapter_amd import Waterfall
    rng = np.random.default_rng(77)
    w, ref = Waterfall(scroll=1), RefWaterfall()
    for k in range(60):
        W = 128 if k < 45 else 256
        row = rng.uniform(-200.0, -110.0, W).astype(np.float32).astype(np.float64)
        w.image_update(row.copy())
        ref.image_update(row.copy(), 1)
        if k % 7 == 0 or k > 50:
            np.testing.assert_array_equal(w.img_array, ref.img_array, err_msg=f"line {k}")
        if k % 11 == 3:
            np.testing.assert_array_equal(w.render(), rr.render(ref.img_array, rr.lookup_table("Default"),
                                                                w.levels), err_msg=f"render {k}")
    w.image_update(rng.uniform(-200.0, -110.0, 256))
    lv = w.autolevel()
    assert lv == rr.autolevel(w.img_array)
    w.close()


def _frames(F, L, N, z, W, seed0=100, fs=2.4e6, f_lo=1.0):
    from pypanadapter_amd import synth
    return np.stack([synth.make_iq(L, fs, seed0 + f, n_fft=N, zoom=z, n_win=W, f_lo=f_lo)
                     for f in range(F)])


@pytest.mark.parametrize("N,z,L,F", [(4096, 8, 299008, 24), (1024, 4, 262144, 8),
                                      (16384, 8, 294912, 4), (2048, 2, 100003, 6),
                                      (1024, 16, 77779, 5), (256, 1, 16411, 7)])
def test_batched_frames_vs_oracle(oracle_lib, N, z, L, F):
    from pypanadapter_amd import ZoomFFT
    W = N // z
    x = _frames(F, L, N, z, W)
    with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, z, W), f"frame {f}")


@pytest.mark.parametrize("N,z,W,F", [(1024, 4, 256, 5), (1024, 2, 1024, 3), (2048, 8, 256, 3),
                                      (2048, 2, 2048, 2), (4096, 8, 512, 3), (4096, 4, 1024, 2),
                                      (8192, 8, 1024, 2), (8192, 2, 4096, 1), (16384, 8, 2048, 1)])
def test_welch_one_workgroup_forms_vs_oracle(oracle_lib, N, z, W, F):
    """Welch mode 1 (one workgroup per frame): the in-place DIF kernel for 1024 <= N <= 8192
    with its pruned (W <= 2N/RL) and full last stage, frames that leave spare slots in a
    multi-frame workgroup (N = 1024: 4 frames each), and the Stockham kernel at N = 16384."""
    from pypanadapter_amd import ZoomFFT
    L = N * z * 6
    x = _frames(F, L, N, z, W, seed0=8800 + N + z)
    with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
        plan.set_welch(1)
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, z, W), f"N={N} W={W} frame {f}")


@pytest.mark.parametrize("N,z,W,L", [(4096, 2, 2048, 299008), (1024, 4, 256, 262144), (16384, 1, 16384, 294912),
                                      (2048, 1, 2047, 100003), (8192, 8, 1024, 1048576), (4096, 1, 1000, 40960)])
def test_welch_split_few_frames_vs_oracle(oracle_lib, N, z, W, L):
    """A call of one or two frames -- the reference's use -- splits each frame's segments over
    several workgroups (welch_dif_split) and sums their partial PSDs in a second launch:
    rows within the gate (pruned and full last stage, odd W, zoom 1), identical on a repeat."""
    from pypanadapter_amd import ZoomFFT
    for F in (1, 2):
        x = _frames(F, L, N, z, W, seed0=9300 + N + z + F)
        with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
            rows = plan.rows(x)
            again = plan.rows(x)
        np.testing.assert_array_equal(rows, again)
        for f in range(F):
            assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, z, W), f"N={N} z={z} F={F} frame {f}")


@pytest.mark.parametrize("welch", [0, 1, 2])
@pytest.mark.parametrize("N,z,W", [(16384, 1, 16384), (16384, 2, 8192), (16384, 1, 12000)])
def test_welch_16384_unpruned_vs_oracle(oracle_lib, welch, N, z, W):
    """N = 16384 where the crop keeps more than the last stage's outputs 0 and RL-1 (zoom 1
    with the full row, zoom 2, a ragged W): the full DIF<16384> form (one 1024-thread frame,
    139 KB of LDS) that the automatic choice (welch 0) takes, the one-workgroup mode and
    the four-step form, all against the float64 oracle."""
    from pypanadapter_amd import ZoomFFT
    L = N * z * 4 + 123
    x = _frames(2, L, N, z, W, seed0=9900 + z + W // 1000)
    with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
        plan.set_welch(welch)
        rows = plan.rows(x)
    for f in range(2):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, z, W), f"welch={welch} W={W} frame {f}")


@pytest.mark.parametrize("N,z,W", [(32768, 8, 4096), (32768, 8, 4100), (65536, 16, 4096),
                                   (65536, 8, 8200), (16384, 8, 2048), (8192, 8, 1024),
                                   (4096, 8, 512), (16384, 4, 4096)])
def test_four_step_pruned_row_pass_vs_oracle(oracle_lib, N, z, W):
    """Four-step Welch (mode 2): the row pass keeps only the last radix-16 pass's outputs 0
    and 15 when the crop keeps |k| < N/16 (W <= N/8, N1 > 16); at W just above N/8 and at
    N1 = 16 it runs the full pass.  Both against the float64 oracle."""
    from pypanadapter_amd import ZoomFFT
    L = N * z * 3
    x = _frames(2, L, N, z, W, seed0=7100 + N // 1024 + z)
    with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
        plan.set_welch(2)
        rows = plan.rows(x)
    for f in range(2):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, z, W), f"N={N} z={z} W={W} frame {f}")


@pytest.mark.parametrize("block,warm", [(512, 192), (1024, 256), (64, 192), (8192, 128)])
def test_block_and_warmup_invariance(oracle_lib, block, warm):
    """The result must not depend on how frames are cut into lanes (within the gate)."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(3, 131072, 1024, 8, 128, seed0=900)
    with ZoomFFT(1024, 8, 2.4e6) as plan:
        plan.tune(block, warm)
        rows = plan.rows(x)
    for f in range(3):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, 1024, 8, 128), f"S={block}")


def test_lo_frequency_per_stream(oracle_lib):
    """Config 4: 8 IF centre frequencies, f_LO,k = 1 Hz + k*150 kHz."""
    from pypanadapter_amd import ZoomFFT
    for k in range(8):
        f_lo = 1.0 + k * 150e3
        x = _frames(1, 299008, 4096, 8, 512, seed0=300 + k, f_lo=f_lo)[0]
        with ZoomFFT(4096, 8, 2.4e6, f_lo=f_lo) as plan:
            row = plan.rows(x)
        assert_row_close(row, oracle_lib.psd_row(x, 2.4e6, 4096, 8, 512, f_lo=f_lo), f"k={k}")


def test_device_path_matches_host_path_bitwise():
    import torch
    from pypanadapter_amd import ZoomFFT
    x = _frames(5, 65536, 1024, 8, 128, seed0=50)
    with ZoomFFT(1024, 8, 2.4e6) as plan:
        host = plan.rows(x)
        d_in = torch.from_numpy(x.view(np.float32)).cuda()
        d_rows = torch.empty((5, 128), dtype=torch.float32, device="cuda")
        stream = torch.cuda.current_stream()
        plan.process_device(d_in.data_ptr(), 65536, 5, d_rows.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_rows.cpu().numpy(), host)
        plan.set_timing(True)
        plan.process_device(d_in.data_ptr(), 65536, 5, d_rows.data_ptr(), stream.cuda_stream)
        t = plan.timings()
        assert len(t) == len(plan.launch_names()) and all(v > 0 for v in t)


@pytest.mark.parametrize("N,z,L", [(4096, 8, 299008), (1024, 4, 262144), (2048, 16, 300000),
                                    (1024, 2, 70001), (4096, 32, 1048576)])
def test_fused_interior_matches_exact_pipeline(oracle_lib, N, z, L):
    """The fused commuted-order interior + exact edge windows (path 2) against the exact
    reference-order pipeline (path 1): decimated IQ within fp32 rounding everywhere,
    including the frame edges, and both rows within the gate of the float64 oracle."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(2, L, N, z, N // z, seed0=4200)
    out = {}
    for path in (1, 2, 3):
        with ZoomFFT(N, z, 2.4e6) as plan:
            plan.set_path(path)
            out[path] = (plan.rows(x), plan.decimate(x[0]))
    ref_dec = oracle_lib.zoomfft(x[0], z, 2.4e6)
    # fp32 relative error of the decimated IQ vs float64: DF2T schedules ~1e-6 per stage;
    # XA (all-pole + FIR + half-rate all-pole, tools/xa_proto.py) ~8e-6 per stage
    tol = {1: 3e-6, 2: 3e-6, 3: 1e-5 * np.log2(z)}
    for path in (1, 2, 3):
        d = out[path][1]
        assert d.shape == ref_dec.shape
        err = np.abs(d - ref_dec) / np.abs(ref_dec).max()
        assert err.max() < tol[path], (path, float(err.max()), int(err.argmax()), len(d))
    for f in range(2):
        ref = oracle_lib.psd_row(x[f], 2.4e6, N, z, N // z)
        assert_row_close(out[1][0][f], ref, "exact")
        assert_row_close(out[2][0][f], ref, "fused")
        assert_row_close(out[3][0][f], ref, "XA tiles")


def test_size_independent_properties():
    """At larger batches: determinism, frame-order equivariance, exact x2 scaling."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(16, 299008, 4096, 8, 512, seed0=7000)
    with ZoomFFT(4096, 8, 2.4e6) as plan:
        a = plan.rows(x)
        b = plan.rows(x)
        perm = np.random.default_rng(0).permutation(16)
        c = plan.rows(x[perm])
        d = plan.rows(2 * x)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(c, a[perm])
    assert np.all(np.isfinite(a))
    np.testing.assert_allclose(d - a, 20 * np.log10(4.0), atol=2e-4)


def test_minimal_and_short_lengths(oracle_lib):
    from pypanadapter_amd import ZoomFFT
    with ZoomFFT(32, 2, 2.4e6) as plan:
        x = _frames(1, 28, 32, 2, 16, seed0=5)[0]  # stage length 28 > padlen 27
        assert_row_close(plan.rows(x), oracle_lib.psd_row(x, 2.4e6, 32, 2, 16), "L=28")
        with pytest.raises(ValueError):
            plan.rows(x[:27])
    with ZoomFFT(2048, 512, 2.4e6) as plan:  # 6000 -> ... -> stage 8 has 24 <= 27 samples
        with pytest.raises(ValueError):
            plan.rows(np.zeros(6000, np.complex64))
    with ZoomFFT(1024, 1, 2.4e6) as plan:  # z=1 short input: nperseg = L
        x = _frames(1, 300, 1024, 1, 1024, seed0=6)[0]
        assert_row_close(plan.rows(x), oracle_lib.psd_row(x, 2.4e6, 1024, 1, 1024), "L<N")


def test_array_window_rejects_short_frames():
    import scipy.signal as ss
    from pypanadapter_amd import ZoomFFT
    with ZoomFFT(2048, 512, 2.4e6, n_win=4, window=ss.get_window(("chebwin", 100), 2048)) as plan:
        with pytest.raises(ValueError):  # scipy: "window is longer than input signal"
            plan.rows(np.zeros(299008, np.complex64))


def test_plans_in_threads(oracle_lib):
    """One plan per thread (the QThreadPool PSD worker shape, T:1485-1549)."""
    from pypanadapter_amd import ZoomFFT
    xs = [_frames(2, 131072, 1024, 4, 256, seed0=400 + 10 * t) for t in range(3)]
    out = [None] * 3

    def work(t):
        with ZoomFFT(1024, 4, 2.4e6) as plan:
            out[t] = plan.rows(xs[t])

    th = [threading.Thread(target=work, args=(t,)) for t in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for t in range(3):
        for f in range(2):
            ddb, damp = row_errors(out[t][f], oracle_lib.psd_row(xs[t][f], 2.4e6, 1024, 4, 256))
            assert ddb <= 1e-3 and damp <= 1e-5


def test_facade_matches_reference_rows():
    from pypanadapter_amd import psd_row, thread_psd_row
    c = {d["name"]: d for d in CASES}
    x = case_input(c["cfg2"])
    row = psd_row(x, 2.4e6, 4096, 8, 512)
    assert row.dtype == np.float64 and row.flags.writeable
    assert_row_close(row, golden_rows()["cfg2"], "psd_row")
    assert_row_close(thread_psd_row(x, 2.4e6, 4096, 8), golden_rows()["T_cfg2"], "thread")
    assert thread_psd_row(x[:4000], 2.4e6, 4096, 8) is None  # T:1522-1523


@pytest.mark.gpu
@pytest.mark.parametrize("z,F,L,want", [(8, 1, 299008, "pc"), (8, 15, 299008, "pc"),
                                        (8, 16, 299008, "fc"), (8, 384, 299008, "fc"),
                                        (8, 768, 1048576, "fc"), (8, 1024, 32768, "fc"),
                                        (8, 1023, 32768, "fc"), (8, 4, 8192, "exact"),
                                        (4, 1, 262144, "pc"), (4, 31, 262144, "pc"),
                                        (4, 32, 262144, "fc"), (4, 256, 262144, "fc"),
                                        (4, 384, 262144, "fc"), (4, 64, 1048576, "fc"),
                                        (4, 511, 65536, "fc"), (4, 512, 65536, "fc"),
                                        (4, 1024, 65536, "fc"), (4, 768, 8192, "xa"),
                                        (2, 512, 65536, "xa"), (2, 511, 65536, "pc2"), (2, 8, 262144, "pc2"),
                                        (2, 600, 1048576, "pc2"), (2, 768, 1048576, "xa"),
                                        (2, 8, 8192, "exact"),
                                        (16, 384, 262144, "fc"), (16, 512, 262144, "fc"),
                                        (16, 8, 262144, "pc")])
def test_auto_schedule_by_batch(z, F, L, want):
    """The automatic decimator schedule follows the measured crossovers (zfft_plan.cpp
    pc_fits / kPcWalkMinFrames / auto_xa / use_fused, tools/sweep_schedule.py,
    profiles/r04l): at zoom 8 the PC polyphase cascade for every batch of frames >= 16384
    samples (one frame per call -- the reference's use -- included), as its walk kernel
    from 1024 frames per call (round 6: profiles/r06k/sweep_walk.json); zoom >= 16 as PC's
    first three stages + XA where XA would take
    the batch and zoom 2's tiles does not (>= 512 frames; zoom 2's tiles below that, then the
    blocked passes under 16384 samples); at zoom 4 PC's tiles below 512 frames per call and
    the zoom-4 walk from there; at zoom 2 the tiles below 512, XA from there where XA takes the batch (the
    tiles, not the blocked passes, for 512-767 frames of > 2^19 samples); for frames < 16384 samples
    >= 384 frames of <= 2^19 samples (768 of longer ones) the XA tiles and smaller batches the
    exact blocked passes (the fused interior with edge windows is reached on request only)."""
    import torch
    from pypanadapter_amd import ZoomFFT
    dev = torch.device("cuda", 0)
    x = torch.zeros((F, L, 2), dtype=torch.float32, device=dev)
    x[..., 0] = 1.0
    N = {2: 2048, 4: 1024, 8: 4096, 16: 4096}[z]
    rows = torch.empty((F, N // z), dtype=torch.float32, device=dev)
    with ZoomFFT(N, z, 2.4e6, n_win=N // z) as plan:
        plan.set_timing(True)
        plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        names = plan.launch_names()
    first = {"exact": ("exact_forward_mix",), "fused": ("exact_forward_mix",),
             "xa": ("xa_stage_mix",), "pc": ("pc_fir",), "pc2": ("pc_tail",), "walk": ("pc_walk",),
             "fc": ("fc_decim",),
             "walk4": ("pc_walk4",)}[want]
    assert names[0] in first, names
    assert ("edge_windows" in names) == (want == "fused"), names
    if z == 16:  # the PC head's tail stage: zoom 2's tiles below 512 frames, else XA's
        assert ("xa_stage" in names) == (F >= 512) and names.count("pc_edge") == (1 if F >= 512 else 2), names
    del x, rows
    torch.cuda.empty_cache()


# frame lengths around the XA tile geometry (T = 2048 input samples per tile, odd
# extension 27 each side): no fast tile, exactly one, a fast tile ending at n + 27, the
# last tile reaching e - 1 exactly, odd and power-of-two lengths
XA_EDGE_LENGTHS = [28, 100, 2048 + 26, 2048 + 27, 2048 + 28, 4096 + 53, 4096 + 54, 4096 + 55,
                   6144 - 27, 8192, 8192 + 1, 10007, 3 * 2048 + 2048 // 2, 32769]


@pytest.mark.gpu
@pytest.mark.parametrize("z", [2, 8])
@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
def test_xa_decimate_tile_boundary_lengths(oracle_lib, z, flip):
    """XA (path 3) decimated IQ at frame lengths around its tile boundaries, every stage,
    against the float64 oracle (relative to the output peak, XA's documented tolerance);
    flip reverses the frame on load as the sources do (S:541-543)."""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(90 + z)
    for L in XA_EDGE_LENGTHS:
        if (L + z - 1) // z < 28:  # the last stage would be <= padlen: the reference raises
            continue
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        with ZoomFFT(32, z, 2.4e6, flip=flip) as plan:
            plan.set_path(3)
            d = plan.decimate(x)
        ref = oracle_lib.zoomfft(x[::-1].copy() if flip else x, z, 2.4e6)
        assert d.shape == ref.shape, (L, d.shape, ref.shape)
        err = np.abs(d - ref).max() / np.abs(ref).max()
        assert err < 1e-5 * np.log2(z), (L, z, flip, float(err))


def test_plan_fed_push_refuses_short_rows():
    """Odd W: the plan's rows hold W - 1 entries (the reference's slice), so pushing the
    plan's own last row into a W-wide waterfall is refused -- the reference's
    img_array[-1:] = psd raises there (S:1640) -- while a full-width host row still goes."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(1, 65536, 1024, 8, 127, seed0=77)[0]
    with ZoomFFT(1024, 8, 2.4e6, n_win=127) as plan:
        assert plan.row_length == 126
        plan.rows(x)
        with pytest.raises(ValueError):
            plan.waterfall_push()
        plan.waterfall_push(np.full(127, -150.0, np.float32))
        # the pushed row, apart from the tick stamps image_update writes (S:1655-1662)
        assert (plan.waterfall_image() == -150.0).sum(axis=1).max() >= 120


def test_xa_refuses_frames_beyond_32bit_offsets():
    """Path 3 addresses a frame's stage arrays with 32-bit buffer offsets: forced on a frame
    of >= 2^31 bytes it refuses before any launch (auto takes a blocked path there)."""
    import torch
    from pypanadapter_amd import ZoomFFT
    d = torch.zeros(64, dtype=torch.float32, device="cuda")
    rows = torch.empty(512, dtype=torch.float32, device="cuda")
    with ZoomFFT(4096, 8, 2.4e6, n_win=512) as plan:
        plan.set_path(3)
        with pytest.raises(NotImplementedError):
            plan.process_device(d.data_ptr(), 1 << 28, 1, rows.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("z,F,L,first,waits", [(8, 1024, 32768, "fc_decim", 1), (4, 2100, 32768, "fc_decim", 1),
                                                (2, 2100, 32768, "xa_stage_mix", 1), (2, 500, 32768, "pc_tail", 1),
                                                (4, 500, 32768, "fc_decim", 1), (4, 20, 32768, "pc_fir", 0)])
def test_batched_host_call_times_every_batch_with_one_schedule(z, F, L, first, waits):
    """zfft_process splits a >= 64 MB call into batches (H2D of k+1 under compute of k): the
    timings cover every batch, and a call the XA tiles would take keeps them in every batch
    (batches of >= 384 frames for these lengths, or a single batch) instead of splitting into
    batches too small for them; zoom 8 and 4 (PC's tiles below FC's batch, FC from it) take any
    batch by its own frame count."""
    from pypanadapter_amd import ZoomFFT
    x = np.zeros((F, L), np.complex64)
    x[:, ::3] = 1.0
    with ZoomFFT(1024, z, 2.4e6) as plan:
        plan.set_timing(True)
        rows = plan.rows(x)
        names = plan.launch_names()
    assert np.all(np.isfinite(rows))
    assert names.count(first) == names.count("batch_wait") + 1, names
    assert names.count("batch_wait") == waits, names


IF_LOS = [1.0 + k * 150e3 for k in range(8)]  # config 4's IF centre frequencies


@pytest.mark.parametrize("path", [1, 2, 3])
@pytest.mark.parametrize("per", [1, 3])
def test_lo_per_frame_every_schedule(oracle_lib, path, per):
    """Config 4 on one plan: 8 IF LOs over one batch, frame f mixed with
    f_lo[(f // per) % 8], on every decimator schedule, each frame vs the float64 oracle."""
    from pypanadapter_amd import ZoomFFT
    F, L = 24, 65536
    x = _frames(F, L, 1024, 8, 128, seed0=1300)
    with ZoomFFT(1024, 8, 2.4e6) as plan:
        plan.set_path(path)
        plan.set_lo_frames(IF_LOS, per)
        rows = plan.rows(x)
        d = plan.decimate(x[5])  # a single-frame call: frame 0 -> f_lo[0]
        plan.set_lo_frames([])   # back to the plan's f_lo
        row0 = plan.rows(x[7])
    for f in range(F):
        f_lo = IF_LOS[(f // per) % 8]
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, 1024, 8, 128, f_lo=f_lo),
                         f"path={path} per={per} frame {f}")
    ref = oracle_lib.zoomfft(x[5], 8, 2.4e6, f_lo=IF_LOS[0])
    assert np.abs(d - ref).max() / np.abs(ref).max() < 3e-5
    assert_row_close(row0, oracle_lib.psd_row(x[7], 2.4e6, 1024, 8, 128), "restored f_lo")


def test_lo_rows_refused_at_zoom_1():
    """Zoom 1 never mixes (the reference skips zoomfft at ratio 1, S:2108): several LO rows
    would be ignored by the rows, so the plan refuses them; one row (a new f_lo) is kept."""
    from pypanadapter_amd import ZoomFFT
    with ZoomFFT(1024, 1, 2.4e6) as plan:
        with pytest.raises(ValueError):
            plan.set_lo_frames([1.0, 2.0], 1)
        plan.set_lo_frames([5.0], 1)
        plan.set_lo_frames([], 1)


@pytest.mark.parametrize("path,first", [(0, "fc_decim"), (5, "pc_walk"), (4, "pc_fir"), (3, "xa_stage_mix")])
def test_lo_per_frame_bench_batch(oracle_lib, path, first):
    """Config 4 at the bench's geometry: 8 IFs x 512 frames of cfg2 in one F = 4096 batch on
    the device (the automatic schedule -- FC at this batch --, the walk, the PC tiles and XA),
    two frames of every IF vs the oracle at that IF's f_LO."""
    import torch
    import bench
    from pypanadapter_amd import ZoomFFT
    cfg = bench.CONFIGS["cfg4"]
    F, L = 4096, cfg["n_fft"] * cfg["n_avg"]
    dev = torch.device("cuda", 0)
    x = bench.make_frames(torch, F, L, cfg, dev, 77)
    rows = torch.empty((F, 512), dtype=torch.float32, device=dev)
    with ZoomFFT(4096, 8, 2.4e6, n_win=512) as plan:
        plan.set_lo_frames(IF_LOS, F // 8)
        plan.set_path(path)
        plan.set_timing(True)
        plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert plan.launch_names()[0] == first
    host = rows.cpu().numpy()
    for k in range(8):
        for f in (512 * k, 512 * k + 511):
            xf = bench.decoded_host(torch, x, f, "complex64")
            assert_row_close(host[f], oracle_lib.psd_row(xf, 2.4e6, 4096, 8, 512, f_lo=IF_LOS[k]),
                             f"IF {k} frame {f}")
    del x, rows
    torch.cuda.empty_cache()


def test_lo_per_frame_batched_host_call(oracle_lib):
    """A batched zfft_process call (H2D pipelined batches): frames keep their call index for
    the LO choice across the batch boundary."""
    from pypanadapter_amd import ZoomFFT
    F, L = 1024, 32768
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((F, L)) + 1j * rng.standard_normal((F, L))).astype(np.complex64)
    with ZoomFFT(1024, 8, 2.4e6) as plan:
        plan.set_lo_frames(IF_LOS, 100)
        plan.set_timing(True)
        rows = plan.rows(x)
        assert "batch_wait" in plan.launch_names()
    for f in (0, 99, 100, 511, 512, 513, 700, 1023):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, 1024, 8, 128,
                                                     f_lo=IF_LOS[(f // 100) % 8]), f"frame {f}")


@pytest.mark.parametrize("z", [4, 8, 32])
def test_xa_cascade_lengths_vs_oracle(oracle_lib, z):
    """XA, one launch per stage, against the float64 oracle within its tolerance at lengths
    around the tile geometry (an intermediate stage shorter than one tile, ragged ends, long
    frames).  (The 2-3-stages-per-launch ring variant this test used to compare against was
    removed in round 4 after measuring slower: DESIGN §3.1.)"""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(700 + z)
    for L in [28 * z, 2048 * 2 + 77, 9000, 65536 + 3, 299008]:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        with ZoomFFT(1024, z, 2.4e6) as plan:
            plan.set_path(3)
            got = plan.decimate(x)
        ref = oracle_lib.zoomfft(x, z, 2.4e6)
        assert got.shape == ref.shape
        err = np.abs(got - ref).max() / np.abs(ref).max()
        assert err < 1e-5 * np.log2(z), (L, z, float(err))
