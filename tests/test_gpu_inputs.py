"""GPU parity of the caller-input formats fused into the stage-0 loads (zfft_config in_dtype,
flip_input): complex64, complex32 (f16, BASELINE cfg5) and RTL-SDR uint8,
each optionally reversed per frame (the sources' np.flip, S:541-543 / 459-460).

The oracle sees the same values the kernel is handed: the fp16 input widened to complex64
exactly, the uint8 bytes normalised as pyrtlsdr's packed_bytes_to_iq does (b/127.5 - 1, fp64;
pyrtlsdr is not vendored in the reference, so that normalisation is "parity unpinned" beyond
its published formula), and np.flip applied per frame.  Gate as every other row test."""
import numpy as np
import pytest

from conftest import assert_row_close, case_input, golden_cases, golden_rows, row_errors

pytestmark = pytest.mark.gpu


def _frames(F, L, N, z, W, seed0):
    from pypanadapter_amd import synth
    return np.stack([synth.make_iq(L, 2.4e6, seed0 + f, n_fft=N, zoom=z, n_win=W)
                     for f in range(F)])


def _encode(x, fmt):
    """complex64 frames -> (array handed to the engine, complex128 values it represents)."""
    if fmt == "complex64":
        return x, x.astype(np.complex128)
    if fmt == "complex32":
        h = np.ascontiguousarray(x).view(np.float32).astype(np.float16)
        v = h.astype(np.float64)
        return h, v[..., 0::2] + 1j * v[..., 1::2]
    # cu8: an 8-bit ADC view of the same signal (RTL-SDR read_bytes layout I,Q,I,Q,...)
    iq = np.ascontiguousarray(x).view(np.float32).astype(np.float64)
    b = np.clip(np.rint(127.5 + 127.5 * 0.25 * iq), 0, 255).astype(np.uint8)
    v = b.astype(np.float64) / 127.5 - 1.0
    return b, v[..., 0::2] + 1j * v[..., 1::2]


CONFIGS = [(1024, 8, 65536, 3), (4096, 8, 299008, 2), (2048, 2, 100003, 2), (256, 1, 16411, 3)]


@pytest.mark.parametrize("fmt", ["complex64", "complex32", "cu8"])
@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
@pytest.mark.parametrize("N,z,L,F", CONFIGS, ids=[f"N{c[0]}_z{c[1]}_L{c[2]}" for c in CONFIGS])
def test_input_format_rows_vs_oracle(oracle_lib, fmt, flip, N, z, L, F):
    from pypanadapter_amd import ZoomFFT
    W = N // z
    x = _frames(F, L, N, z, W, seed0=2000 + N + z)
    arr, vals = _encode(x, fmt)
    ref_in = vals[:, ::-1] if flip else vals
    refs = [oracle_lib.psd_row(ref_in[f], 2.4e6, N, z, W) for f in range(F)]
    for path in ([0, 1, 3] if z > 1 else [0]):
        with ZoomFFT(N, z, 2.4e6, n_win=W, in_dtype=fmt, flip=flip) as plan:
            plan.set_path(path)
            rows = plan.rows(arr)
        for f in range(F):
            assert_row_close(rows[f], refs[f], f"{fmt} flip={flip} path={path} frame {f}")


@pytest.mark.parametrize("fmt", ["complex32", "cu8"])
def test_input_format_decimate(oracle_lib, fmt):
    """zoomfft(x, ratio) on the converted input (S:2088-2100), including ratio 1 (mix only)."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(1, 40000, 1024, 4, 256, seed0=2500)[0]
    arr, vals = _encode(x, fmt)
    for ratio in (1, 4):
        with ZoomFFT(1024, ratio, 2.4e6, in_dtype=fmt, flip=True) as plan:
            y = plan.decimate(arr)
        ref = oracle_lib.zoomfft(vals[::-1], ratio, 2.4e6)
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err < 2e-6, (fmt, ratio, err)


def test_cfg5_fp16_storage_gate():
    """BASELINE cfg5: frames stored as complex32 against the reference's fp32/fp64 rows, under
    SURVEY §8c's fp16-storage gate (|ddB| <= 0.05 within 40 dB of peak, |d amp| <= 1e-3 x
    peak); fp32 arithmetic throughout."""
    from pypanadapter_amd import ZoomFFT
    c = next(c for c in golden_cases()["cases"] if c["name"] == "cfg5")
    x = case_input(c)
    h, _ = _encode(x, "complex32")
    with ZoomFFT(c["n_fft"], c["zoom"], c["fs"], n_win=c["n_win"], in_dtype="complex32") as plan:
        row = plan.rows(h)
    ref = golden_rows()["cfg5"].astype(np.float64)
    pk = ref.max()
    m = ref > pk - 40.0
    assert np.abs(row - ref)[m].max() <= 0.05
    _, damp = row_errors(row, ref)
    assert damp <= 1e-3


def test_input_format_rejects_wrong_arrays():
    from pypanadapter_amd import ZoomFFT
    with ZoomFFT(1024, 4, 2.4e6, in_dtype="cu8") as plan:
        with pytest.raises(ValueError):
            plan.rows(np.zeros(4096, np.float16))
        with pytest.raises(ValueError):
            plan.rows(np.zeros(4097, np.uint8))
    with pytest.raises(ValueError):
        ZoomFFT(1024, 4, 2.4e6, in_dtype="complex128")


def _audio(L, fs, seed):
    """Real float32 'audio': two tones over white noise (AudioPan's paFloat32 stream)."""
    rng = np.random.default_rng(seed)
    n = np.arange(L)
    x = 0.1 * rng.standard_normal(L) + np.sin(2 * np.pi * 0.123 * n) + 0.01 * np.cos(2 * np.pi * 0.31 * n)
    return x.astype(np.float32)


REAL_CASES = [(1024, 1, 1024, 12 * 1024), (1024, 1, 512, 12 * 1024), (2048, 1, 256, 9000),
              (4096, 1, 4096, 40000), (256, 1, 256, 300), (1024, 4, 256, 64 * 1024),
              (2048, 2, 1024, 30000), (16384, 1, 16384, 70000)]


@pytest.mark.parametrize("N,z,W,L", REAL_CASES, ids=[f"N{c[0]}_z{c[1]}_W{c[2]}_L{c[3]}" for c in REAL_CASES])
def test_real_input_rows_vs_reference(N, z, W, L):
    """Real input (AudioPan S:663-721): at zoom 1 scipy's welch is one-sided
    (rfft bins 0..N/2, doubled but for 0 and N/2) and the reference's fftshift/crop slice
    of those N/2+1 bins is shorter than W; when zooming the LO mix makes it complex.  The
    oracle is the reference's own scipy calls on the same float32 samples.  Every schedule
    and every Welch form."""
    from oracle import scipy_path
    from pypanadapter_amd import ZoomFFT
    fs = 44100.0
    x = np.stack([_audio(L, fs, 40 + f) for f in range(2)])
    refs = [scipy_path.psd_row(x[f], fs, N, z, W) for f in range(2)]
    assert (len(refs[0]) < W) == (z == 1)
    paths = [0, 1, 3] if z > 1 else [0]
    welchs = [0, 1, 2] if (z == 1 and N >= 4096) else [0, 1]
    for path in paths:
        for welch in welchs:
            with ZoomFFT(N, z, fs, n_win=W, in_dtype="f32") as plan:
                plan.set_path(path)
                plan.set_welch(welch)
                rows = plan.rows(x)
                assert plan.row_length == len(refs[0])
            for f in range(2):
                assert_row_close(rows[f], refs[f], f"real path={path} welch={welch} frame {f}")


def test_real_chunk_through_the_facade():
    """psd_row with a real chunk (what S:2102-2119 gets from AudioPan) takes the real path."""
    from oracle import scipy_path
    from pypanadapter_amd import psd_row
    x = _audio(20000, 44100.0, 7)
    for z, W in ((1, 1024), (2, 1024)):
        row = psd_row(x, 44100.0, 2048, z, W)
        ref = scipy_path.psd_row(x, 44100.0, 2048, z, W)
        assert row.shape == ref.shape
        assert_row_close(row, ref, f"facade z={z}")


def test_real_zoom1_rows_feed_the_waterfall():
    """AudioPan at zoom 1: psd_row's one-sided row is odd-length (N/2 + 1 = 513 here); the
    reference's Waterfall.image_update takes any width (S:1638-1664), so must the facade."""
    from oracle import scipy_path
    from pypanadapter_amd import Waterfall, psd_row
    fs, N = 44100.0, 1024
    ref_wf, wf = scipy_path.Waterfall(), Waterfall(scroll=1, fs=fs)
    for k in range(12):
        x = _audio(16 * N, fs, 900 + k)
        row = psd_row(x, fs, N, 1)
        want = scipy_path.psd_row(x, fs, N, 1, N)
        assert row.shape == want.shape == (N // 2 + 1,) and row.dtype == np.float64
        assert_row_close(row, want, f"real row {k}")
        ref_row = row.copy()
        wf.image_update(row)
        ref_wf.image_update(ref_row, 1)
        np.testing.assert_array_equal(row, ref_row)  # grid stamped in place, both
    np.testing.assert_array_equal(wf.img_array.astype(np.float32),
                                  ref_wf.img_array.astype(np.float32))


@pytest.mark.parametrize("W", [511, 97])
def test_odd_n_win_is_the_reference_slice(oracle_lib, W):
    """An odd crop width gives the reference's fftshift(P)[N//2 - W//2 : N//2 + W//2], W - 1
    entries (S:2114)."""
    from pypanadapter_amd import ZoomFFT
    N, z = 1024, 4
    x = _frames(2, N * z * 8, N, z, W - 1, seed0=77)
    with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
        assert plan.row_length == W - 1
        rows = plan.rows(x)
    assert rows.shape == (2, W - 1)
    for f in range(2):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, z, W), f"W={W} frame {f}")
