"""GPU parity of the FC decimator (path 6: zoom 8 as overlap-save FFT convolution with the ↓8
folded into the spectrum; fc_kernels.hip) against the float64 oracle of the
reference's decimate(x, 2) x 3 (pypanadapter_spectrum.py:2096-2098), its rows and the golden
rows recorded from the reference.

FC applies the zoom-8 model's response truncated at |k| <= 768 input samples (tail < 1.0e-6 of
sum |g|, tools/fc_model.py) through fp32 FFTs; the frame ends are the walk's maps.  Its fp32
error relative to the output peak is set from the tolerance ledger (conftest.check_rel)."""
import numpy as np
import pytest

from conftest import assert_row_close, case_input, check_rel, golden_cases, golden_rows
from test_gpu_pc import PC_LENGTHS, PC_TOL, _encode, _frames

pytestmark = pytest.mark.gpu
# the bound include/zfft.h documents for path 6: measured worst 6.07e-7 at K = 768 (the 2 GiB frame,
# fc_decim/largest_frame; 5.96e-7 fc8/decimate_lo; tolerance ledger profiles/r06tol/tol_ledger.json)
# + 7 %; FC sums in a fixed order (no atomics), so the worst is the same on every run
FC_TOL = 6.5e-7


@pytest.fixture(scope="module", autouse=True)
def _gpu(zfft_lib):
    from pypanadapter_amd import device_count
    assert device_count() >= 1, "GPU tests need a HIP device"


def _decimate_named(plan, x):
    plan.set_timing(True)
    d = plan.decimate(x)
    return d, plan.launch_names()


@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
def test_fc_decimate_vs_oracle(oracle_lib, flip):
    """Every L mod 8, the shortest frame, windows straddling the frame ends, cfg2 / cfg5 lengths;
    one frame per call (the frame split into runs of blocks over many workgroups)."""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(4400 + flip)
    for L in PC_LENGTHS:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        x += np.exp(2j * np.pi * 0.0071 * np.arange(L)).astype(np.complex64)
        with ZoomFFT(4096, 8, 2.4e6, flip=flip) as plan:
            plan.set_path(6)
            d, names = _decimate_named(plan, x)
        assert "fc_decim" in names, names
        ref = oracle_lib.zoomfft(x[::-1].copy() if flip else x, 8, 2.4e6)
        assert d.shape == ref.shape, (L, d.shape, ref.shape)
        check_rel(d, ref, FC_TOL, "fc8/decimate", (L, flip))


@pytest.mark.parametrize("L,kernel", [((1 << 28) - 3, "fc_decim"), ((1 << 28) + 5, "pc_walk")],
                         ids=["fc_largest_frame", "walk_past_2GiB"])
def test_fc_largest_frames_ends_vs_oracle(oracle_lib, L, kernel):
    """FC addresses a frame through 32-bit buffer offsets (launch_fc_decim, fc_fits): the largest
    complex64 frame it takes (< 2^31 bytes) runs FC, one past it runs the walk even with path 6
    forced.  Size-independent check at 2 GiB, both flips: the first and last 98,304 decimated
    samples equal the oracle's on a 2^20-sample prefix and on an 8-aligned suffix of the frame
    (the cascade has forgotten the far end long before; f_lo = 0 keeps the mix shift-invariant)."""
    from pypanadapter_amd import ZoomFFT
    x = np.random.default_rng(4490).standard_normal(2 * L, dtype=np.float32).view(np.complex64)
    L2, m = (1 << 20) + L % 8, 98304
    tol = FC_TOL if kernel == "fc_decim" else PC_TOL
    for flip in (False, True):
        s = x[::-1] if flip else x
        with ZoomFFT(4096, 8, 2.4e6, f_lo=0.0, flip=flip) as plan:
            plan.set_path(6)
            d, names = _decimate_named(plan, x)
        assert kernel in names and ("fc_decim" in names) == (kernel == "fc_decim"), names
        head = oracle_lib.zoomfft(np.ascontiguousarray(s[:L2]), 8, 2.4e6, f_lo=0.0)
        tail = oracle_lib.zoomfft(np.ascontiguousarray(s[L - L2:]), 8, 2.4e6, f_lo=0.0)
        check_rel(d[:m], head[:m], tol, f"{kernel}/largest_frame", ("head", flip))
        check_rel(d[-m:], tail[-m:], tol, f"{kernel}/largest_frame", ("tail", flip))


def test_fc_lo_offsets_vs_oracle(oracle_lib):
    """The LO moved into the filter: f_lo across the band (and past it), against the oracle's
    mixer on integer n."""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(4470)
    L = 299008 + 5
    x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
    for f_lo in (1.0, 150e3 + 1.0, -300e3 + 1.0, 1.1e6, 0.0):
        with ZoomFFT(4096, 8, 2.4e6, f_lo=f_lo) as plan:
            plan.set_path(6)
            d = plan.decimate(x)
        ref = oracle_lib.zoomfft(x, 8, 2.4e6, f_lo=f_lo)
        check_rel(d, ref, FC_TOL, "fc8/decimate_lo", f_lo)


@pytest.mark.parametrize("N,L,F", [(4096, 299008, 6), (16384, 294912, 3), (65536, 1048576, 2),
                                    (1024, 65536, 4), (32768, 524288 + 3, 2)])
def test_fc_rows_vs_oracle(oracle_lib, N, L, F):
    from pypanadapter_amd import ZoomFFT
    W = N // 8
    x = _frames(F, L, N, 8, W, seed0=5100 + N // 1024)
    with ZoomFFT(N, 8, 2.4e6, n_win=W) as plan:
        plan.set_path(6)
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, 8, W), f"N={N} L={L} frame {f}")


def test_fc_golden_rows():
    """Every zoom-8 golden row the reference recorded whose frame FC takes (>= 16384)."""
    from pypanadapter_amd import ZoomFFT
    from conftest import window_of
    n = 0
    for c in golden_cases()["cases"]:
        if c["zoom"] != 8 or c["n_samples"] < 16384:
            continue
        x = case_input(c)
        with ZoomFFT(c["n_fft"], 8, c["fs"], n_win=c["n_win"], window=window_of(c["window"]),
                     f_lo=c["f_lo"]) as plan:
            plan.set_path(6)
            row = plan.rows(x)
        assert_row_close(row, golden_rows()[c["name"]], c["name"])
        n += 1
    assert n >= 3


@pytest.mark.parametrize("fmt", ["complex32", "cu8", "f32"])
@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
def test_fc_input_formats(oracle_lib, fmt, flip):
    """complex32 / RTL-SDR u8 / real f32 and np.flip in the window loads (buffer loads, zero
    past the frame)."""
    from pypanadapter_amd import ZoomFFT
    F, L, N = 3, 299008 + 3, 4096
    x = _frames(F, L, N, 8, 512, seed0=6100)
    arr, vals = _encode(x, fmt)
    ref_in = vals[:, ::-1] if flip else vals
    with ZoomFFT(N, 8, 2.4e6, n_win=512, in_dtype=fmt, flip=flip) as plan:
        plan.set_path(6)
        rows = plan.rows(arr)
        d = plan.decimate(arr[1])
    check_rel(d, oracle_lib.zoomfft(ref_in[1].copy(), 8, 2.4e6), FC_TOL, f"fc8/format/{fmt}", flip)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(ref_in[f], 2.4e6, N, 8, 512),
                         f"{fmt} flip={flip} frame {f}")


def test_fc_lo_per_frame(oracle_lib):
    """Config 4 on one plan: frame f mixed with f_lo[f % 3] -- one filter table per LO row."""
    from pypanadapter_amd import ZoomFFT
    f_lo = [1.0, 150e3 + 1.0, -300e3 + 1.0]
    L, F = 299008, 6
    x = np.stack([_frames(1, L, 4096, 8, 512, seed0=6500 + f, f_lo=f_lo[f % 3])[0] for f in range(F)])
    with ZoomFFT(4096, 8, 2.4e6, n_win=512) as plan:
        plan.set_path(6)
        plan.set_lo_frames(f_lo, 1)
        rows = plan.rows(x)
        plan.set_lo_frames([], 1)          # back to cfg.f_lo: the tables follow
        rows0 = plan.rows(x[:1])
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, 4096, 8, 512, f_lo=f_lo[f % 3]),
                         f"frame {f}")
    assert_row_close(rows0[0], oracle_lib.psd_row(x[0], 2.4e6, 4096, 8, 512), "reset")


def test_fc_batch_rows_vs_oracle(oracle_lib):
    """A 1024-frame batch: one workgroup walks each frame, every window after the first taking
    the previous window's last 2048 samples from registers and the rest from the prefetch (the
    few-frame calls above split frames into one-block runs and never carry).  Picked frames
    against the oracle, the others zero."""
    import torch
    from pypanadapter_amd import ZoomFFT
    F, L, N, W = 1024, 299008 + 1, 4096, 512
    picks = (0, 511, F - 1)
    dev = torch.device("cuda:0")
    x = torch.zeros((F, L, 2), device=dev, dtype=torch.float32)
    xs = {f: _frames(1, L, N, 8, W, seed0=8100 + f)[0] for f in picks}
    for f, v in xs.items():
        x[f] = torch.from_numpy(np.ascontiguousarray(v).view(np.float32).reshape(L, 2)).to(dev)
    rows = torch.empty((F, W), device=dev, dtype=torch.float32)
    with ZoomFFT(N, 8, 2.4e6, n_win=W) as plan:
        plan.set_path(6)
        plan.set_timing(True)
        st = torch.cuda.current_stream()
        plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        names = plan.launch_names()
    assert "fc_decim" in names, names
    got = rows.cpu().numpy()
    for f in picks:
        assert_row_close(got[f], oracle_lib.psd_row(xs[f], 2.4e6, N, 8, W), f"frame {f}")


def test_fc_close_to_walk_at_a_batch():
    """FC and the walk (path 5) on the same 8 frames: two fp32 forms of one model."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(8, 299008, 4096, 8, 512, seed0=6950)
    out = {}
    for path in (5, 6):
        with ZoomFFT(4096, 8, 2.4e6) as plan:
            plan.set_path(path)
            out[path] = np.stack([plan.decimate(x[f]) for f in (0, 7)])
    check_rel(out[6], out[5], 8.6e-6, "fc8/vs_walk")


def test_fc_size_independent_properties():
    """Determinism, frame-order equivariance and exact x2 scaling (+12.04 dB) at a batch."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(12, 299008, 4096, 8, 512, seed0=7300)
    with ZoomFFT(4096, 8, 2.4e6) as plan:
        plan.set_path(6)
        a = plan.rows(x)
        b = plan.rows(x)
        perm = np.random.default_rng(1).permutation(12)
        c = plan.rows(x[perm])
        d = plan.rows(2 * x)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(c, a[perm])
    np.testing.assert_allclose(d - a, 20 * np.log10(4.0), atol=2e-4)


@pytest.mark.parametrize("zoom", [16, 32])
def test_fc_head_decimate_vs_oracle(oracle_lib, zoom):
    """Zoom >= 16: FC for the first three stages (the reference's stages apply one after
    another, S:2096-2098), then zoom 2's tiles / the blocked passes as after the walk."""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(4650 + zoom)
    for L in [16384, 16390, 262144 + 5, 299008]:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        x += np.exp(2j * np.pi * 0.0023 * np.arange(L)).astype(np.complex64)
        with ZoomFFT(4096, zoom, 2.4e6) as plan:
            plan.set_path(6)
            d, names = _decimate_named(plan, x)
        assert names[0] == "fc_decim", names
        ref = oracle_lib.zoomfft(x, zoom, 2.4e6)
        check_rel(d, ref, 7.5e-6, f"fc_head/zoom{zoom}", L)


# ---- zoom 4 (cfg1): four residues of 2048 points, the zoom-4 model truncated at |k| <= 512 ----

@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
def test_fc4_decimate_vs_oracle(oracle_lib, flip):
    """decimate(x, 2) twice (cfg1's decimator, S:2096-2098 at fft_ratio 4) at every L mod 4 and
    across the 1792-output block geometry, against the float64 oracle."""
    from pypanadapter_amd import ZoomFFT
    from test_gpu_pc import PC4_LENGTHS
    rng = np.random.default_rng(4800 + flip)
    for L in PC4_LENGTHS + [7168 * 3 + 5, 1048576 + 3]:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        x += np.exp(2j * np.pi * 0.013 * np.arange(L)).astype(np.complex64)
        with ZoomFFT(1024, 4, 2.4e6, flip=flip) as plan:
            plan.set_path(6)
            d, names = _decimate_named(plan, x)
        assert names[0] == "fc_decim", names
        ref = oracle_lib.zoomfft(x[::-1].copy() if flip else x, 4, 2.4e6)
        assert d.shape == ref.shape, (L, d.shape, ref.shape)
        check_rel(d, ref, FC_TOL, "fc4/decimate", (L, flip))


@pytest.mark.parametrize("N,L,F", [(1024, 262144, 5), (4096, 299008, 3), (2048, 131072 + 3, 4)])
def test_fc4_rows_vs_oracle(oracle_lib, N, L, F):
    from pypanadapter_amd import ZoomFFT
    W = N // 4
    x = _frames(F, L, N, 4, W, seed0=5300 + N // 1024)
    with ZoomFFT(N, 4, 2.4e6, n_win=W) as plan:
        plan.set_path(6)
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, 4, W), f"N={N} L={L} frame {f}")


@pytest.mark.parametrize("fmt", ["complex32", "cu8", "f32"])
def test_fc4_input_formats_and_lo(oracle_lib, fmt):
    """The raw formats with np.flip, and per-frame LO rows (one zoom-4 filter table each)."""
    from pypanadapter_amd import ZoomFFT
    F, L, N = 3, 262144 + 1, 1024
    x = _frames(F, L, N, 4, 256, seed0=6300)
    arr, vals = _encode(x, fmt)
    with ZoomFFT(N, 4, 2.4e6, n_win=256, in_dtype=fmt, flip=True) as plan:
        plan.set_path(6)
        d = plan.decimate(arr[1])
        f_lo = [1.0, 150e3 + 1.0, -300e3 + 1.0]
        plan.set_lo_frames(f_lo, 1)
        rows = plan.rows(arr)
    check_rel(d, oracle_lib.zoomfft(vals[1, ::-1].copy(), 4, 2.4e6), FC_TOL, f"fc4/format/{fmt}")
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(vals[f, ::-1].copy(), 2.4e6, N, 4, 256, f_lo=f_lo[f % 3]),
                         f"{fmt} frame {f}")


def test_fc4_batch_rows_vs_oracle(oracle_lib):
    """cfg1's geometry at a 1024-frame batch: one workgroup walks each frame, windows carried."""
    import torch
    from pypanadapter_amd import ZoomFFT
    F, L, N, W = 1024, 262144 + 3, 1024, 256
    picks = (0, 700, F - 1)
    dev = torch.device("cuda:0")
    x = torch.zeros((F, L, 2), device=dev, dtype=torch.float32)
    xs = {f: _frames(1, L, N, 4, W, seed0=8300 + f)[0] for f in picks}
    for f, v in xs.items():
        x[f] = torch.from_numpy(np.ascontiguousarray(v).view(np.float32).reshape(L, 2)).to(dev)
    rows = torch.empty((F, W), device=dev, dtype=torch.float32)
    with ZoomFFT(N, 4, 2.4e6, n_win=W) as plan:
        plan.set_path(6)
        plan.set_timing(True)
        st = torch.cuda.current_stream()
        plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        names = plan.launch_names()
    assert names[0] == "fc_decim", names
    got = rows.cpu().numpy()
    for f in picks:
        assert_row_close(got[f], oracle_lib.psd_row(xs[f], 2.4e6, N, 4, W), f"frame {f}")
