"""GPU parity of the PC decimator (path 4: polyphase cascade, zoom 8; pc_kernels.hip) against
the float64 oracle of the reference's decimate(x, 2) x 3 (pypanadapter_spectrum.py:2096-2098)
and its rows, and against the golden rows recorded from the reference.

Decimated IQ: relative to the output peak, PC's fp32 error is 2-6e-6 (the bounds below are
the measured worst + ~20 %, from the tolerance ledger).  Rows: the §8(c) gate."""
import numpy as np
import pytest

from conftest import assert_row_close, case_input, check_rel, golden_cases, golden_rows

pytestmark = pytest.mark.gpu
# Bounds = the largest error measured over every check below on the shipped kernels (the
# tolerance ledger, profiles/r06h/tol_ledger.json; tests/conftest.py check_rel) + ~20 %:
#   PC_TOL    zoom 8 / 4 / 2 decimated IQ vs the float64 oracle, and PC vs XA: worst 5.35e-6
#             (zoom 8, tiles); the walk on the zf_n512_z8 fixture 6.07e-6 (test_gpu_parity)
#   HEAD_TOL  zoom >= 16 (PC's x8, then zoom 2's tiles or the blocked passes): worst 6.02e-6
#   CMP_TOL   PC against the exact blocked passes (two fp32 paths, errors add): worst 7.10e-6
# DESIGN §3.5 has where PC's 5-6e-6 comes from (the FIR taps summed in order).
PC_TOL = 6.5e-6
HEAD_TOL = 7.5e-6
CMP_TOL = 8.6e-6
# 4: K1 + K2 tiles (y2 through device memory), 5: KW (one workgroup walks each frame)
PC_PATHS = pytest.mark.parametrize("path", [4, 5], ids=["tiles", "walk"])


@pytest.fixture(scope="module", autouse=True)
def _gpu(zfft_lib):
    from pypanadapter_amd import device_count
    assert device_count() >= 1, "GPU tests need a HIP device"


def _frames(F, L, N, z, W, seed0, f_lo=1.0):
    from pypanadapter_amd import synth
    return np.stack([synth.make_iq(L, 2.4e6, seed0 + f, n_fft=N, zoom=z, n_win=W, f_lo=f_lo)
                     for f in range(F)])


# every L mod 8 (the frame-end map depends on it), the shortest frame PC takes, the K1 / K2
# tile geometry (992 y2 outputs, 2048 outputs) straddled, BASELINE's cfg2/cfg5 lengths
PC_LENGTHS = [16384, 16385, 16386, 16387, 16388, 16389, 16390, 16391, 3968 * 5 + 1,
              16384 * 2 - 3, 299008, 299008 + 5, 1048576 + 7]


@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
@PC_PATHS
def test_pc_decimate_vs_oracle(oracle_lib, flip, path):
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(4400 + flip)
    for L in PC_LENGTHS:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        x += np.exp(2j * np.pi * 0.0071 * np.arange(L)).astype(np.complex64)
        with ZoomFFT(4096, 8, 2.4e6, flip=flip) as plan:
            plan.set_path(path)
            d = plan.decimate(x)
        ref = oracle_lib.zoomfft(x[::-1].copy() if flip else x, 8, 2.4e6)
        assert d.shape == ref.shape, (L, d.shape, ref.shape)
        check_rel(d, ref, PC_TOL, f"pc8/decimate/path{path}", (L, flip))


@pytest.mark.parametrize("N,L,F", [(4096, 299008, 6), (16384, 294912, 3), (65536, 1048576, 2),
                                    (1024, 65536, 4), (32768, 524288 + 3, 2)])
@PC_PATHS
def test_pc_rows_vs_oracle(oracle_lib, N, L, F, path):
    from pypanadapter_amd import ZoomFFT
    W = N // 8
    x = _frames(F, L, N, 8, W, seed0=5100 + N // 1024)
    with ZoomFFT(N, 8, 2.4e6, n_win=W) as plan:
        plan.set_path(path)
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, 8, W), f"N={N} L={L} frame {f}")


@PC_PATHS
def test_pc_golden_rows(path):
    """Every zoom-8 golden row the reference recorded whose frame PC takes (>= 16384)."""
    from pypanadapter_amd import ZoomFFT
    from conftest import window_of
    n = 0
    for c in golden_cases()["cases"]:
        if c["zoom"] != 8 or c["n_samples"] < 16384:
            continue
        x = case_input(c)
        with ZoomFFT(c["n_fft"], 8, c["fs"], n_win=c["n_win"], window=window_of(c["window"]),
                     f_lo=c["f_lo"]) as plan:
            plan.set_path(path)
            row = plan.rows(x)
        assert_row_close(row, golden_rows()[c["name"]], c["name"])
        n += 1
    assert n >= 3


def _encode(x, fmt):
    if fmt == "complex32":
        h = np.ascontiguousarray(x).view(np.float32).astype(np.float16)
        v = h.astype(np.float64)
        return h, v[..., 0::2] + 1j * v[..., 1::2]
    if fmt == "cu8":
        iq = np.ascontiguousarray(x).view(np.float32).astype(np.float64)
        b = np.clip(np.rint(127.5 + 127.5 * 0.25 * iq), 0, 255).astype(np.uint8)
        v = b.astype(np.float64) / 127.5 - 1.0
        return b, v[..., 0::2] + 1j * v[..., 1::2]
    r = np.ascontiguousarray(x.real).astype(np.float32)
    return r, r.astype(np.complex128)


@pytest.mark.parametrize("fmt", ["complex32", "cu8", "f32"])
@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
@PC_PATHS
def test_pc_input_formats(oracle_lib, fmt, flip, path):
    """The raw-source formats (complex32 / RTL-SDR u8 / AudioPan real f32) and np.flip fused
    into the K1 loads and the frame-end maps' loads."""
    from pypanadapter_amd import ZoomFFT
    F, L, N = 3, 299008 + 3, 4096
    x = _frames(F, L, N, 8, 512, seed0=6100)
    arr, vals = _encode(x, fmt)
    ref_in = vals[:, ::-1] if flip else vals
    with ZoomFFT(N, 8, 2.4e6, n_win=512, in_dtype=fmt, flip=flip) as plan:
        plan.set_path(path)
        rows = plan.rows(arr)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(ref_in[f], 2.4e6, N, 8, 512),
                         f"{fmt} flip={flip} frame {f}")


@PC_PATHS
def test_pc_lo_per_frame(oracle_lib, path):
    """Config 4 on one plan: frame f mixed with f_lo[f % 3] in K1 and the edge maps."""
    from pypanadapter_amd import ZoomFFT
    f_lo = [1.0, 150e3 + 1.0, -300e3 + 1.0]
    L, F = 299008, 6
    x = np.stack([_frames(1, L, 4096, 8, 512, seed0=6500 + f, f_lo=f_lo[f % 3])[0] for f in range(F)])
    with ZoomFFT(4096, 8, 2.4e6, n_win=512) as plan:
        plan.set_path(path)
        plan.set_lo_frames(f_lo, 1)
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, 4096, 8, 512, f_lo=f_lo[f % 3]),
                         f"frame {f}")


def test_pc_matches_xa_and_exact_rows(oracle_lib):
    """Schedules agree on a batch: PC, XA and the exact blocked passes all within the gate of
    the oracle, and PC's decimated IQ close to the exact path's."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(4, 299008, 4096, 8, 512, seed0=6900)
    out = {}
    for path in (1, 3, 4, 5):
        with ZoomFFT(4096, 8, 2.4e6) as plan:
            plan.set_path(path)
            out[path] = (plan.rows(x), plan.decimate(x[1]))
    for p in (4, 5):
        check_rel(out[p][1], out[1][1], CMP_TOL, f"pc8/vs_exact_path/path{p}")
    for f in range(4):
        ref = oracle_lib.psd_row(x[f], 2.4e6, 4096, 8, 512)
        for path in (1, 3, 4, 5):
            assert_row_close(out[path][0][f], ref, f"path {path} frame {f}")


@PC_PATHS
def test_pc_refuses_outside_its_domain(path):
    """PC needs frames of >= 16384 samples at every zoom it covers (2 and up)."""
    from pypanadapter_amd import ZoomFFT
    with ZoomFFT(1024, 8, 2.4e6) as plan:
        plan.set_path(path)
        with pytest.raises(NotImplementedError):
            plan.rows(np.zeros(16383, np.complex64))


@PC_PATHS
def test_pc_size_independent_properties(path):
    """Determinism, frame-order equivariance and exact x2 scaling (+12.04 dB) at a batch."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(12, 299008, 4096, 8, 512, seed0=7300)
    with ZoomFFT(4096, 8, 2.4e6) as plan:
        plan.set_path(path)
        a = plan.rows(x)
        b = plan.rows(x)
        perm = np.random.default_rng(1).permutation(12)
        c = plan.rows(x[perm])
        d = plan.rows(2 * x)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(c, a[perm])
    np.testing.assert_allclose(d - a, 20 * np.log10(4.0), atol=2e-4)


@PC_PATHS
def test_pc_ragged_lengths_on_a_caller_stream(oracle_lib, zfft_lib, path):
    """L mod 8 = 0..7 in turn through zfft_process_device on a caller stream.  Every frame-end
    map is resident from the plan's first PC call (pc_edge_maps.h), so after a first call at
    the longest length none of these calls waits on the host, and every
    row passes the oracle gate."""
    import ctypes
    import torch
    from pypanadapter_amd import ZoomFFT
    count = zfft_lib.zfft__plan_quiesce_count
    count.argtypes, count.restype = [ctypes.c_void_p], ctypes.c_int64
    Ls = [20000 + k for k in (3, 0, 7, 1, 6, 2, 5, 4)]  # every L mod 8, shuffled
    F, N, W = 2, 1024, 128
    dev = torch.device("cuda:0")
    xs = {L: _frames(F, L, N, 8, W, seed0=7700 + L) for L in Ls}
    d_in = {L: torch.from_numpy(np.ascontiguousarray(x).view(np.float32)).to(dev) for L, x in xs.items()}
    rows = {L: torch.empty((F, W), dtype=torch.float32, device=dev) for L in Ls}
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    with ZoomFFT(N, 8, 2.4e6, n_win=W) as plan:
        plan.set_path(path)
        Lmax = max(Ls)
        plan.process_device(d_in[Lmax].data_ptr(), Lmax, F, rows[Lmax].data_ptr(), st.cuda_stream)
        st.synchronize()
        q0 = count(plan._plan)
        for L in Ls:
            plan.process_device(d_in[L].data_ptr(), L, F, rows[L].data_ptr(), st.cuda_stream)
        q1 = count(plan._plan)
        st.synchronize()
    assert q0 >= 0 and q1 == q0, (q0, q1)
    for L in Ls:
        got = rows[L].cpu().numpy()
        for f in range(F):
            assert_row_close(got[f], oracle_lib.psd_row(xs[L][f], 2.4e6, N, 8, W), f"L={L} frame {f}")


# ---- zoom >= 16: PC for the first three stages, XA for the rest (run_pc_head) ----

@pytest.mark.parametrize("zoom", [16, 32])
@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
@PC_PATHS
def test_pc_head_decimate_vs_oracle(oracle_lib, zoom, flip, path):
    """decimate(x, 2) x log2(zoom) as PC's exact x8 (frame-end maps at every L mod 8) followed,
    for one frame per call, by zoom 2's tiles while a stage's input has >= 16384 samples and
    the exact blocked passes after that (both on a unit LO table), against the float64 oracle;
    1e-5 per tail stage on top."""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(4600 + zoom + flip)
    for L in [16384, 16387, 16390, 3968 * 5 + 1, 262144 + 5, 299008]:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        x += np.exp(2j * np.pi * 0.0023 * np.arange(L)).astype(np.complex64)
        with ZoomFFT(4096, zoom, 2.4e6, flip=flip) as plan:
            plan.set_path(path)
            plan.set_timing(True)
            d = plan.decimate(x)
            names = plan.launch_names()
        # one frame: zoom 2's tiles for the tail stages whose input has >= 16384 samples,
        # then the blocked passes
        n = [L]
        while len(n) <= {16: 4, 32: 5}[zoom]:
            n.append((n[-1] + 1) // 2)
        tiles = next((k - 3 for k in range(3, len(n) - 1) if n[k] < 16384), len(n) - 4)
        assert names.count("exact_backward") == len(n) - 4 - tiles, (L, names)
        assert names.count("pc_tail") == tiles + (path == 4), (L, names)
        ref = oracle_lib.zoomfft(x[::-1].copy() if flip else x, zoom, 2.4e6)
        assert d.shape == ref.shape, (L, d.shape, ref.shape)
        check_rel(d, ref, HEAD_TOL, f"head/zoom{zoom}/path{path}", (L, flip))


@PC_PATHS
def test_pc_head_golden_rows(path):
    """Every golden row the reference recorded at zoom >= 16 whose frame PC takes."""
    from pypanadapter_amd import ZoomFFT
    from conftest import window_of
    n = 0
    for c in golden_cases()["cases"]:
        if c["zoom"] < 16 or c["n_samples"] < 16384:
            continue
        x = case_input(c)
        with ZoomFFT(c["n_fft"], c["zoom"], c["fs"], n_win=c["n_win"], window=window_of(c["window"]),
                     f_lo=c["f_lo"]) as plan:
            plan.set_path(path)
            row = plan.rows(x)
        assert_row_close(row, golden_rows()[c["name"]], c["name"])
        n += 1
    assert n >= 3


def test_pc_head_auto_batch_rows(oracle_lib):
    """At a batch XA would take (384 frames), zoom 16 runs the head (FC from 16 frames per call)
    + one XA stage on its own (the XA tail); rows of three frames against the oracle."""
    from pypanadapter_amd import ZoomFFT
    F, L, N = 384, 65536 + 3, 2048
    x = np.zeros((F, L), np.complex64)
    for f in (0, 191, F - 1):
        x[f] = _frames(1, L, N, 16, 128, seed0=7900 + f)[0]
    with ZoomFFT(N, 16, 2.4e6, n_win=128) as plan:
        plan.set_timing(True)
        rows = plan.rows(x)
        names = plan.launch_names()
    assert names[0] == "fc_decim" and "xa_stage" in names and "pc_edge" in names, names
    for f in (0, 191, F - 1):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, 16, 128), f"frame {f}")


# ---- zoom 2: the tail kernel on the mixed input (pc_tail_kernel<2>; paths 4 / 5) ----

PC2_LENGTHS = [16384, 16385, 2048 * 9 + 3, 4096 * 4 + 17, 262144, 262144 + 1, 299008 + 3]


@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
def test_pc2_decimate_vs_oracle(oracle_lib, flip):
    """Zoom 2 -- the UI's default fft_ratio (S:1497), one decimate(x, 2) (S:2096-2098) -- at
    both L mod 2 and across the tile geometry (2048 outputs from a 5376-sample span), against
    the float64 oracle."""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(4900 + flip)
    for L in PC2_LENGTHS:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        x += np.exp(2j * np.pi * 0.031 * np.arange(L)).astype(np.complex64)
        with ZoomFFT(2048, 2, 2.4e6, flip=flip) as plan:
            plan.set_path(4)
            plan.set_timing(True)
            d = plan.decimate(x)
            names = plan.launch_names()
        assert names[-1] == "pc_edge", names
        ref = oracle_lib.zoomfft(x[::-1].copy() if flip else x, 2, 2.4e6)
        assert d.shape == ref.shape, (L, d.shape, ref.shape)
        check_rel(d, ref, PC_TOL, "pc2/decimate", (L, flip))


@pytest.mark.parametrize("N,L,F", [(2048, 262144, 4), (4096, 299008, 3), (1024, 65536 + 1, 5)])
def test_pc2_rows_vs_oracle(oracle_lib, N, L, F):
    from pypanadapter_amd import ZoomFFT
    W = N // 2
    x = _frames(F, L, N, 2, W, seed0=8700 + N // 1024)
    with ZoomFFT(N, 2, 2.4e6, n_win=W) as plan:
        plan.set_path(5)  # (the same tiles as path 4: zoom 2 has no walk)
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, 2, W), f"N={N} L={L} frame {f}")


def test_pc2_golden_rows():
    """Every zoom-2 golden row the reference recorded whose frame PC takes (>= 16384)."""
    from pypanadapter_amd import ZoomFFT
    from conftest import window_of
    n = 0
    for c in golden_cases()["cases"]:
        if c["zoom"] != 2 or c["n_samples"] < 16384:
            continue
        x = case_input(c)
        with ZoomFFT(c["n_fft"], 2, c["fs"], n_win=c["n_win"], window=window_of(c["window"]),
                     f_lo=c["f_lo"]) as plan:
            plan.set_path(4)
            row = plan.rows(x)
        assert_row_close(row, golden_rows()[c["name"]], c["name"])
        n += 1
    assert n >= 1


@pytest.mark.parametrize("fmt", ["complex32", "cu8", "f32"])
def test_pc2_input_formats_and_lo(oracle_lib, fmt):
    """Raw-source formats, np.flip and per-frame LOs read straight into zoom 2's tail kernel."""
    from pypanadapter_amd import ZoomFFT
    F, L, N = 3, 131072 + 1, 2048
    f_lo = [1.0, 150e3 + 1.0, -300e3 + 1.0]
    x = np.stack([_frames(1, L, N, 2, 1024, seed0=8900 + f, f_lo=f_lo[f])[0] for f in range(F)])
    arr, vals = _encode(x, fmt)
    with ZoomFFT(N, 2, 2.4e6, n_win=1024, in_dtype=fmt, flip=True) as plan:
        plan.set_path(4)
        plan.set_lo_frames(f_lo, 1)
        rows = plan.rows(arr)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(vals[f, ::-1], 2.4e6, N, 2, 1024, f_lo=f_lo[f]),
                         f"{fmt} frame {f}")


def test_pc2_size_independent_properties():
    """Determinism, frame-order equivariance, exact x2 scaling, and the tiles against the XA
    schedule on the same batch."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(8, 262144, 2048, 2, 1024, seed0=9100)
    with ZoomFFT(2048, 2, 2.4e6) as plan:
        plan.set_path(4)
        plan.set_timing(True)
        a = plan.rows(x)
        assert plan.launch_names()[:2] == ["pc_tail", "pc_edge"], plan.launch_names()
        b = plan.rows(x)
        perm = np.random.default_rng(3).permutation(8)
        c = plan.rows(x[perm])
        d = plan.rows(2 * x)
        da = plan.decimate(x[5])
        plan.set_path(3)
        xa = plan.rows(x)
        dx = plan.decimate(x[5])
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(c, a[perm])
    np.testing.assert_allclose(d - a, 20 * np.log10(4.0), atol=2e-4)
    check_rel(da, dx, PC_TOL, "pc2/vs_xa")
    np.testing.assert_allclose(xa, a, atol=2e-3)


# ---- zoom 4: the tiles (path 4; automatic below XA's batch) and the walk (path 5) ----

PC4_LENGTHS = [16384, 16385, 16386, 16387, 2048 * 9 + 3, 262144, 262144 + 2, 299008 + 1]


@pytest.mark.parametrize("flip", [False, True], ids=["noflip", "flip"])
@PC_PATHS
def test_pc4_decimate_vs_oracle(oracle_lib, flip, path):
    """Zoom 4's two-stage cascade (cfg1's decimator, S:2096-2098 at fft_ratio 4) at every
    L mod 4, against the float64 oracle of decimate(x, 2) twice."""
    from pypanadapter_amd import ZoomFFT
    rng = np.random.default_rng(4800 + flip)
    for L in PC4_LENGTHS:
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64)
        x += np.exp(2j * np.pi * 0.013 * np.arange(L)).astype(np.complex64)
        with ZoomFFT(1024, 4, 2.4e6, flip=flip) as plan:
            plan.set_path(path)
            d = plan.decimate(x)
        ref = oracle_lib.zoomfft(x[::-1].copy() if flip else x, 4, 2.4e6)
        assert d.shape == ref.shape, (L, d.shape, ref.shape)
        check_rel(d, ref, PC_TOL, f"pc4/decimate/path{path}", (L, flip))


@pytest.mark.parametrize("N,L,F", [(1024, 262144, 5), (4096, 299008, 3), (2048, 131072 + 3, 4)])
@PC_PATHS
def test_pc4_rows_vs_oracle(oracle_lib, N, L, F, path):
    from pypanadapter_amd import ZoomFFT
    W = N // 4
    x = _frames(F, L, N, 4, W, seed0=8100 + N // 1024)
    with ZoomFFT(N, 4, 2.4e6, n_win=W) as plan:
        plan.set_path(path)
        rows = plan.rows(x)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(x[f], 2.4e6, N, 4, W), f"N={N} L={L} frame {f}")


@PC_PATHS
def test_pc4_golden_rows(path):
    """Every zoom-4 golden row the reference recorded whose frame PC takes (tiles and walk)."""
    from pypanadapter_amd import ZoomFFT
    from conftest import window_of
    n = 0
    for c in golden_cases()["cases"]:
        if c["zoom"] != 4 or c["n_samples"] < 16384:
            continue
        x = case_input(c)
        with ZoomFFT(c["n_fft"], 4, c["fs"], n_win=c["n_win"], window=window_of(c["window"]),
                     f_lo=c["f_lo"]) as plan:
            plan.set_path(path)
            row = plan.rows(x)
        assert_row_close(row, golden_rows()[c["name"]], c["name"])
        n += 1
    assert n >= 1


@pytest.mark.parametrize("fmt", ["complex32", "cu8", "f32"])
@PC_PATHS
def test_pc4_input_formats_and_lo(oracle_lib, fmt, path):
    """Raw-source formats, np.flip and per-frame LOs through zoom 4's tiles and walk."""
    from pypanadapter_amd import ZoomFFT
    F, L, N = 3, 262144 + 1, 1024
    f_lo = [1.0, 150e3 + 1.0, -300e3 + 1.0]
    x = np.stack([_frames(1, L, N, 4, 256, seed0=8300 + f, f_lo=f_lo[f])[0] for f in range(F)])
    arr, vals = _encode(x, fmt)
    with ZoomFFT(N, 4, 2.4e6, n_win=256, in_dtype=fmt, flip=True) as plan:
        plan.set_path(path)
        plan.set_lo_frames(f_lo, 1)
        rows = plan.rows(arr)
    for f in range(F):
        assert_row_close(rows[f], oracle_lib.psd_row(vals[f, ::-1], 2.4e6, N, 4, 256, f_lo=f_lo[f]),
                         f"{fmt} frame {f}")


@PC_PATHS
def test_pc4_size_independent_properties(path):
    """Determinism, frame-order equivariance, exact x2 scaling, and PC against the XA schedule
    on the same batch."""
    from pypanadapter_amd import ZoomFFT
    x = _frames(8, 262144, 1024, 4, 256, seed0=8500)
    with ZoomFFT(1024, 4, 2.4e6) as plan:
        plan.set_path(path)
        a = plan.rows(x)
        b = plan.rows(x)
        perm = np.random.default_rng(2).permutation(8)
        c = plan.rows(x[perm])
        d = plan.rows(2 * x)
        da = plan.decimate(x[3])
        plan.set_path(3)
        xa = plan.rows(x)
        dx = plan.decimate(x[3])
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(c, a[perm])
    np.testing.assert_allclose(d - a, 20 * np.log10(4.0), atol=2e-4)
    check_rel(da, dx, PC_TOL, "pc4/vs_xa")
    np.testing.assert_allclose(xa, a, atol=2e-3)
