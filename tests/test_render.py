"""On-device waterfall rendering: colormap LUTs, levels, autolevel, RGBA.

Oracle: oracle/render.py, a numpy restatement of the reference's Waterfall colormap /
levels / autolevel (pypanadapter_spectrum.py:1579-1623, 1667-1685) and of what pyqtgraph
draws from them.  pyqtgraph is absent from this image, so parity with pyqtgraph itself is
unpinned; the device path must equal the restatement bit for bit."""
import ctypes

import numpy as np
import pytest

from oracle import render as rr

NAMES = ["Default", "Matrix", "Red Green", "Tropical", "no such map"]


@pytest.mark.parametrize("name", NAMES)
def test_colormap_lut_matches_restatement(zfft_lib, name):
    out = np.empty((256, 4), dtype=np.uint8)
    assert zfft_lib.zfft_colormap_lut(name.encode(), out.ctypes.data_as(ctypes.c_void_p)) == 0
    np.testing.assert_array_equal(out, rr.lookup_table(name))


def test_restatement_facts():
    """Stops land where Waterfall.Colors puts them; 'Default' carries the numpy<2 wrap."""
    d = rr.lookup_table("Default")
    np.testing.assert_array_equal(d[0], [0, 0, 90, 255])
    np.testing.assert_array_equal(d[255], [255, 0, 0, 255])
    assert 2020 % 256 == 228 and d[102, 1] > 200  # near pos 0.4: the wrapped 228 green
    np.testing.assert_array_equal(rr.lookup_table("no such map"), d)
    img = np.array([[-500.0, 0.0, -220.0, -120.0, -170.0, np.float32(-119.9)]])
    px = rr.render(img, rr.lookup_table("Matrix"), (-220, -120))
    np.testing.assert_array_equal(px[0, :, 1], [0, 255, 0, 255, 128, 255])


def _filled_plan(W=512, scroll=1, seed=0, rows=None):
    from pypanadapter_amd import ZoomFFT
    plan = ZoomFFT(max(1024, W), 2, 2.4e6, n_win=W, scroll=scroll)
    rng = np.random.default_rng(seed)
    H = W // 4
    for _ in range(rows if rows is not None else H // 2):
        r = (-170 + 40 * rng.standard_normal(W)).astype(np.float32)
        r[0] = r[W // 2] = r[W - 1] = 0
        plan.waterfall_push(r)
    return plan


@pytest.mark.gpu
@pytest.mark.parametrize("name,levels", [("Default", None), ("Tropical", (-200.0, -140.0)),
                                         ("Red Green", (-150.0, -150.0)), ("Matrix", (-260.5, -90.25))])
def test_render_matches_restatement(name, levels):
    plan = _filled_plan(seed=len(name))
    try:
        plan.waterfall_colormap(name)
        if levels is not None:
            plan.waterfall_levels(*levels)
        lv = plan.waterfall_levels()
        assert lv == (levels if levels is not None else (-220.0, -120.0))
        px = plan.waterfall_render()
        img = plan.waterfall_image().astype(np.float64)
        np.testing.assert_array_equal(px, rr.render(img, rr.lookup_table(name), lv))
    finally:
        plan.close()


@pytest.mark.gpu
@pytest.mark.parametrize("W,rows,scroll", [(512, 64, 1), (512, 200, -1), (64, 3, 1), (2048, 40, 1)])
def test_autolevel_matches_numpy_percentile(W, rows, scroll):
    plan = _filled_plan(W=W, scroll=scroll, seed=W + rows, rows=rows)
    try:
        got = plan.waterfall_autolevel()
        img = plan.waterfall_image().astype(np.float64)
        assert got == rr.autolevel(img)  # bit-exact: same order statistics, numpy's lerp
        assert plan.waterfall_levels() == got
        np.testing.assert_array_equal(plan.waterfall_render(),
                                      rr.render(img, rr.lookup_table("Default"), got))
    finally:
        plan.close()


@pytest.mark.gpu
def test_waterfall_facade_rendering():
    """Waterfall.lookuptable / newlevel / autolevel / render on the facade, through a width
    change (init_image) that keeps the chosen map and levels."""
    from pypanadapter_amd import Waterfall
    wf = Waterfall(scroll=1)
    wf.lookuptable("Tropical")
    wf.newlevel(-210.0, -130.0)
    rng = np.random.default_rng(5)
    for W in (256, 512):
        for _ in range(20):
            wf.image_update((-170 + 30 * rng.standard_normal(W)).astype(np.float32))
        assert wf.levels == (-210.0, -130.0)
        img = wf.img_array
        np.testing.assert_array_equal(wf.render(), rr.render(img, rr.lookup_table("Tropical"),
                                                             (-210.0, -130.0)))
    lv = wf.autolevel()
    assert lv == rr.autolevel(wf.img_array)
    np.testing.assert_array_equal(wf.render(), rr.render(wf.img_array, rr.lookup_table("Tropical"), lv))
    wf.lookuptable("nope")
    np.testing.assert_array_equal(wf.render(), rr.render(wf.img_array, rr.lookup_table("Default"), lv))


@pytest.mark.gpu
@pytest.mark.parametrize("side_stream", [False, True])
def test_render_device_matches_host_render(side_stream):
    """zfft_waterfall_render_device (into a device buffer, on a caller stream) gives the
    same pixels as the host-buffer render; the plan's scroll survives a reset."""
    import torch
    plan = _filled_plan(W=256, seed=11, rows=50)
    try:
        plan.waterfall_colormap("Tropical")
        want = plan.waterfall_render()
        d = torch.zeros(want.size, dtype=torch.uint8, device="cuda")
        st = torch.cuda.Stream() if side_stream else torch.cuda.current_stream()
        with torch.cuda.stream(st):
            plan.waterfall_render_device(d.data_ptr(), st.cuda_stream)
        st.synchronize()
        np.testing.assert_array_equal(d.cpu().numpy().reshape(want.shape), want)
        plan.waterfall_reset(-1)
        assert plan.scroll == -1
        plan.waterfall_push((-170 + np.zeros(256)).astype(np.float32))
        img = plan.waterfall_image()
        assert img.shape == (64, 256) and np.all(img[:-1] <= 0)
    finally:
        plan.close()


@pytest.mark.gpu
def test_render_into_page_locked_buffers():
    """render() without `out` lands in two engine-owned page-locked buffers used in turn (VERDICT
    r04 item 7): consecutive images are distinct arrays, the earlier one intact after the later
    render; `out` takes a caller's array, page-locked (pinned_empty) or pageable."""
    from pypanadapter_amd import pinned_empty
    plan = _filled_plan(W=2048, seed=11)
    try:
        want = rr.render(plan.waterfall_image().astype(np.float64), rr.lookup_table("Default"),
                         plan.waterfall_levels())
        a = plan.waterfall_render()
        b = plan.waterfall_render()
        assert a.ctypes.data != b.ctypes.data
        np.testing.assert_array_equal(a, want)
        np.testing.assert_array_equal(b, want)
        c = plan.waterfall_render()
        assert c.ctypes.data == a.ctypes.data  # the third render reuses the first buffer
        mine = pinned_empty(want.shape, np.uint8)
        assert plan.waterfall_render(out=mine) is mine
        np.testing.assert_array_equal(mine, want)
        pageable = np.zeros_like(want)
        plan.waterfall_render(out=pageable)
        np.testing.assert_array_equal(pageable, want)
        with pytest.raises(ValueError):
            plan.waterfall_render(out=np.zeros((3, 3, 4), np.uint8))
    finally:
        plan.close()
