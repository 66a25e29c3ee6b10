"""Host-side engine: one `ZoomFFT` plan per (N, zoom, W, window, fs, f_lo, scroll).

Mirrors the reference's per-frame DSP (pypanadapter_spectrum.py:2088-2119) and its
waterfall model (S:1625-1664) behind libzfft.so.  Host numpy buffers go through the
synchronous C-ABI calls; device tensors (torch, on the plan's device) go through
`process_device`, which enqueues on a caller-supplied HIP stream and does not sync.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, zfft_config


def _window_spec(window):
    """AppState.fft_tapering value -> (kind, params, array_or_None).

    Accepts what the reference stores (S:1358-1363): a scipy window name, a
    (name, p0[, p1]) tuple, or an explicit array (any other scipy window).  Absent
    parameters are NaN: the native generator applies scipy's default or refuses the window
    as get_window does.
    """
    if isinstance(window, np.ndarray) or (isinstance(window, (list,)) and window and
                                          not isinstance(window[0], str)):
        return _lib.WIN_ARRAY, (0.0, 0.0), np.ascontiguousarray(window, dtype=np.float32)
    name, params = (window, ()) if isinstance(window, str) else (window[0], tuple(window[1:]))
    name = _lib.WINDOW_ALIASES.get(name.lower(), name.lower())
    if name not in _lib.WINDOW_KINDS:
        raise ValueError(f"window {window!r} has no native generator; pass it as an array "
                         "(e.g. scipy.signal.get_window(window, n_fft))")
    if len(params) > 2:
        raise ValueError(f"window {window!r}: at most two parameters")
    p = [float(v) for v in params] + [float("nan")] * 2
    return _lib.WINDOW_KINDS[name], (p[0], p[1]), None


# in_dtype name -> (zfft_config.in_dtype, numpy element type of the host array)
IN_DTYPES = {"complex64": (0, np.complex64), "complex32": (1, np.float16), "cu8": (2, np.uint8),
             "f32": (3, np.float32)}


class ZoomFFT:
    """A plan: IQ frames -> dB rows (+ the on-device waterfall ring)."""

    def __init__(self, n_fft: int, zoom: int, fs: float, n_win: int | None = None,
                 window="hamming", f_lo: float = 1.0, scroll: int = 1, device: int = 0,
                 in_dtype: str = "complex64", flip: bool = False):
        """in_dtype: "complex64" (complex ndarray), "complex32" (float16 interleaved I,Q,
        shape (..., 2L)), "cu8" (RTL-SDR uint8 interleaved I,Q, value b/127.5 - 1) or "f32"
        (real samples, AudioPan; at zoom 1 the rows are one-sided and `row_length` long).
        flip: reverse every frame on load (the sources' np.flip, S:541-543)."""
        self.lib = _lib.load()
        if in_dtype not in IN_DTYPES:
            raise ValueError(f"in_dtype must be one of {sorted(IN_DTYPES)}")
        self.in_dtype, self.flip = in_dtype, bool(flip)
        self.n_fft, self.zoom, self.fs, self.f_lo = int(n_fft), int(zoom), float(fs), float(f_lo)
        self.n_win = int(n_win) if n_win is not None else self.n_fft // self.zoom
        kind, params, arr = _window_spec(window)
        cfg = zfft_config()
        cfg.n_fft, cfg.zoom, cfg.n_win, cfg.window_kind = self.n_fft, self.zoom, self.n_win, kind
        cfg.fs, cfg.f_lo = self.fs, self.f_lo
        cfg.window_param[0], cfg.window_param[1] = params
        cfg.scroll, cfg.device = int(scroll), int(device)
        cfg.in_dtype, cfg.flip_input = IN_DTYPES[in_dtype][0], int(self.flip)
        if arr is not None and arr.size != self.n_fft:
            raise ValueError("array window must have length n_fft (welch nperseg)")
        self._window_array = arr  # kept alive for the call
        self._plan = ctypes.c_void_p()
        check(self.lib.zfft_plan_create(ctypes.byref(cfg),
                                        arr.ctypes.data_as(ctypes.c_void_p) if arr is not None else None,
                                        ctypes.byref(self._plan)), "zfft_plan_create")
        self.scroll = int(scroll)
        self.device = int(device)

    # ---------------------------------------------------------------- lifetime
    def close(self):
        if getattr(self, "_plan", None) and self._plan.value:
            self.lib.zfft_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def tune(self, block: int = 0, warmup: int = 0):
        check(self.lib.zfft_plan_tune(self._plan, int(block), int(warmup)), "zfft_plan_tune")

    def set_timing(self, enable: bool) -> None:
        check(self.lib.zfft_plan_timing(self._plan, int(bool(enable))), "zfft_plan_timing")

    def timings(self) -> list:
        """Per-launch ms of the last process call (needs set_timing(True)), in launch order,
        one per name of `launch_names()`: XA schedule [xa_stage_mix, xa_stage, ..., welch_rows
        | welch4]; blocked schedules a forward and a backward pass per stage; a batched host
        call repeats the sequence per batch after a "batch_wait" interval."""
        buf = (ctypes.c_float * 1024)()
        n = ctypes.c_int32()
        check(self.lib.zfft_plan_timings(self._plan, buf, 1024, ctypes.byref(n)), "zfft_plan_timings")
        return [float(buf[i]) for i in range(n.value)]

    def launch_names(self) -> list:
        """Names of the intervals `timings()` returns (from the last timed call)."""
        raw = self.lib.zfft_plan_timing_names(self._plan) or b""
        return [n for n in raw.decode().split(",") if n]

    def set_path(self, path: int) -> None:
        """0 auto, 1 exact reference pass order (blocked; the auto choice for small batches,
        e.g. one frame per call), 2 fused interior + exact edges (blocked; auto from 2^27
        samples per call), 3 XA tiles (all-pole + FIR + half-rate all-pole, one wave per
        frame; auto for >= 768 frames, or >= 384 frames of <= 2^19 samples), 4 PC polyphase
        cascade tiles (zoom 8, frames >= 16384 samples; the auto choice there below 4096
        frames per call), 5 the PC walk (one workgroup per frame; zoom 8: auto from 4096
        frames; zoom 4: the two-stage walk, on request only -- XA is faster there; path 4 at
        zoom 4 is its tiles, automatic below 1024 frames per call; at zoom 2, 4 and 5 are
        one-stage tiles in XA's factorisation, automatic below 512).  At zoom
        >= 16, 4 / 5 run PC for the first three stages and XA for the rest; automatic wherever
        XA would take the batch."""
        check(self.lib.zfft_plan_path(self._plan, int(path)), "zfft_plan_path")

    def set_welch(self, mode: int) -> None:
        """0 auto, 1 one workgroup per frame (n_fft <= 16384), 2 four-step (n_fft >= 4096)."""
        check(self.lib.zfft_plan_welch(self._plan, int(mode)), "zfft_plan_welch")

    def set_lo_frames(self, f_lo, frames_per_lo: int = 1) -> None:
        """Batched multi-IF (config 4): frame f of each call is mixed with
        f_lo[(f // frames_per_lo) % len(f_lo)] (the reference's f_demod per IF, S:2090);
        an empty list restores the plan's f_lo.  Zoom 1 never mixes (S:2108): several
        rows raise ValueError there."""
        arr = np.ascontiguousarray(f_lo, dtype=np.float64).ravel()
        check(self.lib.zfft_plan_set_lo_frames(self._plan, arr.ctypes.data_as(ctypes.c_void_p) if arr.size else None,
                                               int(arr.size), int(frames_per_lo)), "zfft_plan_set_lo_frames")
        if arr.size == 1:
            self.f_lo = float(arr[0])

    # ---------------------------------------------------------------- DSP
    def _as_iq(self, x) -> np.ndarray:
        """The caller's frames in the plan's input format, C-contiguous; the last axis holds
        L complex samples (complex64) or 2L interleaved I,Q values (complex32, cu8)."""
        x = np.asarray(x)
        dt = IN_DTYPES[self.in_dtype][1]
        if self.in_dtype == "complex64":
            if x.dtype != dt:
                x = x.astype(dt)
        elif self.in_dtype == "f32":
            if np.iscomplexobj(x):
                raise ValueError("f32 input must be real")
            x = x.astype(dt, copy=False)
        elif x.dtype != dt or x.shape[-1] % 2:
            raise ValueError(f"{self.in_dtype} input must be {np.dtype(dt).name} with "
                             "interleaved I,Q on the last axis")
        return np.ascontiguousarray(x)

    def _samples(self, x) -> int:
        return x.shape[-1] if self.in_dtype in ("complex64", "f32") else x.shape[-1] // 2

    @property
    def row_length(self) -> int:
        """Valid floats per row: n_win, or the one-sided slice for real input at zoom 1."""
        n = self.lib.zfft_plan_row_length(self._plan)
        if n < 0:
            check(n, "zfft_plan_row_length")
        return n

    def rows(self, frames) -> np.ndarray:
        """(F, L) or (L,) complex IQ -> (F, W) or (W,) float32 dB rows."""
        x = self._as_iq(frames)
        single = x.ndim == 1
        x2 = x.reshape(1, -1) if single else x
        F, L = x2.shape[0], self._samples(x2)
        out = np.empty((F, self.n_win), dtype=np.float32)
        check(self.lib.zfft_process(self._plan, x2.ctypes.data_as(ctypes.c_void_p), L, F,
                                    out.ctypes.data_as(ctypes.c_void_p)), "zfft_process")
        n = self.row_length
        if n != self.n_win:  # one-sided rows (real input at zoom 1)
            out = np.ascontiguousarray(out[:, :n])
        return out[0] if single else out

    def process_host(self, iq_ptr: int, n_samples: int, n_frames: int, rows_ptr: int) -> None:
        """zfft_process on raw host pointers (e.g. a pinned torch tensor's data_ptr()): frames in
        the plan's input format, rows n_frames * n_win floats.  Synchronous; large inputs go in
        batches whose H2D copy overlaps the previous batch's compute."""
        check(self.lib.zfft_process(self._plan, ctypes.c_void_p(iq_ptr), int(n_samples),
                                    int(n_frames), ctypes.c_void_p(rows_ptr)), "zfft_process")

    def process_device(self, d_iq_ptr: int, n_samples: int, n_frames: int, d_rows_ptr: int,
                       stream: int = 0) -> None:
        """Device pointers (e.g. torch .data_ptr()); enqueued on `stream`, no sync."""
        check(self.lib.zfft_process_device(self._plan, ctypes.c_void_p(d_iq_ptr), int(n_samples),
                                           int(n_frames), ctypes.c_void_p(d_rows_ptr),
                                           ctypes.c_void_p(stream or None)), "zfft_process_device")

    def decimate(self, x) -> np.ndarray:
        """zoomfft(x, zoom) of the reference (S:2088-2100) -> complex64."""
        x = self._as_iq(x).ravel()
        L = self._samples(x)
        m = self.lib.zfft_decimated_length(L, self.zoom)
        out = np.empty(max(m, 1), dtype=np.complex64)
        n_out = ctypes.c_int64()
        check(self.lib.zfft_decimate(self._plan, x.ctypes.data_as(ctypes.c_void_p), L,
                                     out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n_out)),
              "zfft_decimate")
        return out[:n_out.value]

    # ---------------------------------------------------------------- waterfall
    def waterfall_push(self, row=None) -> None:
        if row is None:
            check(self.lib.zfft_waterfall_push(self._plan, None), "zfft_waterfall_push")
            return
        r = np.ascontiguousarray(row, dtype=np.float32)
        if r.size != self.n_win:
            raise ValueError("row length must equal n_win")
        check(self.lib.zfft_waterfall_push(self._plan, r.ctypes.data_as(ctypes.c_void_p)),
              "zfft_waterfall_push")

    def waterfall_push_device(self, d_rows_ptr: int, count: int, stream: int = 0) -> None:
        check(self.lib.zfft_waterfall_push_device(self._plan, ctypes.c_void_p(d_rows_ptr),
                                                  int(count), ctypes.c_void_p(stream or None)),
              "zfft_waterfall_push_device")

    def waterfall_shape(self):
        h, w = ctypes.c_int32(), ctypes.c_int32()
        check(self.lib.zfft_waterfall_shape(self._plan, ctypes.byref(h), ctypes.byref(w)),
              "zfft_waterfall_shape")
        return h.value, w.value

    def waterfall_image(self) -> np.ndarray:
        h, w = self.waterfall_shape()
        img = np.empty((h, w), dtype=np.float32)
        check(self.lib.zfft_waterfall_read(self._plan, img.ctypes.data_as(ctypes.c_void_p)),
              "zfft_waterfall_read")
        return img

    def waterfall_reset(self, scroll: int) -> None:
        """Waterfall.init_image with a (possibly new) scroll direction (S:1625-1636, 2074-2077)."""
        check(self.lib.zfft_waterfall_reset(self._plan, int(scroll)), "zfft_waterfall_reset")
        self.scroll = int(scroll)

    # ---------------------------------------------------------------- rendering (§8f-2)
    def waterfall_colormap(self, name: str) -> None:
        """Waterfall.lookuptable (S:1611-1623): unknown names fall back to 'Default'."""
        check(self.lib.zfft_waterfall_colormap(self._plan, str(name).encode()), "zfft_waterfall_colormap")

    def waterfall_levels(self, low: float | None = None, high: float | None = None):
        """Waterfall.newlevel (S:1680-1684) when given; returns the current (low, high)."""
        if low is not None:
            check(self.lib.zfft_waterfall_levels(self._plan, float(low), float(high)),
                  "zfft_waterfall_levels")
        lo, hi = ctypes.c_double(), ctypes.c_double()
        check(self.lib.zfft_waterfall_get_levels(self._plan, ctypes.byref(lo), ctypes.byref(hi)),
              "zfft_waterfall_get_levels")
        return lo.value, hi.value

    def waterfall_autolevel(self):
        """Waterfall.autolevel (S:1667-1678) as intended: levels = percentiles 2, 98 of the
        pixels below 0, computed on the device; returns (low, high)."""
        lo, hi = ctypes.c_double(), ctypes.c_double()
        check(self.lib.zfft_waterfall_autolevel(self._plan, ctypes.byref(lo), ctypes.byref(hi)),
              "zfft_waterfall_autolevel")
        return lo.value, hi.value

    def waterfall_render(self, out: np.ndarray | None = None) -> np.ndarray:
        """RGBA uint8 (H, W, 4): the pixels pyqtgraph's ImageItem draws for the ring image.

        Without `out` the image lands in one of two page-locked buffers the engine owns and
        uses in turn (the D2H copy then runs at PCIe DMA rate; a pageable array is staged
        through the runtime's bounce buffer at a fraction of it): the returned array stays
        valid until the render after next -- what `setImage` each line needs.  Pass `out`
        (any C-contiguous (H, W, 4) uint8 array; page-locked from `pinned_empty` for speed)
        to keep an image longer."""
        h, w = self.waterfall_shape()
        if out is None:
            slots = getattr(self, "_render_slots", None)
            if not slots or slots[0].shape != (h, w, 4):
                slots = self._render_slots = [pinned_empty((h, w, 4), np.uint8) for _ in range(2)]
                self._render_k = 0
            out = slots[self._render_k % 2]
            self._render_k += 1
        elif out.shape != (h, w, 4) or out.dtype != np.uint8 or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous uint8 array of shape {(h, w, 4)}")
        check(self.lib.zfft_waterfall_render(self._plan, out.ctypes.data_as(ctypes.c_void_p)),
              "zfft_waterfall_render")
        return out

    def waterfall_push_emit(self, rows, f64: bool, out: np.ndarray | None = None) -> np.ndarray:
        """`rows` ((count, n_win) float32 host rows, or None) pushed, then the image in one
        round trip (zfft_waterfall_push_render / _push_read64): RGBA uint8 (H, W, 4), or the
        float64 (H, W) image when `f64`.  Without `out` the image lands in one of two
        page-locked buffers the engine owns and uses in turn, valid until the call after next
        (as waterfall_render); pass `out` to keep one.  (The per-line display path: kept to a
        few attribute reads and two integer pointers on the Python side.)"""
        st = self.__dict__.get("_emit_state")
        if st is None:
            h, w = self.waterfall_shape()  # fixed per plan (n_win / 4 x n_win)
            st = self._emit_state = {
                True: [[pinned_empty((h, w), np.float64) for _ in range(2)], 0, (h, w), np.float64,
                       self.lib.zfft_waterfall_push_read64, "zfft_waterfall_push_read64"],
                False: [[pinned_empty((h, w, 4), np.uint8) for _ in range(2)], 0, (h, w, 4), np.uint8,
                        self.lib.zfft_waterfall_push_render, "zfft_waterfall_push_render"],
                "w": w}
        slot = st[bool(f64)]
        if out is None:
            out = slot[0][slot[1] & 1]
            slot[1] += 1
        elif out.shape != slot[2] or out.dtype != slot[3] or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous {np.dtype(slot[3]).name} array of shape {slot[2]}")
        if rows is None:
            count, ptr = 0, None
        else:
            r = rows if (rows.dtype == np.float32 and rows.flags.c_contiguous) else \
                np.ascontiguousarray(rows, dtype=np.float32)
            count, ptr = r.size // st["w"], r.ctypes.data
        check(slot[4](self._plan, ptr, count, out.ctypes.data), slot[5])
        return out

    def waterfall_render_device(self, d_rgba_ptr: int, stream: int = 0) -> None:
        """RGBA8 pixels of the ring into device memory (H*W*4 bytes), enqueued on `stream`."""
        check(self.lib.zfft_waterfall_render_device(self._plan, ctypes.c_void_p(d_rgba_ptr),
                                                    ctypes.c_void_p(stream or None)),
              "zfft_waterfall_render_device")


_IN_DTYPES = {"complex64": (0, np.complex64, 1), "complex32": (1, np.float16, 2),
              "cu8": (2, np.uint8, 2), "f32": (3, np.float32, 1)}


class IQRing:
    """Host IQ accumulation ring: pypanadapter_thread.py's `Data`
    (T:1400-1483) in pinned host memory, between the reader thread (`add`) and the PSD
    worker (`take` / `process`).  See include/zfft.h zfft_ring_* for the semantics."""

    def __init__(self, chunk_size: int = 8196 * 2, in_dtype: str = "complex64"):
        self.lib = _lib.load()
        if in_dtype not in _IN_DTYPES:
            raise ValueError(f"in_dtype must be one of {sorted(_IN_DTYPES)}")
        self.in_dtype = in_dtype
        code, self._np, self._per = _IN_DTYPES[in_dtype]
        self._ring = ctypes.c_void_p()
        check(self.lib.zfft_ring_create(int(chunk_size), code, ctypes.byref(self._ring)),
              "zfft_ring_create")
        self.chunk_size = int(chunk_size)
        self.max_size = 16 * self.chunk_size

    def close(self):
        if self._ring:
            self.lib.zfft_ring_destroy(self._ring)
            self._ring = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _raw(self, chunk) -> tuple:
        a = np.ascontiguousarray(chunk)
        if self.in_dtype in ("complex64", "f32"):
            a = np.ascontiguousarray(a, dtype=self._np).reshape(-1)
            return a, a.shape[0]
        a = np.ascontiguousarray(a, dtype=self._np).reshape(-1)
        if a.size % 2:
            raise ValueError("interleaved I,Q input needs an even number of values")
        return a, a.size // 2

    def add(self, chunk) -> None:
        """Data.add (T:1433-1457) without the pacing sleep."""
        a, n = self._raw(chunk)
        check(self.lib.zfft_ring_add(self._ring, a.ctypes.data_as(ctypes.c_void_p), n),
              "zfft_ring_add")

    def state(self):
        """(size, real_size, total_size) as Data holds them."""
        v = [ctypes.c_int64() for _ in range(3)]
        check(self.lib.zfft_ring_state(self._ring, *(ctypes.byref(x) for x in v)), "zfft_ring_state")
        return tuple(x.value for x in v)

    def take(self):
        """get_data_start / data[:real_size] / get_data_end (T:1516-1520): the frame (a view
        of the drained buffer, valid until the next take) and total_size."""
        p, n, tot = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.zfft_ring_take(self._ring, ctypes.byref(p), ctypes.byref(n),
                                      ctypes.byref(tot)), "zfft_ring_take")
        count = n.value * self._per
        if count == 0:
            return np.empty(0, dtype=self._np), tot.value
        buf = (ctypes.c_char * (count * np.dtype(self._np).itemsize)).from_address(p.value)
        return np.frombuffer(buf, dtype=self._np, count=count), tot.value

    def process(self, plan: "ZoomFFT"):
        """PSD.update (T:1513-1548): the next row from the drained frame, or None when the
        frame is shorter than fft_size (T:1522-1523)."""
        row = np.empty(plan.n_win, dtype=np.float32)
        produced = ctypes.c_int32()
        check(self.lib.zfft_ring_process(self._ring, plan._plan, row.ctypes.data_as(ctypes.c_void_p),
                                         ctypes.byref(produced)), "zfft_ring_process")
        return row[:plan.row_length] if produced.value else None


class _PinnedBlock:
    """One zfft_host_alloc block; arrays made by `pinned_empty` hold a reference to it."""

    def __init__(self, nbytes: int):
        self._lib = _lib.load()
        p = ctypes.c_void_p()
        check(self._lib.zfft_host_alloc(max(1, int(nbytes)), ctypes.byref(p)), "zfft_host_alloc")
        self.ptr = p.value

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.zfft_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


def pinned_empty(shape, dtype) -> np.ndarray:
    """An uninitialised numpy array in page-locked host memory (zfft_host_alloc), freed when
    the last array viewing it is collected: the fast destination for D2H copies (renders,
    rows) and source for H2D."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    blk = _PinnedBlock(n)
    raw = (ctypes.c_char * max(1, n)).from_address(blk.ptr)
    raw._zfft_owner = blk  # the ctypes array keeps the block alive; the ndarray keeps it
    return np.frombuffer(raw, dtype=dt, count=int(np.prod(shape))).reshape(shape)


def colormap_lut(name: str) -> np.ndarray:
    """The 256 x 4 RGBA lookup table of a Waterfall colormap (host-side, no GPU needed)."""
    lib = _lib.load()
    out = np.empty((256, 4), dtype=np.uint8)
    check(lib.zfft_colormap_lut(str(name).encode(), out.ctypes.data_as(ctypes.c_void_p)),
          "zfft_colormap_lut")
    return out


def native_window(window, length: int) -> np.ndarray:
    """fp64 window from the library's native generator (no scipy needed)."""
    lib = _lib.load()
    kind, params, arr = _window_spec(window)
    if arr is not None:
        raise ValueError("array windows are not generated")
    out = np.empty(length, dtype=np.float64)
    p = (ctypes.c_double * 2)(*params)
    check(lib.zfft_window_values(kind, p, int(length), out.ctypes.data_as(ctypes.c_void_p)),
          "zfft_window_values")
    return out


def device_count() -> int:
    return int(_lib.load().zfft_device_count())
