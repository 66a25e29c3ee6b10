#!/usr/bin/env python3
"""Generate golden fixtures by RUNNING THE REFERENCE in this container.

Container-only test tooling: it needs `/root/reference` (absent on the GPU box)
and exits quietly without it.  It loads the reference scripts unmodified through
`tools/ref_stub.py` and drives:

  * `ApplicationDisplay.update(fake_self, chunk)`  pypanadapter_spectrum.py:2102-2130
    (calls `zoomfft` S:2088-2100, `scipy.signal.welch` S:2111, fftshift/crop S:2114,
    20*log10 S:2117-2119) -> the row handed to `waterfall.image_update`.
  * `PSD.update(fake_self)`                        pypanadapter_thread.py:1513-1549
  * `Waterfall.image_update(psd)`                  pypanadapter_spectrum.py:1638-1664
  * `ApplicationDisplay.zoomfft(fake_self, x, r)`  pypanadapter_spectrum.py:2088-2100
  * `Data` (new_complex / new_real / add / get_data_start / data[:real_size] /
    get_data_end / target)                      pypanadapter_thread.py:1400-1483, 1516-1520

Outputs (all data, no reference source): tests/golden/cases.json (metadata, input
digests), rows.npz (float64 rows), inputs.npz (small stored complex64 inputs),
zoomfft.npz (decimated IQ), waterfall.npz (image snapshots), ring.npz (Data sequences).

Run:  python tools/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from pypanadapter_amd import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
FS = 2.4e6


class Obj:
    def __init__(self, **k):
        self.__dict__.update(k)


def _window_json(w):
    return list(w) if isinstance(w, tuple) else w


# ----------------------------------------------------------------------------- cases
def spectrum_cases():
    """(name, kw) for the single-thread variant S.  L = fft_avg*N as S:1764 reads it."""
    c = []

    def add(name, n_fft, zoom, n_avg, seed, window="hamming", f_lo=1.0, n_win=None,
            store_input=False, tones=((0.31, 1.0), (-0.57, 0.1)), noise=1.0, fs=FS):
        n_win = n_fft // zoom if n_win is None else n_win
        c.append((name, dict(n_fft=n_fft, zoom=zoom, n_avg=n_avg, L=n_fft * n_avg, seed=seed,
                             window=window, f_lo=f_lo, n_win=n_win, store_input=store_input,
                             tones=tones, noise=noise, fs=fs)))

    # BASELINE.json configs
    add("cfg1", 1024, 4, 256, 101)
    add("cfg2", 4096, 8, 73, 201)
    add("cfg2_b", 4096, 8, 73, 202)
    add("cfg3", 16384, 8, 18, 301)
    add("cfg4_lo150k", 4096, 8, 73, 401, f_lo=1.0 + 150e3)
    add("cfg4_lo-450k", 4096, 8, 73, 402, f_lo=1.0 - 450e3)
    add("cfg5", 65536, 8, 16, 501)
    add("n32768_z4", 32768, 4, 8, 502)               # largest N of the UI list (S:1397)
    add("n32768_z64_short", 32768, 64, 8, 503)       # L_d=4096 < N: short-input four-step
    # zoom edge cases
    add("z1_n2048", 2048, 1, 146, 601)
    add("z1_n256_small", 256, 1, 64, 602, store_input=True)
    add("z2_default_ui", 2048, 2, 146, 701)
    add("z16_n4096", 4096, 16, 73, 801)
    add("z512_short", 2048, 512, 146, 901)          # L_d=584 < N: short-input Welch
    add("z64_n16384_short", 16384, 64, 18, 902)      # L_d=4608 < N
    add("z256_short", 2048, 256, 146, 903)
    add("tiny_n32_z2", 32, 2, 2, 904, store_input=True)   # minimal lengths (stage len 64 > 27)
    add("small_n256_z4", 256, 4, 64, 905, store_input=True)
    add("small_n512_z8", 512, 8, 64, 906, store_input=True)
    # stale-W behaviour of S (N_WIN != N/zoom until fft_change, S:1712/1757)
    add("cfg2_stale_w1024", 4096, 8, 73, 907, n_win=1024)
    # windows (taper list S:1222-1243), small frames
    wins = ["hann", "blackmanharris", ("kaiser", 14), "boxcar", ("tukey", 0.3), "flattop",
            "bartlett", ("gaussian", 7), ("general_gaussian", 1.5, 7), "triang", "bohman",
            "parzen", "nuttall", "barthann", "blackman", ("chebwin", 100), ("dpss", 3)]
    for i, w in enumerate(wins):
        nm = w if isinstance(w, str) else "_".join(str(v) for v in w)
        add(f"win_{nm}", 1024, 4, 64, 1001 + i, window=w)
    add("win_kaiser14_short", 2048, 512, 146, 1101, window=("kaiser", 14))
    # known-answer inputs
    add("kat_tone_bin37", 1024, 4, 64, 1201, tones=((37.0 / 128.0, 1.0),), noise=0.0)
    add("kat_noise_z1", 1024, 1, 256, 1202, tones=(), noise=1.0)
    add("kat_noise_z8", 1024, 8, 256, 1203, tones=(), noise=1.0)
    add("fs_2p56M", 2048, 2, 156, 1301, fs=2.56e6)  # fft_avg=int(fs/N/8)=156, S:1546
    return c


def thread_cases():
    """(name, kw) for the threaded variant T: chunk length is `real_size` (T:1516-1527)."""
    c = []

    def add(name, n_fft, zoom, L, seed, window="hamming"):
        c.append((name, dict(n_fft=n_fft, zoom=zoom, L=L, seed=seed, window=window, f_lo=1.0,
                             n_win=2 * int(0.5 * n_fft / zoom), store_input=False,
                             tones=((0.31, 1.0), (-0.57, 0.1)), noise=1.0, fs=FS)))

    add("T_cfg2", 4096, 8, 299008, 201)        # same input as S cfg2: rows must agree
    add("T_odd_len", 1024, 8, 100003, 1401)    # ragged frame length, ceil() at every stage
    add("T_odd_len_z2", 2048, 2, 77777, 1402)   # breaks T's float arange: skipped
    add("T_odd_len_z2b", 2048, 2, 77779, 1405)
    add("T_z1_ragged", 1024, 1, 50001, 1403)
    add("T_len_not_pow2_z4", 4096, 4, 163840 + 5, 1404)
    return c


# ----------------------------------------------------------------------------- drivers
def run_S(S, kw, x):
    AppState = S.AppState
    AppState._panadapter = Obj(SampleRate=kw["fs"], driver=True)
    AppState.fft_size = kw["n_fft"]
    AppState.fft_ratio = kw["zoom"]
    AppState.fft_avg = kw["n_avg"]
    AppState.fft_tapering = kw["window"]
    cap = S_cap = __import__("ref_stub").Capture()
    fake = Obj(N_WIN=kw["n_win"], waterfall=cap, spectrum_plot=S_cap, win=cap)
    fake.zoomfft = lambda xx, r: S.ApplicationDisplay.zoomfft(fake, xx, r)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        S.ApplicationDisplay.update(fake, x)
    rows = [c[1] for c in cap.calls if c[0] == "image_update"]
    assert len(rows) == 1
    return rows[0]


def run_T(T, kw, x):
    AppState = T.AppState
    AppState._panadapter = Obj(SampleRate=kw["fs"], driver=True)
    AppState.fft_size = kw["n_fft"]
    AppState.fft_ratio = kw["zoom"]
    AppState.fft_tapering = kw["window"]
    ref_stub = __import__("ref_stub")
    data = Obj(real_size=len(x), data=x, get_data_start=lambda: None, get_data_end=lambda: None)
    psd = T.PSD.__new__(T.PSD)
    psd.dataclass = data
    psd.lock = ref_stub._Any()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        T.PSD.update(psd)
    return np.asarray(psd.psd)


def premix(x, f_lo, fs):
    """Reference hard-codes f_demod=1 Hz (S:2090).  Feeding x*exp(-2pi i (f_lo-1) n/fs)
    makes the reference's own code compute the zoom-FFT at LO frequency f_lo."""
    if f_lo == 1.0:
        return x
    n = np.arange(len(x))
    return x.astype(np.complex128) * synth.tone(n, -(f_lo - 1.0), fs, 1.0)


def lo_len_ok(kw):
    """S builds t with float arange (S:2091-2093); it can yield L+1 points and then
    x*lo raises.  The build defines the LO on integer n; skip combos that break S."""
    fs, L = kw["fs"], kw["L"]
    t_total = (1 / fs) * kw["n_fft"] * kw.get("n_avg", 0) if "n_avg" in kw else (1 / fs) * L
    return len(np.arange(0, t_total, 1 / fs)) == L


def waterfall_sequences(S):
    """Waterfall.image_update (S:1638-1664) on a __new__ instance (its __init__ needs Qt LUTs)."""
    ref_stub = __import__("ref_stub")
    AppState = S.AppState
    AppState._panadapter = Obj(SampleRate=FS, driver=True)
    AppState.fft_size = 4096
    AppState.fft_ratio = 8
    seqs = {}
    meta = []

    def run(name, widths, scrolls, snap_at, seed, invert_at=()):
        rng = np.random.default_rng(seed)
        wf = S.Waterfall.__new__(S.Waterfall)
        wf.fftwidth = 0
        AppState.scroll = scrolls
        rows, stamped, snaps = [], [], {}
        for k, w in enumerate(widths):
            if k in invert_at:  # ApplicationDisplay.on_invertscroll_clicked, S:2074-2077
                AppState.scroll *= -1
                if wf.fftwidth:
                    S.Waterfall.init_image(wf)
            row = rng.normal(-170.0, 15.0, w).astype(np.float32).astype(np.float64)
            rows.append(row.copy())
            S.Waterfall.image_update(wf, row)
            stamped.append(row.copy())
            if (k + 1) in snap_at:
                snaps[k + 1] = wf.img_array.astype(np.float32)
        for i, r in enumerate(rows):
            seqs[f"{name}/row{i}"] = r.astype(np.float32)
            seqs[f"{name}/stamped{i}"] = stamped[i].astype(np.float32)
        for k, s in snaps.items():
            seqs[f"{name}/img{k}"] = s
        meta.append(dict(name=name, widths=list(widths), scroll=scrolls, snaps=sorted(snaps),
                         invert_at=list(invert_at)))

    run("w64_up", [64] * 40, 1, set(range(1, 41)), 11)
    run("w64_down", [64] * 40, -1, set(range(1, 41)), 12)
    run("w128_up", [128] * 100, 1, {1, 31, 32, 33, 100}, 13)
    run("w512_up", [512] * 150, 1, {150}, 14)
    run("w_change", [64] * 10 + [128] * 10, 1, {10, 11, 20}, 15)
    run("w_invert", [64] * 30, 1, {10, 11, 20, 30}, 16, invert_at=(10, 20))
    run("w40_down", [40] * 12, -1, {12}, 17)   # smallest W valid for scroll=-1
    return seqs, meta


def ring_sequences(T):
    """T's own `Data` ring (T:1400-1483) driven by seeded add / drain / target sequences.

    `Data.add` sleeps `delay_time` (the NewtRap pacing, T:1455-1457): the loaded module's
    `time` is replaced by one whose sleep returns at once (the module namespace, not the
    reference source).  A drain is the PSD worker's T:1516-1520: get_data_start(); size =
    real_size; chunk = data[:size]; get_data_end().  Recorded per step: the op, its input,
    (size, real_size, total_size, target_size) after it, and every drained frame."""
    import contextlib
    import io
    import time
    import types
    T.time = types.SimpleNamespace(sleep=lambda s: None, monotonic=time.monotonic)
    T.AppState.fft_size = 1024  # the target setter's lower bound (T:1477)
    out, meta = {}, []

    def run(name, chunk, real, n_ops, seed, p_add=0.75, p_target=0.08, max_len=3):
        rng = np.random.default_rng(seed)
        d = T.Data(chunk)
        (d.new_real if real else d.new_complex)()
        ops, states, lens, targets = [], [], [], []
        n_drain = 0
        for i in range(n_ops):
            u = rng.random()
            if u < p_target:
                t = float(rng.choice([100.0, 1023.0, 1024.0, 5000.0, 9000.0, 16.0 * chunk,
                                      16.0 * chunk + 1.0, 40000.0]))
                d.target = t
                ops.append(2)
                targets.append(t)
                lens.append(0)
            elif u < p_target + p_add:
                n = int(rng.integers(0, max_len * chunk + 1))
                if real:
                    x = rng.standard_normal(n).astype(np.float32)
                else:
                    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
                out[f"{name}/in{i}"] = x
                if n > d.max_size:
                    with contextlib.suppress(ValueError):  # numpy refuses the slice assignment
                        d.add(x)
                    ops.append(3)
                else:
                    d.add(x)
                    ops.append(0)
                lens.append(n)
                targets.append(0.0)
            else:
                with contextlib.redirect_stdout(io.StringIO()):  # get_data_end prints delay_time
                    d.get_data_start()
                    size = d.real_size
                    frame = np.array(d.data[:size])
                    total = d.total_size
                    d.get_data_end()
                out[f"{name}/frame{i}"] = frame.astype(np.float32 if real else np.complex64)
                out[f"{name}/frame_total{i}"] = np.array([total], np.int64)
                ops.append(1)
                lens.append(size)
                targets.append(0.0)
                n_drain += 1
            states.append([d.size, d.real_size, d.total_size, float(d.target_size)])
        out[f"{name}/ops"] = np.array(ops, np.int8)
        out[f"{name}/lens"] = np.array(lens, np.int64)
        out[f"{name}/targets"] = np.array(targets, np.float64)
        out[f"{name}/states"] = np.array(states, np.float64)
        meta.append(dict(name=name, chunk_size=chunk, real=real, n_ops=n_ops, seed=seed,
                         drains=n_drain, fft_size=1024, max_size=16 * chunk))

    run("c64", 64, False, 300, 1)
    run("c520", 520, False, 160, 2, max_len=1)       # target_size clip: 16*520 = 8320 > 8192
    run("real64", 64, True, 200, 3)                  # new_real (T:1413-1417)
    run("c64_overlong", 64, False, 80, 4, max_len=20)  # chunks past max_size raise
    return out, meta


def main():
    if not os.path.isdir("/root/reference"):
        print("gen_golden: /root/reference absent, nothing to do")
        return 0
    import ref_stub
    S = ref_stub.load("spectrum")
    T = ref_stub.load("thread")
    os.makedirs(OUT, exist_ok=True)
    cases, rows, inputs, zf = [], {}, {}, {}

    for variant, mod, lst, runner in (("S", S, spectrum_cases(), run_S),
                                      ("T", T, thread_cases(), run_T)):
        for name, kw in lst:
            if kw["zoom"] > 1 and not lo_len_ok(kw):
                print("skip (reference arange length bug)", name)
                continue
            x = synth.make_iq(kw["L"], kw["fs"], kw["seed"], n_fft=kw["n_fft"], zoom=kw["zoom"],
                              n_win=kw["n_win"], f_lo=kw["f_lo"], tones=kw["tones"],
                              noise=kw["noise"])
            xin = premix(x, kw["f_lo"], kw["fs"])
            row = runner(mod, kw, xin)
            # zoom>1 rows are float64 (complex128 after the LO mix); at zoom==1 welch runs on
            # the complex64 chunk directly, so the reference row itself is float32.
            assert row.shape == (kw["n_win"],), (name, row.shape)
            ref_dtype = str(row.dtype)
            rows[name] = row.astype(np.float64)
            if kw["store_input"]:
                inputs[name] = x
            meta = dict(name=name, variant=variant, fs=kw["fs"], n_fft=kw["n_fft"],
                        zoom=kw["zoom"], n_win=kw["n_win"], window=_window_json(kw["window"]),
                        n_samples=kw["L"], seed=kw["seed"], f_lo=kw["f_lo"],
                        tones=[list(t) for t in kw["tones"]], noise=kw["noise"],
                        input_sha256=synth.digest(x), stored_input=kw["store_input"],
                        ref_row_dtype=ref_dtype)
            cases.append(meta)
            print(f"{variant} {name:24s} L={kw['L']:8d} N={kw['n_fft']:6d} z={kw['zoom']:4d} "
                  f"W={kw['n_win']:5d} max={row.max():8.2f} min={row.min():8.2f}")

    # zoomfft (a-1 + a-2) outputs, S:2088-2100
    AppState = S.AppState
    for name, n_fft, n_avg, ratio, seed in (("zf_n256_z4", 256, 64, 4, 905),
                                             ("zf_n512_z8", 512, 64, 8, 906),
                                             ("zf_n1024_z2_odd_pad", 1024, 31, 2, 1501)):
        AppState._panadapter = Obj(SampleRate=FS, driver=True)
        AppState.fft_size, AppState.fft_avg = n_fft, n_avg
        x = synth.make_iq(n_fft * n_avg, FS, seed, n_fft=n_fft, zoom=ratio, n_win=n_fft // ratio)
        y = S.ApplicationDisplay.zoomfft(Obj(), x, ratio)
        zf[name + "/x"] = x
        zf[name + "/y"] = y
        zf[name + "/meta"] = np.array([n_fft, n_avg, ratio, seed], dtype=np.int64)

    wf, wf_meta = waterfall_sequences(S)
    ring, ring_meta = ring_sequences(T)

    np.savez_compressed(os.path.join(OUT, "rows.npz"), **rows)
    np.savez_compressed(os.path.join(OUT, "inputs.npz"), **inputs)
    np.savez_compressed(os.path.join(OUT, "zoomfft.npz"), **zf)
    np.savez_compressed(os.path.join(OUT, "waterfall.npz"), **wf)
    np.savez_compressed(os.path.join(OUT, "ring.npz"), **ring)
    with open(os.path.join(OUT, "cases.json"), "w") as fh:
        json.dump(dict(generator="tools/gen_golden.py",
                       reference="alfille/pypanadapter @ /root/reference (S, T variants)",
                       numpy=np.__version__, scipy=__import__("scipy").__version__,
                       cases=cases, waterfall=wf_meta, ring=ring_meta), fh, indent=1)
    print("wrote", len(cases), "row cases,", len(wf_meta), "waterfall sequences")
    return 0


if __name__ == "__main__":
    sys.exit(main())
