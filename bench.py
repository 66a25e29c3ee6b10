#!/usr/bin/env python3
"""Benchmark of the IQ -> log-PSD -> waterfall-line hot path (BASELINE.json metric).

One step = one pass of the hot path over one batch of F synthetic IQ frames resident in
HBM: LO mix + log2(zoom) x decimate(x, 2) + Welch PSD + fftshift/crop + 20*log10 (the
reference's ApplicationDisplay.update, pypanadapter_spectrum.py:2102-2119) and the
waterfall row-roll of all F lines (Waterfall.image_update, S:1638-1664).

Workload (BASELINE.json configs[1]): 2.4 MS/s synthetic IQ, N_FFT=4096, zoom=8, fp32,
W=512, L = fft_avg*N = 73*4096 = 299,008 samples per line (fft_avg = int(fs/N/8), S:1546).

Multi-GPU (`torch.distributed.run --nproc-per-node N`): frames are independent, so every
rank processes its own F frames on its own GPU with no data-path collective (weak
scaling); the barrier and the max-over-ranks time are the only collectives.

CPU baseline: the reference's numpy/scipy library path (oracle/scipy_path.py, the same
decimate/welch calls) on a bounded sample of frames, rank 0 at N=1 only, run in a
spawn-context process pool BEFORE the GPU is touched.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "IQ Msamples/s + waterfall lines/s @ N_FFT=4096 zoom=8; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    "cfg2": dict(n_fft=4096, zoom=8, fs=2.4e6, n_avg=73, frames=4096,
                 desc="2.4 MS/s synthetic IQ stream, N_FFT=4096, zoom=8, fp32, 1 MI355X"),
    "cfg3": dict(n_fft=16384, zoom=8, fs=2.4e6, n_avg=18, frames=4096,
                 desc="N_FFT=16384 with 50%-overlap Welch averaging, fp32, 1 MI355X"),
    "cfg1": dict(n_fft=1024, zoom=4, fs=2.4e6, n_avg=256, frames=4096,
                 desc="256k-sample frames, N_FFT=1024, zoom=4"),
    "cfg4": dict(n_fft=4096, zoom=8, fs=2.4e6, n_avg=73, frames=4096, lo_step=150e3,
                 desc="8 independent IF centre frequencies (f_LO = 1 Hz + rank*150 kHz), one "
                      "stream per GPU"),
    "cfg5": dict(n_fft=65536, zoom=8, fs=2.4e6, n_avg=16, frames=2048,
                 desc="1M-sample frames, N_FFT=65536, four-step Welch; --in-dtype complex32 "
                      "for fp16 IQ storage"),
}
IN_BYTES = {"complex64": 8, "complex32": 4, "cu8": 2}
TONES = ((0.31, 1.0), (-0.57, 0.1))


# ----------------------------------------------------------------------------- CPU leg
def _cpu_worker(args):
    """Runs in a spawned process: time the reference's library path on fresh frames."""
    cfg, seconds, seed = args
    import numpy as np  # noqa: F401
    from oracle import scipy_path
    from pypanadapter_amd import synth
    L = cfg["n_fft"] * cfg["n_avg"]
    W = cfg["n_fft"] // cfg["zoom"]
    x = synth.make_iq(L, cfg["fs"], seed, n_fft=cfg["n_fft"], zoom=cfg["zoom"], n_win=W)
    scipy_path.psd_row(x, cfg["fs"], cfg["n_fft"], cfg["zoom"], W)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        scipy_path.psd_row(x, cfg["fs"], cfg["n_fft"], cfg["zoom"], W)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return n, el


def cpu_baseline(cfg, seconds: float, workers: int):
    import multiprocessing as mp
    L = cfg["n_fft"] * cfg["n_avg"]
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    ctx = mp.get_context("spawn")
    # single core
    n1, t1 = _cpu_worker((cfg, max(2.0, seconds / 3), 11))
    single = n1 * L / t1 / 1e6
    # all worker processes, one frame stream each
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(cfg, seconds, 100 + i) for i in range(workers)])
    wall = time.perf_counter() - t0
    frames = sum(r[0] for r in res)
    span = max(r[1] for r in res)
    value = frames * L / span / 1e6
    try:
        model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo")
                 if ln.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(value, 3), "unit": "MS/s", "cores": workers, "kind": "port",
            "lines_per_s": round(frames / span, 2),
            "single_core_MS_per_s": round(single, 3),
            "sample": (f"oracle/scipy_path.psd_row (the reference's decimate/welch/fftshift/log10 "
                       f"library calls) on {frames} frames of L={L} complex64 in {workers} spawned "
                       f"processes for ~{seconds:.0f}s each (+1 core for {t1:.1f}s); "
                       f"wall {wall:.1f}s; host {model}, os.cpu_count()={os.cpu_count()}")}


# ----------------------------------------------------------------------------- GPU leg
def make_frames(torch, F, L, cfg, device, seed):
    """Synthetic IQ on the device: complex white noise (sigma 1/sqrt(2) per component) plus
    two in-band tones, the generator of pypanadapter_amd/synth.py re-expressed in torch."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn((F, L, 2), generator=g, device=device, dtype=torch.float32)
    x.mul_(1.0 / math.sqrt(2.0))
    n = torch.arange(L, device=device, dtype=torch.float64)
    hw = 0.5 * (cfg["n_fft"] // cfg["zoom"]) * cfg["fs"] / (cfg["zoom"] * cfg["n_fft"])
    for frac, amp in TONES:
        turns = torch.remainder(n * ((1.0 + frac * hw) / cfg["fs"]), 1.0)
        ph = 2 * math.pi * turns
        x[:, :, 0] += (amp * torch.cos(ph)).to(torch.float32)
        x[:, :, 1] += (amp * torch.sin(ph)).to(torch.float32)
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=0, help="frames per rank (default: config)")
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--warm", type=int, default=0)
    ap.add_argument("--path", type=int, default=0,
                    help="0 auto, 1 exact order, 2 fused interior, 3 DF2T exact tiles, 4 XA tiles")
    ap.add_argument("--welch", type=int, default=0,
                    help="Welch kernel: 0 auto, 1 one workgroup per frame, 2 four-step (A/B runs)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--in-dtype", default="complex64", choices=sorted(IN_BYTES),
                    help="IQ storage format in HBM (cfg5: complex32 = fp16)")
    args = ap.parse_args()

    cfg = dict(CONFIGS[args.config])
    F = args.frames or cfg["frames"]
    N, zoom, fs = cfg["n_fft"], cfg["zoom"], cfg["fs"]
    L = N * cfg["n_avg"]
    W = N // zoom
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
        cpu = cpu_baseline(cfg, args.cpu_seconds, workers)

    import torch
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from pypanadapter_amd import ZoomFFT
    f_lo = 1.0 + cfg.get("lo_step", 0.0) * rank
    plan = ZoomFFT(N, zoom, fs, n_win=W, device=local, f_lo=f_lo, in_dtype=args.in_dtype)
    if args.block or args.warm:
        plan.tune(args.block, args.warm)
    if args.path:
        plan.set_path(args.path)
    if args.welch:
        plan.set_welch(args.welch)
    stream = torch.cuda.Stream(dev)  # a real stream: the null stream's handle (0) would be
    torch.cuda.set_stream(stream)    # read by the C-ABI as "the plan's own stream"
    sp = stream.cuda_stream
    x = make_frames(torch, F, L, cfg, dev, 1234 + rank)
    if args.in_dtype == "complex32":
        x = x.to(torch.float16).contiguous()
    elif args.in_dtype == "cu8":
        x = torch.clamp(torch.round(127.5 + 127.5 * 0.25 * x), 0, 255).to(torch.uint8).contiguous()
    rows = torch.empty((F, W), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)

    def step():
        plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), sp)
        plan.waterfall_push_device(rows.data_ptr(), F, sp)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    gpu_ms = ev0.elapsed_time(ev1)
    t = torch.tensor([wall, gpu_ms / 1e3], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max, ev_max = float(t[0]), float(t[1])

    # per-launch breakdown from one instrumented step (events on the launch stream)
    plan.set_timing(True)
    plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), sp)
    launch_ms = plan.timings()
    plan.set_timing(False)
    torch.cuda.synchronize(dev)
    finite = bool(torch.isfinite(rows).all().item())

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    ms_per_step = wall_max / args.steps * 1e3
    total_samples = F * L * args.steps * world
    value = total_samples / wall_max / 1e6
    lines = F * args.steps * world / wall_max
    bps = IN_BYTES[args.in_dtype]
    alg_bytes_step = F * (bps * L + 8 * W)  # bps*L in + 4*W row + 4*W ring row
    ev_ms_step = ev_max / args.steps * 1e3
    achieved = alg_bytes_step / (ev_ms_step / 1e3) / 1e9
    names = plan.launch_names()
    kernels = {}
    for i, (nm, ms) in enumerate(zip(names, launch_ms)):
        kernels[f"{i}:{nm}"] = round(ms, 4)
    dominant = max(kernels, key=lambda k: kernels[k]) if kernels else None
    dom_roof = None
    if dominant is not None and "stage_mix" in dominant:
        # the stage-0 decimator: reads the caller's IQ (bps*L per frame), writes the first
        # decimated stage (complex64, ceil(L/2) per frame)
        dom_bytes = F * (bps * L + 8 * ((L + 1) // 2))
        dom_gbs = dom_bytes / (kernels[dominant] / 1e3) / 1e9
        dom_roof = {"kernel": dominant, "algorithmic_bytes_per_launch": dom_bytes,
                    "achieved": round(dom_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(dom_gbs / HBM_PEAK_GBS, 4), "launch_ms": kernels[dominant]}
    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if (tj.get("frames") == F and tj.get("in_dtype", "complex64") == args.in_dtype
                    and tj.get("schedule") == "xa"  # measured on the current auto schedule
                    and not args.path and not args.welch and not args.block and not args.warm):
                traffic = tj.get("hbm_bytes_per_step")
        except Exception:
            traffic = None
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MS/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.in_dtype == "complex64" else f"f32 ({args.in_dtype} IQ storage)",
        "data": "synthetic (device-generated complex white noise + 2 in-band tones, seed per rank)",
        "config": {"workload": f"{args.config}: {cfg['desc']}", "n_fft": N, "zoom": zoom,
                   "n_win": W, "samples_per_line": L, "frames_per_rank": F, "fs": fs,
                   "window": "hamming", "in_dtype": args.in_dtype, "f_lo_rank0": 1.0,
                   "parallelism": f"frame-sharded x{world}, no collective"},
        "lines_per_s": round(lines, 1),
        "roofline": {"bound": "hbm", "kernel": "IQ->log-PSD path (all launches of one step)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_step": alg_bytes_step,
                     "event_ms_per_step": round(ev_ms_step, 4)},
        "kernels": kernels,
        "dominant_kernel": dominant,
        "dominant_roofline": dom_roof,
        "rows_finite": finite,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
