#!/usr/bin/env python3
"""Benchmark of the IQ -> log-PSD -> waterfall-line hot path (BASELINE.json metric).

One step = one pass of the hot path over one batch of F synthetic IQ frames resident in
HBM: LO mix + log2(zoom) x decimate(x, 2) + Welch PSD + fftshift/crop + 20*log10 (the
reference's ApplicationDisplay.update, pypanadapter_spectrum.py:2102-2119) and the
waterfall row-roll of all F lines (Waterfall.image_update, S:1638-1664).

Workload (BASELINE.json configs[1]): 2.4 MS/s synthetic IQ, N_FFT=4096, zoom=8, fp32,
W=512, L = fft_avg*N = 73*4096 = 299,008 samples per line (fft_avg = int(fs/N/8), S:1546).

Multi-GPU: frames are independent (S:2091-2111, T:1516-1538), so every rank processes its
own F frames on its own GPU with no data-path collective (weak scaling).  Under
torch.distributed.run the ranks come from the environment; `--gpus N` without it spawns N
rank processes itself (before anything touches a GPU).  The barrier and the max-over-ranks
time go through gloo on the host: no RCCL on this path.

Outside the timed region: per-launch HIP-event times (the dominant kernel's roofline), a
parity check of sampled frames against the float64 oracle (checker only), and the
end-to-end host path (single-frame latency; streaming from pinned host memory with the H2D
copy of batch k+1 overlapping the compute of batch k).

CPU baseline: the reference's numpy/scipy library path (oracle/scipy_path.py, the same
decimate/welch calls) on a bounded sample of frames, rank 0 at N=1 only, in a spawn-context
process pool of the job's CPU share, run BEFORE the GPU is touched.
"""
from __future__ import annotations

import argparse
import datetime
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

def metric_of(n_fft: int, zoom: int) -> str:
    """BASELINE.json's metric string (cfg2's N_FFT=4096 zoom=8), with the config's own N/zoom."""
    return f"IQ Msamples/s + waterfall lines/s @ N_FFT={n_fft} zoom={zoom}; % HBM roofline"


METRIC = metric_of(4096, 8)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    "cfg2": dict(n_fft=4096, zoom=8, fs=2.4e6, n_avg=73, frames=4096,
                 desc="2.4 MS/s synthetic IQ stream, N_FFT=4096, zoom=8, fp32, 1 MI355X"),
    "cfg3": dict(n_fft=16384, zoom=8, fs=2.4e6, n_avg=18, frames=4096,
                 desc="N_FFT=16384 with 50%-overlap Welch averaging, fp32, 1 MI355X"),
    "cfg1": dict(n_fft=1024, zoom=4, fs=2.4e6, n_avg=256, frames=4096,
                 desc="256k-sample frames, N_FFT=1024, zoom=4"),
    "cfg4": dict(n_fft=4096, zoom=8, fs=2.4e6, n_avg=73, frames=4096, lo_step=150e3,
                 desc="8 independent IF centre frequencies (f_LO,k = 1 Hz + k*150 kHz), batched "
                      "on one plan per rank (8/N IFs per rank; one per GPU at N = 8)"),
    "cfg5": dict(n_fft=65536, zoom=8, fs=2.4e6, n_avg=16, frames=2048,
                 desc="1M-sample frames, N_FFT=65536, four-step Welch; --in-dtype complex32 "
                      "for fp16 IQ storage"),
}
IN_BYTES = {"complex64": 8, "complex32": 4, "cu8": 2}
TONES = ((0.31, 1.0), (-0.57, 0.1))
# plan launch name -> kernel-name prefix in the rocprofv3 / PMC summaries
KERNEL_OF = {"xa_stage_mix": "xa_stage_kernel<32, true", "xa_stage": "xa_stage_kernel<32, false",
             "pc_fir": "pc_fir_kernel", "pc_tail": "pc_tail_kernel", "pc_edge": "pc_edge_kernel",
             "pc_walk": "pc_walk_kernel", "fc_decim": "fc_decim_kernel",
             "welch_rows": "welch_", "welch4": "welch4_"}


def alg_bytes_per_line(bps: int, L: int, W: int) -> int:
    """bps*L of IQ in + 4*W row out + 4*W waterfall ring row."""
    return bps * L + 8 * W


def stage_lengths(L: int, zoom: int) -> list:
    n = [L]
    while zoom > 1:
        n.append((n[-1] + 1) // 2)
        zoom //= 2
    return n


def own_bytes_per_frame(name: str, bps: int, L: int, zoom: int, W: int, stage: int) -> int | None:
    """A launch's OWN minimal bytes per frame: what it must read and write (its input and its
    output arrays, intermediates included when they are its input or output) -- the basis of
    kernels_roofline.  None for the blocked schedules (FGI intermediates, several passes)."""
    n = stage_lengths(L, zoom)
    if name == "pc_fir":  # IQ in, y2 (rate 1/4 from q = -16, complex64) out
        y2 = ((L + 15) // 2 + 24) // 2 + 17
        return bps * L + 8 * y2
    if name == "pc_tail":
        y2 = ((L + 15) // 2 + 24) // 2 + 17
        return 8 * y2 + 8 * n[-1]
    if name in ("pc_walk", "fc_decim"):  # IQ in, decimated IQ out (intermediates on chip)
        return bps * L + 8 * n[-1]
    if name == "pc_edge":  # ~1070 IQ samples at each end in, ~160 outputs read and written
        return bps * 2 * 1100 + 16 * 2 * 170
    if name in ("xa_stage_mix", "xa_stage"):
        k = stage
        return (bps if k == 0 else 8) * n[k] + 8 * n[k + 1]
    if name in ("welch_rows", "welch4"):
        return 8 * n[-1] + 4 * W
    return None


# ----------------------------------------------------------------------------- CPU leg
def cpu_share() -> tuple:
    """(cores, how): the CPUs this job may use -- the cgroup quota, else OMP_NUM_THREADS
    (the GPU box sets it to the job's share), else the affinity mask."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(p))), "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        return int(os.environ["OMP_NUM_THREADS"]), "OMP_NUM_THREADS (the job's CPU share)"
    return len(os.sched_getaffinity(0)), "sched_getaffinity"


def _cpu_worker(args):
    """Runs in a spawned process: time the reference's library path on fresh frames."""
    cfg, seconds, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
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


def cpu_baseline(cfg, seconds: float, workers: int, how: str):
    import multiprocessing as mp
    L = cfg["n_fft"] * cfg["n_avg"]
    ctx = mp.get_context("spawn")
    n1, t1 = _cpu_worker((cfg, max(2.0, seconds / 3), 11))  # one core
    single = n1 * L / t1 / 1e6
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:  # one frame stream per worker process
        res = pool.map(_cpu_worker, [(cfg, seconds, 100 + i) for i in range(workers)])
    wall = time.perf_counter() - t0
    frames = sum(r[0] for r in res)
    span = max(r[1] for r in res)
    try:
        model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo")
                 if ln.startswith("model name")][0]
    except (OSError, IndexError):
        model = "unknown"
    return {"value": round(frames * L / span / 1e6, 3), "unit": "MS/s", "cores": workers,
            "kind": "port", "lines_per_s": round(frames / span, 2),
            "single_core_MS_per_s": round(single, 3),
            "single_core_ms_per_frame": round(t1 / n1 * 1e3, 2),
            "sample": (f"oracle/scipy_path.psd_row (the reference's decimate/welch/fftshift/log10 "
                       f"library calls) on {frames} frames of L={L} complex64 in {workers} spawned "
                       f"processes for ~{seconds:.0f}s each (+1 core for {t1:.1f}s); wall {wall:.1f}s; "
                       f"cores = {how}; host {model}, os.cpu_count()={os.cpu_count()}")}


def parity_check(frames: dict, rows: dict, cfg, f_lo_of) -> dict:
    """Checker only: sampled frames of the timed batch against the float64 oracle under the
    fp32 gate (|ddB| <= 1e-3 within 100 dB of the peak, |d amp| <= 1e-5 peak)."""
    import numpy as np
    from oracle import coracle
    coracle.build()
    N, z = cfg["n_fft"], cfg["zoom"]
    W = N // z
    worst_db = worst_amp = 0.0
    for f, x in frames.items():
        ref = coracle.psd_row(x, cfg["fs"], N, z, W, f_lo=f_lo_of(f))
        row = rows[f].astype(np.float64)
        pk = ref.max()
        m = ref > pk - 100.0
        worst_db = max(worst_db, float(np.abs(row - ref)[m].max()))
        worst_amp = max(worst_amp, float(np.abs(10 ** (row / 20) - 10 ** (ref / 20)).max() / 10 ** (pk / 20)))
    return {"frames": sorted(frames), "max_abs_ddb_within_100dB": worst_db, "max_amp_err_rel_peak": worst_amp,
            "gate": "|ddB| <= 1e-3 within 100 dB of peak and |d amp| <= 1e-5 x peak",
            "pass": bool(worst_db <= 1e-3 and worst_amp <= 1e-5)}


def provenance() -> dict:
    """Ties this line to the profiles/ it is judged against: the kernel-source hash (the
    stamp PMC/SQ summaries carry), the git commit the library was built at (the GPU box has
    no .git: build() records it next to the .so), and whether that build matches the tree."""
    from pypanadapter_amd import build
    info = build.build_info()
    head = None
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
    except (OSError, subprocess.SubprocessError):
        pass
    return {"source_hash": build.source_hash(), "git_head": head or info.get("git_head"),
            "git_head_from": "git" if head else "build_info", "built_source_hash": info.get("source_hash"),
            "built_git_dirty": info.get("git_dirty"), "host": socket.gethostname()}


# ----------------------------------------------------------------------------- launcher
def spawn_ranks(argv) -> int:
    """`--gpus N` outside torch.distributed.run: N rank processes, one per GPU, started
    before this process touches any GPU; returns the worst exit code."""
    n = int(argv.gpus)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    # a rank that fails ends the others (which would wait in the barrier for it)
    while any(p.poll() is None for p in procs):
        if any(p.returncode not in (None, 0) for p in procs):
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    return max(abs(p.wait()) for p in procs)


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


def encode(torch, x, in_dtype):
    """Device frames in the plan's input format (complex32 = fp16 I,Q; cu8 = RTL-SDR bytes)."""
    if in_dtype == "complex32":
        return x.to(torch.float16).contiguous()
    if in_dtype == "cu8":
        return torch.clamp(torch.round(127.5 + 127.5 * 0.25 * x), 0, 255).to(torch.uint8).contiguous()
    return x


def decoded_host(torch, xe, f, in_dtype):
    """Frame f exactly as the kernels read it, complex128 on the host (for the checker)."""
    import numpy as np
    a = xe[f].cpu().numpy()
    if in_dtype == "cu8":
        a = (a.astype(np.float64) - 127.5) / 127.5
    a = a.astype(np.float64)
    return a[:, 0] + 1j * a[:, 1]


def stamped_profile(path, F, in_dtype):
    """A committed profile summary, if it was measured on these kernel sources."""
    from pypanadapter_amd import build
    try:
        tj = json.load(open(path))
    except (OSError, ValueError):
        return None, "absent"
    if tj.get("source_hash") != build.source_hash():
        return None, f"stale (measured on sources {tj.get('source_hash')}, now {build.source_hash()})"
    if tj.get("frames") != F or tj.get("in_dtype", "complex64") != in_dtype:
        return None, "other workload"
    return tj, "ok"


def end_to_end(torch, args, cfg, x_dev, dev):
    """Host-path numbers (PCIe-inclusive; never `value`): single-frame psd latency as the
    reference calls it (one chunk per update(), S:2102), and streaming throughput from pinned
    host memory through zfft_process (batched, H2D of batch k+1 under compute of batch k)."""
    import numpy as np
    from pypanadapter_amd import ZoomFFT, synth
    N, z, fs = cfg["n_fft"], cfg["zoom"], cfg["fs"]
    L, W = N * cfg["n_avg"], N // z
    out = {}
    x1 = synth.make_iq(L, fs, 4242, n_fft=N, zoom=z, n_win=W)
    with ZoomFFT(N, z, fs, n_win=W, device=dev.index) as plan:
        for _ in range(3):
            plan.rows(x1)
        lat = []
        for _ in range(40):
            t0 = time.perf_counter()
            plan.rows(x1)
            lat.append((time.perf_counter() - t0) * 1e3)
    lat = np.sort(lat)
    out["single_frame_latency_ms"] = {"p50": round(float(np.percentile(lat, 50)), 3),
                                      "p99": round(float(np.percentile(lat, 99)), 3),
                                      "what": "psd_row of one host complex64 frame (H2D, decimate, "
                                              "Welch, D2H) through zfft_process"}
    Fs = min(args.e2e_frames, x_dev.shape[0])
    stream = {}
    for fmt in ("complex64", "cu8"):
        xe = encode(torch, x_dev[:Fs], fmt)
        host = torch.empty(xe.shape, dtype=xe.dtype, pin_memory=True)
        host.copy_(xe)
        nbytes = host.numel() * host.element_size()
        tmp = torch.empty_like(xe)  # the PCIe H2D ceiling: a plain pinned -> device copy
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(3):
            tmp.copy_(host, non_blocking=True)
        torch.cuda.synchronize(dev)
        h2d = 3 * nbytes / (time.perf_counter() - t0) / 1e9
        del tmp
        rows = np.empty((Fs, W), np.float32)
        with ZoomFFT(N, z, fs, n_win=W, device=dev.index, in_dtype=fmt) as plan:
            plan.process_host(host.data_ptr(), L, Fs, rows.ctypes.data)
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                plan.process_host(host.data_ptr(), L, Fs, rows.ctypes.data)
            el = (time.perf_counter() - t0) / reps
        rate = Fs * L / el / 1e6
        bound = h2d * 1e3 / IN_BYTES[fmt]
        stream[fmt] = {"MS_per_s": round(rate, 1), "lines_per_s": round(Fs / el, 1),
                       "frames": Fs, "bytes_per_sample": IN_BYTES[fmt],
                       "pcie_h2d_GBps": round(h2d, 1), "pcie_bound_MS_per_s": round(bound, 1),
                       "frac_of_pcie_bound": round(rate / bound, 3)}
        del host, xe
    out["streaming_pinned"] = stream
    out["display"] = display_timing(dev)
    return out


def display_timing(dev, widths=(512, 8192), lines=12) -> dict:
    """The display side SURVEY §8f-2 exists for, per waterfall line: the facade's
    `image_update(psd)` (device ring push, O(W)) then either `render()` (RGBA8 on the device +
    D2H, what pyqtgraph's setImage turns the image into, S:1664) or `img_array` (the float64
    image materialised on the host every line, the pre-r04 INTEGRATION.md binding); beside
    them the reference's own `Waterfall.image_update` (oracle/scipy_path.py: full-image
    np.roll per line, S:1638-1664) on the CPU.  Since round 6 the facade's image_update
    stages the row on the host and the next read pushes it (zfft_waterfall_push_render /
    _push_read64: one kernel, one copy, one wait per line), so "push" alone is host work and
    the device push is inside the other two columns."""
    import numpy as np
    from oracle.scipy_path import Waterfall as RefWaterfall
    from pypanadapter_amd import Waterfall
    out = {}
    rng = np.random.default_rng(5)
    for W in widths:
        rows = rng.uniform(-200.0, -110.0, (lines + 2, W))
        wf = Waterfall(scroll=1, device=dev.index)
        res = {}
        for what in ("push", "push_render", "push_img_array"):
            ts = []
            for k in range(lines + 2):
                r = rows[k].astype(np.float32)
                t0 = time.perf_counter()
                wf.image_update(r)
                if what == "push_render":
                    wf.render()
                elif what == "push_img_array":
                    _ = wf.img_array
                # "push" alone: the facade stages the row (the next read pushes it)
                if k >= 2:
                    ts.append((time.perf_counter() - t0) * 1e3)
            res[what + "_ms_per_line"] = round(float(np.median(ts)), 3)
        ref = RefWaterfall()
        ts = []
        for k in range(lines + 2):
            t0 = time.perf_counter()
            ref.image_update(rows[k].copy(), 1)
            if k >= 2:
                ts.append((time.perf_counter() - t0) * 1e3)
        res["reference_cpu_image_update_ms_per_line"] = round(float(np.median(ts)), 3)
        res["H"] = W // 4
        out[f"W{W}"] = res
        wf.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200,
                    help="timed steps; raised so that the timed region lasts >= --min-seconds")
    ap.add_argument("--min-seconds", type=float, default=1.0,
                    help="lower bound on the timed region (0: exactly --steps)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=0, help="frames per rank (default: config)")
    ap.add_argument("--zoom", type=int, default=0, help="override the config's zoom (not a BASELINE line)")
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--warm", type=int, default=0)
    ap.add_argument("--path", type=int, default=0,
                    help="0 auto, 1 exact order, 2 fused interior, 3 XA tiles, 4 PC cascade")
    ap.add_argument("--welch", type=int, default=0,
                    help="Welch kernel: 0 auto, 1 one workgroup per frame, 2 four-step (A/B runs)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-workers", type=int, default=0, help="0: the job's CPU share")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--e2e-frames", type=int, default=1024)
    ap.add_argument("--dry-run", action="store_true",
                    help="rank/launcher check only: no GPU call (CPU tests of --gpus N)")
    ap.add_argument("--in-dtype", default="complex64", choices=sorted(IN_BYTES),
                    help="IQ storage format in HBM (cfg5: complex32 = fp16)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))

    cfg = dict(CONFIGS[args.config])
    if args.zoom:  # e.g. the PC head + XA tail at zoom 16 on cfg2's frames
        cfg["zoom"] = args.zoom
        cfg["desc"] += f" (zoom overridden to {args.zoom}: not a BASELINE config)"
    F = args.frames or cfg["frames"]
    N, zoom, fs = cfg["n_fft"], cfg["zoom"], cfg["fs"]
    L = N * cfg["n_avg"]
    W = N // zoom
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        share, how = cpu_share()
        workers = args.cpu_workers or share
        cpu = cpu_baseline(cfg, args.cpu_seconds, workers, how if not args.cpu_workers else "--cpu-workers")

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo on the host: barrier + max-reduce only
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=600))
    if args.dry_run and os.environ.get("BENCH_DRY_RUN_FAIL_RANK") == str(rank):
        sys.exit(3)  # launcher test: a rank that dies before the barrier
    if args.dry_run:  # the launcher's contract without touching a GPU
        # plan_device: the GPU this rank's plan and streams would use (cuda:LOCAL_RANK)
        me = torch.tensor([rank, local, world, os.getpid(), local], dtype=torch.int64)
        allr = [torch.zeros(5, dtype=torch.int64) for _ in range(world)] if dist else [me]
        if dist:
            dist.all_gather(allr, me)
            dist.barrier()
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"dry_run": True, "world": world,
                              "ranks": [dict(zip(("rank", "local_rank", "world", "pid", "plan_device"), map(int, r)))
                                        for r in allr]}))
        return
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from pypanadapter_amd import ZoomFFT
    # config 4: 8 IF centre frequencies f_k = 1 Hz + k * 150 kHz over the job, 8 / world of
    # them per rank, each on F / (its IFs) consecutive frames of the rank's one batch
    ifs = [0]
    if "lo_step" in cfg:
        n_if = max(1, 8 // world)
        ifs = [(rank * n_if + i) % 8 for i in range(n_if)]
    f_los = [1.0 + cfg.get("lo_step", 0.0) * k for k in ifs]
    per = max(1, F // len(f_los))

    def f_lo_of(f):
        return f_los[(f // per) % len(f_los)]

    plan = ZoomFFT(N, zoom, fs, n_win=W, device=local, f_lo=f_los[0], in_dtype=args.in_dtype)
    if len(f_los) > 1:
        plan.set_lo_frames(f_los, per)
    if args.block or args.warm:
        plan.tune(args.block, args.warm)
    if args.path:
        plan.set_path(args.path)
    if args.welch:
        plan.set_welch(args.welch)
    stream = torch.cuda.Stream(dev)  # a real stream: the null stream's handle (0) would be
    torch.cuda.set_stream(stream)    # read by the C-ABI as HIP's default stream
    sp = stream.cuda_stream
    x = make_frames(torch, F, L, cfg, dev, 1234 + rank)
    xe = encode(torch, x, args.in_dtype)
    if xe is not x and (args.no_e2e or rank != 0):
        x = None  # only the e2e leg re-encodes from the float frames
    rows = torch.empty((F, W), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)

    def step():
        plan.process_device(xe.data_ptr(), L, F, rows.data_ptr(), sp)
        plan.waterfall_push_device(rows.data_ptr(), F, sp)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    t_w = time.perf_counter()  # a warm probe for the step time (the first warmup step also
    for _ in range(3):         # allocates the plan's workspaces)
        step()
    torch.cuda.synchronize(dev)
    est = (time.perf_counter() - t_w) / 3
    # >= min_seconds of timed work whatever --steps says (a 20-step region at ~6 ms/step is
    # 0.13 s, inside the box-to-box noise); every rank runs the same count (max over ranks)
    steps = max(args.steps, math.ceil(1.05 * args.min_seconds / max(est, 1e-6)))
    if dist:
        ts = torch.tensor([steps], dtype=torch.int64)
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        steps = int(ts[0])
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    gpu_ms = ev0.elapsed_time(ev1)
    t = torch.tensor([wall, gpu_ms / 1e3], dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max, ev_max = float(t[0]), float(t[1])

    # per-launch HIP-event times (events on the launch stream) over a few instrumented steps
    plan.set_timing(True)
    acc, n_inst = {}, max(1, min(steps, 10))
    for _ in range(n_inst):
        plan.process_device(xe.data_ptr(), L, F, rows.data_ptr(), sp)
        for i, (nm, ms) in enumerate(zip(plan.launch_names(), plan.timings())):
            acc[f"{i}:{nm}"] = acc.get(f"{i}:{nm}", 0.0) + ms
    plan.set_timing(False)
    torch.cuda.synchronize(dev)
    kernels = {k: round(v / n_inst, 4) for k, v in acc.items()}
    finite = bool(torch.isfinite(rows).all().item())

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    check = None
    if not args.no_check:
        pick = sorted({0, F // 2, F - 1} | ({per * i + per - 1 for i in range(len(f_los))} if len(f_los) > 1 else set()))
        host_rows = rows.cpu().numpy()
        frames = {f: decoded_host(torch, xe, f, args.in_dtype) for f in pick}
        check = parity_check(frames, {f: host_rows[f] for f in pick}, cfg, f_lo_of)
    e2e = None
    if not args.no_e2e:
        plan.close()
        del rows
        e2e = end_to_end(torch, args, cfg, x if x is not None else xe, dev)

    ms_per_step = wall_max / steps * 1e3
    total_samples = F * L * steps * world
    value = total_samples / wall_max / 1e6
    lines = F * steps * world / wall_max
    bps = IN_BYTES[args.in_dtype]
    alg_step = F * alg_bytes_per_line(bps, L, W)
    ev_ms_step = ev_max / steps * 1e3
    path_gbs = alg_step / (ev_ms_step / 1e3) / 1e9
    traffic_j, traffic_status = stamped_profile(
        os.path.join(ROOT, "profiles", f"traffic_{args.config}.json"), F, args.in_dtype)
    sq_j, sq_status = stamped_profile(os.path.join(ROOT, "profiles", f"sq_{args.config}.json"), F,
                                      args.in_dtype)
    default_sched = not (args.path or args.welch or args.block or args.warm)
    step_traffic = None
    if traffic_j and default_sched:
        step_traffic = traffic_j.get("hbm_bytes_per_step")
    # per-launch component rooflines, each priced on its OWN input + output bytes
    kroof, stage_k = {}, 0
    for key, ms in kernels.items():
        name = key.split(":", 1)[1]
        ob = own_bytes_per_frame(name, bps, L, zoom, W, stage_k)
        if name.startswith("xa_stage"):
            stage_k += 1
        ent = {"ms": ms}
        if ob is not None and ms:
            gbs = F * ob / (ms / 1e3) / 1e9
            ent.update({"own_bytes": F * ob, "achieved_GBps": round(gbs, 1),
                        "frac": round(gbs / HBM_PEAK_GBS, 4)})
        pref = KERNEL_OF.get(name)
        if pref and traffic_j and default_sched:
            t = sum(v["hbm_bytes_per_step_fetch_x2"] for k2, v in traffic_j["per_kernel"].items()
                    if k2.startswith(pref))
            ent["traffic"] = t or None
        if pref and sq_j and default_sched:
            vk = [v for k2, v in sq_j["per_kernel"].items() if k2.startswith(pref)]
            ent["valu_util"] = vk[0].get("valu_busy") if vk else None
        kroof[key] = ent
    dominant = max(kernels, key=lambda k: kernels[k]) if kernels else None
    out = {
        "metric": metric_of(N, zoom),
        "value": round(value, 2),
        "unit": "MS/s",
        "n_gpus": world,
        "steps": steps,
        "steps_requested": args.steps,
        "warmup": args.warmup,
        "timed_seconds": round(wall_max, 4),
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.in_dtype == "complex64" else f"f32 ({args.in_dtype} IQ storage)",
        "data": "synthetic (device-generated complex white noise + 2 in-band tones, seed per rank)",
        "config": {"workload": f"{args.config}: {cfg['desc']}", "n_fft": N, "zoom": zoom,
                   "n_win": W, "samples_per_line": L, "frames_per_rank": F, "fs": fs,
                   "window": "hamming", "in_dtype": args.in_dtype,
                   "f_lo_hz": f_los, "frames_per_lo": per,
                   "parallelism": f"frame-sharded x{world}, no collective (gloo barrier only)"},
        "lines_per_s": round(lines, 1),
        "roofline": {"bound": "hbm",
                     "kernel": "the whole IQ -> log-PSD -> waterfall chain of a step (all launches)",
                     "achieved": round(path_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(path_gbs / HBM_PEAK_GBS, 4),
                     "traffic": step_traffic,
                     "traffic_ratio": round(step_traffic / alg_step, 3) if step_traffic else None,
                     "algorithmic_bytes_per_launch": alg_step,
                     "bytes_basis": "SURVEY §8(d) per line (bps*L IQ in + 4W row + 4W ring row) x F lines "
                                    "per step; intermediates excluded",
                     "avg_launch_ms": round(ev_ms_step, 4),
                     "avg_launch_ms_is": "HIP-event time of one step on the launch stream (the sum of "
                                         "the chain's launches; rocprofv3: sum of their averages)",
                     "dominant_component": dominant,
                     "profiles": {"traffic": traffic_status, "sq": sq_status}},
        "kernels_roofline": kroof,
        "path_roofline": {"what": "same as roofline (the whole chain) since round 4; kept for the "
                                  "earlier rounds' readers", "frac": round(path_gbs / HBM_PEAK_GBS, 4),
                          "event_ms_per_step": round(ev_ms_step, 4)},
        "kernels": kernels,
        "rows_finite": finite,
        "parity_checked_frames": check,
        "end_to_end": e2e,
        "cpu_baseline": cpu,
        "provenance": provenance(),
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
