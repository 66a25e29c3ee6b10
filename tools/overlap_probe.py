#!/usr/bin/env python3
"""Does Welch hide inside FC?  cfg2's step (zoom 8, FC + edge + Welch, stream A) and a
stand-alone Welch over decimated-length frames (zoom 1, stream B): each alone, one after the
other, and both submitted together (B forked from A's start).  ms per pair, HIP events, median of
7 after 2 warm runs.  A pipelined FC -> Welch over frame chunks saves at most
(A + B) - (A || B).  usage: python tools/overlap_probe.py OUT.json [frames]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out, F):
    import torch
    from pypanadapter_amd import ZoomFFT, build
    dev = torch.device("cuda", 0)
    N, z, L, W = 4096, 8, 299008, 512
    x = torch.randn((F, L, 2), device=dev, dtype=torch.float32)
    Ld = L // z
    y = torch.randn((F, Ld, 2), device=dev, dtype=torch.float32)
    ra = torch.empty((F, W), device=dev, dtype=torch.float32)
    rb = torch.empty((F, W), device=dev, dtype=torch.float32)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    pa, pb = ZoomFFT(N, z, 2.4e6, n_win=W), ZoomFFT(N, 1, 2.4e6, n_win=W)

    def run(mode):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        jb = torch.cuda.Event()
        e0.record(sa)
        if mode in ("a", "seq", "par"):
            pa.process_device(x.data_ptr(), L, F, ra.data_ptr(), sa.cuda_stream)
        if mode == "seq":
            pb.process_device(y.data_ptr(), Ld, F, rb.data_ptr(), sa.cuda_stream)
        if mode == "b":
            pb.process_device(y.data_ptr(), Ld, F, rb.data_ptr(), sa.cuda_stream)
        if mode == "par":
            sb.wait_event(e0)
            pb.process_device(y.data_ptr(), Ld, F, rb.data_ptr(), sb.cuda_stream)
            jb.record(sb)
            sa.wait_event(jb)
        e1.record(sa)
        e1.synchronize()
        return e0.elapsed_time(e1)

    res = {"source_hash": build.source_hash(), "frames": F, "what": __doc__.split("\n")[0]}
    for rep in range(2):
        for mode in ("a", "b", "seq", "par"):
            run(mode)
    for mode in ("a", "b", "seq", "par"):
        ts = sorted(run(mode) for _ in range(7))
        res[mode] = round(ts[3], 4)
        print(mode, res[mode], flush=True)
    res["hidden_ms"] = round(res["seq"] - res["par"], 4)
    pa.close()
    pb.close()
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4096)
