#!/usr/bin/env python3
"""Per-call time against frames per call near cfg2's 4096: the stand-alone Welch (zoom 1 over
decimated-length frames, N = 4096) and the whole cfg2 chain (zoom 8).  A launch whose last round
of workgroups is partial shows up as a step in ms per frame.  HIP events, median of 7 after 2 warm
calls.  usage: python tools/tail_probe.py OUT.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import torch
    from pypanadapter_amd import ZoomFFT, build
    dev = torch.device("cuda", 0)
    N, z, L, W = 4096, 8, 299008, 512
    Ld = L // z
    Fs = [2304, 3072, 3584, 3840, 4096, 4352, 4608]
    Fmax = max(Fs)
    x = torch.randn((Fmax, L, 2), device=dev, dtype=torch.float32)
    y = torch.randn((Fmax, Ld, 2), device=dev, dtype=torch.float32)
    rows = torch.empty((Fmax, W), device=dev, dtype=torch.float32)
    st = torch.cuda.current_stream()
    res = {"source_hash": build.source_hash(), "what": __doc__.split("\n")[0], "welch": {}, "chain": {}}
    for key, zoom, src, n in (("welch", 1, y, Ld), ("chain", z, x, L)):
        with ZoomFFT(N, zoom, 2.4e6, n_win=W) as plan:
            for F in Fs:
                ts = []
                for r in range(9):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    plan.process_device(src.data_ptr(), n, F, rows.data_ptr(), st.cuda_stream)
                    e1.record(st)
                    e1.synchronize()
                    if r >= 2:
                        ts.append(e0.elapsed_time(e1))
                ts.sort()
                ms = ts[3]
                res[key][F] = {"ms": round(ms, 4), "us_per_frame": round(ms * 1e3 / F, 4)}
                print(key, F, res[key][F], flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
