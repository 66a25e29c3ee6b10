#!/usr/bin/env python3
"""Walk crossovers after round 6's walk changes (zfft_plan.cpp kPcWalkMinFrames and the zoom-4
choice between XA, the tiles and the walk): per-call device time (HIP events, median of 5 after
2 warm calls) of the PC tiles (path 4), the walk (path 5) and XA (path 3, zoom 4 only) over batch
sizes, zoom 8 at cfg2's and cfg5's frame lengths (N = 4096), zoom 4 at cfg1's (N = 1024).
Stamped with the kernel-source hash.  usage: python tools/sweep_walk.py OUT.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import torch
    from pypanadapter_amd import ZoomFFT, build
    dev = torch.device("cuda", 0)
    res = {"source_hash": build.source_hash(), "what": "ms per process_device call (HIP events, median "
           "of 5 after 2 warm calls)", "series": {}}
    Fs = [256, 512, 768, 1024, 1536, 2048, 3072, 4096]
    cases = {"z8_L299008": (8, 4096, 299008, (4, 5)), "z8_L1048576": (8, 4096, 1048576, (4, 5)),
             "z4_L262144": (4, 1024, 262144, (3, 4, 5))}
    for name, (z, N, L, paths) in cases.items():
        x = torch.randn((max(Fs), L, 2), device=dev, dtype=torch.float32)
        W = N // z
        rows = torch.empty((max(Fs), W), device=dev, dtype=torch.float32)
        ser = {}
        for F in Fs:
            for path in paths:
                with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
                    plan.set_path(path)
                    st = torch.cuda.current_stream()
                    ts = []
                    for r in range(7):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), st.cuda_stream)
                        e1.record(st)
                        e1.synchronize()
                        if r >= 2:
                            ts.append(e0.elapsed_time(e1))
                ts.sort()
                ser[f"F{F}_path{path}"] = round(ts[len(ts) // 2], 4)
                print(name, F, path, ser[f"F{F}_path{path}"], flush=True)
        res["series"][name] = ser
        res[f"{name}_best_by_frames"] = {F: min(paths, key=lambda p: ser[f"F{F}_path{p}"]) for F in Fs}
        del x, rows
        torch.cuda.empty_cache()
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "series"}))


if __name__ == "__main__":
    main(sys.argv[1])
