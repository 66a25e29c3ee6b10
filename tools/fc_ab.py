#!/usr/bin/env python3
"""Same-box A/B of the zoom-8 and zoom-4 decimators: per-call device time (HIP events, median of 5 after 2
warm calls) of the PC tiles (path 4, small batches), the walk (path 5) and FC (path 6) at cfg2's
and cfg5's frame lengths over batch sizes, and of zoom 16 (PC head + tail, walk vs FC head);
paths alternate per size; per-launch times of the largest batch.  Stamped with the kernel-source
hash.  usage: python tools/fc_ab.py OUT.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {  # name: (n_fft, zoom, L, {paths: frame counts})
    "cfg2_L299008": (4096, 8, 299008, {(4, 5, 6): [1, 16, 64, 256, 512, 1024], (5, 6): [2048, 4096]}),
    "cfg5_L1048576": (65536, 8, 1048576, {(4, 5, 6): [1, 64, 512, 1024], (5, 6): [2048]}),
    "z16_L299008": (4096, 16, 299008, {(5, 6): [1, 64, 512, 4096]}),
    "cfg1_z4_L262144": (1024, 4, 262144, {(4, 5, 6): [1, 16, 64, 256, 512, 1024], (5, 6): [2048, 4096]}),
}


def main(out):
    import torch
    from pypanadapter_amd import ZoomFFT, build
    dev = torch.device("cuda", 0)
    res = {"source_hash": build.source_hash(), "what": "ms per process_device call (HIP events, median "
           "of 5 after 2 warm calls)", "series": {}, "launches": {}}
    for name, (N, z, L, plan_fs) in CASES.items():
        Fmax = max(max(v) for v in plan_fs.values())
        x = torch.randn((Fmax, L, 2), device=dev, dtype=torch.float32)
        W = N // z
        rows = torch.empty((Fmax, W), device=dev, dtype=torch.float32)
        ser = {}
        for paths, Fs in plan_fs.items():
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
                        if F == Fmax:
                            plan.set_timing(True)
                            plan.process_device(x.data_ptr(), L, F, rows.data_ptr(), st.cuda_stream)
                            torch.cuda.synchronize()
                            res["launches"][f"{name}_F{F}_path{path}"] = dict(zip(
                                plan.launch_names(), [round(v, 4) for v in plan.timings()]))
                    ts.sort()
                    ser[f"F{F}_path{path}"] = round(ts[len(ts) // 2], 4)
                    print(name, F, path, ser[f"F{F}_path{path}"], flush=True)
        res["series"][name] = ser
        del x, rows
        torch.cuda.empty_cache()
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["launches"]))


if __name__ == "__main__":
    main(sys.argv[1])
