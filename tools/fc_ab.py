#!/usr/bin/env python3
"""Same-box A/B of the zoom-8 decimators: per-call device time (HIP events, median of 5 after 2
warm calls) of the walk (path 5) and FC (path 6) at cfg2's and cfg5's frame lengths over batch
sizes, alternating the two paths per size; per-launch times of the FC call at the largest batch.
Stamped with the kernel-source hash.  usage: python tools/fc_ab.py OUT.json [Fs...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out, Fs):
    import torch
    from pypanadapter_amd import ZoomFFT, build
    dev = torch.device("cuda", 0)
    res = {"source_hash": build.source_hash(), "what": "ms per process_device call (HIP events, median "
           "of 5 after 2 warm calls)", "series": {}, "launches": {}}
    cases = {"cfg2_L299008": (4096, 299008), "cfg5_L1048576": (65536, 1048576)}
    for name, (N, L) in cases.items():
        Fmax = max(f for f in Fs if f * L * 8 <= 40 << 30)
        x = torch.randn((Fmax, L, 2), device=dev, dtype=torch.float32)
        W = N // 8
        rows = torch.empty((Fmax, W), device=dev, dtype=torch.float32)
        ser = {}
        for F in [f for f in Fs if f <= Fmax]:
            for path in (5, 6):
                with ZoomFFT(N, 8, 2.4e6, n_win=W) as plan:
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
                        res["launches"][f"{name}_F{F}_path{path}"] = dict(zip(plan.launch_names(),
                                                                             [round(v, 4) for v in plan.timings()]))
                ts.sort()
                ser[f"F{F}_path{path}"] = round(ts[len(ts) // 2], 4)
                print(name, F, path, ser[f"F{F}_path{path}"], flush=True)
        res["series"][name] = ser
        del x, rows
        torch.cuda.empty_cache()
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["launches"]))


if __name__ == "__main__":
    main(sys.argv[1], [int(a) for a in sys.argv[2:]] or [1, 16, 256, 1024, 2048, 4096])
