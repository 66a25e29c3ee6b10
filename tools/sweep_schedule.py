#!/usr/bin/env python3
"""Re-derive the automatic decimator-schedule crossovers (zfft_plan.cpp auto_xa / use_fused /
pc_fits / kPcWalkMinFrames) from one GPU run: per-call device time of each schedule (path 1
exact blocked, 2 fused blocked + edge windows, 3 XA tiles, 4 PC polyphase cascade tiles, 5 PC
walk: one workgroup per frame) over batch sizes, for cfg2-length
frames (L = 299,008 <= 2^19) and cfg5-length frames (L = 2^20).  Writes a JSON stamped with the kernel-source
hash; DESIGN.md cites it, and the constants in zfft_plan.cpp are the crossovers it finds.
usage: python tools/sweep_schedule.py OUT.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import torch
    from pypanadapter_amd import ZoomFFT, build
    dev = torch.device("cuda", 0)
    res = {"source_hash": build.source_hash(), "what": "ms per process_device call (HIP events, "
           "median of 5 after 2 warm calls); N = 4096, zoom 8, W = 512", "series": {}}
    cases = {"L299008": (299008, [1, 2, 4, 8, 16, 32, 64, 128, 256, 384, 512, 768, 1024, 1536, 2048, 4096]),
             "L1048576": (1048576, [1, 2, 4, 8, 16, 32, 64, 128, 256, 384, 512, 768, 1024, 2048])}
    for name, (L, Fs) in cases.items():
        x = torch.randn((max(Fs), L, 2), device=dev, dtype=torch.float32)
        rows = torch.empty((max(Fs), 512), device=dev, dtype=torch.float32)
        ser = {}
        for F in Fs:
            for path in (1, 2, 3, 4, 5):
                if path == 2 and F * L < (1 << 24):
                    continue  # edge windows dominate tiny batches; not a contender
                with ZoomFFT(4096, 8, 2.4e6, n_win=512) as plan:
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
        # crossovers: the smallest batch from which XA is fastest, and from which path 2 beats 1
        def best(F):
            c = {p: ser.get(f"F{F}_path{p}") for p in (1, 2, 3, 4, 5)}
            return min((v, p) for p, v in c.items() if v is not None)[1]
        xa_from = next((F for F in Fs if all(best(G) == 3 for G in Fs if G >= F)), None)
        res[f"{name}_xa_fastest_from_frames"] = xa_from
        res[f"{name}_best_by_frames"] = {F: best(F) for F in Fs}
        res[f"{name}_walk_vs_tiles"] = {F: round(ser[f"F{F}_path5"] / ser[f"F{F}_path4"], 3) for F in Fs}
        del x, rows
        torch.cuda.empty_cache()
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "series"}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep_schedule.json")
