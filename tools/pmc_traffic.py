#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into HBM bytes per zfft launch.

Recipe (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE come from separate
--pmc passes (they do not fit one pass); both are in KiB; on gfx950 FETCH_SIZE reports
exactly half the bytes of a wide coalesced streaming read, so it is doubled here
("fetch_corrected"), WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Other access
widths are uncalibrated, so both raw and corrected figures are written.

usage: tools/pmc_traffic.py <fetch_dir> <write_dir> <frames> <config> [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    for key in ("iir_forward_mix", "iir_forward_fgi", "iir_backward_kernel<true>",
                "iir_backward_kernel<false>", "welch_rows", "waterfall_push", "waterfall_init",
                "waterfall_read", "mix_kernel"):
        if key.split("<")[0] in name and (("<" not in key) or key.split("<")[1].rstrip(">") in name):
            return key
    return name[:60]


def load(d, counter):
    rows = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "zfft" in r["Kernel_Name"]:
                rows[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return rows


def main():
    fetch_dir, write_dir, frames, config = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    out = sys.argv[5] if len(sys.argv) > 5 else None
    fetch = load(fetch_dir, "FETCH_SIZE")
    write = load(write_dir, "WRITE_SIZE")
    per = {}
    total_raw = total_corr = 0.0
    for k in sorted(set(fetch) | set(write)):
        fr = fetch.get(k, [])
        wr = write.get(k, [])
        f_kib = sum(fr) / max(len(fr), 1)
        w_kib = sum(wr) / max(len(wr), 1)
        per[k] = {"dispatches": max(len(fr), len(wr)), "fetch_KiB_raw": round(f_kib, 1),
                  "write_KiB": round(w_kib, 1),
                  "hbm_bytes_raw": int((f_kib + w_kib) * 1024),
                  "hbm_bytes_fetch_x2": int((2 * f_kib + w_kib) * 1024)}
    # per step: sum over the distinct launches of one step (dispatch counts per step differ
    # only for kernels launched several times per step: iir_forward_fgi / iir_backward)
    res = {"frames": frames, "config": config, "per_kernel_avg_dispatch": per,
           "note": "FETCH doubled per the gfx950 calibration; per-step = sum over one step's "
                   "launches (see launches_per_step)"}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))
    _ = (total_raw, total_corr)


if __name__ == "__main__":
    main()
