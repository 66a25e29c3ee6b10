#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into HBM bytes per bench step.

Recipe (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are collected in
separate --pmc passes (they do not fit one pass), both in KiB; on gfx950 FETCH_SIZE
reports exactly half the bytes of a wide coalesced streaming read, so it is doubled
("fetch x2"); WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Other access
widths are uncalibrated; both raw and corrected sums are kept.

Per step = (sum over every zfft dispatch) / (number of Welch row dispatches): each
process call launches exactly one of welch_rows / welch_dif / welch4_rows.

The summary is stamped with the kernel-source hash (bench.py uses it only while the sources
are unchanged).

usage: tools/pmc_traffic.py <fetch_dir> <write_dir> <frames> <config> [out.json] [in_dtype]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypanadapter_amd import build  # noqa: E402


def kname(name: str) -> str:
    m = re.search(r"zfft::(?:xa::|pc::|fc::)?([a-z_0-9]+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def load(d, counter):
    per = defaultdict(float)
    count = defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "zfft::" in r["Kernel_Name"]:
                k = kname(r["Kernel_Name"])
                per[k] += float(r["Counter_Value"])
                count[k] += 1
    return per, count


def main():
    fetch_dir, write_dir, frames, config = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    out = sys.argv[5] if len(sys.argv) > 5 else None
    in_dtype = sys.argv[6] if len(sys.argv) > 6 else "complex64"
    fetch, fc = load(fetch_dir, "FETCH_SIZE")
    write, wc = load(write_dir, "WRITE_SIZE")
    step_kernel = ("welch_rows", "welch_dif", "welch4_rows")
    steps_f = sum(v for k, v in fc.items() if k.startswith(step_kernel))
    steps_w = sum(v for k, v in wc.items() if k.startswith(step_kernel))
    per_kernel = {}
    tot_raw = tot_x2 = 0.0
    for k in sorted(set(fetch) | set(write)):
        f_kib = fetch.get(k, 0.0) / max(steps_f, 1)
        w_kib = write.get(k, 0.0) / max(steps_w, 1)
        per_kernel[k] = {"fetch_KiB_per_step_raw": round(f_kib, 1),
                         "write_KiB_per_step": round(w_kib, 1),
                         "hbm_bytes_per_step_fetch_x2": int((2 * f_kib + w_kib) * 1024)}
        tot_raw += (f_kib + w_kib) * 1024
        tot_x2 += (2 * f_kib + w_kib) * 1024
    res = {"frames": frames, "config": config, "in_dtype": in_dtype,
           "source_hash": build.source_hash(),
           "steps_counted": [steps_f, steps_w],
           "hbm_bytes_per_step": int(tot_x2), "hbm_bytes_per_step_raw": int(tot_raw),
           "per_kernel": per_kernel,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of "
                     "bench.py; FETCH doubled per the gfx950 calibration (calibrated for 16-B-per-lane "
                     "streaming reads: the XA tile loads and the Welch loads are 16 B per lane); "
                     "the raw sum is kept as the lower bound"}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
