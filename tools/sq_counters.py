#!/usr/bin/env python3
"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (counter_collection.csv), stamped
with the kernel-source hash so bench.py uses it only while the sources are unchanged.

Counters (one pass: 8 SQ + 1 GRBM): SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_ACTIVE_INST_VALU,
SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_INSTS_VALU, SQ_LDS_BANK_CONFLICT,
GRBM_GUI_ACTIVE.  SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles summed over
waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, rocprofv3 section and
the per-instruction table).  Derived per dispatch:
  valu_busy      = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE / 8): the share of
                   SIMD cycles in which a VALU instruction issued (the gfx9 VALUBusy formula)
  waves_per_simd = 4 * SQ_WAVE_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8): resident waves
  wave_valu      = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: one wave's VALU issue share
  wave_wait      = SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier),
  wave_stall     = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls)
  valu_per_tile  = SQ_INSTS_VALU / (frames * samples / 2048) for the stage-0 kernel (its input
                   is the frame: `samples` per frame, 2048-sample tiles; SQ_INSTS_VALU counts
                   wave instructions)

usage: sq_counters.py <dir> [frames config in_dtype out.json [samples_per_frame]]
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

SIMDS = 1024
XCDS = 8


def kname(name):
    m = re.search(r"zfft::(?:xa::|pc::|fc::)?([a-z_0-9]+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else None


def summarise(d):
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[k][r["Counter_Name"]] += 1
    out = {}
    for k in sorted(acc):
        v = {c: acc[k][c] / cnt[k][c] for c in acc[k]}
        g = v.get("GRBM_GUI_ACTIVE")
        wc = v.get("SQ_WAVE_CYCLES")
        if g and "SQ_ACTIVE_INST_VALU" in v:
            v["valu_busy"] = round(4 * v["SQ_ACTIVE_INST_VALU"] / (SIMDS * g / XCDS), 4)
        if g and wc:
            v["waves_per_simd"] = round(4 * wc / (SIMDS * g / XCDS), 3)
        if wc:
            for c, nm in (("SQ_ACTIVE_INST_VALU", "wave_valu"), ("SQ_WAIT_ANY", "wave_wait"),
                          ("SQ_WAIT_INST_ANY", "wave_stall"), ("SQ_ACTIVE_INST_ANY", "wave_any")):
                if c in v:
                    v[nm] = round(v[c] / wc, 4)
        out[k] = v
    return out


def main():
    d = sys.argv[1]
    per = summarise(d)
    res = {"source_hash": build.source_hash(), "per_kernel": per,
           "method": __doc__.split("usage:")[0].strip()}
    if len(sys.argv) > 4:
        res.update(frames=int(sys.argv[2]), config=sys.argv[3], in_dtype=sys.argv[4])
    if len(sys.argv) > 6:
        frames, samples = int(sys.argv[2]), int(sys.argv[6])
        for k, v in per.items():
            if k.startswith("xa_stage_kernel<32, true") and "SQ_INSTS_VALU" in v:
                v["valu_per_tile"] = round(v["SQ_INSTS_VALU"] / (frames * samples / 2048), 1)
    if len(sys.argv) > 5:
        json.dump(res, open(sys.argv[5], "w"), indent=1)
    for k, v in per.items():
        print(k, {c: v[c] for c in ("valu_busy", "waves_per_simd", "wave_valu", "wave_wait",
                                    "wave_stall", "valu_per_tile") if c in v})


if __name__ == "__main__":
    main()
