#!/usr/bin/env python3
"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (counter_collection.csv):
average per dispatch of each counter, grouped by kernel name.  usage: sq_counters.py <dir>"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"zfft::(?:xa::)?([a-z_0-9]+)(<[^>(]*>)?", r["Kernel_Name"])
        if not m:
            continue
        k = m.group(1) + (m.group(2) or "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k in sorted(acc):
    vals = {c: acc[k][c] / cnt[k][c] for c in acc[k]}
    print(k)
    for c in sorted(vals):
        print(f"   {c:24s} {vals[c]:.4g}")
    wc = vals.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if c in vals:
                print(f"   {c}/WAVE_CYCLES = {vals[c] / wc:.3f}")
