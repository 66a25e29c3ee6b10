#!/usr/bin/env python3
"""VALU census of the zoom-8 walk (pc_walk_kernel<DT, FLIP, 8>), per phase and per class
(VERDICT r05 item 1).

Builds pc_kernels.hip to gfx950 assembly (device only, the product's flags plus
`-DZFFT_DIAG -DPC_CENSUS`, which makes every sub-tile take the interior ("fast") path so the
frame-edge code is dead and the listing is the steady-state tile), cuts the tile loop at its
s_barrier instructions into the walk's phases, classifies every VALU instruction, and
multiplies each phase by its trip count (the FIR sub-tile loop runs SUB = 4 times per tile).

Per input sample: lane-instructions = wave-instructions x 4 waves x 64 lanes / 16384 input
samples per tile, times ntiles x 16384 / L for the bench frame (19 tiles for L = 299,008).
The dynamic total is checked against SQ_INSTS_VALU per dispatch / (frames x 4 waves x ntiles).

usage: tools/isa_census.py [--asm FILE.s] [--dt 0] [--flip 0] [--defines A=1,B] [--json OUT]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter, OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pypanadapter_amd", "csrc")

# phase names of the zoom-8 tile loop in barrier order (pc_kernels.hip, pc_walk_kernel):
# the sub-tile loop (x SUB) has 4 barriers, the rest of the tile 10
SUB_PHASES = ["load+LO mix+x to LDS", "FIR alpha reads", "FIR alpha + y1 to LDS",
              "FIR beta + y2 to LDS"]
TILE_PHASES = ["causal sec 0 (run+scan)", "causal sec 0 fix + sec 1 (run+scan)",
               "causal sec 1 fix + store", "cz read",
               "anticausal sec 0 (run+scan)", "anticausal sec 0 fix + sec 1",
               "anticausal sec 1 fix + store", "FIR gamma", "output-rate sections",
               "stores + loop"]

CLASSES = ["pk_fma", "pk_mul/add", "fma/mul/add f32", "dpp move", "readlane/writelane",
           "mov", "cndmask", "cmp", "cvt", "int/addr", "other valu"]


def classify(op: str, line: str) -> str | None:
    """VALU class of one instruction, None for non-VALU (SALU, LDS, VMEM, SMEM, waits)."""
    if not op.startswith("v_"):
        return None
    if op.startswith("v_pk_fma"):
        return "pk_fma"
    if op.startswith(("v_pk_mul", "v_pk_add")):
        return "pk_mul/add"
    if re.match(r"v_(fma|fmac|mul|add|sub|subrev|mac)_f32", op):
        return "fma/mul/add f32"
    if "_dpp" in op or " row_" in line or "wave_sh" in line or "quad_perm" in line:
        return "dpp move"
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "readlane/writelane"
    if op.startswith("v_mov"):
        return "mov"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith("v_cmp"):
        return "cmp"
    if op.startswith("v_cvt"):
        return "cvt"
    if re.match(r"v_(lshl|lshr|ashr|and|or|xor|add|sub|mad|mul_lo|mul_hi|bfe|bfi|alignbit)", op):
        return "int/addr"
    return "other valu"


def build_asm(defines: list[str]) -> str:
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    out = os.path.join(tempfile.mkdtemp(prefix="census_"), "pc.s")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
           "-I", CSRC, "--cuda-device-only", "-S", os.path.join(CSRC, "pc_kernels.hip"), "-o", out]
    cmd += [f"-D{d}" for d in defines]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return out


def kernel_lines(asm: str, dt: int, flip: int, zoom: int = 8) -> list[str]:
    sym = f"_ZN4zfft2pc14pc_walk_kernelILi{dt}ELi{flip}ELi{zoom}E"
    lines = open(asm).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) and l.split(":")[0].endswith("E"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def census(lines: list[str]) -> dict:
    # loop structure from the compiler's block comments
    hdr2 = next(i for i, l in enumerate(lines) if re.search(r"This (Inner )?Loop Header: Depth=2", l))
    if not lines[hdr2].startswith(".L"):  # the comment continues the label's line
        hdr2 -= 1
    bb2 = re.search(r"(BB\d+_\d+)", lines[hdr2]).group(1)
    bb1 = re.search(r"Parent Loop (BB\d+_\d+)", lines[hdr2] + lines[hdr2 + 1]).group(1)
    hdr1 = next(i for i, l in enumerate(lines) if l.startswith(".L" + bb1 + ":"))
    # blocks: label line indices
    labels = [i for i, l in enumerate(lines) if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", l)]
    def block_end(i):
        nxt = [j for j in labels if j > i]
        return nxt[0] if nxt else len(lines)
    in_loop1, in_loop2 = [], []
    for i in labels:
        blk = lines[i] + lines[i + 1] if i + 1 < len(lines) else lines[i]
        if i == hdr1 or f"Header={bb1}" in blk or f"Parent Loop {bb1}" in blk:
            in_loop1.append(i)
        if i == hdr2 or f"Header={bb2}" in blk:
            in_loop2.append(i)
    # also the block that jumps back to the sub-tile header (its latch) is "in Loop: Header=bb2"
    sub_ranges = [(i, block_end(i)) for i in in_loop2]
    tile_ranges = [(i, block_end(i)) for i in sorted(set(in_loop1) | {hdr1})]
    sub_lines = sorted(set(j for a, b in sub_ranges for j in range(a, b)))
    tile_lines = sorted(set(j for a, b in tile_ranges for j in range(a, b)) - set(sub_lines))

    def segs(idx, names):
        out = OrderedDict((n, Counter()) for n in names)
        k = 0
        extra = Counter()
        for j in idx:
            l = lines[j].strip()
            if not l or l.startswith((";", ".")):
                continue
            op = l.split()[0]
            if op == "s_barrier":
                k += 1
                continue
            c = classify(op, l)
            if c is None:
                continue
            if k < len(names):
                out[names[k]][c] += 1
            else:
                extra[c] += 1
        return out, k, extra

    # the sub-tile loop's body in textual order starts at its header; rotate so the phase after
    # the loop-closing barrier (the latch, placed before the header) comes last
    lat = [j for j in sub_lines if j < hdr2]
    body = [j for j in sub_lines if j >= hdr2] + lat
    sub, nb_sub, sub_extra = segs(body, SUB_PHASES)
    # tile loop: from its header past the sub-tile loop, then the latch block placed before it
    t_after = [j for j in tile_lines if j >= hdr1]
    t_before = [j for j in tile_lines if j < hdr1]
    pre = [j for j in t_after if j < hdr2]
    post = [j for j in t_after if j > hdr2]
    tile, nb_tile, tile_extra = segs(post + t_before + pre, TILE_PHASES)
    return {"sub": sub, "tile": tile, "sub_barriers": nb_sub, "tile_barriers": nb_tile,
            "sub_unassigned": sub_extra, "tile_unassigned": tile_extra}


def report(c: dict, sub_trips: int = 4, L: int = 299008, ntiles: int = 19) -> dict:
    per_sample = 4 * 64 / 16384.0 * (ntiles * 16384.0 / L)
    rows = []
    tot = Counter()
    for name, cnt in c["sub"].items():
        rows.append((f"[x{sub_trips}] {name}", cnt, sub_trips))
        for k, v in cnt.items():
            tot[k] += v * sub_trips
    for name, cnt in c["tile"].items():
        rows.append((name, cnt, 1))
        for k, v in cnt.items():
            tot[k] += v
    hdr = f"{'phase':44s} {'wave-instr/tile':>15s} {'lane-instr/sample':>17s}  " + "  ".join(
        f"{k[:10]:>10s}" for k in CLASSES)
    print(hdr)
    out = {"phases": {}, "classes_per_sample": {}, "total_per_tile": 0, "total_per_sample": 0.0}
    for name, cnt, trips in rows:
        n = sum(cnt.values()) * trips
        print(f"{name:44s} {n:15d} {n * per_sample:17.2f}  " + "  ".join(
            f"{cnt.get(k, 0) * trips * per_sample:10.2f}" for k in CLASSES))
        out["phases"][name] = {"per_tile": n, "per_sample": round(n * per_sample, 3),
                               "classes": {k: cnt.get(k, 0) * trips for k in CLASSES if cnt.get(k)}}
    n = sum(tot.values())
    print(f"{'TOTAL':44s} {n:15d} {n * per_sample:17.2f}  " + "  ".join(
        f"{tot.get(k, 0) * per_sample:10.2f}" for k in CLASSES))
    out["total_per_tile"] = n
    out["total_per_sample"] = round(n * per_sample, 3)
    out["classes_per_sample"] = {k: round(tot.get(k, 0) * per_sample, 3) for k in CLASSES}
    out["barriers"] = {"sub": c["sub_barriers"], "tile": c["tile_barriers"]}
    if c["sub_unassigned"] or c["tile_unassigned"]:
        print("unassigned:", dict(c["sub_unassigned"]), dict(c["tile_unassigned"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--dt", type=int, default=0)
    ap.add_argument("--flip", type=int, default=0)
    ap.add_argument("--defines", default="")
    ap.add_argument("--json")
    a = ap.parse_args()
    asm = a.asm or build_asm(["ZFFT_DIAG", "PC_CENSUS"] + [d for d in a.defines.split(",") if d])
    c = census(kernel_lines(asm, a.dt, a.flip))
    r = report(c)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(r, fh, indent=1)


if __name__ == "__main__":
    sys.exit(main())
