#!/usr/bin/env python3
"""Build A/B variants of libzfft.so (kernel build knobs) into pypanadapter_amd/lib/variants/;
run one with ZFFT_LIB_PATH=<path> python bench.py ...   usage: build_variants.py NAME=D1,D2 ...
Every variant is a diagnostic build (-DZFFT_DIAG: the knobs XA_STAMPS, XA_EXP, PC_KO exist only
there; the shipped library never has them)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pypanadapter_amd import build  # noqa: E402


def one(spec):
    name, _, defs = spec.partition("=")
    out = os.path.join(build.LIB_DIR, "variants", f"libzfft_{name}.so")
    build.build(out=out, defines=("ZFFT_DIAG",) + tuple(d for d in defs.split(",") if d))
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for p in ex.map(one, sys.argv[1:]):
            print(p)
