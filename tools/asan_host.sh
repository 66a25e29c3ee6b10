#!/bin/bash
# Host-code AddressSanitizer run (CPU only, no GPU): libzfft.so rebuilt with ASan on the
# host side only (-Xarch_host; device code untouched), loaded into the CPU test suites that
# drive host code -- the IQ ring (zfft_ring.cpp), native windows (windows.cpp), plan
# validation / error paths and the exports (zfft_plan.cpp host side).
# usage: tools/asan_host.sh [pytest args]     (log: gpurun_out/asan_host.log)
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
LIB=pypanadapter_amd/lib/variants/libzfft_asan.so
python3 -c "
import sys; sys.path.insert(0, '.')
from pypanadapter_amd import build
build.build(out='$LIB', defines=('-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fno-omit-frame-pointer', '-g'))"
ASAN_LIB=$(gcc -print-file-name=libasan.so)
mkdir -p gpurun_out
# python itself is not instrumented: preload the runtime, no leak check (CPython's arenas)
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 LD_PRELOAD="$ASAN_LIB" ZFFT_LIB_PATH="$LIB" \
  python3 -m pytest tests/test_ring.py tests/test_ring_golden.py tests/test_host.py -m "not gpu" -q \
  -p no:cacheprovider "$@" 2>&1 | tee gpurun_out/asan_host.log
