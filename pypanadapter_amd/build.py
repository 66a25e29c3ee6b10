"""Build libzfft.so in-tree with hipcc for gfx950 (no JIT cache, so it travels with gpurun)."""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libzfft.so")
SOURCES = ["zfft_kernels.hip", "xa_kernels.hip", "pc_kernels.hip", "fc_kernels.hip", "zfft_plan.cpp",
           "pc_tables.cpp", "zfft_ring.cpp", "windows.cpp"]
HEADERS = ["zfft_internal.h", "zfft_device.h", "zfft_fft.h", "zfft_pairs.h", "cheby1_q2.h", "pc_edge_maps.h", os.path.join("..", "..", "include", "zfft.h")]
ARCH = os.environ.get("ZFFT_OFFLOAD_ARCH", "gfx950")


def _newest_input_mtime() -> float:
    paths = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return max(os.path.getmtime(p) for p in paths)


def needs_build() -> bool:
    """The shipped .so is missing, or was built from other sources, for another arch or with
    build knobs (the record build() keeps next to it; file times when there is none)."""
    if not os.path.exists(LIB_PATH):
        return True
    info = build_info()
    if info.get("source_hash"):
        return (info["source_hash"] != source_hash() or info.get("arch") != ARCH
                or bool(info.get("defines")))
    return os.path.getmtime(LIB_PATH) < _newest_input_mtime()


def build(force: bool = False, verbose: bool = False, out: str = LIB_PATH,
          defines: tuple = ()) -> str:
    """hipcc all sources into `out`; `defines` ("NAME=VALUE", ...) select kernel build knobs
    (A/B variants written elsewhere than the shipped LIB_PATH); an entry starting with "-" is
    passed to hipcc as it is (e.g. "-mllvm", "-amdgpu-sched-strategy=max-ilp")."""
    if not force and not defines and out == LIB_PATH and not needs_build():
        return LIB_PATH
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    tmp = out + ".tmp"
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-Wall", "-I", os.path.join(ROOT, "include"), "-I", CSRC]
    flags += [d if d.startswith("-") else f"-D{d}" for d in defines]
    with tempfile.TemporaryDirectory(prefix="zfft_build_") as td:
        # one object per source, compiled in parallel (the kernel files dominate), then linked
        def obj(s):
            o = os.path.join(td, s + ".o")
            cmd = [hipcc, *flags, "-c", os.path.join(CSRC, s), "-o", o]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
            return o
        with ThreadPoolExecutor(min(len(SOURCES), os.cpu_count() or 1)) as ex:
            objs = list(ex.map(obj, SOURCES))
        subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp],
                       check=True)
    os.replace(tmp, out)
    if out == LIB_PATH:  # a knob build there is recorded as such: the next build() replaces it
        _write_build_info(defines)
    return out


INFO_PATH = os.path.join(LIB_DIR, "build_info.json")


def _git(*args):
    try:
        r = subprocess.run(["git", "-C", ROOT, *args], capture_output=True, text=True, timeout=10)
        return r.stdout.strip() if r.returncode == 0 else None
    except (OSError, subprocess.SubprocessError):
        return None


def _write_build_info(defines: tuple = ()) -> None:
    """Next to the shipped .so (it travels with it; the GPU box has no .git): the source hash,
    git commit, arch and build knobs it was built from, so a bench line can name them."""
    import json
    st = _git("status", "--porcelain", "--untracked-files=no")
    info = {"source_hash": source_hash(), "git_head": _git("rev-parse", "HEAD"),
            "git_dirty": None if st is None else bool(st), "arch": ARCH,
            "defines": list(defines)}
    with open(INFO_PATH, "w") as fh:
        json.dump(info, fh)


def build_info() -> dict:
    import json
    try:
        with open(INFO_PATH) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def source_hash() -> str:
    """Digest of the kernel/library sources: profiles measured on other sources (PMC traffic,
    SQ counters) are stamped with it, and bench.py uses them only while it still matches."""
    import hashlib
    h = hashlib.sha256()
    for name in sorted(SOURCES + HEADERS):
        with open(os.path.join(CSRC, name), "rb") as fh:
            h.update(name.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(build(force=True, verbose=True))
