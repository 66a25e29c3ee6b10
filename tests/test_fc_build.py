"""CPU check of the FC kernel's register budget (fc_kernels.hip): every
fc_decim_kernel<Z, dtype, flip> instantiation compiles for gfx950 without VGPR spills or scratch
at its launch bound (256 threads, two workgroups per CU).  fc_hold() keeps as many of the
filter-table pairs in registers as each instantiation holds without spilling; a change that makes
one spill (a larger hold, more live values in a pass) fails here before it reaches a GPU."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pypanadapter_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _resource_usage(tmp_path):
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    out = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", CSRC,
                          "-I", os.path.join(ROOT, "include"), "--cuda-device-only", "-c",
                          os.path.join(CSRC, "fc_kernels.hip"), "-o", str(tmp_path / "fc.o"),
                          "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    usage, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            usage[name] = {}
            continue
        m = re.search(r"(VGPRs Spill|SGPRs Spill|VGPRs|ScratchSize \[bytes/lane\]): (\d+)", line)
        if m and name:
            usage[name][m.group(1)] = int(m.group(2))
    return {k: v for k, v in usage.items() if "fc_decim_kernel" in k}


def test_fc_decim_instantiations_do_not_spill(tmp_path):
    usage = _resource_usage(tmp_path)
    assert len(usage) == 16, sorted(usage)     # zoom {8, 4} x 4 input formats x 2 flips
    for name, u in usage.items():
        assert u.get("VGPRs Spill") == 0 and u.get("SGPRs Spill") == 0, (name, u)
        assert u.get("ScratchSize [bytes/lane]") == 0, (name, u)
        assert 0 < u.get("VGPRs", 0) <= 256, (name, u)
