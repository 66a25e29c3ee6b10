#!/bin/bash
# Register / spill / LDS report of the XA stage kernels for a set of -D knobs (CPU only):
#   tools/xa_resources.sh [-DNAME=VALUE ...]
R="$(cd "$(dirname "$0")/.." && pwd)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I "$R/include" -I "$R/pypanadapter_amd/csrc" \
  --cuda-device-only -c -o /dev/null "$@" -Rpass-analysis=kernel-resource-usage \
  "$R/pypanadapter_amd/csrc/xa_kernels.hip" 2>&1 |
  awk '/Function Name: _ZN4zfft2xa15xa_stage_kernelILi32ELb[01]ELi0ELi0E/ {p=1; print; next}
       /Function Name/ {p=0} p && /VGPRs:|Spill|Occupancy|LDS Size|SGPRs:|ScratchSize/ {print}'
