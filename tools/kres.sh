#!/bin/bash
# Per-kernel resource usage (VGPRs, scratch, LDS, occupancy) of one .hip file:
#   bash tools/kres.sh csrc/kernels/hevc_kernels.hip [KERNEL-REGEX]
SRC=$1; PAT=${2:-.}
C=$(cd "$(dirname "$0")/.." && pwd)/csrc
/opt/rocm/bin/hipcc -x hip -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -c "$SRC" -o /dev/null \
    -I"$C" -I"$C/codec" -I"$C/runtime" -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v pat="$PAT" '/Function Name:/ {name=$(NF-1); show = (name ~ pat)} show && /VGPRs:|ScratchSize|Occupancy|LDS Size|Function Name/ {sub(/.*remark: /,""); print}'
