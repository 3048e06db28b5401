#!/bin/bash
# Register / LDS / scratch (spill) usage of every engine kernel for gfx950, from the compiler's
# kernel-resource-usage remarks.  Usage: tools/kernel_resources.sh > profiles/<round>_kernel_resources.txt
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC --cuda-device-only -c \
  -Iinclude -Iartis_amd/csrc/engine artis_amd/csrc/engine/engine.hip -o /dev/null \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "remark: .*(Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size|SGPRs:)" |
  sed -E 's/^.*remark: //' |
  awk '/Function Name/ {printf "\n%s", $0; next} {printf " | %s", $0} END {print ""}'
