#!/bin/bash
# Per-kernel VGPR / spill / LDS usage of the gfx950 build (compile-only, no GPU).
SRC="$(cd "$(dirname "$0")/.." && pwd)/yacy_search_server_amd/csrc/yrwi_kernels.hip"
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -c "$SRC" \
  -o /tmp/yrwi_kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name:/ {n=$NF} / VGPRs:/ {v=$NF} /VGPRs Spill:/ {sp=$NF} /LDS Size/ {printf "%-70s vgpr=%s spill=%s lds=%s\n", substr(n,1,70), v, sp, $NF}'
