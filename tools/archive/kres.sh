#!/bin/bash
# per-kernel VGPR / AGPR / scratch / occupancy / LDS of a .hip file (our kernels only)
f=$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math --cuda-device-only -c -o /tmp/kres.o "$f" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -v rocprim | grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size" \
  | sed -E 's/.*remark: //; s/ \[-Rpass.*//; s/^ +//' | paste -d'|' - - - - - - | sed -E 's/Function Name: _ZN5prgpu[0-9]*//'
