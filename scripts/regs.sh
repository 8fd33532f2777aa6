#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy of a HIP source (dev tool).
# usage: scripts/regs.sh concurrent-raytracer-go_amd/csrc/rt_wavefront.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics -x hip -c "$1" \
  -o /tmp/regs.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: [^ ]+ +//; s/ \[-Rpass.*//' | paste - - - -
