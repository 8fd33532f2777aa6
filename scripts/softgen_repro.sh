#!/bin/bash
# Builds and runs scripts/softgen_repro.hip (the wf_softgen queue-write
# repro) and keeps the ISA of both loops under gpurun_out/softgen_isa.
set -eu
cd "$(dirname "$0")"
mkdir -p ../gpurun_out/softgen_isa
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I ../include -I ../concurrent-raytracer-go_amd/csrc \
  --save-temps softgen_repro.hip -o ../gpurun_out/softgen_isa/softgen_repro 2> /dev/null
mv softgen_repro-hip-amdgcn-amd-amdhsa-gfx950.s ../gpurun_out/softgen_isa/ 2>/dev/null || true
rm -f softgen_repro-hip-* softgen_repro-host-*
timeout -k 10 120 ../gpurun_out/softgen_isa/softgen_repro
