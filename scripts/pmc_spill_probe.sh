#!/bin/bash
# WRITE_SIZE of the headline render launch with the product build and with
# a no-spill build (RT_WAVES_PER_SIMD=2: 183 VGPRs, no scratch), to attribute
# the launch's HBM writes beyond the framebuffer (dev tool).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
RTGO_LIB=concurrent-raytracer-go_amd/build/var_w2/librtgo.so timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/w2_w -o run --output-format csv -- python3 scripts/pmc_workload.py 5 > gpurun_out/pmc/w2_w.log 2>&1
RTGO_LIB=concurrent-raytracer-go_amd/build/var_w2/librtgo.so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/w2_f -o run --output-format csv -- python3 scripts/pmc_workload.py 5 > gpurun_out/pmc/w2_f.log 2>&1
echo spill probe done
