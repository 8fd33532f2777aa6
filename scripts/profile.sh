#!/bin/bash
# GPU-box profiling of round NN: kernel-trace stats of the bench command and
# two PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench workload.
# usage: scripts/profile.sh r01   (writes gpurun_out/prof_r01*; copy gpurun_out/profiles_r01/* into profiles/)
set -eu
R=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles_${R}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_trace -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-e2e > gpurun_out/prof_${R}_bench.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${R}_fetch -o run --output-format csv \
  -- python3 scripts/pmc_workload.py 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${R}_write -o run --output-format csv \
  -- python3 scripts/pmc_workload.py 5
python3 scripts/pmc_traffic.py gpurun_out/prof_${R}_fetch gpurun_out/prof_${R}_write gpurun_out/profiles_${R}/${R}_pmc_traffic.json
cp "$(find gpurun_out/prof_${R}_trace -name '*kernel_stats.csv' | head -1)" gpurun_out/profiles_${R}/${R}_kernel_stats.csv
cp gpurun_out/prof_${R}_bench.json gpurun_out/profiles_${R}/${R}_bench_under_rocprof.json
echo "profile ${R} done"
