#!/bin/bash
# GPU-box profiling of round NN: rocprofv3 kernel-trace stats of the bench
# commands (c2 headline, c4) and two PMC passes (FETCH_SIZE, WRITE_SIZE) of
# every config's workload, reduced to HBM bytes of its dominant kernel.
# usage: scripts/profile.sh r03   (writes gpurun_out/profiles_r03/*; copy them into profiles/)
set -eu
R=${1:-r03}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/profiles_${R}
mkdir -p $O
# (one frame per launch, one launch in flight: the launches rocprof averages
# are the one-frame launches whose HIP-event time the roofline uses)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_trace -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-e2e --frames-per-launch 1 --frames-in-flight 1 \
  > $O/${R}_bench_under_rocprof.json
cp "$(find gpurun_out/prof_${R}_trace -name '*kernel_stats.csv' | head -1)" $O/${R}_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_c4trace -o run --output-format csv \
  -- python3 bench.py --config c4 --steps 2 --no-cpu-baseline > $O/${R}_c4_bench_under_rocprof.json
cp "$(find gpurun_out/prof_${R}_c4trace -name '*kernel_stats.csv' | head -1)" $O/${R}_c4_kernel_stats.csv
for cfg in c2 c3 c4 c5; do
  n=5; [ $cfg = c4 ] && n=2; [ $cfg = c5 ] && n=1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PMC_CONFIG=$cfg timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${R}_${cfg}_${ctr} -o run \
      --output-format csv -- python3 scripts/pmc_workload.py $n
  done
  python3 scripts/pmc_traffic.py $cfg gpurun_out/pmc_${R}_${cfg}_FETCH_SIZE gpurun_out/pmc_${R}_${cfg}_WRITE_SIZE \
    $O/${R}_pmc_traffic.json $n
done
echo "profile ${R} done"
