#!/bin/bash
# GPU-box profiling of round NN: rocprofv3 kernel-trace stats of the bench
# commands and PMC passes (FETCH_SIZE, WRITE_SIZE) of every config's
# workload, reduced to HBM bytes of its dominant kernel.
# usage: scripts/profile.sh r05   (writes gpurun_out/profiles_r05/*; copy them into profiles/)
#   PROFILE_PARTS="driver onefr c4 pmc"  (default: all four); PMC_CONFIGS="c2 c2b c3 c4 c5" (default)
set -eu
R=${1:-r05}
PARTS=${PROFILE_PARTS:-driver onefr c4 pmc}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/profiles_${R}
mkdir -p $O
has() { case " $PARTS " in *" $1 "*) return 0 ;; esac; return 1; }
if has driver; then
  # the driver's own command, unmodified: its timed launches (batched frames,
  # launches in flight) are the ones the line's value and roofline describe
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_driver -o run --output-format csv \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${R}_driver_bench_under_rocprof.json
  cp "$(find gpurun_out/prof_${R}_driver -name '*kernel_stats.csv' | head -1)" $O/${R}_driver_kernel_stats.csv
  python3 scripts/batched_trace.py gpurun_out/prof_${R}_driver $O/${R}_driver_bench_under_rocprof.json \
    $O/${R}_driver_batched_trace.json
fi
if has onefr; then
  # one frame per launch, one launch in flight: the launches whose HIP-event
  # time the roofline's kernel_ms uses
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_trace -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-e2e --frames-per-launch 1 --frames-in-flight 1 \
    > $O/${R}_bench_under_rocprof.json
  cp "$(find gpurun_out/prof_${R}_trace -name '*kernel_stats.csv' | head -1)" $O/${R}_kernel_stats.csv
fi
if has c4; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_c4trace -o run --output-format csv \
    -- python3 bench.py --config c4 --steps 2 --no-cpu-baseline > $O/${R}_c4_bench_under_rocprof.json
  cp "$(find gpurun_out/prof_${R}_c4trace -name '*kernel_stats.csv' | head -1)" $O/${R}_c4_kernel_stats.csv
fi
if has pmc; then
  for cfg in ${PMC_CONFIGS:-c2 c2b c3 c4 c5}; do
    c=$cfg; n=5; fpl=1
    [ $cfg = c2b ] && { c=c2; n=2; fpl=10; }
    [ $cfg = c4 ] && n=2
    [ $cfg = c5 ] && n=1
    for ctr in FETCH_SIZE WRITE_SIZE; do
      PMC_CONFIG=$c PMC_FRAMES=$fpl timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${R}_${cfg}_${ctr} \
        -o run --output-format csv -- python3 scripts/pmc_workload.py $n
    done
    python3 scripts/pmc_traffic.py $c gpurun_out/pmc_${R}_${cfg}_FETCH_SIZE gpurun_out/pmc_${R}_${cfg}_WRITE_SIZE \
      $O/${R}_pmc_traffic.json $n $fpl
  done
fi
echo "profile ${R} done"
