#!/bin/bash
# GPU-box: PMC HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the headline
# workload's render kernel, one frame per launch.  usage: scripts/pmc_c2.sh TAG
set -eu
TAG=${1:-r04}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_${TAG}
for ctr in FETCH_SIZE WRITE_SIZE; do
  PMC_CONFIG=c2 timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_c2_${ctr} -o run \
    --output-format csv -- python3 scripts/pmc_workload.py 5
done
python3 scripts/pmc_traffic.py c2 gpurun_out/pmc_${TAG}_c2_FETCH_SIZE gpurun_out/pmc_${TAG}_c2_WRITE_SIZE \
  gpurun_out/pmc_${TAG}/${TAG}_pmc_traffic_c2.json 5
cat gpurun_out/pmc_${TAG}/${TAG}_pmc_traffic_c2.json
