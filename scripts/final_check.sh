#!/bin/bash
# GPU-box: the round-end sequence the driver runs, in order and bounded:
# smoke(), the default bench (N=1), then the driver's command.
# usage: scripts/final_check.sh TAG  (writes gpurun_out/TAG_*)
set -eu
TAG=${1:-final}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.json 2> gpurun_out/${TAG}_bench_driver.err
echo done
