#!/bin/bash
# GPU-box: bench.py throughput lines for a list of variants (no CPU baseline,
# no end-to-end probes), one "label value ms_per_step one_frame_kernel_ms"
# line each into gpurun_out/sweep_TAG.txt.
# usage: sweep_bench.sh TAG 'label|bench args' ['label|bench args' ...]
set -u
TAG=$1
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/sweep_$TAG.txt
: > "$O"
for spec in "$@"; do
  label=${spec%%|*}
  args=${spec#*|}
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-e2e $args > gpurun_out/sweep_${TAG}_$label.json \
    2> gpurun_out/sweep_${TAG}_$label.err
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "$label rc=$rc" >> "$O"
    exit $rc
  fi
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('one_frame_in_flight') or {}).get('kernel_ms'))
" gpurun_out/sweep_${TAG}_$label.json "$label" >> "$O"
  tail -1 "$O"
done
