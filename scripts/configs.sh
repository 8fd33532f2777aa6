#!/bin/bash
# GPU-box: one bench line per BASELINE config (c1 as committed, c2 headline,
# c3, c4, c5 on one GPU) with their CPU baselines, into gpurun_out/TAG_configs.jsonl
set -eu
TAG=${1:-r05}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/${TAG}_configs.jsonl
: > $O
for cfg in c2_committed c2 c3 c4 c5; do
  echo "== $cfg"
  timeout -k 10 400 python3 bench.py --config $cfg > gpurun_out/${TAG}_$cfg.log 2> gpurun_out/${TAG}_$cfg.err
  grep '^{' gpurun_out/${TAG}_$cfg.log | tail -1 >> $O
  tail -c 300 $O
done
