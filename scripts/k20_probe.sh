#!/bin/bash
# GPU-box: the driver's command (--steps 20 --warmup 5) against --steps 100,
# and K = 20 under other launch shapes (frames per launch x launches in
# flight), each twice; one JSON line per run into gpurun_out/k20_probe.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/k20_probe.jsonl
: > $O
run() {
  local tag="$1"; shift
  timeout -k 10 120 python3 bench.py --gpus 1 --no-cpu-baseline --no-e2e "$@" > gpurun_out/k20_tmp.log 2>&1 || return $?
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/k20_tmp.log') if x.startswith('{')][-1]
d=json.loads(l); print(json.dumps({'tag':'$tag','value':d['value'],'ms_per_step':d['ms_per_step'],'launch_frames':d.get('launch_frames')}))" >> $O
  tail -1 $O
}
for i in 1 2 3; do
  run driver --steps 20 --warmup 5 || exit $?
  run k100 --steps 100 --warmup 5 || exit $?
  run k20_f3 --steps 20 --warmup 5 --frames-in-flight 3 || exit $?
  run k100_f3 --steps 100 --warmup 5 --frames-in-flight 3 || exit $?
  run k20_f1x20 --steps 20 --warmup 5 --frames-in-flight 1 --frames-per-launch 20 || exit $?
done
