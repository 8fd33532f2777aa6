#!/bin/bash
# GPU-box: the driver's command (--steps 20 --warmup 5) under schedule
# tunings (rt_tuning: no tuning changes an output bit), twice each; one JSON
# line per run into gpurun_out/k20_tuning.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/k20_tuning.jsonl
: > $O
run() {
  local tag="$1"; shift
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${K20_EXTRA:-} --no-cpu-baseline --no-e2e "$@" \
    > gpurun_out/k20_tmp.log 2>&1 || return $?
  python3 -c "
import json
l=[x for x in open('gpurun_out/k20_tmp.log') if x.startswith('{')][-1]
d=json.loads(l); print(json.dumps({'tag':'$tag','value':d['value'],'ms_per_step':d['ms_per_step'],'check':d.get('check_equals_oracle')}))" >> $O
  tail -1 $O
}
for i in 1 2; do
  run default || exit $?
  [ -n "${K20_ALSO100:-}" ] && { run "default k100" --steps 100 || exit $?; }
  for t in ${K20_TUNINGS:-block_work=1536 block_work=2048 block_work=3072 block_work=4096 \
           block_work=2048,measure=1 block_work=3072,measure=1 block_work=2048,block_samples=2048}; do
    run "$t" --tuning "$t" || exit $?
    [ -n "${K20_ALSO100:-}" ] && { run "$t k100" --tuning "$t" --steps 100 || exit $?; }
  done
done
