#!/bin/bash
# Dev tool (runs HERE, not on the box): retry gpurun only on infrastructure transients
# (status=transient: nothing ran, nothing charged), after the backoff it names.
# usage: gpu_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6; do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > "$OUT" 2>&1
  if grep -q "status=transient" "$OUT"; then
    w=$(grep -o "retry in [0-9]*s" "$OUT" | grep -o "[0-9]*" | head -1)
    w=${w:-120}
    echo "transient (try $i), waiting $((w + 10))s" >> "$OUT.log"
    sleep $((w + 10))
    continue
  fi
  break
done
