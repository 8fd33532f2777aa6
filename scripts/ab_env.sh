#!/bin/bash
# A/B of environment settings on one config (dev tool):
#   scripts/ab_env.sh CONFIG "ENV=.. ENV2=.." "ENV=.." ...
# (each setting in its own process; RTGO_X=1 is a no-op placeholder)
cfg=$1; shift
for e in "$@"; do
  echo "### $e"
  env $e timeout -k 10 60 python scripts/bench_configs.py --only "$cfg" --reps 5 | grep config
done
