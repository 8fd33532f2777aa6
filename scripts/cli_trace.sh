#!/bin/bash
# GPU-box: where the drop-in CLI's first Render goes (a fresh process per
# frame, like cmd/raytracer/main.go:46-51).  Three plain runs (their
# benchmark_data.json), then one under rocprofv3 with the HIP API, kernel and
# memory-copy traces (no counters).  usage: scripts/cli_trace.sh [TAG]
# -> gpurun_out/cli_trace_TAG/{run*.json, trace/...csv}
set -eu
TAG=${1:-r04}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/cli_trace_${TAG}
mkdir -p $O
EXE=concurrent-raytracer-go_amd/build/raytracer
SCENE=scenes/sphere_reflections_light_facing.json
for i in 1 2 3; do
  s=$(date +%s.%N)
  timeout -k 10 60 $EXE $SCENE $O/out$i.png 800 600 > $O/stdout$i.txt
  e=$(date +%s.%N)
  python3 - "$O/benchmark_data.json" "$O/run$i.json" "$s" "$e" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
d["process_wall_s"] = float(sys.argv[4]) - float(sys.argv[3])
json.dump(d, open(sys.argv[2], "w"), indent=1)
print(sys.argv[2], d["render_time_seconds"], d.get("render_breakdown_seconds"), d["process_wall_s"])
EOF
done
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv \
  -- $EXE $SCENE $O/out_traced.png 800 600 > $O/stdout_traced.txt
cp $O/benchmark_data.json $O/run_traced.json
echo "cli trace ${TAG} done"
