#!/bin/bash
# Build an experiment variant of librtgo.so (dev tool): the kernel sources
# recompiled with extra defines, linked with the host objects of the main
# build.  usage: scripts/build_variant.sh NAME "-DFOO -DBAR=2" [PATCH ...]
# -> concurrent-raytracer-go_amd/build/var_NAME/librtgo.so (time it with
#    scripts/ab_bench.py or RTGO_LIB=... python bench.py)
# PATCH: a name under scripts/variants/ (e.g. no_soft, fastdiv, cheap_rng,
# free_skip, no_soft_trace, no_soft_norm).  The image-changing timing
# experiments live ONLY as these patches: they are applied to a scratch copy
# of csrc/ and include/, so the product sources never carry them.
# VARIANT_SRC=DIR compiles the .hip files from DIR (a patched copy of csrc/)
# instead, so the in-tree sources and build stay untouched.
set -eu
NAME=$1
DEFS=${2:-}
shift $(( $# >= 2 ? 2 : $# ))
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT/concurrent-raytracer-go_amd"
make -s -j8 >/dev/null
OUT=build/var_$NAME
mkdir -p "$OUT"
HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function -munsafe-fp-atomics"
SRC=${VARIANT_SRC:-csrc}
if [ $# -gt 0 ]; then
  # scratch tree with the repo's layout (csrc includes ../../include/...)
  SCR=$(mktemp -d)
  mkdir -p "$SCR/concurrent-raytracer-go_amd"
  cp -r "$ROOT/include" "$SCR/include"
  cp -r "$SRC" "$SCR/concurrent-raytracer-go_amd/csrc"
  for p in "$@"; do
    patch -s -p1 -d "$SCR" < "$ROOT/scripts/variants/$p.patch"
  done
  SRC="$SCR/concurrent-raytracer-go_amd/csrc"
fi
for k in rt_kernel rt_wavefront rt_schedule; do
  /opt/rocm/bin/hipcc $HIPFLAGS $DEFS -I"$SRC" -x hip -c $SRC/$k.hip -o "$OUT/$k.o" &
done
wait
OBJS="$OUT/rt_kernel.o $OUT/rt_wavefront.o $OUT/rt_schedule.o"
for o in rt_api scene_json image_io bvh schedule rt_multi scene_flat dev_pool; do OBJS="$OBJS build/$o.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/librtgo.so" $OBJS -L/opt/rocm/lib -lrccl -lz \
  -Wl,-soname,librtgo.so -Wl,-rpath,/opt/rocm/lib
echo "$OUT/librtgo.so"
