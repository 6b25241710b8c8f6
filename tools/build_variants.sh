#!/usr/bin/env bash
# Build librtg variants with measurement knobs into humanoid-real-time-retarget_amd/variants/<name>.so
# usage: tools/build_variants.sh "name:-DKNOB=1 -DOTHER=0" ...   (time them with tools/variant_bench.sh)
set -eu
cd "$(dirname "$0")/../humanoid-real-time-retarget_amd/csrc"
mkdir -p ../variants
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -I../../include"
for spec in "$@"; do
  name="${spec%%:*}"; defs="${spec#*:}"
  /opt/rocm/bin/hipcc $FLAGS $defs -c rtg_kernels.hip -o /tmp/v_$name.k.o &
  /opt/rocm/bin/hipcc $FLAGS $defs -x hip -c rtg_api.cpp -o /tmp/v_$name.a.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC /tmp/v_$name.k.o /tmp/v_$name.a.o -o ../variants/$name.so
  echo "built variants/$name.so ($defs)"
done
