#!/usr/bin/env bash
# Build librtg variants with measurement knobs into humanoid-real-time-retarget_amd/variants/<name>.so
# usage: tools/build_variants.sh "name:-DKNOB=1 -DOTHER=0" ...   (time them with tools/variant_bench.sh)
# A variant built with a wrong-answer knob (RTG_EXP_STUB_SVD / _NO_TABLE / _HOT_INPUTS) reports it in
# rtg_build_info(); rtg._lib refuses to load it unless RTG_ALLOW_MEASUREMENT_BUILD=1 (variant_bench.sh sets it).
set -eu
cd "$(dirname "$0")/../humanoid-real-time-retarget_amd/csrc"
mkdir -p ../variants
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -I../../include"
TUS="rtg_solve_fbp_aos rtg_solve_fbp_soa rtg_solve_fbp_small rtg_solve_other rtg_fk rtg_ops"
SMALL_FLAGS="-mllvm -amdgpu-sched-strategy=max-ilp"   # rtg_solve_fbp_small only (csrc/Makefile)
for spec in "$@"; do
  name="${spec%%:*}"; defs="${spec#*:}"
  objs=""
  for t in $TUS; do
    extra=""; { [ "$t" = rtg_solve_fbp_small ] || [ "$t" = rtg_fk ]; } && extra="$SMALL_FLAGS"
    /opt/rocm/bin/hipcc $FLAGS $extra $defs -c $t.hip -o /tmp/v_$name.$t.o &
    objs="$objs /tmp/v_$name.$t.o"
  done
  /opt/rocm/bin/hipcc $FLAGS $defs -x hip -c rtg_api.cpp -o /tmp/v_$name.api.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/v_$name.api.o -o ../variants/$name.so
  echo "built variants/$name.so ($defs)"
done
