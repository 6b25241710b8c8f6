#!/usr/bin/env bash
# Time every librtg variant in humanoid-real-time-retarget_amd/variants/ with the
# secondary solver bench (RTG_LIB selects the library).  One process per variant.
set -u
mkdir -p gpurun_out
for so in humanoid-real-time-retarget_amd/variants/*.so; do
  n=$(basename "$so" .so)
  RTG_ALLOW_MEASUREMENT_BUILD=1 RTG_LIB="$PWD/$so" timeout -k 10 120 python tools/extra_bench.py ${1:-solvers} > "gpurun_out/var_$n.log" 2>&1
  rc=$?
  echo "$n rc=$rc $(grep -o '"frames_per_s": [0-9.e+]*' gpurun_out/var_$n.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
