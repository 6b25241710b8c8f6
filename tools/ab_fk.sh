#!/usr/bin/env bash
# Interleaved A/B of the kinematics kernels (tools/extra_bench.py fk): the product library against variants, R rounds.
# usage: tools/ab_fk.sh ROUNDS variant1.so [variant2.so ...]   (logs into gpurun_out/ab_<mode>_<name>_<round>.log; AB_MODE=fk|aux|solvers|latency)
set -u
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for so in humanoid-real-time-retarget_amd/librtg_hip.so "$@"; do
    n=$(basename "$so" .so)
    RTG_ALLOW_MEASUREMENT_BUILD=1 RTG_LIB="$PWD/$so" timeout -k 10 120 python tools/extra_bench.py ${AB_MODE:-fk} > "gpurun_out/ab_${AB_MODE:-fk}_${n}_$r.log" 2>&1
    rc=$?
    echo "round $r $n rc=$rc $(python -c "import json,sys; t=open(sys.argv[1]).read(); d=json.loads(t[t.index('{'):])[sys.argv[2]]; print(' '.join('%s=%.1fus' % (k, v['ms']*1e3) for k, v in d.items()))" "gpurun_out/ab_${AB_MODE:-fk}_${n}_$r.log" "${AB_MODE:-fk}" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
