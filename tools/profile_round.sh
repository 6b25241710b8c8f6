#!/usr/bin/env bash
# The committed evidence for one round, on the GPU box: the bench line, rocprofv3 kernel-trace stats of the same
# bench command, and the PMC passes tools/pmc_summary.py turns into profiles/pmc_<tag>.json (one counter family per
# rocprofv3 run; FETCH_SIZE and WRITE_SIZE never share a pass; no --pmc run combines a trace domain):
#   fetch / write / sq / cyc    the headline solver (bench.py --steps 10)
#   notab_fetch                 the RTG_EXP_NO_TABLE build (humanoid-real-time-retarget_amd/variants/notab.so)
#   calib_fetch / calib_write   tools/fetch_calib (known-byte micro-kernels for the FETCH_SIZE calibration)
# usage (on the GPU box): tools/profile_round.sh <tag>     -> gpurun_out/prof_<tag>/...
set -eu
tag=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
# the PMC passes count bytes and instructions, which the clock does not change: no clock-settle phase there
export RTG_BENCH_SETTLE_MS=0
pmc() {   # pmc <name> <lib or -> <counters...>
  name=$1; lib=$2; shift 2
  if [ "$lib" = "-" ]; then env_lib=""; else env_lib="$lib"; fi
  RTG_ALLOW_MEASUREMENT_BUILD=1 RTG_LIB=${env_lib:-$PWD/humanoid-real-time-retarget_amd/librtg_hip.so} timeout -s KILL 120 \
    rocprofv3 --pmc "$@" -d $out/$name -o $name --output-format csv -- $B > $out/$name.log 2>&1
}
RTG_BENCH_SETTLE_MS=200 timeout -k 10 300 python bench.py > $out/bench.log 2>&1
RTG_BENCH_SETTLE_MS=200 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv \
  -- python bench.py --steps 20 --no-cpu-baseline > $out/trace.log 2>&1
python tools/trace_summary.py $out/trace/trace_kernel_trace.csv 12 10 > $out/trace_by_grid.txt 2>&1 || true
pmc fetch - FETCH_SIZE
pmc write - WRITE_SIZE
pmc sq - SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
  SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32
pmc cyc - SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_INSTS_VMEM_RD
if [ -f humanoid-real-time-retarget_amd/variants/notab.so ]; then
  pmc notab_fetch $PWD/humanoid-real-time-retarget_amd/variants/notab.so FETCH_SIZE
fi
timeout -k 10 60 tools/fetch_calib > $out/calib.json
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $out/calib_fetch -o calib_fetch --output-format csv -- tools/fetch_calib \
  > $out/calib_fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $out/calib_write -o calib_write --output-format csv -- tools/fetch_calib \
  > $out/calib_write.log 2>&1
timeout -k 10 200 python tools/extra_bench.py latency fk solvers > $out/extra.log 2>&1
echo "profile_round $tag done"
