#!/usr/bin/env bash
# PMC passes over a short bench run, one rocprofv3 run per pass (gfx950 slot limits:
# <= 8 SQ counters per pass).  Output: gpurun_out/pmc_<tag>_<pass>/...
# usage: tools/pmc_passes.sh <tag> [pass ...]   (passes: sq valu misc icache; default all)
set -eu
tag=${1:-r01}
shift || true
passes=${*:-sq valu misc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_${tag}_$name -o $name --output-format csv \
    -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_${tag}_$name.log 2>&1
}
for p in $passes; do
  case $p in
    sq) run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE ;;
    valu) run valu SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
          SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 ;;
    misc) run misc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
          SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_BUSY_CYCLES ;;
    icache) run icache SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES ;;
  esac
done
