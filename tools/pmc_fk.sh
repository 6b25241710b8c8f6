#!/usr/bin/env bash
# FK-family profile on the GPU box: kernel trace + PMC passes (one counter family per rocprofv3 run) over
# `tools/extra_bench.py fk` (Hu FK, inverse FK, HuForwardModel, the mixed 4-skeleton launch at 4 x 65536).
# usage: tools/pmc_fk.sh <tag>   -> gpurun_out/fk_<tag>/...
set -eu
tag=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/fk_$tag
mkdir -p $out
C="python tools/extra_bench.py fk"
pmc() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $out/$name -o $name --output-format csv -- $C > $out/$name.log 2>&1
}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- $C > $out/trace.log 2>&1
pmc cyc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc mix SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH
echo "pmc_fk $tag done"
