#!/usr/bin/env bash
# PMC passes over the §8(f) kernels around the solver (tools/extra_bench.py aux: ingest, linear / angular velocity
# tiles), one rocprofv3 run per counter family, plus a kernel trace of the same command.
# usage (on the GPU box): tools/pmc_aux.sh <tag>      -> gpurun_out/pmc_aux_<tag>/...
# summarise with: python tools/pmc_table.py gpurun_out/pmc_aux_<tag> ingest velocity
set -eu
tag=${1:-r05}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_aux_$tag
mkdir -p $out
run() {   # run <name> <counters...>
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $out/$name -o $name --output-format csv \
    -- python tools/extra_bench.py aux > $out/$name.log 2>&1
}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv \
  -- python tools/extra_bench.py aux > $out/trace.log 2>&1
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
echo "pmc_aux $tag done"
