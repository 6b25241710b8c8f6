#!/usr/bin/env bash
# The committed evidence for one round: bench line, kernel-trace stats of the same bench command, the two PMC
# traffic passes (FETCH_SIZE / WRITE_SIZE, one rocprofv3 run each), and the instruction-mix passes.
# usage (on the GPU box): tools/profile_round.sh <tag>     -> gpurun_out/prof_<tag>/...
set -eu
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 300 python bench.py > $out/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv \
  -- python bench.py --steps 20 --no-cpu-baseline > $out/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv \
  -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv \
  -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/write.log 2>&1
timeout -k 10 200 python tools/extra_bench.py latency fk solvers > $out/extra.log 2>&1
