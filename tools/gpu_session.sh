#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box.  Each step has its own time
# limit; an ordinary failure (exit 1) lets later steps run, but a fault-like
# exit (abort 134, segfault 139, timeout 124/137, or a signal) ends the session.
# usage: tools/gpu_session.sh "<name>:<seconds>:<command>" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (${secs}s) $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|4|5) ;;   # pass / test failures / usage errors: keep going
    *) echo "=== fault-like exit ($rc): stopping session" | tee -a gpurun_out/session.log; exit $rc ;;
  esac
done
