#!/bin/bash
# GPU session script: each GPU step has its own time limit; a fault/abort/timeout stops the script.
mkdir -p gpurun_out
step() {  # step <seconds> <logfile> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  tail -5 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
"$@"
