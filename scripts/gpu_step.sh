#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a fault/abort/timeout.
# usage: scripts/gpu_step.sh NAME SECONDS cmd...   (log -> gpurun_out/NAME.log)
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "== $name: $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
tail -n 25 "gpurun_out/$name.log"
case $rc in
  0|1|5) exit 0 ;;          # ok / test failures / no tests: keep going
  *) echo "STOP: $name rc=$rc"; exit $rc ;;
esac
