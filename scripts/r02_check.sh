#!/bin/bash
# Round-2 GPU check: the whole -m gpu suite, the default bench line, a kernel trace of the bench.
# usage (GPU box, repo root): scripts/r02_check.sh TAG [pytest selection...]
tag=$1; shift
sel=${*:-tests}
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.log; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
scripts/gpu_step.sh pytest_$tag 1000 python3 -u -m pytest $sel -m gpu -x -v -s --timeout 700 --timeout-method thread || exit $?
scripts/gpu_step.sh bench_$tag 300 python3 bench.py || exit $?
scripts/kt.sh $tag || exit $?
