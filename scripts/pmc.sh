#!/bin/bash
# One rocprofv3 PMC pass (counters restricted to the SpMV kernels) over a short bench run.
# usage: scripts/pmc.sh NAME "COUNTERS" [bench args...]   -> gpurun_out/pmc_NAME/
name=$1; ctrs=$2; shift 2
out=gpurun_out/pmc_$name
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "spmv" -d $out -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $out/log.txt 2>&1
rc=$?; echo "pmc $name rc=$rc"; tail -n 2 $out/log.txt
exit $rc
