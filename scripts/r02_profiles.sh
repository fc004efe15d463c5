#!/bin/bash
# Round-2 profile artefacts (GPU box, repo root): kernel trace + PMC traffic passes of the bench
# workload (collect_profiles.sh), the traffic summary, and a roctx marker trace of the same run.
# usage: scripts/r02_profiles.sh TAG
tag=$1
export TMPDIR=/tmp
scripts/collect_profiles.sh $tag --steps 5 --warmup 1 || exit $?
python3 scripts/traffic.py gpurun_out/prof_$tag rmat-s26-ef16-p1 gpurun_out/traffic_$tag.json || exit $?
timeout -k 10 180 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/prof_$tag/marker -o run \
  --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 \
  > gpurun_out/prof_$tag/marker.log 2>&1 || exit $?
echo marker rc=0
PR_VERBOSE=1 timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 \
  > gpurun_out/prof_$tag/verbose.out 2> gpurun_out/prof_$tag/verbose.log || exit $?
python3 scripts/traffic_breakdown.py gpurun_out/prof_$tag gpurun_out/prof_$tag/verbose.log \
  gpurun_out/prof_$tag/traffic_breakdown.json
