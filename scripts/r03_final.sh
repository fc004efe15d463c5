#!/bin/bash
# Round-3 closing check (GPU box, repo root): the whole -m gpu suite, the default bench line,
# a 60-case soak against the exact oracle, and the profile artefacts of the bench workload.
# usage: scripts/r03_final.sh TAG
tag=$1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.log; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
# (the bench line first: as the first process on a fresh box, the state the driver's run starts
# from -- under the kernel trace, so that the committed trace and the bench line are one process)
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$tag
scripts/gpu_step.sh bench_$tag 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag/kt -o run --output-format csv -- python3 bench.py || exit $?
scripts/gpu_step.sh smoke_$tag 200 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
scripts/gpu_step.sh pytest_$tag 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
scripts/gpu_step.sh soak_$tag 400 python3 -u scripts/soak.py 60 || exit $?
SKIP_KT=1 scripts/r02_profiles.sh $tag || exit $?
PR_PIECE_STATS=1 timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/piece_stats_$tag.log 2>&1
echo "final check done"
