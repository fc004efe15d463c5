#!/bin/bash
# per-phase timing of the stream launch (PR_STAMPS) for several knob settings
# usage: scripts/stamps.sh TAG "VAR=v ..." ...
tag=$1; shift
i=0
for v in "$@"; do
  i=$((i+1))
  echo "### $tag.$i: ${v:-defaults}" >> gpurun_out/stamps_$tag.txt
  env PR_STAMPS=1 PR_VERBOSE=1 $v timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/stamps_${tag}_$i.log 2>&1 || { echo "variant $i rc=$?"; tail -5 gpurun_out/stamps_${tag}_$i.log; exit 1; }
  grep -h "stamps\|pieces=" gpurun_out/stamps_${tag}_$i.log | head -80 >> gpurun_out/stamps_$tag.txt
done
cat gpurun_out/stamps_$tag.txt
