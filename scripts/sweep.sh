#!/bin/bash
# Kernel-trace sweep over engine knobs: one short bench per variant under rocprofv3.
# usage: scripts/sweep.sh TAG "VAR=v VAR2=w" "VAR=x" ...   (empty string = defaults)
tag=$1; shift
i=0
for v in "$@"; do
  i=$((i+1))
  echo "### $tag.$i: ${v:-defaults}" | tee -a gpurun_out/sweep_$tag.txt
  scripts/kt.sh ${tag}_$i PR_VERBOSE=1 $v >> gpurun_out/sweep_$tag.txt 2>&1 || { echo "variant $i failed rc=$?"; tail -5 gpurun_out/kt_${tag}_$i.log; exit 1; }
  grep -h "pieces=" gpurun_out/kt_${tag}_$i.log | head -1 | sed 's/.*pairs=/  pairs=/' >> gpurun_out/sweep_$tag.txt
  grep -h '"value"' gpurun_out/kt_${tag}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  GTEPS', d['value'], 'kernel_ms', d['roofline']['kernel_ms'])" >> gpurun_out/sweep_$tag.txt
done
cat gpurun_out/sweep_$tag.txt
