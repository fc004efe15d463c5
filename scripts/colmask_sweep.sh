#!/bin/bash
# Timing-only experiment: restrict every gather to the first (mask+1) x entries (PR_COLMASK)
# to separate the stream/issue cost from the gather cost.  usage: scripts/colmask_sweep.sh
set -e
for cm in 0x0 0x3FFF 0xFFFFF 0xFFFFFFFF; do
  for hl in 0 20480; do
    r=$(PR_COLMASK=$cm PR_HOTLDS=$hl timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2)
    echo "cm=$cm hotlds=$hl $(echo "$r" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'GTEPS', d['roofline']['kernel_ms'], 'ms')")"
  done
done
