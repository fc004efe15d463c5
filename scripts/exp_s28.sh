#!/bin/bash
# Layout knobs at R-MAT scale 28 (cfg5's graph, seed 5) on one GPU: LDS blocks per slice and the
# L2-hot range.  usage: scripts/exp_s28.sh TAG "ENV=.." ...
tag=$1; shift
out=gpurun_out/s28_$tag.txt
for cfg in "$@"; do
  line=$(env PR_VERBOSE=1 $cfg timeout -k 10 300 python3 bench.py --scale 28 --seed 5 --no-cpu-baseline --steps 6 --warmup 1 2> gpurun_out/s28_err.log) || { echo "'$cfg' failed"; tail -5 gpurun_out/s28_err.log; exit 1; }
  pcs=$(grep -h -o "segments/slice=[0-9]* .*pieces=[0-9]*" gpurun_out/s28_err.log | head -1)
  echo "${cfg:-defaults} | $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'GTEPS', d['roofline']['kernel_ms'], 'ms SpMV kernels')") | $pcs" | tee -a "$out"
done
