#!/bin/bash
# Layout knobs at another R-MAT scale on one GPU.  usage: scripts/exp_scale.sh TAG SCALE SEED "ENV=.." ...
tag=$1; scale=$2; seed=$3; shift 3
out=gpurun_out/scale_$tag.txt
for cfg in "$@"; do
  line=$(env PR_VERBOSE=1 $cfg timeout -k 10 300 python3 bench.py --scale $scale --seed $seed --no-cpu-baseline --steps 8 --warmup 2 2> gpurun_out/scale_err.log) || { echo "'$cfg' failed"; tail -5 gpurun_out/scale_err.log; exit 1; }
  pcs=$(grep -h -o "segments/slice=[0-9]* .*pieces=[0-9]*" gpurun_out/scale_err.log | head -1)
  echo "s$scale ${cfg:-defaults} | $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'GTEPS', d['roofline']['kernel_ms'], 'ms SpMV kernels')") | $pcs" | tee -a "$out"
done
