#!/bin/bash
# Where the round's time goes by row in-degree (timing only): SpMV kernel time with the rows
# below D dropped (PR_DROPDEG) or the rows at or above K dropped (PR_KEEPDEG).
# usage: scripts/exp_bins.sh TAG "ENV=.. ENV=.." ...
tag=$1; shift
out=gpurun_out/bins_$tag.txt
mkdir -p gpurun_out
for cfg in "$@"; do
  line=$(env PR_VERBOSE=1 $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 2> gpurun_out/bins_err.log) || { echo "'$cfg' failed"; tail -5 gpurun_out/bins_err.log; exit 1; }
  pcs=$(grep -h -o "local_nnz=[0-9]* .*pieces=[0-9]*" gpurun_out/bins_err.log | head -1)
  echo "${cfg:-defaults} | $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], 'ms SpMV kernels', d['ms_per_step'], 'ms/step')") | $pcs" | tee -a "$out"
done
