#!/bin/bash
# Interleaved A/B of engine knobs on one box: each variant's bench (no CPU leg) REPS times in
# A B C A B C order, so clock drift between runs spreads over every variant.
# usage: scripts/ab.sh TAG REPS "VAR=v ..." "VAR=w ..." ...   ("" = defaults)
tag=$1; reps=$2; shift 2
out=gpurun_out/ab_$tag.txt
mkdir -p gpurun_out
for r in $(seq 1 "$reps"); do
  for cfg in "$@"; do
    line=$(env $cfg timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3) || { echo "variant '$cfg' failed rc=$?"; exit 1; }
    echo "rep $r | ${cfg:-defaults} | $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'GTEPS', d['roofline']['kernel_ms'], 'ms kernels', d['ms_per_step'], 'ms/step')")" | tee -a "$out"
  done
done
