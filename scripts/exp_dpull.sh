#!/bin/bash
# Direct-pull experiment (timing only): for each in-degree bound D, the SpMV kernels' time with
# the rows below D (a) in the streams as usual, (b) dropped from the streams (PR_DROPDEG), and
# (c) dropped and summed by the direct-pull kernel instead (PR_DPULL); piece statistics of (a).
# usage: scripts/exp_dpull.sh TAG D1 D2 ...
tag=$1; shift
out=gpurun_out/dpull_$tag.txt
mkdir -p gpurun_out
run() {  # label, env...
  lbl=$1; shift
  line=$(env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 2> gpurun_out/dpull_err.log) || { echo "$lbl failed"; tail -5 gpurun_out/dpull_err.log; exit 1; }
  grep -h "direct-pull experiment" gpurun_out/dpull_err.log | tee -a "$out"
  grep -h "dpull check" gpurun_out/dpull_err.log | tee -a "$out"
  echo "$lbl | $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], 'ms SpMV kernels', d['ms_per_step'], 'ms/step')")" | tee -a "$out"
}
PR_DPULL=8 PR_DPULL_CHECK=1 timeout -k 10 100 python3 bench.py --no-cpu-baseline --steps 2 --warmup 0 --scale 16 2>&1 | grep -E "dpull|direct-pull" | tee -a "$out"
run "defaults" PR_X=0
for D in "$@"; do
  run "D=$D dropped from the streams" PR_DROPDEG=$D
  run "D=$D dropped + direct pull" PR_DROPDEG=$D PR_DPULL=$D
done
run "defaults again" PR_X=0
