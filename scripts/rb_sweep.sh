#!/bin/bash
# Row-launch block geometry at 8 ranks on one GPU (one HW queue: each rank's launches run
# alone; per-rank kernel times from rocprofv3) and at 1 rank (bench).
# usage: scripts/rb_sweep.sh "ENV=.. ENV=.." ...
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg GPU_MAX_HW_QUEUES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rbs$i -o run --output-format csv -- python3 scripts/group_split.py 26 ${GP:-8} > gpurun_out/rbs$i.log 2>&1 || exit $?
  echo "$cfg p=${GP:-8} per-rank kernels (calls, total ns, avg ns):"; grep spmv gpurun_out/rbs$i/run_kernel_stats.csv | cut -d, -f1-4
  [ -n "$NOBENCH" ] || scripts/exp.sh "$cfg" || exit $?
done
