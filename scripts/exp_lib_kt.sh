#!/bin/bash
# per-kernel averages (rocprofv3 kernel trace) of two engine libraries on one box, interleaved
# usage: scripts/exp_lib_kt.sh REPS LIB_A LIB_B
reps=$1; a=$2; b=$3
export TMPDIR=/tmp
for i in $(seq $reps); do
  k=0
  for l in $a $b; do
    k=$((k + 1))
    d=gpurun_out/libkt_${i}_$k
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- scripts/probes/lib_ab $l 26 20 | grep GTEPS || exit 1
    python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("spmv", "finalize", "reduce")):
        print(f"    {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
  done
done
