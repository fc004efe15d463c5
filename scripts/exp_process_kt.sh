#!/bin/bash
# per-process kernel averages (rocprofv3 kernel trace) of N processes back to back
# usage: scripts/exp_process_kt.sh N [ENV=..]
n=$1; shift
export TMPDIR=/tmp
for i in $(seq $n); do
  d=gpurun_out/pkt_$i
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- scripts/probes/lib_ab page-rank-and-tfidf-using-apache-spark_amd/_build/libprmi355x.so 26 20 2>/dev/null | grep GTEPS | sed 's/.*build/build/' || exit 1
  python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
o = []
for r in csv.DictReader(open(sys.argv[1])):
    if "spmv_stream" in r["Name"]: o.append("stream %.1f us" % (float(r["AverageNs"]) / 1e3))
    if "spmv_rows<0>" in r["Name"]: o.append("rows %.1f us" % (float(r["AverageNs"]) / 1e3))
print("    " + "  ".join(o))
PY
done
