#!/bin/bash
# Hardware counters of the stream launch before and after the partial array moves behind a
# ballast (scripts/probes/placement_probe), one counter set per process.
# usage: scripts/exp_place_pmc.sh GB "COUNTERS" ["COUNTERS" ...]
gb=$1; shift
export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i + 1))
  d=gpurun_out/place_pmc_$i
  rm -rf $d
  timeout -s KILL 200 rocprofv3 --pmc $set -d $d -o run --output-format csv -- scripts/probes/placement_probe 26 $gb:partial 2>/dev/null | grep GTEPS
  python3 - $d/run_counter_collection.csv <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "spmv_stream" in r["Kernel_Name"]]
ids = sorted({int(r["Dispatch_Id"]) for r in rows})
half = ids[len(ids) // 2]
acc = collections.defaultdict(lambda: [0.0, 0, 0.0, 0])
for r in rows:
    a = acc[r["Counter_Name"]]
    k = 0 if int(r["Dispatch_Id"]) < half else 2
    a[k] += float(r["Counter_Value"]); a[k + 1] += 1
for n, a in sorted(acc.items()):
    nb = len({int(r["Dispatch_Id"]) for r in rows if r["Counter_Name"] == n and int(r["Dispatch_Id"]) < half})
    na = len({int(r["Dispatch_Id"]) for r in rows if r["Counter_Name"] == n and int(r["Dispatch_Id"]) >= half})
    print(f"    {n:44s} before {a[0] / max(nb, 1):16.0f}   after {a[2] / max(na, 1):16.0f}   ratio {a[2] / max(na, 1) / max(a[0] / max(nb, 1), 1e-9):.3f}")
PY
done
