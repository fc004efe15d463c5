#!/bin/bash
# per-kernel time of a short bench run under rocprofv3 (optionally with env knobs)
# usage: scripts/kt.sh TAG [VAR=value ...]
tag=$1; shift
export TMPDIR=/tmp
env "$@" timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$tag -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/kt_$tag.log 2>&1 || exit $?
python3 - "$tag" <<'PY'
import csv, sys
tag = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/kt_{tag}/run_kernel_stats.csv")))
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("spmv", "reduce_shards", "finalize")):
        print(f"{tag:10s} {n[:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
