#!/bin/bash
# Per-rank kernel times of a p-rank group on ONE GPU (LocalGroup, peer copies instead of RCCL):
# with one hardware queue every rank's launches run alone, so rocprofv3's per-kernel averages
# are the per-rank stream / row launch times at p ranks.
# usage: [PRMI_SCALE=26] [PRMI_SEED=4] scripts/group_kt.sh TAG p...
tag=$1; shift
scale=${PRMI_SCALE:-26}
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=1
for p in "$@"; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/gkt_${tag}_p$p -o run --output-format csv \
    -- python3 scripts/group_split.py $scale $p > gpurun_out/gkt_${tag}_p$p.log 2>&1 || { echo "p=$p failed"; exit 1; }
  tail -n 2 gpurun_out/gkt_${tag}_p$p.log | grep "scale"
  python3 - "gpurun_out/gkt_${tag}_p$p/run_kernel_stats.csv" "$p" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("spmv", "finalize", "reduce_shards")):
        print(f"p={sys.argv[2]} {r['Name'][:52]:52s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
