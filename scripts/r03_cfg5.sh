#!/bin/bash
# cfg5 evidence (R-MAT scale 28, seed 5) on one GPU: the single-GPU bench line, the per-rank
# kernel times of the 8-rank deal, and the L2 hit / miss counters of the stream launch at
# scale 26 and scale 28 (what bounds the lower roofline fraction at scale 28).
# usage: scripts/r03_cfg5.sh TAG
tag=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench s28 seed 5"
timeout -k 10 400 python3 bench.py --scale 28 --seed 5 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_s28_seed5_$tag.json 2> gpurun_out/bench_s28_seed5_$tag.err || { echo "bench s28 failed"; tail -5 gpurun_out/bench_s28_seed5_$tag.err; exit 1; }
cat gpurun_out/bench_s28_seed5_$tag.json
echo "== per-rank kernels, 8 ranks of scale 28"
PRMI_SCALE=28 PRMI_SEED=5 scripts/group_kt.sh s28_$tag 8 | tee gpurun_out/s28_p8_$tag.txt || exit 1
echo "== L2 counters of the SpMV kernels"
for cfg in "26 4" "28 5"; do
  set -- $cfg
  for pass in "TCC_HIT_sum TCC_MISS_sum" "TCC_REQ_sum TCC_READ_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" "GRBM_GUI_ACTIVE"; do
    d=gpurun_out/l2c_${tag}_s$1_$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 240 rocprofv3 --pmc $pass -d $d -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --scale $1 --seed $2 > $d.log 2>&1 || { echo "pass '$pass' s$1 rc=$?"; tail -3 $d.log; }
  done
done
python3 - $tag <<'PY' | tee gpurun_out/l2_counters_$tag.txt
import csv, sys, glob, collections
tag = sys.argv[1]
for s in ("26", "28"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/l2c_{tag}_s{s}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "spmv" not in n: continue
            acc["stream" if "spmv_stream" in n else "rows"][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in sorted(acc.items()):
        print(f"scale {s} {k} launch (mean per launch):")
        for c, v in sorted(d.items()):
            print(f"   {c:36s} {sum(v)/len(v):16.5g}")
PY
