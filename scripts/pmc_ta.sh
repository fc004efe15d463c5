#!/bin/bash
# Vector-memory pipeline counters of the SpMV kernels (one rocprofv3 --pmc run per pass) and the
# box's list of available counters.  usage (GPU box): scripts/pmc_ta.sh TAG [VAR=value ...]
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmcta_$tag
mkdir -p $out
timeout -s KILL 60 rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
i=0
for pass in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum" \
            "TD_BUSY_sum TD_TC_STALL_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum" \
            "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  env "$@" timeout -s KILL 90 rocprofv3 --pmc $pass -d $out/p$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $out/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $out/p$i.log; }
done
python3 - $out <<'PY'
import csv, sys, glob, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "spmv" not in n: continue
        acc[n.split("(")[0][-30:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:40s} {sum(v)/len(v):16.4g}")
PY
