#!/bin/bash
# SQ counter passes over a short bench run (one rocprofv3 --pmc run per pass)
# usage: scripts/pmc_stream.sh TAG [VAR=value ...]
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum"; do
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
        print(f"   {c:28s} {sum(v)/len(v):16.4g}")
PY
