#!/bin/bash
# Kernel timeline of a rank group on one GPU under an injected exchange delay: which launches of
# round t+1 start before round t's exchange has finished.
# usage: [GPU_MAX_HW_QUEUES=n] scripts/trace_overlap.sh TAG SCALE p DELAY_US OVERLAP
tag=$1; scale=$2; p=$3; d=$4; ov=$5
export TMPDIR=/tmp
out=gpurun_out/trace_$tag
PR_XDELAY_US=$d PR_XOVERLAP=$ov timeout -k 10 300 rocprofv3 --kernel-trace -d $out -o run --output-format csv -- python3 scripts/group_split.py $scale $p > $out.log 2>&1 || { echo "trace failed"; tail -5 $out.log; exit 1; }
tail -1 $out.log
python3 - $out/run_kernel_trace.csv <<'PY' | tee gpurun_out/trace_$tag.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
def short(n):
    for k, v in (("spmv_stream", "stream"), ("spmv_rows", "rows"), ("k_delay", "DELAY"), ("k_sx_pack", "pack"),
                 ("k_sx_unpack", "unpack"), ("finalize_round", "finalize"), ("reduce_shards", "reduce")):
        if k in n: return v
    return None
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", "?"), r.get("Stream_Id", "?")) for r in rows if short(r["Kernel_Name"])]
ev.sort()
# the last two rounds: everything after the third-last 'finalize' group
fins = [i for i, e in enumerate(ev) if e[2] == "finalize"]
p = max(1, len(set(e[3] for e in ev if e[2] == "stream")))
start = fins[-3 * p] if len(fins) >= 3 * p else 0
t0 = ev[start][0]
for s, e, n, q, st in ev[start:]:
    if n in ("pack", "unpack", "reduce"): continue
    print(f"{(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  {n:9s} queue {q} stream {st}")
PY
