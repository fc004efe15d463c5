#!/bin/bash
# How long the exchange's small kernels (pack, unpack, finalize) take when they run beside a
# stream launch that holds all but one compute unit of every XCD: a p-rank group on one GPU with
# many hardware queues, kernel trace, durations split by "started inside some stream launch".
# usage: [PR_PACKCOMM=..] scripts/trace_small_kernels.sh TAG SCALE p
tag=$1; scale=$2; p=$3
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
out=gpurun_out/small_$tag
timeout -k 10 300 rocprofv3 --kernel-trace -d $out -o run --output-format csv -- python3 scripts/group_split.py $scale $p > $out.log 2>&1 || { echo "trace failed"; tail -5 $out.log; exit 1; }
tail -1 $out.log
python3 - $out/run_kernel_trace.csv <<'PY' | tee gpurun_out/small_$tag.txt
import csv, sys, bisect
rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
streams = sorted((s, e) for s, e, n in ev if "spmv_stream" in n)
starts = [s for s, _ in streams]
def inside(t):
    i = bisect.bisect_right(starts, t) - 1
    return any(streams[k][0] <= t < streams[k][1] for k in range(max(0, i - 16), i + 1))
for key in ("k_sx_pack", "k_sx_unpack", "finalize_round", "reduce_shards", "spmv_rows"):
    a = [(e - s) / 1e3 for s, e, n in ev if key in n and inside(s)]
    b = [(e - s) / 1e3 for s, e, n in ev if key in n and not inside(s)]
    f = lambda v: f"n {len(v):5d} avg {sum(v) / len(v):8.1f} max {max(v):8.1f} us" if v else "n     0"
    print(f"{key:15s} beside a stream launch: {f(a)} | alone: {f(b)}")
PY
