#!/bin/bash
# which launch pays for a physically contiguous partial array: kernel trace of the placement
# probe, averages before and after the move
export TMPDIR=/tmp
PR_CONTIG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/contig_kt -o run --output-format csv -- scripts/probes/placement_probe 26 0:partial 2>/dev/null | grep GTEPS
python3 - gpurun_out/contig_kt/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
st = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "spmv_stream" in r["Kernel_Name"]]
rw = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "spmv_rows" in r["Kernel_Name"]]
h = len(st) // 2
f = lambda v: sum(v) / len(v)
print("as built:   stream %.1f us  rows %.1f us" % (f(st[3:h]), f(rw[3:h])))
print("contiguous: stream %.1f us  rows %.1f us" % (f(st[h + 1:]), f(rw[h + 1:])))
PY
