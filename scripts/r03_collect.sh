#!/bin/bash
# Copy the closing run's artefacts (scripts/r03_final.sh TAG on the GPU box, merged back into
# gpurun_out/) into profiles/r03/ and refresh profiles/traffic.json.  usage: scripts/r03_collect.sh TAG
set -e
tag=$1
src=gpurun_out
dst=profiles/r03
mkdir -p $dst/pmc
grep -h '^{' $src/bench_$tag.log | tail -1 > $dst/bench.json
cp $src/prof_$tag/kt/run_kernel_stats.csv $dst/kernel_stats.csv
# the same trace restricted to the round loop: a stream launch counts when the next SpMV launch
# is a row launch (the build's placement search runs stream launches of its own, back to back)
python3 - $src/prof_$tag/kt/run_kernel_trace.csv $dst/kernel_stats_round_loop.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sp = [r for r in rows if "spmv_stream" in r["Kernel_Name"] or "spmv_rows" in r["Kernel_Name"]]
acc = {}
for i, r in enumerate(sp):
    n = r["Kernel_Name"]
    if "spmv_stream" in n and not (i + 1 < len(sp) and "spmv_rows" in sp[i + 1]["Kernel_Name"]):
        continue
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    a = acc.setdefault(n, [0, 0, 1 << 62, 0])
    a[0] += 1; a[1] += d; a[2] = min(a[2], d); a[3] = max(a[3], d)
with open(sys.argv[2], "w") as f:
    f.write('"Name","Calls","TotalDurationNs","AverageNs","MinNs","MaxNs"\n')
    for n, a in acc.items():
        f.write('"%s",%d,%d,%.1f,%d,%d\n' % (n, a[0], a[1], a[1] / a[0], a[2], a[3]))
PY
for p in rd wr fetch write l2; do cp $src/prof_$tag/$p/run_counter_collection.csv $dst/pmc/$p.csv; done
cp $src/prof_$tag/traffic_breakdown.json $dst/traffic_breakdown.json
cp $src/prof_$tag/marker/run_marker_api_stats.csv $dst/marker_stats.csv 2>/dev/null || cp $src/prof_$tag/marker/run_marker_stats.csv $dst/marker_stats.csv 2>/dev/null || ls $src/prof_$tag/marker
cp $src/pytest_$tag.log $dst/pytest_gpu.log
cp $src/soak_$tag.log $dst/soak.log
cp $src/smoke_$tag.log $dst/smoke.log
grep -h "piece stats" $src/piece_stats_$tag.log > $dst/piece_stats.log || true
cp $src/traffic_$tag.json profiles/traffic.json
python3 - <<'PY'
import json
d = json.load(open("profiles/r03/bench.json"))
print("bench:", d["value"], "GTEPS", d["ms_per_step"], "ms/step frac", d["roofline"]["frac"], "cpu", d["cpu_baseline"]["value"], "build", d["build_id"])
t = json.load(open("profiles/traffic.json"))
print("traffic:", {k: round(v["hbm_bytes_per_launch"] / 1e9, 3) for k, v in t.items()})
PY
