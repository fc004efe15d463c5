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
