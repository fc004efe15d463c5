#!/bin/bash
# HBM read/write bytes per SpMV kernel launch (TCC EA request counters by size), optionally
# with env knobs.  usage (GPU box, repo root): scripts/pmc_kernels.sh TAG [VAR=value ...]
tag=$1; shift
out=gpurun_out/pmck_$tag
mkdir -p $out
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
set --
for pass in "rd TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  set -- $pass
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex spmv -d $out/$name -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $out/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
done
python3 - "$out" "$tag" <<'PY'
import csv, collections, sys
d, tag = sys.argv[1], sys.argv[2]
size = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}
for name in ("rd", "wr"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f"{d}/{name}/run_counter_collection.csv")):
        agg[row["Kernel_Name"].split("(")[0]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if name == "rd":
            b = sum(m[c] * size[c] for c in size if c in m)
        else:
            b = m["TCC_EA0_WRREQ_64B_sum"] * 64 + (m["TCC_EA0_WRREQ_sum"] - m["TCC_EA0_WRREQ_64B_sum"]) * 32
        print(f"{tag:8s} {name} {k[:48]:48s} {b / 1e9:7.3f} GB")
PY
