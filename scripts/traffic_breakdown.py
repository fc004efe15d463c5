#!/usr/bin/env python3
"""Per-array HBM traffic of one round: the algorithmic bytes of every array the two SpMV
kernels touch (the engine's `round bytes:` verbose line, PR_VERBOSE=1) beside the measured
read/write bytes of each kernel (rocprofv3 PMC passes of collect_profiles.sh: TCC EA requests
by size).  The difference per kernel and direction is the re-read / partial-line overhead.
usage: scripts/traffic_breakdown.py gpurun_out/prof_TAG VERBOSE_LOG OUT_JSON
"""
import collections, csv, json, re, sys

d, vlog, dst = sys.argv[1], sys.argv[2], sys.argv[3]
line = [ln for ln in open(vlog) if "round bytes:" in ln][0]
a = {k: int(v) for k, v in re.findall(r"(\w+)=(\d+)", line.split("round bytes:")[1])}
arrays = {
    "spmv_stream": {"read": ["col16", "col32", "bits", "task_piece", "x_lds", "x_rest"],
                    "write": ["piece_w"]},
    "spmv_rows": {"read": ["piece_r", "roff", "row_maps", "meta"], "write": ["x_out"]},
}
size = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}


def measured(name):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f"{d}/{name}/run_counter_collection.csv")):
        k = row["Kernel_Name"].split("(")[0]
        if "spmv_rows<1" in k or "spmv_rows<2" in k:
            continue  # the last / tracked rounds' row-launch variants
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        key = "spmv_stream" if "spmv_stream" in k else "spmv_rows"
        if name == "rd":
            out[key] = sum(m[c] * size[c] for c in size if c in m)
        else:
            out[key] = m["TCC_EA0_WRREQ_64B_sum"] * 64 + (m["TCC_EA0_WRREQ_sum"] - m["TCC_EA0_WRREQ_64B_sum"]) * 32
    return out


meas = {"read": measured("rd"), "write": measured("wr")}
res = {"arrays_bytes": {k: v for k, v in a.items() if not k.startswith(("n_", "lines", "runs"))},
       "counts": {k: a[k] for k in ("n_col16", "n_col32", "lines", "runs") if k in a},
       "kernels": {}}
for k, dirs in arrays.items():
    e = {}
    for dr, names in dirs.items():
        alg = sum(a[n] for n in names)
        got = meas[dr].get(k, 0.0)
        e[dr] = {"algorithmic": alg, "measured": got, "excess": got - alg,
                 "arrays": {n: a[n] for n in names}}
    res["kernels"][k] = e
tot_alg = sum(e[dr]["algorithmic"] for e in res["kernels"].values() for dr in e)
tot_got = sum(e[dr]["measured"] for e in res["kernels"].values() for dr in e)
res["round"] = {"algorithmic": tot_alg, "measured": tot_got}
json.dump(res, open(dst, "w"), indent=1)
for k, e in res["kernels"].items():
    for dr, v in e.items():
        print(f"{k:12s} {dr:5s} algorithmic {v['algorithmic'] / 1e9:6.3f} GB  measured {v['measured'] / 1e9:6.3f} GB"
              f"  excess {v['excess'] / 1e9:+6.3f} GB  " +
              " ".join(f"{n}={b / 1e9:.3f}" for n, b in v["arrays"].items()))
print(f"round: algorithmic {tot_alg / 1e9:.3f} GB, measured {tot_got / 1e9:.3f} GB")
