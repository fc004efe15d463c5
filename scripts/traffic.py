#!/usr/bin/env python3
"""Turn a collect_profiles.sh run into per-round HBM traffic of the SpMV kernels.

Reads use the L2->EA request counters by size (TCC_EA0_RDREQ_{32,64,128}B x bytes): on
gfx950 FETCH_SIZE tallies 128-B requests at 64 B (MI355X_MICROARCH.md, HBM), so the sized
counters give the byte count directly; FETCH_SIZE x 1024 is reported beside it.  Writes
use TCC_EA0_WRREQ_64B x 64 + (WRREQ - WRREQ_64B) x 32, with WRITE_SIZE beside it.
usage: scripts/traffic.py gpurun_out/prof_TAG WORKLOAD_KEY [profiles/traffic.json]
"""
import collections, csv, json, os, sys

d, key = sys.argv[1], sys.argv[2]
dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")


def load(name):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(os.path.join(d, name, "run_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].split("(")[0]
            agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return agg


def per_round(agg, ctr):
    """sum over the SpMV kernels of one round (mean per dispatch of each kernel, summed
    over the distinct kernels that run once per round: stream launch + row launch)."""
    tot = 0.0
    for k, cs in agg.items():
        if ctr in cs and ("spmv_stream" in k or "spmv_rows" in k):
            tot += sum(cs[ctr]) / len(cs[ctr])
    return tot


rd, wr, fe, ws, l2 = (load(x) for x in ("rd", "wr", "fetch", "write", "l2"))
# spmv_rows<0> (plain rounds) and <1> (last round) both appear: keep one row-launch variant
for agg in (rd, wr, fe, ws, l2):
    for k in list(agg):
        if "spmv_rows<1" in k or "spmv_rows<2" in k:
            del agg[k]
read_b = (per_round(rd, "TCC_EA0_RDREQ_32B_sum") * 32 + per_round(rd, "TCC_EA0_RDREQ_64B_sum") * 64
          + per_round(rd, "TCC_EA0_RDREQ_128B_sum") * 128)
w_all, w64 = per_round(wr, "TCC_EA0_WRREQ_sum"), per_round(wr, "TCC_EA0_WRREQ_64B_sum")
write_b = w64 * 64 + (w_all - w64) * 32
entry = {
    "hbm_bytes_per_launch": read_b + write_b,
    "read_bytes": read_b, "write_bytes": write_b,
    "fetch_size_x1024": per_round(fe, "FETCH_SIZE") * 1024,
    "write_size_x1024": per_round(ws, "WRITE_SIZE") * 1024,
    "l2_hit": per_round(l2, "TCC_HIT_sum"), "l2_miss": per_round(l2, "TCC_MISS_sum"),
    "note": "per round = one spmv_stream + one spmv_rows launch; rocprofv3 PMC passes",
}
cur = json.load(open(dst)) if os.path.exists(dst) else {}
cur[key] = entry
json.dump(cur, open(dst, "w"), indent=1, sort_keys=True)
print(key, json.dumps(entry, indent=1))
