#!/usr/bin/env python3
"""Benchmark: PageRank rounds/s on R-MAT scale 26 (BASELINE.json config 4) on MI355X.

A "step" is one PageRank round (PageRank.java:92-164): the fused pull SpMV over every
distinct edge, dangling redistribution and damping, plus -- on more than one GPU -- the
exchange of the contribution vector (grouped RCCL send/recv per row-launch chunk on a comm
stream, and an all-gather of the exact per-rank record).  The graph (R-MAT scale 26, edge factor 16, seed 4,
generated on the device; ~1.06e9 distinct edges) is resident in HBM before timing starts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--no-cpu-baseline]
                  [--exchange rccl|external] [--watchdog SECONDS]
  (N > 1: launched by torch.distributed.run, one process per GPU; RCCL over xGMI; the
   graph is the same for every N -> strong scaling.  --exchange external moves every round's
   x slot and exact record through the gloo world instead (host-staged, pr_ext_*): the same
   launch harness and per-rank engine work with only the transport changed, so an N-process
   world also runs on one GPU.  At N > 1 a watchdog thread follows the rounds the device has
   finished (pr_progress) and ends the process with a message naming the round when nothing
   completes for --watchdog seconds.)

Prints ONE JSON line on rank 0 (metric GTEPS = distinct edges / round time / 1e9).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "page-rank-and-tfidf-using-apache-spark_amd"))

import prmi355x as P  # noqa: E402

P.lib()  # load the engine (and ROCm's HIP + RCCL) before torch brings its own copies

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
# achievable streaming-read bandwidth measured on the box (8 x dwordx4 per lane, 1 WG/CU;
# profiles/r01/stream_probe.log, scripts/probes/): SURVEY.md 8d's "STREAM-copy" reference
STREAM_READ_GBS = 6330.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rounds", type=int, default=40)   # ~10 s of host CPU work at scale 26
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--exchange", choices=("rccl", "external"), default="rccl",
                    help="N > 1: RCCL over xGMI (one GPU per rank), or the caller-staged "
                         "exchange over the gloo world (any number of ranks per GPU)")
    ap.add_argument("--watchdog", type=float, default=90.0,
                    help="N > 1: seconds without a finished round before the process exits "
                         "with a diagnostic (0 = off)")
    return ap.parse_args()


class Watchdog(threading.Thread):
    """Ends the process (os._exit: a fresh exit, nothing is re-executed) when the engine's
    round loop stops finishing rounds.  `phase` names what the main thread is doing; only the
    phases in `watched` are timed."""

    def __init__(self, eng, rank, world, exchange, limit):
        super().__init__(daemon=True)
        self.eng, self.rank, self.world, self.exchange, self.limit = eng, rank, world, exchange, limit
        self.phase = "setup"
        self.rounds = 0
        self._stop = threading.Event()

    def enter(self, phase, rounds=0):
        self.phase, self.rounds = phase, rounds
        self._last = (None, time.monotonic())

    def stop(self):
        self._stop.set()

    def run(self):
        self._last = (None, time.monotonic())
        while not self._stop.wait(0.5):
            if not self.phase.startswith("rounds"):
                continue
            prog = self.eng.progress()
            now = time.monotonic()
            if prog != self._last[0]:
                self._last = (prog, now)
            elif now - self._last[1] > self.limit:
                sys.stderr.write(
                    f"[bench watchdog] rank {self.rank}/{self.world} ({self.exchange} exchange): no "
                    f"round finished for {self.limit:.0f} s in phase '{self.phase}' "
                    f"({self.rounds} rounds requested): {prog[0]} rounds handed to the device, "
                    f"{prog[1]} finished -- the exchange after round {prog[1]} did not complete "
                    f"on this rank; exiting\n")
                sys.stderr.flush()
                os._exit(86)


def cpu_baseline(eng, rounds: int):
    """The oracle's plain-fp64 OpenMP restatement ("port") on this host's cores, timed on a
    bounded sample: `rounds` rounds over the SAME graph (exported CSR, relabelled)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    rp, col, od, dw = eng.export_csr()
    info = eng.info()
    t0 = time.time()
    res = O.pagerank_csr(rp, col, od, dw, int(info["n_tot"]), rounds, exact=False,
                         threads=cores)
    wall = time.time() - t0
    gteps = info["nnz"] / res["sec_per_iter"] / 1e9
    return {"value": round(gteps, 4), "unit": "GTEPS", "cores": cores, "kind": "port",
            "sample": f"{rounds} rounds of the same R-MAT graph ({int(info['nnz'])} edges), "
                      f"oracle/pagerank_oracle.c fast mode (plain fp64 OpenMP pull), "
                      f"{res['sec_per_iter']:.3f} s/round, {wall:.1f} s total"}


def load_traffic(path: str, workload: str):
    """Per-launch HBM bytes of the SpMV kernel from the committed rocprofv3 PMC summary."""
    try:
        d = json.load(open(path))
        e = d.get(workload)
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if a.gpus != world and world > 1:
        a.gpus = world
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)   # rendezvous only
    eng = P.Engine(n_ranks=world, rank=rank)
    external = world > 1 and a.exchange == "external"
    allgather = None
    if world > 1 and external:
        import torch
        eng.comm_init_external()

        def allgather(send):                      # host buffers only: gloo never sees the GPU
            t = torch.from_numpy(send)
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            return torch.cat(parts).numpy()
    elif world > 1:
        import torch
        uid = P.comm_unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        eng.comm_init(bytes(t.tolist()))
    comm = eng.comm_query()
    dog = None
    if world > 1 and a.watchdog > 0:
        dog = Watchdog(eng, rank, world, a.exchange, a.watchdog)
        dog.start()
    t0 = time.time()
    eng.generate_rmat(a.scale, a.edge_factor, a.seed)
    info = eng.info()
    build_s = time.time() - t0

    def barrier():
        if dist is not None:
            dist.barrier()

    def rounds(k, phase):
        if dog is not None:
            dog.enter(phase, k)
        st_ = eng.run_external(k, allgather) if external else eng.run(k)
        if dog is not None:
            dog.enter("idle")
        return st_

    # (at p > 1 the first exchanged run builds and cross-checks the sparse-exchange lists:
    # at least one untimed round, whatever --warmup says)
    if a.warmup > 0 or world > 1:
        rounds(max(a.warmup, 1 if world > 1 else 0), "rounds (warm-up)")
    barrier()
    t1 = time.perf_counter()
    st = rounds(a.steps, "rounds (timed)")
    t2 = time.perf_counter()
    barrier()
    if dog is not None:
        dog.stop()
    wall = t2 - t1
    if external:                                  # pr_ext_end reports no loop time of its own
        st["ms_per_iter"] = wall * 1e3 / a.steps
    exposed_rank = None
    if dist is not None:
        import torch
        w = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
        # per rank: what the exchange, the record all-gather and finalize leave exposed on
        # top of that rank's own SpMV launches
        mine = torch.tensor([(t2 - t1) * 1e3 / a.steps - st["ms_spmv_kernel"]], dtype=torch.float64)
        parts = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, mine)
        exposed_rank = [round(max(float(x.item()), 0.0), 4) for x in parts]
        k = torch.tensor([st["ms_spmv_kernel"]], dtype=torch.float64)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        st["ms_spmv_kernel"] = float(k.item())
    ms_step = wall * 1e3 / a.steps
    nnz = int(info["nnz"])
    n = int(info["n_vertices"])
    gteps = nnz / (ms_step * 1e-3) / 1e9
    workload = f"rmat-s{a.scale}-ef{a.edge_factor}"
    # roofline of the SpMV of one round (stream launch + row launch, bracketed by HIP events on
    # the engine stream): SURVEY.md 8d algorithmic bytes per launch.  p = 1: 4 nnz + 24 N + 8.
    # p > 1, per rank: its own edges' columns, the WHOLE x (every rank gathers from all
    # sources), its share of row pointers and rank writes: 4 local_nnz + 8 N + 16 N / p + 8.
    local_nnz = int(info["local_nnz"])
    if world == 1:
        bytes_launch = 4 * local_nnz + 24 * n + 8
    else:
        bytes_launch = 4 * local_nnz + 8 * n + 16 * n // world + 8
    kms = st["ms_spmv_kernel"]
    achieved = bytes_launch / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    traffic = load_traffic(a.traffic_json, f"{workload}-p{world}")
    sparse_x = world > 1 and not external and os.environ.get("PR_SPARSE_X", "1") != "0"  # api.cpp want_sx
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(eng, a.cpu_rounds)
    if rank == 0:
        line = {
            "metric": f"PageRank GTEPS per round (distinct edges / round time), R-MAT scale-{a.scale}",
            "value": round(gteps, 3),
            "unit": "GTEPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (Graph500 R-MAT generated on device, Philox seed %d)" % a.seed,
            "config": {"workload": workload, "scale": a.scale, "edge_factor": a.edge_factor,
                       "vertices": n, "distinct_edges": nnz, "rounds_per_step": 1,
                       "parallelism": (f"rows dealt over {world} ranks, x' slots and exact records "
                                       f"all-gathered over the gloo world (host-staged, pr_ext_*)"
                                       if external else
                                       f"rows dealt over {world} GPUs, chunked RCCL p2p "
                                       f"exchange of x' overlapped with the row launch"
                                       + (" (sparse: referenced entries only)" if sparse_x else ""))
                       if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": "spmv_stream+spmv_rows (the SpMV of one round)",
                         "time_source": "HIP events on the engine stream around the two "
                                        "launches of each round, mean over the timed rounds "
                                        "(pr_stats.ms_spmv_kernel)",
                         "kernel_ms": round(kms, 4),
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "achievable_stream_read_gbs": STREAM_READ_GBS,
                         "frac_of_achievable": round(achieved / STREAM_READ_GBS, 4)},
            "cpu_baseline": cpu,
            "device_ms_per_round": round(st["ms_per_iter"], 4),
            # per round: the SpMV launches (slowest rank) and what the exchange, the record
            # all-gather and finalize leave exposed on top of them
            "round_breakdown_ms": {"spmv_kernels": round(kms, 4),
                                   "exposed_exchange_and_finalize": round(max(ms_step - kms, 0.0), 4)},
            # the transport the rounds used: for RCCL, ncclCommCount / ncclCommUserRank of
            # this rank's communicator (must equal n_gpus / 0 on rank 0)
            "exchange": {"transport": comm["transport"], "comm_ranks": comm["comm_ranks"],
                         "comm_rank": comm["comm_rank"],
                         "exposed_ms_per_rank": exposed_rank},
            "build_s": round(build_s, 2),
            # the build may move the per-piece sums to faster physical memory (PR_PLACE=0: off):
            # placements it timed beyond the first, stream launch with the first and with the
            # one it kept (rank 0)
            "placement": {"tried": int(info.get("place_tried", 0)),
                          "stream_ms_first": round(info.get("place_ms_first", 0.0), 4),
                          "stream_ms_kept": round(info.get("place_ms_best", 0.0), 4)},
            "build_id": P.build_id(),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
