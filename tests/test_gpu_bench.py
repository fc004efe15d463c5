"""bench.py keeps the driver's JSON contract: one line on rank 0 with the metric, the roofline
object of the SpMV launches and the CPU baseline of the oracle port (small R-MAT scale, so the
whole run takes seconds)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--scale", "14",
                          "--steps", "3", "--warmup", "1", "--cpu-rounds", "2"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["unit"] == "GTEPS" and d["value"] > 0 and d["n_gpus"] == 1
    assert d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["dtype"] == "f64" and d["config"]["workload"] == "rmat-s14-ef16"
    assert d["config"]["distinct_edges"] > 0
    # GTEPS is distinct edges over the measured time per round
    assert abs(d["value"] - d["config"]["distinct_edges"] / (d["ms_per_step"] * 1e6)) \
        <= 1e-3 * d["value"] + 1e-3
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert rf["achieved"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # no committed PMC summary for this small workload
    assert rf["traffic"] is None
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "GTEPS" and cb["value"] > 0 and cb["cores"] >= 1


@pytest.mark.gpu
def test_bench_two_process_world_external():
    """The driver's multi-process launch line (torch.distributed.run, one process per rank) on
    this one GPU with --exchange external: the rounds' x slots and exact records travel through
    the gloo world instead of RCCL, everything else is the multi-GPU bench path (ranks' row
    deals, the untimed warm-up, barriers, max over ranks, rank 0's single JSON line)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--steps", "3", "--warmup", "1", "--scale", "15",
                          "--exchange", "external", "--watchdog", "60"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "strong"
    assert d["config"]["workload"] == "rmat-s15-ef16" and d["value"] > 0
    assert abs(d["value"] - d["config"]["distinct_edges"] / (d["ms_per_step"] * 1e6)) \
        <= 1e-3 * d["value"] + 1e-3
    ex = d["exchange"]
    assert ex["transport"] == "external" and ex["comm_ranks"] == 2 and ex["comm_rank"] == 0
    assert len(ex["exposed_ms_per_rank"]) == 2 and all(x >= 0 for x in ex["exposed_ms_per_rank"])
    assert d["roofline"]["kernel_ms"] > 0 and d["cpu_baseline"] is None
