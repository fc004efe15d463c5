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
