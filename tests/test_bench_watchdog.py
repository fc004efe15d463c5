"""bench.py's multi-rank watchdog (CPU): when the engine reports no finished round for the
limit, the process ends itself with exit code 86 and a message naming the rank, the exchange and
the round -- a fresh exit (os._exit), nothing is re-executed."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SNIPPET = r"""
import sys, time
sys.path.insert(0, {root!r})
import bench

class Stuck:
    def progress(self):
        return (7, 4)          # seven rounds handed to the device, four finished, forever

dog = bench.Watchdog(Stuck(), rank=1, world=2, exchange="rccl", limit=0.6)
dog.start()
dog.enter("rounds (timed)", 20)
time.sleep(30)
print("not reached")
"""


def test_watchdog_ends_a_stuck_round_loop(engine_mod):
    out = subprocess.run([sys.executable, "-c", SNIPPET.format(root=ROOT)], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 86, (out.returncode, out.stderr[-2000:])
    assert "not reached" not in out.stdout
    msg = out.stderr
    assert "rank 1/2" in msg and "rccl exchange" in msg and "4 finished" in msg
    assert "after round 4" in msg and "20 rounds requested" in msg


def test_watchdog_stays_quiet_while_rounds_finish(engine_mod):
    snippet = SNIPPET.replace("return (7, 4)", "import time as t; return (9, int(t.monotonic() * 10))") \
                     .replace("time.sleep(30)", "time.sleep(2.0); dog.stop()") \
                     .replace('print("not reached")', 'print("alive")')
    out = subprocess.run([sys.executable, "-c", snippet.format(root=ROOT)], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 0 and "alive" in out.stdout, out.stderr[-2000:]
