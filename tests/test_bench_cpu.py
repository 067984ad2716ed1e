"""CPU checks of bench.py's ride-along guard (no GPU): a failing key-switch leg is reported inside
the line, and a leg that never finishes makes rank 0 print the line without it and exit -- so the
driver's scaling runs always get the headline line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_guarded_leg_reports_exceptions():
    sys.path.insert(0, ROOT)
    import bench

    def boom():
        raise RuntimeError("no communicator")

    res = bench.guarded_leg(boom, {"metric": "m"}, 0, "keyswitch_leg", timeout_s=30)
    assert res == {"error": "RuntimeError: no communicator"}
    assert bench.guarded_leg(lambda: {"value": 1}, {}, 0, "x", timeout_s=30) == {"value": 1}


def test_guarded_leg_timeout_emits_the_line():
    code = f"""
import argparse, os, sys, time
sys.path.insert(0, {ROOT!r})
import bench
bench._EMIT.update(json_fd=os.dup(1), args=argparse.Namespace(steps=3, warmup=1), world=1)
out = {{"metric": "m", "value": 42.0, "unit": "HomMult/s", "ms_per_step": 1.0,
        "config": {{"workload": "w"}}}}
bench.guarded_leg(lambda: time.sleep(60), out, 0, "keyswitch_leg", timeout_s=1.0)
print("not reached")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=50)
    assert r.returncode == 0
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] == 42.0 and "did not finish" in line["keyswitch_leg"]["error"]
    assert "not reached" not in r.stdout
