"""bench.py's output contract on the GPU: one JSON line with the driver's keys, the roofline and
cpu_baseline objects, and the streaming figure's detail (a short run: 3 timed steps)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--no-traffic", "--no-per-sample", "--side-steps", "0", "--stream-blocks", "16"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["dtype"] == "f64"
    assert "workload" in d["config"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["bound"] in ("hbm", "mfma") and 0 < rf["frac"] < 1.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    st = d["streaming"]
    assert st["block"] == 1024 and st["us_per_block"] > 0
    assert st["kernels"] and st["roofline"]["bound"].startswith("latency")
    # 1024-sample calls of the stationary C2 bank take the streaming engine: one launch per block
    assert st["path"] == "stream" and st["launches_per_block"] == 1, st
    assert st["end_to_end_host_buffers"]["us_per_block"] > 0
    assert st["per_band_engine"]["path"] == "lti"
