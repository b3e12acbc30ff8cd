"""bench.py --gpus N: outside a launcher, N > 1 reruns bench.py under
torch.distributed.run as a child process (no GPU touched by the parent) and forwards rank 0's
JSON line; under a launcher, WORLD_SIZE must equal --gpus or the run exits non-zero.  CPU only:
HZ_BENCH_DRY=1 stops every rank right after the launch check, before any torch import."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_plan():
    assert bench.launch_plan(1, {}) == ("run", None)
    assert bench.launch_plan(4, {})[0] == "relaunch"
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == ("run", None)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("run", None)
    for gpus, ws in ((1, "2"), (8, "4"), (2, "x")):
        plan, why = bench.launch_plan(gpus, {"WORLD_SIZE": ws})
        assert plan == "mismatch" and why
    assert bench.launch_plan(0, {})[0] == "mismatch"


def test_relaunch_cmd():
    cmd = bench.relaunch_cmd(8, ["--gpus", "8", "--steps", "5"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5].endswith("bench.py")


def test_forward_child_prints_only_the_json_line(capfd):
    code = ("import json,sys; print('noise'); print(json.dumps({'metric': 'm', 'value': 1})); "
            "sys.stderr.write('err\\n'); sys.exit(3)")
    rc = bench.forward_child([sys.executable, "-c", code])
    out, err = capfd.readouterr()
    assert rc == 3
    assert out.strip().splitlines() == ['{"metric": "m", "value": 1}']
    assert "noise" in err


def _run(args, env_extra, timeout=120):
    env = dict(os.environ, HZ_BENCH_DRY="1", **env_extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        if k not in env_extra:
            env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def test_gpus_2_relaunches_two_ranks():
    """the driver's own command line: `python bench.py --gpus 2` with no launcher"""
    r = _run(["--gpus", "2", "--steps", "1"], {})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["gpus_arg"] == 2


def test_gpus_1_runs_in_process():
    r = _run(["--gpus", "1"], {})
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip())["n_gpus"] == 1


@pytest.mark.parametrize("gpus,ws", [(1, "2"), (4, "2")])
def test_mismatch_exits_nonzero(gpus, ws):
    r = _run(["--gpus", str(gpus)], {"WORLD_SIZE": ws, "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr and not r.stdout.strip()
