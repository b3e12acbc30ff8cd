"""Multi-rank decomposition on CPU: world_size 2 (and 3) over gloo, one process per rank,
each rank computing its contiguous shard of units (huygens_amd.shard.shard_of) and the
partial mixes summed to rank 0 by dist.reduce -- the same decomposition bench.py runs over
RCCL on one GPU per rank."""
import json
import os
import socket
import subprocess
import sys

import pytest

from huygens_amd.shard import shard_of

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(kind, world, tmp_path):
    port = _free_port()
    out = tmp_path / f"{kind}.json"
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), kind, str(out)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        o, _ = p.communicate(timeout=240)
        assert p.returncode == 0, o.decode()[-2000:]
    if kind.startswith(("protocol", "row:", "c2split")):
        return [json.loads((tmp_path / f"{kind}.json.{r}").read_text()) for r in range(world)]
    return json.loads(out.read_text())


@pytest.mark.parametrize("kind", ["filterbank", "oscbank", "bowl", "delaybank"])
def test_world2_reduce_matches_unsharded(kind, tmp_path):
    res = _run(kind, 2, tmp_path)
    assert res["err"] < 1e-12
    assert sum(c for _, c in res["shards"]) == {"filterbank": 96, "oscbank": 50, "bowl": 40, "delaybank": 6}[kind]


def test_world3_uneven(tmp_path):
    res = _run("filterbank", 3, tmp_path)
    assert res["err"] < 1e-12
    assert [c for _, c in res["shards"]] == [32, 32, 32]


@pytest.mark.parametrize("world", [2, 3])
def test_time_shares_gather(world, tmp_path):
    """Stationary calls split by time (bench.py at N > 1): the ranks' shares, gathered to rank 0
    in fixed-size slots, reassemble the whole call (gloo standing in for RCCL)."""
    res = _run("timeshare", world, tmp_path)
    assert res["err"] == 0.0
    shares = res["shares"]
    assert shares[0][0] == 0 and sum(c for _, c in shares) == 3000
    assert all(f1 == f0 + c0 for (f0, c0), (f1, _) in zip(shares, shares[1:]))


def test_time_share_split():
    from huygens_amd.shard import time_share
    assert [time_share(r, 8, 480000) for r in (0, 7)] == [(0, 59392), (419840, 60160)]
    assert sum(time_share(r, 3, 100003)[1] for r in range(3)) == 100003
    assert [time_share(r, 3, 100) for r in range(3)] == [(0, 0), (0, 0), (0, 100)]   # one block: the last rank


def test_shard_of():
    assert [shard_of(r, 3, 10) for r in range(3)] == [(0, 4), (4, 3), (7, 3)]
    assert [shard_of(r, 8, 4096)[1] for r in range(8)] == [512] * 8
    assert shard_of(1, 4, 2) == (1, 1) and shard_of(3, 4, 2) == (2, 0)
    with pytest.raises(ValueError):
        shard_of(2, 2, 5)


@pytest.mark.parametrize("world", [2, 3])
def test_time_shard_protocol(world, tmp_path):
    """huygens_amd.shard.set_time_shards + arm_when_ready through their real code over gloo (a
    fake handle stands in for the HIP object): the bank response is the sum of the shards' over the
    largest horizon on every rank, and the ranks -- ready after different numbers of calls -- are
    armed in the same call, the one after the slowest rank is ready."""
    res = _run("protocol:normal", world, tmp_path)
    for r, rr in enumerate(res):
        assert rr["ok"] is True
        assert rr["bank_len"] == 8192 * world and rr["bank_err"] < 1e-12
        assert rr["shard"] == [r, world]
        assert rr["armed_at"] == 1 + 2 * (world - 1)          # the slowest rank's readiness
    logs = [rr["log"] for rr in res]
    assert all(lg == logs[0] for lg in logs)                # every call: same engine on every rank
    assert res[0]["gather_err"] == 0.0


def test_time_shard_protocol_no_horizon(tmp_path):
    """One shard without a finite horizon: every rank returns False from set_time_shards (no rank
    left waiting in a collective) -- ADVICE r2."""
    res = _run("protocol:no_horizon", 2, tmp_path)
    assert [rr["ok"] for rr in res] == [False, False]

@pytest.mark.parametrize("row", ["c3", "c4"])
def test_bench_row_reduce_world2(row, tmp_path):
    """bench_rows.run_c3 / run_c4 at world 2 through their real multi-rank code -- shard
    construction, the per-step reduce to rank 0, max-over-ranks timing -- over gloo, with fake
    handles on a CPU device (tests/dist_worker.py FakeAdditive / FakeSTFT): rank 0's reduced output
    is the whole job's (C3's N > 1 path had never executed)."""
    res = _run(f"row:{row}", 2, tmp_path)
    assert [r["n_gpus"] for r in res] == [2, 2]
    assert res[0]["ms"] == res[1]["ms"]          # max over ranks on both
    assert res[0]["err"] < 1e-12


@pytest.mark.parametrize("world", [2, 3])
def test_c2_time_split_value_path(world, tmp_path):
    """bench.py's N > 1 C2 value path through its real helpers over gloo:
    every rank arms in the same call although the ranks are ready after different numbers of
    calls (the priming decision agrees across ranks), every rank issues the same
    number of reduces before arming and none after, an armed step writes the whole bank's output
    on the rank's share only (share-only fill, the rest untouched: no collective), and the shares
    gathered to rank 0 (side.gather_to_rank0) are the whole call."""
    res = _run("c2split", world, tmp_path)
    for r, rr in enumerate(res):
        assert rr["ok"] is True and rr["fill"] is False and rr["armed"] is True
        assert rr["calls"] == 1 + 2 * (world - 1)          # the slowest rank's readiness
        assert rr["reduces"] == rr["calls"]                # same collectives on every rank
        assert rr["share_err"] == 0.0 and rr["outside_untouched"]
        assert rr["before_armed_partial"] == 0.0
    assert all(rr["log"] == res[0]["log"] for rr in res)
    shares = [rr["share"] for rr in res]
    assert shares[0][0] == 0 and sum(c for _, c in shares) == 100000
    assert res[0]["gather_err"] == 0.0
