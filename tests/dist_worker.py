"""world_size-N gloo worker for tests/test_dist_cpu.py (TEST INFRASTRUCTURE).

Each rank runs ITS shard of a bank -- the oracle stands in for the GPU kernel, which the
CPU container cannot run -- and the partial mixes are summed to rank 0 with the same
dist.reduce the GPU path issues over RCCL (bench.py).  Rank 0 compares with the unsharded
bank and writes the error to a result file.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def _filterbank(b0, cnt, N, x):
    from golden.spec_numpy import resonant_coefficients
    from oracle import OracleFilterbank
    fwd, back = resonant_coefficients(N, 0.999, 1.0)
    fb = OracleFilterbank(2, cnt)
    for i in range(cnt):
        fb.coefficients(i, fwd[b0 + i], back[b0 + i])
    fb.boost(np.ones(cnt))
    fb.open()
    return fb.process(x)


def _oscbank(b0, cnt, N, n):
    from oracle import OracleOscbank
    f = 20.0 * 1.0007 ** np.arange(N)
    o = OracleOscbank(cnt)
    for i in range(cnt):
        o.freqmod(i, f[b0 + i])
    o.open()
    mix = o.fill(n)
    return np.concatenate([mix.real, mix.imag])


def _bowl(b0, cnt, N, n):
    from oracle_bowl import OracleBowl
    rng = np.random.default_rng(5)
    f = np.exp(rng.uniform(np.log(20.0), np.log(16000.0), N))
    a = rng.uniform(1e-4, 5e-2, N)
    d = rng.uniform(0.05, 15.0, N)
    return OracleBowl(cnt, f[b0:b0 + cnt], a[b0:b0 + cnt], d[b0:b0 + cnt]).render(n)


def _delaybank(b0, cnt, N, x):
    from oracle_delay import OracleDelaybank
    b = OracleDelaybank(cnt, 3, 2000)
    for k in range(cnt):
        g = b0 + k
        b.coefficients(k, [(0, 1.0)], [(500 + 37 * g, 0.5), (900 + 53 * g, 0.45)])
    return b.process(x).sum(axis=0)   # unscaled line sum; / N after the reduce


def _timeshare(rank, world, N, x):
    """Time-sharded stationary calls: each rank holds the WHOLE bank's output (the oracle stands
    in for the convolution with the whole-bank response) only on its share, zeros elsewhere; the
    shares are assembled on rank 0 by the same ShareGather bench.py uses over RCCL."""
    import torch
    from huygens_amd.shard import ShareGather, time_share
    full = _filterbank(0, N, N, x)
    f, c = time_share(rank, world, len(x), block=256)
    y = torch.zeros(len(x), dtype=torch.float64)
    y[f:f + c] = torch.from_numpy(full[f:f + c])
    return y, full, ShareGather(len(x), rank, world, y, block=256)


def main():
    import torch
    import torch.distributed as dist
    from huygens_amd.shard import shard_of
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    kind, out_path = sys.argv[1], sys.argv[2]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N = {"filterbank": 96, "oscbank": 50, "bowl": 40, "delaybank": 6, "timeshare": 96}[kind]
    n = 3000
    x = np.random.default_rng(1).uniform(-1, 1, n).astype(np.float32).astype(np.float64)
    if kind == "timeshare":
        import torch.distributed as dist_
        y, full, g = _timeshare(rank, world, 96, x)
        g(y, dist_)
        if rank == 0:
            err = float(np.max(np.abs(y.numpy() - full)) / np.max(np.abs(full)))
            with open(out_path, "w") as fh:
                json.dump({"err": err, "shares": g.shares}, fh)
        dist.barrier()
        dist.destroy_process_group()
        return
    b0, cnt = shard_of(rank, world, N)
    fn = {"filterbank": lambda b, c: _filterbank(b, c, N, x), "oscbank": lambda b, c: _oscbank(b, c, N, n),
          "bowl": lambda b, c: _bowl(b, c, N, n), "delaybank": lambda b, c: _delaybank(b, c, N, x)}[kind]
    part = torch.from_numpy(np.ascontiguousarray(fn(b0, cnt)))
    dist.reduce(part, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        full = fn(0, N)
        got = part.numpy()
        err = float(np.max(np.abs(got - full)) / np.max(np.abs(full)))
        with open(out_path, "w") as fh:
            json.dump({"err": err, "shards": [shard_of(r, world, N) for r in range(world)]}, fh)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
