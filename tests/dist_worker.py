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


class FakeShardHandle:
    """Stands in for huygens_amd.Filterbank on a CPU rank (no GPU here): the methods
    huygens_amd.shard calls, with a horizon, a response and a readiness schedule chosen per rank,
    so set_time_shards / arm_when_ready / time_share / ShareGather run through their real code."""

    def __init__(self, rank, K, ready_after, fail_probe=False):
        self.rank, self.K, self.ready_after, self.fail_probe = rank, K, ready_after, fail_probe
        self.calls = 0
        self.bank = None
        self.shard = None
        self.armed = False
        self.log = []

    def response(self, count):
        if self.fail_probe:
            raise RuntimeError("HZ_E_UNSUPPORTED: no finite horizon")
        t = np.arange(count, dtype=np.float64)
        return np.where(t < self.K, (self.rank + 1) * 0.5 ** (t / 4096.0), 0.0)

    def response_info(self):
        return self.K, 0, False, 0

    def set_bank_response(self, h):
        self.bank = np.array(h)

    def set_time_shard(self, rank, world):
        self.shard = (rank, world)

    def stationary_ready(self, n):
        return self.calls >= self.ready_after

    def arm_time_shard(self, armed=True):
        self.armed = bool(armed)

    def call(self):
        self.calls += 1
        self.log.append(self.armed)


def _shard_protocol(rank, world, variant):
    """set_time_shards + arm_when_ready over gloo with FakeShardHandle ranks."""
    import torch
    import torch.distributed as dist
    from huygens_amd.shard import ShareGather, arm_when_ready, set_time_shards, time_share

    def ar_sum(a):
        t = torch.from_numpy(np.array(a, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    def ar_max(k):
        t = torch.tensor([int(k)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    def ar_min(k):
        t = torch.tensor([int(k)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    K = 8192 * (rank + 1)                       # the ranks' horizons differ
    fb = FakeShardHandle(rank, K, ready_after=1 + 2 * rank,
                         fail_probe=(variant == "no_horizon" and rank == world - 1))
    ok = set_time_shards(fb, rank, world, ar_sum, ar_max)
    res = {"ok": ok}
    if ok:
        K_all = 8192 * world
        t = np.arange(K_all, dtype=np.float64)
        want = sum(np.where(t < 8192 * (r + 1), (r + 1) * 0.5 ** (t / 4096.0), 0.0) for r in range(world))
        res["bank_err"] = float(np.max(np.abs(fb.bank - want)))
        res["bank_len"] = len(fb.bank)
        res["shard"] = list(fb.shard)
        armed_at = None
        for c in range(8):                      # calls, with the arming protocol between them
            fb.call()
            if not fb.armed and arm_when_ready(fb, 480000, ar_min):
                armed_at = fb.calls
        res["armed_at"] = armed_at
        res["log"] = fb.log
        # the armed calls' output shares, assembled on rank 0 through ShareGather
        n = 100000
        f, c = time_share(rank, world, n)
        y = torch.zeros(n, dtype=torch.float64)
        y[f:f + c] = torch.arange(f, f + c, dtype=torch.float64)
        ShareGather(n, rank, world, y)(y, dist)
        if rank == 0:
            res["gather_err"] = float(torch.max(torch.abs(y - torch.arange(n, dtype=torch.float64))).item())
    return res


class FakeC2Handle(FakeShardHandle):
    """Stands in for the C2 Filterbank shard in bench.py's N > 1 value path (bench.c2_setup_time_split,
    bench.c2_prime, the share-only step): before arming, a call writes its own bands' partial mix over
    the whole call (here (rank + 1) x); once armed, the WHOLE bank's output (here sum over ranks of
    (r + 1) x) on this rank's time share only, leaving the rest of the buffer untouched."""

    def __init__(self, rank, world, K, ready_after):
        super().__init__(rank, K, ready_after)
        self.world, self.fill = world, True

    def set_time_shard_fill(self, zero_outside=True):
        self.fill = bool(zero_outside)

    def time_shard_info(self, n):
        from huygens_amd.shard import time_share
        f, c = time_share(self.shard[0], self.shard[1], n)
        return True, f, c

    def process_device(self, xp, yp, n):
        import ctypes
        x = np.ctypeslib.as_array((ctypes.c_double * n).from_address(xp)).copy()
        y = np.ctypeslib.as_array((ctypes.c_double * n).from_address(yp))
        self.call()
        if self.armed:
            _, f, c = self.time_shard_info(n)
            whole = sum(r + 1 for r in range(self.world)) * x
            if self.fill:
                y[:] = 0.0
            y[f:f + c] = whole[f:f + c]
        else:
            y[:] = (self.rank + 1) * x

    def last_path(self):
        return 3 if self.armed else 2


def _c2_split(rank, world):
    """bench.py's N > 1 C2 value path through its real helpers over gloo: c2_setup_time_split (the
    whole-bank response and the share-only fill on every rank), c2_prime (ranks ready after
    different numbers of calls are armed in the same call), the share-only steps (no collective),
    and ShareGather.start / finish (side.gather_to_rank0) assembling the whole call on rank 0."""
    import torch
    import torch.distributed as dist
    import bench
    from huygens_amd.shard import ShareGather

    def ar_sum(a):
        t = torch.from_numpy(np.array(a, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    def ar_op(op):
        def f(k):
            t = torch.tensor([int(k)], dtype=torch.int64)
            dist.all_reduce(t, op=op)
            return int(t.item())
        return f
    coll = (ar_sum, ar_op(dist.ReduceOp.MAX), ar_op(dist.ReduceOp.MIN))
    fb = FakeC2Handle(rank, world, 8192 * (rank + 1), ready_after=1 + 2 * rank)
    ok = bench.c2_setup_time_split(fb, rank, world, coll)
    n = 100000
    x = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, n))
    y = torch.full((n,), 7.0, dtype=torch.float64)
    armed = [False]
    reduces = [0]

    def step():
        fb.process_device(x.data_ptr(), y.data_ptr(), n)
        if not armed[0]:   # (band shards before arming: partial mixes reduced, as bench.step)
            t = y.clone()
            dist.reduce(t, dst=0)
            reduces[0] += 1
    calls = bench.c2_prime(fb, step, n, ok, coll[2], 3, armed=armed)
    before = y.clone()
    y.fill_(7.0)
    step()                                   # an armed (timed) step: the share only, no collective
    _, f, c = fb.time_shard_info(n)
    whole = sum(r + 1 for r in range(world)) * x
    res = {"ok": ok, "fill": fb.fill, "armed": armed[0], "calls": calls, "reduces": reduces[0],
           "log": fb.log, "share": [f, c],
           "share_err": float(torch.max(torch.abs(y[f:f + c] - whole[f:f + c])).item()),
           "outside_untouched": bool(torch.all(torch.cat([y[:f], y[f + c:]]) == 7.0).item()),
           "before_armed_partial": float(torch.max(torch.abs(before - (rank + 1) * x)).item())}
    g = ShareGather(n, rank, world, y)
    w = g.start(y, dist, async_op=True)
    w.wait()
    g.finish(y)
    if rank == 0:
        res["gather_err"] = float(torch.max(torch.abs(y - whole)).item())
    return res


class FakeAdditive:
    """Stands in for huygens_amd.Additive in bench_rows.run_c3 on a CPU device: fill_device writes
    the shard's partial mix y[t] = sum over its overtones o of cos(1e-3 (o + 1) t), t the handle's
    running sample count, into the (CPU) buffer at the pointer."""

    def __init__(self, V, O, k_p, k_g, device=0, shard=None):
        self.o0, self.oc = shard if shard is not None else (0, O)
        self.t = 0

    def makenote(self, *a):
        pass

    def release(self, v):
        pass

    def set_stream(self, s):
        pass

    def fill_device(self, ptr, n):
        import ctypes
        t = np.arange(self.t, self.t + n, dtype=np.float64)
        o = np.arange(self.o0, self.o0 + self.oc, dtype=np.float64)[:, None]
        y = np.ascontiguousarray(np.cos(1e-3 * (o + 1) * t).sum(axis=0) if self.oc else np.zeros(n))
        ctypes.memmove(ptr, y.ctypes.data, 8 * n)
        self.t += n

    def profile(self, on):
        pass

    def profile_read(self):
        return 1.0, 1


class FakeSTFT:
    """Stands in for StaticSTFT / Fourier in bench_rows.run_c4 on a CPU device: process_block_device
    writes x[t] for the samples of this rank's frame runs (runs of `per` 1024-sample hops rotating
    over the ranks) and 0 elsewhere, so the reduced output is x."""

    def __init__(self, *a):
        self.rank, self.world, self.per, self.f = 0, 1, 1, 0

    def set_stream(self, s):
        pass

    def set_frame_shard(self, rank, world, per):
        self.rank, self.world, self.per = rank, world, per

    def process_block_device(self, xp, _, yrp, yip, n):
        import ctypes
        x = np.ctypeslib.as_array((ctypes.c_double * n).from_address(xp)).copy()
        run = (np.arange(n) // 1024) // max(1, self.per)
        y = np.where(run % self.world == self.rank, x, 0.0)
        ctypes.memmove(yrp, np.ascontiguousarray(y).ctypes.data, 8 * n)
        ctypes.memmove(yip, np.zeros(n).ctypes.data, 8 * n)
        self.f += n // 1024

    def frames(self):
        return (self.f, 0)

    def profile(self, on, repeat=1):
        pass

    def profile_read(self):
        return 1.0, 1.0, 1


def _row(kind, rank, world, dist):
    """bench_rows.run_c3 / run_c4 through their real multi-rank code (the reduce to rank 0, the
    max-over-ranks timing) over gloo, fake handles standing in for the HIP objects."""
    import argparse
    import torch
    import bench_rows
    import huygens_amd
    bench_rows.COLL = dist
    args = argparse.Namespace(samples=4800, warmup=1, steps=2, no_cpu_baseline=True, no_traffic=True)
    got = {}
    if kind == "c3":
        huygens_amd.Additive = FakeAdditive
        body = bench_rows.run_c3(args, torch, torch.device("cpu"), rank, world,
                                 probe=lambda y: got.setdefault("y", y.clone()))
        t = np.arange((args.warmup + args.steps - 1) * args.samples, (args.warmup + args.steps) * args.samples)
        full = np.cos(1e-3 * (np.arange(256)[:, None] + 1) * t).sum(axis=0)
    else:
        huygens_amd.StaticSTFT = FakeSTFT
        huygens_amd.Fourier = FakeSTFT
        body = bench_rows.run_c4(args, torch, torch.device("cpu"), rank, world,
                                 probe=lambda y: got.setdefault("y", y.clone()))
        full = bench_rows.c4_signal(args.samples)
    res = {"n_gpus": body["n_gpus"], "value": body["value"], "ms": body["ms_per_step"]}
    if rank == 0 and got.get("y") is not None:
        res["err"] = float(np.max(np.abs(got["y"].numpy() - full)) / np.max(np.abs(full)))
    return res


def main():
    import torch
    import torch.distributed as dist
    from huygens_amd.shard import shard_of
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    kind, out_path = sys.argv[1], sys.argv[2]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if kind.startswith("row:"):
        res = _row(kind.split(":")[1], rank, world, dist)
        with open(f"{out_path}.{rank}", "w") as fh:
            json.dump(res, fh)
        dist.barrier()
        dist.destroy_process_group()
        return
    if kind == "c2split":
        res = _c2_split(rank, world)
        with open(f"{out_path}.{rank}", "w") as fh:
            json.dump(res, fh)
        dist.barrier()
        dist.destroy_process_group()
        return
    if kind.startswith("protocol"):
        res = _shard_protocol(rank, world, kind.split(":")[1])
        with open(f"{out_path}.{rank}", "w") as fh:
            json.dump(res, fh)
        dist.barrier()
        dist.destroy_process_group()
        return
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
