#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: band-samples/s of the 4096-band Filterbank<double>.

Workload (BASELINE.json configs[1]): Filterbank<double>(2, 4096),
resonant band-pass bank f_i = 0.5 (i+1) SR / 4096, R = 0.999 (tests/resynthesis.cpp:48-54
recipe), boost(all 1) + open(), k_p = 0.1, k_g = 1, synthetic white noise (uniform[-1,1)
float32 -> double), kernel time tile = the reference's BSIZE 1024.

One step = one Filterbank::process() call over 10 s of 48 kHz audio (480,000 samples),
input already resident in HBM; the result is identical to 469 x {1024-sample block} calls
(tests/test_filterbank_gpu.py::test_block_split_and_per_sample).  A streaming figure
(one call per 1024-sample block) is reported beside it.

Multi-GPU (torchrun, one process per GPU): the 4096 bands are split contiguously over ranks
(each rank keeps its shard's band states).  Once the bank is stationary the
stream is split by TIME: a step is one call of N x 10 s and every rank outputs its 10 s from the
shared input with a K-sample halo, convolving with the whole bank's response (summed over the
band shards by one all-reduce at setup) -- no data-path collective, weak scaling (`--gather`
collects the shares on rank 0 inside the step).  Per-band calls (before the bank is stationary)
sum the band shards' partial mixes to rank 0 with an RCCL reduce.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SR = 48000
N_BANDS = 4096
R_POLE = 0.999
SAMPLES_PER_STEP = 480_000
FP64_PEAK_TFLOPS = 78.6       # MI355X FP64 vector (= FP64 matrix) peak, SURVEY.md 8(d)
HBM_PEAK_GBS = 8000.0
FLOPS_PER_BAND_SAMPLE = 18    # 4*O + 10 with O = 2


def c2_coefficients(N=N_BANDS, R=R_POLE):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden.spec_numpy import resonant_coefficients
    return resonant_coefficients(N, R, 1.0)


def shard_of(rank, world, N=N_BANDS):
    from huygens_amd.shard import shard_of as _shard_of
    return _shard_of(rank, world, N)


def cpu_baseline(fwd, back, seconds_target=1.5):
    """The oracle (C restatement, -O2, no FMA contraction) on the host cores: bands
    split over threads (ctypes releases the GIL), one Filterbank per thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import OracleFilterbank
    threads = max(1, min(16, os.cpu_count() or 1))
    N = fwd.shape[0]
    rng = np.random.default_rng(1)
    nsamp = 480_000
    x = rng.uniform(-1, 1, nsamp).astype(np.float32).astype(np.float64)
    banks = []
    for t in range(threads):
        b0, cnt = shard_of(t, threads, N)
        fb = OracleFilterbank(2, cnt)
        for i in range(cnt):
            fb.coefficients(i, fwd[b0 + i], back[b0 + i])
        fb.boost(np.ones(cnt))
        fb.open()
        banks.append(fb)
    outs = [None] * threads

    def run(i):
        outs[i] = banks[i].process(x)

    t0 = time.perf_counter()
    ths = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    return {"value": N * nsamp / dt, "unit": "band-samples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/hz_oracle.c restatement, {N} bands x {nsamp} samples "
                      f"({nsamp / SR:.2f} s audio), bands split over {threads} threads, {dt:.2f} s wall"}


def fb_executed_flops(lti, L=32, O=2, N=N_BANDS):
    """FP64 flops the kernel actually issues per band-sample.  LTI engine:
    chunk end states on the matrix cores 2 O ceil((L+O)/4) 4 / L, the correction (group mix,
    or the bank-wide GEMM at L >= 64) 2 O, the 64-lane scan 2 (6 O^2 + 2 O^2) 64 / (64 L) per
    chunk; at L >= 64 the GEMM also carries the zero-state term as ceil((L+O)/32) 32 extra K rows
    (2 flops per row and sample, shared by the N bands); general engine ~2 x 10."""
    if not lti:
        return 20.0
    import math
    e = 2.0 * O * 4 * math.ceil((L + O) / 4) / L
    mix = 2.0 * O
    scan = 2.0 * 8 * O * O / L
    zs = 2.0 * math.ceil((L + O) / 32) * 32 / N if L >= 64 else 0.0
    return e + mix + scan + zs


def resp_step_flops(K, S, N, O=2):
    """FP64 flops of one stationary-engine call (hz_fb_resp.hip) of S samples, horizon K:
    packed window FFTs (Q + D - 1) and output FFTs (D) at 5 F log2 F each, the partition MACs
    (8 flops per complex MAC, D x F x Q), and the end-state pass (the chunk-128 state kernel in
    prepass mode over the K history samples: E 2 O 4 ceil((128+O)/4) / 128 + the weighted chunk
    sum 2 (O^2 + 6 O) / 128 flops per band-sample)."""
    import math
    P, F, lgF = 2048, 4096, 12
    Q = K // P
    B = -(-S // P)
    D = -(-B // 2)
    fft = 5.0 * F * lgF
    conv = (Q + D - 1) * fft + D * F * Q * 8.0 + D * fft
    state = N * K * (2.0 * O * 4 * math.ceil((128 + O) / 4) / 128 + 2.0 * (O * O + 6 * O) / 128)
    return conv, state


def pmc_traffic(kernels=("fb_mix_kernel",), extra=()):
    """HBM bytes per step of the engine's kernels from two separate rocprofv3 --pmc passes
    (FETCH_SIZE, WRITE_SIZE; kernel-trace only), run as child processes on a short bench.
    Per kernel name (substring) the mean of its two largest launches (the per-step ones) is
    taken; the kernels are summed.  Correction per MI355X_MICROARCH.md 'HBM': FETCH_SIZE counts
    wide coalesced streaming reads at 1/2 of their bytes, so it is doubled; WRITE_SIZE is taken
    as is.  Returns (bytes, detail) or (None, reason)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    vals = {}
    per_kernel = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="hz_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = [exe, "--pmc", counter, "--kernel-trace", "-d", d, "-o", "pmc", "--output-format", "csv",
               "--", sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "3",
               "--no-cpu-baseline", "--stream-blocks", "0", "--no-traffic", *extra]
        try:
            subprocess.run(cmd, check=True, capture_output=True, timeout=300,
                           env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
        except Exception as e:  # noqa: BLE001
            return None, f"rocprofv3 --pmc {counter} failed: {e}"
        rows = []
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    rows += [r for r in csv.DictReader(open(os.path.join(root, f)))
                             if r["Counter_Name"] == counter]
        shutil.rmtree(d, ignore_errors=True)
        total = 0.0
        for k in kernels:
            v = sorted(float(r["Counter_Value"]) for r in rows if k in r["Kernel_Name"])[-2:]
            if not v:
                if k == kernels[0]:
                    return None, f"no {counter} rows for {k}"
                continue
            b = sum(v) / len(v) * 1024.0  # KB -> bytes
            per_kernel.setdefault(k, {})[counter] = b
            total += b
        vals[counter] = total
    fetch = 2.0 * vals["FETCH_SIZE"]
    write = vals["WRITE_SIZE"]
    return fetch + write, {"fetch_bytes": fetch, "write_bytes": write, "per_kernel": per_kernel,
                           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes; FETCH x2 (gfx950); "
                                     "summed over " + ", ".join(kernels)}


class _HostDist:
    """(rehearsal only, HZ_BENCH_REHEARSAL=1: several ranks on one GPU over gloo) the collectives
    bench.py issues, run through host copies of the device tensors."""

    def __init__(self, d):
        self.d = d
        self.ReduceOp = d.ReduceOp

    def _via(self, fn, t, **kw):
        c = t.detach().cpu()
        r = fn(c, **kw)
        t.copy_(c)
        return r

    def all_reduce(self, t, op=None):
        return self._via(self.d.all_reduce, t, op=op or self.d.ReduceOp.SUM)

    def reduce(self, t, dst=0, op=None):
        return self._via(self.d.reduce, t, dst=dst, op=op or self.d.ReduceOp.SUM)

    def gather(self, t, lst, dst=0):
        c = t.detach().cpu()
        lc = [torch_empty_like(c) for _ in lst] if lst is not None else None
        self.d.gather(c, lc, dst=dst)
        if lst is not None:
            for a, b in zip(lst, lc):
                a.copy_(b)

    def barrier(self):
        self.d.barrier()

    def destroy_process_group(self):
        self.d.destroy_process_group()


def torch_empty_like(t):
    import torch
    return torch.empty_like(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 x 0.38 ms: short runs carry a fixed start-up cost in the timed region (20 steps read
    # 0.42 ms/step on the same box, 200 steps 0.377, 2000 steps 0.373)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--samples", type=int, default=SAMPLES_PER_STEP)
    ap.add_argument("--stream-blocks", type=int, default=469, help="1024-sample calls for the streaming figure")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 --pmc child passes")
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--bands-per-wave", type=int, default=0)
    ap.add_argument("--lti", default="", help="LTI engine geometry 'chunk,bands_per_wave,waves' (default engine choice)")
    ap.add_argument("--general", action="store_true", help="force the general engine (no converged fast path)")
    ap.add_argument("--response", type=int, default=-1,
                    help="stationary engine: 0 off (per-band engines only), 1 eager (default), 2 lazy")
    ap.add_argument("--gather", action="store_true",
                    help="N > 1, time-sharded stationary calls: gather the shares on rank 0 inside each step")
    ap.add_argument("--side-steps", type=int, default=50,
                    help="timed steps of the side figures (per-band engine, lazy stationary engine)")
    ap.add_argument("--target-groups", type=int, default=0, help="(tuning) workgroups wanted per launch")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="(1 GPU, diagnostics) run rank 0's shard of an N-GPU job alone: per-GPU time at N")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5", "c6", "c7", "c8", "c9"], default="c2",
                    help="c2 = the BASELINE.json metric (default); c3/c4/c5 = the other SURVEY.md 8(d) rows; c6 = Granulator, c7 = Freezer, c8 = heterodyne chain, c9 = per-sample coefficient streams (8(f) rows 1-4)")
    args = ap.parse_args()
    if args.workload != "c2":
        return run_row(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and os.environ.get("HZ_BENCH_REHEARSAL") == "1":
        # (rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0, gloo via host copies)
        local = 0
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
        dist = _HostDist(dist)
    elif world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from huygens_amd import Filterbank
    from huygens_amd._lib import HZ_FB_PATH_RESPONSE
    fwd, back = c2_coefficients()
    b0, cnt = shard_of(rank, world) if not args.emulate_world else shard_of(0, args.emulate_world)
    fb = Filterbank(2, N_BANDS, 0.1, 1.0, device=local, shard=(b0, cnt))
    for n in range(b0, b0 + cnt):
        fb.coefficients(n, fwd[n], back[n])
    fb.boost(np.ones(N_BANDS))
    fb.open()
    if args.waves or args.bands_per_wave:
        fb.tune(args.waves, args.bands_per_wave)
    if args.lti:
        fb.tune_lti(*[int(v) for v in args.lti.split(",")])
    if args.target_groups:
        fb.set_target_groups(args.target_groups)
    if args.general:
        from huygens_amd._lib import HZ_FB_PATH_GENERAL
        fb.set_path(HZ_FB_PATH_GENERAL)
    if args.response >= 0:
        fb.set_response(args.response)
    stream = torch.cuda.current_stream(dev)
    fb.set_stream(stream.cuda_stream)

    # N > 1: once stationary, the ranks split the call by TIME (each convolves its share of the
    # output blocks with the whole bank's response, summed over the band shards by one all-reduce
    # at setup) and keep their own bands' states; rank 0 gathers the shares
    tshard = False
    if world > 1 and not args.general and args.response != 0:
        from huygens_amd.shard import set_time_shards

        def all_reduce_sum(h):
            t = torch.from_numpy(h).to(dev)
            dist.all_reduce(t)
            return t.cpu().numpy()

        def all_reduce_max(k):
            t = torch.tensor([k], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return int(t.item())
        try:
            tshard = set_time_shards(fb, rank, world, all_reduce_sum, all_reduce_max)
        except Exception as e:  # noqa: BLE001 -- fall back to band shards + reduce
            print(f"rank {rank}: time shards not set ({e}); band shards + reduce", file=sys.stderr)
            tshard = False
    elif args.emulate_world > 1 and not args.general and args.response != 0:
        # (1 GPU, diagnostics) rank 0 of a time-sharded job: the other shards' handles exist only
        # to sum the whole bank's response
        from huygens_amd.shard import set_time_shards
        others = []
        for r in range(1, args.emulate_world):
            ob, oc = shard_of(r, args.emulate_world)
            o = Filterbank(2, N_BANDS, 0.1, 1.0, device=local, shard=(ob, oc))
            for n in range(ob, ob + oc):
                o.coefficients(n, fwd[n], back[n])
            o.boost(np.ones(N_BANDS))
            o.open()
            o.response(8192)
            others.append(o)
        k_max = max([o.response_info()[0] for o in others])
        tshard = set_time_shards(fb, 0, args.emulate_world,
                                 lambda h: h + sum(o.response(len(h)) for o in others),
                                 lambda k: max(k, k_max))
        for o in others:
            o.close()

    # Time-sharded stationary calls partition the stream: each rank produces the final output of
    # its run of blocks from the shared input (a K-sample halo, no exchange), so a step at N > 1 is
    # a call of N x 10 s with 10 s of output per rank -- weak scaling, no data-path collective
    # (the per-band warmup calls still sum band shards with one reduce)
    P_t = (world if world > 1 else max(1, args.emulate_world)) if tshard else 1
    S = args.samples * P_t
    gbuf = None   # ShareGather (--gather: collect the shares on rank 0 inside the step)
    rng = np.random.default_rng(1234)
    x = torch.from_numpy(rng.uniform(-1, 1, S).astype(np.float32).astype(np.float64)).to(dev)
    y = torch.empty_like(x)

    def step():
        nonlocal gbuf
        fb.process_device(x.data_ptr(), y.data_ptr(), S)
        if world > 1:
            active, first, count = fb.time_shard_info(S) if tshard else (False, 0, S)
            if active and fb.last_path() == HZ_FB_PATH_RESPONSE:
                # every rank holds the final samples of its share: nothing to exchange (--gather
                # collects them on rank 0 inside the step: fixed-size slots, one gather)
                if args.gather:
                    if gbuf is None:
                        from huygens_amd.shard import ShareGather
                        gbuf = ShareGather(S, rank, world, y)
                    gbuf(y, dist)
            else:
                dist.reduce(y, dst=0, op=dist.ReduceOp.SUM)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the engine's GPU time per step (roofline): a separate pass of the same steps with HIP events
    # on the handle's stream (no event records inside the timed region above)
    fb.profile(True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    seg_ms, mix_ms, red_ms, launches = fb.profile_read()
    from huygens_amd._lib import (HZ_FB_PATH_LTI, HZ_FB_PATH_RESPONSE, HZ_FB_RESP_EAGER, HZ_FB_RESP_LAZY,
                                  HZ_FB_RESP_OFF)
    path = fb.last_path()
    lti = path == HZ_FB_PATH_LTI
    resp = path == HZ_FB_PATH_RESPONSE
    chunk = fb.lti_chunk()   # the timed steps' chunk (the streaming calls below use a shorter one)
    horizon = fb.response_info()[0]
    fb.profile(False)

    def side_rate(mode, warm):
        """ms per step of the same workload with the stationary engine in `mode` (timed like the
        main loop, fewer steps): the per-band engine's figure and the lazy-state figure"""
        if args.side_steps <= 0:
            return None
        fb.set_response(mode)
        for _ in range(warm):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        ts = time.perf_counter()
        for _ in range(args.side_steps):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return {"ms_per_step": 1e3 * dt / args.side_steps, "value": N_BANDS * S * args.side_steps / dt,
                "path": {1: "general", 2: "lti", 3: "response"}.get(fb.last_path(), "?")}

    side = {}
    if resp:
        side["per_band_engine"] = side_rate(HZ_FB_RESP_OFF, 3)
        side["stationary_lazy_states"] = side_rate(HZ_FB_RESP_LAZY, 3)
        fb.set_response(HZ_FB_RESP_EAGER if args.response < 0 else args.response)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        mm = torch.tensor([seg_ms + mix_ms + red_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(mm, op=dist.ReduceOp.MAX)
        eng_ms_max = float(mm.item())
    else:
        eng_ms_max = seg_ms + mix_ms + red_ms

    # streaming figure: one process() call per 1024-sample block
    stream_rate = None
    if args.stream_blocks > 0:
        B = 1024
        nb = min(args.stream_blocks, S // B)
        for i in range(min(8, nb)):   # untimed: the short-call geometry's records are built on first use
            fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        ts = time.perf_counter()
        for i in range(nb):
            fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
            if world > 1:
                dist.reduce(y[i * B:(i + 1) * B], dst=0, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        tstream = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([tstream], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tstream = float(t.item())
        stream_rate = N_BANDS * B * nb / tstream

    total_band_samples = N_BANDS * S * args.steps
    value = total_band_samples / elapsed
    if rank == 0:
        # Roofline over the engine's whole per-step GPU time (HIP events on the handle's stream):
        # the LTI engine = segment prepass (+ carry) + mix kernel + cross-group reduce, the general
        # engine = its mix + reduce.  One process() call can be several launches (the partial slab
        # bounds a launch's length).  achieved = algorithmic 18 FP64 flops per band-sample (SURVEY.md
        # 8(d), the reference recurrence); `executed` = the flops the engine actually issues.
        step_ms = eng_ms_max   # max over ranks
        launch_avg_s = (step_ms / 1e3) / max(1, launches)
        band_samples_per_launch = cnt * S * args.steps / max(1, launches)
        if resp:   # this GPU's outputs: its time share of the whole bank (all of it at N = 1)
            band_samples_per_launch = N_BANDS * (S // P_t) * args.steps / max(1, launches)
        flops_per_launch = FLOPS_PER_BAND_SAMPLE * band_samples_per_launch
        achieved = flops_per_launch / launch_avg_s / 1e12 if launch_avg_s > 0 else None
        xflops = fb_executed_flops(lti, chunk, N=cnt)
        if resp:   # the stationary engine's flops per call (its share's convolution, its bands'
            # states), spread over the share's band-samples
            conv_f, state_f = resp_step_flops(horizon, S // P_t, cnt)
            xflops = (conv_f + state_f) / (N_BANDS * (S // P_t))
        executed = xflops * band_samples_per_launch / launch_avg_s / 1e12 if launch_avg_s > 0 else None
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(fwd, back)
        kernels = (("fb_lti_kernel", "fb_lti_gemm", "fb_lti_reduce", "fb_lti_seg_carry", "fb_lti_sum",
                    "fb_lti_xrows") if lti
                   else ("resp_fwd_kernel", "resp_mac_kernel", "resp_inv_kernel", "fb_lti_kernel<2, 128, 1",
                         "fb_lti_seg_carry") if resp
                   else ("fb_mix_kernel", "fb_reduce"))
        traffic, traffic_detail = None, "skipped"
        if not args.no_traffic and world == 1 and S == SAMPLES_PER_STEP:
            traffic, traffic_detail = pmc_traffic(kernels, extra=(["--lti", args.lti] if args.lti else [])
                                                  + (["--general"] if args.general else []))
        line = {
            "metric": "band-samples/s (bands x frames/s) for 4096-band Filterbank",
            "value": value,
            "unit": "band-samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak" if P_t > 1 and resp else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic white noise uniform[-1,1) (float32 -> double), seed 1234",
            "config": {"workload": "C2 Filterbank<double>(order 2, 4096 bands), resonant band-pass "
                                   "f_i=0.5(i+1)SR/4096 R=0.999, boost 1 + open, k_p=0.1 k_g=1"
                                   + (f", {P_t} x 10 s per step split by time" if P_t > 1 and resp else ""),
                       "samples_per_step": S, "samples_per_gpu": S // P_t, "block": 1024, "bands": N_BANDS,
                       "bands_per_gpu": cnt,
                       "parallelism": (f"stream split by time x{P_t}: each GPU outputs 10 s of the N x 10 s "
                                       f"call from the shared input with a {horizon}-sample halo (whole-bank "
                                       f"response, one all-reduce at setup), band states sharded x{P_t}; no "
                                       f"data-path collective" + (" (+ gather to rank 0)" if args.gather else "")
                                       if tshard and resp else f"bands sharded x{world}, RCCL reduce")},
            "engine": "stationary (bank response convolution, eager band states)" if resp
                      else "per-band LTI" if lti else "per-band general",
            "roofline": {"bound": "mfma" if (lti or resp) else "valu", "achieved": executed, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": (executed / FP64_PEAK_TFLOPS) if executed else None,
                         "traffic": traffic,
                         "traffic_detail": traffic_detail,
                         "algorithmic_bytes_per_launch": (16 * S + 120 * cnt) * args.steps / max(1, launches),
                         "launches_per_step": launches / max(1, args.steps),
                         "kernel": ("stationary engine step: resp_fwd_kernel + resp_mac_kernel<8> + resp_inv_kernel "
                                    "(partitioned FFT convolution, history and smoother upkeep) + "
                                    "fb_lti_kernel<2,128,SEGEND> (band states over the %d-sample horizon)" % horizon)
                                   if resp else
                                   (("LTI engine step: fb_lti_kernel<2,%d,STATE>%s + "
                                     "fb_lti_gemm_pp_kernel<%d> + fb_lti_sum_kernel (+ segment prepass)"
                                     % (chunk, " (+ x rows)" if chunk >= 128 else " + fb_lti_xrows_kernel", chunk))
                                    if lti and chunk >= 64 else
                                    ("LTI engine step: fb_lti_kernel<2,%d,MIX> + fb_lti_reduce_kernel (+ segment "
                                     "prepass)" % chunk) if lti
                                    else "general engine step: fb_mix_kernel<2,NONE,1,MIX> + fb_reduce_kernel"),
                         "kernel_avg_ms": 1e3 * launch_avg_s,
                         "components_ms_per_launch": {"segment_prepass": seg_ms / max(1, launches),
                                                      "mix_or_state": mix_ms / max(1, launches),
                                                      "gemm_and_reduce": red_ms / max(1, launches)},
                         "flops_per_band_sample": xflops,
                         "horizon": horizon if resp else None,
                         "flops_per_launch": xflops * band_samples_per_launch,
                         "reference_equivalent": {"flops_per_band_sample": FLOPS_PER_BAND_SAMPLE,
                                                  "achieved": achieved,
                                                  "frac": (achieved / FP64_PEAK_TFLOPS) if achieved else None},
                         "note": ("stationary engine: achieved = the FP64 flops of the call (packed window and output "
                                  "FFTs at 5 F log2 F, partition MACs, the end-state pass over the horizon; "
                                  "bench.resp_step_flops) over the engine's whole per-step GPU time (HIP events on the "
                                  "handle's stream): components mix_or_state = the convolution (fwd + MAC + inv), "
                                  "gemm_and_reduce = history + band states. reference_equivalent = the reference "
                                  "recurrence's 18 flops per band-sample over the same time (far above the peak: the "
                                  "stationary engine's cost does not grow with the bands). peak = FP64 vector = FP64 MFMA "
                                  "peak.") if resp else
                                 "achieved = the FP64 flops the engine's algorithm performs per band-sample "
                                 "(chunked state space: chunk end states + 64-lane scan + correction GEMM with the "
                                 "zero-state rows, DESIGN.md 3.3; PMC-verified in profiles/r2/flops_pmc.txt) over the "
                                 "whole per-step GPU time of the engine (kernel_avg_ms, HIP events on the handle's "
                                 "stream). reference_equivalent = the reference recurrence's 18 flops per band-sample "
                                 "(SURVEY.md 8(d)) over the same time -- it can exceed the peak because the engine "
                                 "needs fewer than half of them. peak = FP64 vector = FP64 MFMA peak."},
            "side": side or None,
            "streaming": {"band_samples_per_s": stream_rate, "block": 1024,
                          "note": "one process() call per 1024-sample block, device-resident I/O"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_row(args):
    """One 1-GPU line for a secondary config (bench_rows.py)."""
    import torch
    import bench_rows
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.workload not in ("c3", "c4"):
        raise SystemExit("--workload c5..c9 are single-GPU configs (SURVEY.md 8(d)); c3 and c4 shard")
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=dev)
        body = (bench_rows.run_c3 if args.workload == "c3" else bench_rows.run_c4)(args, torch, dev, rank, world)
    elif args.workload in ("c3", "c4") and args.emulate_world:
        body = (bench_rows.run_c3 if args.workload == "c3" else bench_rows.run_c4)(args, torch, dev, 0, 1,
                                                                                  args.emulate_world)
    else:
        fn = {"c3": bench_rows.run_c3, "c4": bench_rows.run_c4, "c5": bench_rows.run_c5,
              "c6": bench_rows.run_c6, "c7": bench_rows.run_c7, "c8": bench_rows.run_c8,
              "c9": bench_rows.run_c9}[args.workload]
        body = fn(args, torch, dev)
    line = {"metric": body.pop("metric"), "value": body.pop("value"), "unit": body.pop("unit"),
            "n_gpus": body.pop("n_gpus", 1), "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": body.pop("ms_per_step"), "higher_is_better": True,
            "scaling": body.pop("scaling", "weak"), "vs_baseline": None}
    line.update(body)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
