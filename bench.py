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

Multi-GPU (one process per GPU): `bench.py --gpus N` outside a launcher reruns itself under
`torch.distributed.run --nproc-per-node N` as a child process before any torch / HIP import and
forwards rank 0's JSON line; under a launcher WORLD_SIZE must equal --gpus (else exit 2).  At
N > 1 `value` is the fixed 10 s call split by TIME over the ranks (STRONG scaling): every rank holds
the whole bank's response (one all-reduce at setup) and its own band shard's states, convolves its
run of 2048-sample output blocks from the shared input, and keeps its share -- no data-path
collective in the step.  side.gather_to_rank0 adds one RCCL gather of the shares per
step; side.band_partition_stationary is north_star's band partition (each rank's band shard over the
whole call, partial mixes summed to rank 0 by an RCCL reduce).  `--emulate-world P --emulate-rank r`
runs rank r of P alone on one GPU (its per-rank step; value = the whole job's band-samples over it).
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


def cpu_quota():
    """CPUs this process may use: min(affinity, cgroup CPU quota); without a cgroup quota, the
    pool's per-GPU share when it is exported as OMP_NUM_THREADS (the GPU box sets it), else the
    affinity.  -> (cpus, source)"""
    import math
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):                       # cgroup v2: "<quota|max> <period>"
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = (float(q) / float(per), f"cgroup v2 {path} = {q}/{per}")
        except (OSError, ValueError):
            pass
    if quota is None:                                                # cgroup v1
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = (q / per, f"cgroup v1 cpu.cfs_quota_us/cfs_period_us = {q}/{per}")
        except (OSError, ValueError):
            pass
    if quota is not None:
        return max(1, min(aff, int(math.floor(quota[0] + 1e-9)))), quota[1] + f", affinity {aff}"
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return min(aff, int(omp)), f"no cgroup CPU quota; OMP_NUM_THREADS={omp} (the pool's per-GPU CPU share), affinity {aff}"
    return aff, f"no cgroup CPU quota, no OMP_NUM_THREADS: sched_getaffinity = {aff}"


def cpu_info():
    """Host CPU model (/proc/cpuinfo), logical CPUs of the machine, of this process, and its quota."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    q, src = cpu_quota()
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable, "cpu_quota": q, "quota_source": src}


def native_oracle():
    """The oracle's C sources built -O3 -march=native -ffp-contract=off for THIS host (SURVEY.md
    8(d)), into a temporary directory; None when gcc is unavailable (then the in-tree -O3
    generic build is timed and the line says so)."""
    import glob
    import shutil
    import subprocess
    import tempfile
    cc = shutil.which("gcc")
    if not cc:
        return None
    d = tempfile.mkdtemp(prefix="hz_oracle_native_", dir=os.environ.get("TMPDIR", "/tmp"))
    so = os.path.join(d, "libhz_oracle_native.so")
    srcs = sorted(glob.glob(os.path.join(ROOT, "oracle", "hz_oracle*.c")))
    try:
        subprocess.run([cc, "-O3", "-march=native", "-std=c11", "-fPIC", "-ffp-contract=off", "-shared", "-o", so,
                        *srcs, "-lm", "-lpthread"], check=True, capture_output=True, timeout=120)
    except Exception:  # noqa: BLE001
        return None
    return so


def per_sample_rates(device, samples=12000):
    """The drop-ins' per-sample form -- `out = bank(x); bank.tick();` once per sample, as every
    reference demo's audio callback does -- called from Python (ctypes) like a demo callback, for
    every bank: Filterbank at C1 (128 bands) and C2 (4096), eight 864-band Filterbanks interleaved
    (tests/filterbanks.cpp), Delay(10, 2 SR) (tests/delay.cpp), Granulator with 512 voices and
    grain requests (tests/granny.cpp), Additive 10 x 7 (tests/additive.cpp) and 64 x 256 (C3),
    Sinusoids, Oscbank<72> operator() + mixdown() + tick() (tests/oscbank.cpp) and Bowl<303>
    (tests/bowl.cpp).  Input-driven banks go through the per-sample server (hz_rt.hip), generator
    banks through speculative blocks (huygens_hip.h, hz_add_fill)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from huygens_amd import Additive, Bowl, Delay, Filterbank, Granulator, Oscbank, Sinusoids, rt_info
    from golden.spec_numpy import resonant_coefficients
    out = {}
    rng = np.random.default_rng(7)
    xs = rng.uniform(-1, 1, samples + 500)

    def timed(name, step, n=samples, warm=500, frames=1, **extra):
        for i in range(warm):
            step(i)
        t0 = time.perf_counter()
        for i in range(n):
            step(warm + i)
        dt = time.perf_counter() - t0
        rate = n / dt
        out[name] = {"samples_per_s": rate, "us_per_sample": 1e6 * dt / n, "real_time_48k": rate >= 48000.0,
                     "calls_per_sample": frames, **extra}

    def fb_bank(N, boost=1.0):
        fwd, back = resonant_coefficients(N, 0.999, 1.0)
        fb = Filterbank(2, N, 0.1, 1.0, device=device)
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        fb.boost(np.full(N, boost))
        fb.open()
        return fb

    for name, N in (("filterbank_c1_128_bands", 128), ("filterbank_c2_4096_bands", 4096)):
        fb = fb_bank(N)

        def st(i, fb=fb):
            fb(xs[i % len(xs)])
            fb.tick()
        timed(name, st, path="per-sample server (hz_rt.hip OP_FB)")
        fb.close()
    fbs = [fb_bank(864, 1.0 + 0.1 * k) for k in range(8)]

    def st8(i):
        for fb in fbs:
            fb(xs[i % len(xs)])
            fb.tick()
    timed("filterbank_8x864_interleaved", st8, n=samples // 4, frames=8, path="per-sample server, 8 handles")
    from huygens_amd import sample_many
    from huygens_amd._lib import HZ_DIST_SOFTCLIP
    xs8 = rng.uniform(-1, 1, (samples // 4 + 500, 8))

    def stm(i):   # tests/filterbanks.cpp:191-211: 8 channels, &softclip, one request per frame
        sample_many(fbs, xs8[i % len(xs8)], HZ_DIST_SOFTCLIP)   # &softclip: width 0.125
        for fb in fbs:
            fb.tick()
    timed("filterbank_8x864_sample_many_softclip", stm, n=samples // 4, frames=1,
          path="per-sample server, OP_FB_MANY: one request per frame for the 8 handles (hz_fb_sample_many)")
    for fb in fbs:
        fb.close()
    d = Delay(10, 2 * 48000, device=device)
    d.coefficients([(0, 1.0)], [(20000, 0.5), (10000, 0.5)])
    timed("delay_10_taps_2s", lambda i: d(xs[i % len(xs)]), path="per-sample server (OP_DLY)")
    g = Granulator(3 * 48000, 512, device=device)

    def gran(i):
        g.sample(xs[i % len(xs)])
        if i % 2400 == 0:
            g.request(0.0, 0.15, 1.0 + 0.1 * ((i // 2400) % 5), 0.5, ticked=True)
    timed("granulator_512_voices", gran, path="per-sample server (OP_GRAN)")
    for name, (V, O) in (("additive_10x7_demo", (10, 7)), ("additive_64x256_c3", (64, 256))):
        a = Additive(V, O, 0.75, 1.0, device=device)
        for v in range(V):
            a.makenote(36 + v, 1.0)
        timed(name, lambda i, a=a: a.fill(1), path="speculative blocks (1024 samples)")
        a.close()
    sn = Sinusoids(220.0, 12, 0.8, 1.0, device=device)
    timed("sinusoids_12", lambda i: sn.fill(1), path="speculative blocks")
    ob = Oscbank(72, device=device)
    for k in range(72):
        ob.freqmod(k, 55.0 * 2 ** (k / 12))
    ob.open()

    def osc(i):
        ob.phases()
        ob.mixdown()
        ob.tick()
    timed("oscbank_72_operator_mixdown_tick", osc, path="speculative blocks")
    frng = np.random.default_rng(5)
    f = np.exp(frng.uniform(np.log(20), np.log(16000), 303))
    bw = Bowl(303, f, frng.uniform(1e-4, 5e-2, 303), frng.uniform(0.05, 15, 303), device=device)
    bw.trigger()
    timed("bowl_303_modes", lambda i: bw.render(1), path="speculative blocks")
    req, launches, _ = rt_info(device)
    out["note"] = ("one call per sample (operator() + tick(); Oscbank: operator() + mixdown() + tick()) from a Python "
                   "ctypes caller, after 500 warm-up samples; per-sample server requests %d, launches %d" % (req, launches))
    return out


def cpu_baseline(fwd, back, runs=5):
    """The CPU restatement (oracle/hz_oracle.c, the reference's operation order) timed on this
    host, SURVEY.md 8(d): (a) ONE thread -- the reference's execution model (one PortAudio
    callback thread) -- over the whole 4096-band bank for 1 s of audio, and (b) all usable cores
    (bands split over threads, partial mixes summed) over the full 10 s step; each the median of
    `runs` runs on fresh banks, built -O3 -march=native -ffp-contract=off.  A restatement of the
    reference semantics, not the reference (unbuildable here: Eigen / FFTW / PortAudio absent)."""
    info = cpu_info()
    so = native_oracle()
    if so:
        os.environ["HZ_ORACLE_SO"] = so
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import OracleFilterbank
    N = fwd.shape[0]
    rng = np.random.default_rng(1)
    x = rng.uniform(-1, 1, SAMPLES_PER_STEP).astype(np.float32).astype(np.float64)

    def bank(b0, cnt):
        fb = OracleFilterbank(2, cnt)
        for i in range(cnt):
            fb.coefficients(i, fwd[b0 + i], back[b0 + i])
        fb.boost(np.ones(cnt))
        fb.open()
        return fb

    def leg(threads, nsamp):
        xs = x[:nsamp]
        times = []
        for _ in range(runs):
            banks = [bank(*shard_of(t, threads, N)) for t in range(threads)]
            outs = [None] * threads

            def run(i):
                outs[i] = banks[i].process(xs)
            ths = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
            t0 = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            _ = np.sum(outs, axis=0)   # the partial mixes summed, as the reference's one sum
            times.append(time.perf_counter() - t0)
        dt = float(np.median(times))
        return {"value": N * nsamp / dt, "unit": "band-samples/s", "threads": threads, "samples": nsamp,
                "median_s": dt, "runs_s": times}

    def stream_leg(nblocks, B=1024):
        """the reference's execution model: ONE thread, one call per 1024-sample block"""
        times = []
        for _ in range(3):
            fb = bank(0, N)
            t0 = time.perf_counter()
            for b in range(nblocks):
                fb.process(x[b * B:(b + 1) * B])
            times.append(time.perf_counter() - t0)
        dt = float(np.median(times))
        return {"value": N * B * nblocks / dt, "unit": "band-samples/s", "threads": 1, "blocks": nblocks,
                "block": B, "us_per_block": 1e6 * dt / nblocks, "median_s": dt, "runs_s": times}

    one = leg(1, SR)                                       # 1 s of audio, whole bank, 1 thread
    cores = info["cpu_quota"]                               # cgroup quota / the pool's share / affinity
    allc = leg(cores, SAMPLES_PER_STEP)
    streaming = stream_leg(94)                              # 2 s of audio in 1024-sample calls
    build = "-O3 -march=native -ffp-contract=off" if so else "-O3 -ffp-contract=off (in-tree build; gcc unavailable)"
    return {"value": allc["value"], "unit": "band-samples/s", "cores": cores, "kind": "port",
            "sample": (f"oracle/hz_oracle.c restatement of src/filterbank.h:170-187, {build}, median of {runs}: "
                       f"all {N} bands; 1 thread over {SR} samples (1 s), {cores} threads (bands split) over "
                       f"{SAMPLES_PER_STEP} samples (10 s); streaming: 1 thread, 94 calls of 1024 samples "
                       f"(median of 3)"),
            "threads_1": one, "all_cores": allc, "streaming_1_thread": streaming, "build": build, **info}


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
    """FP64 flops of one stationary-engine call (hz_fb_resp.hip) of S samples, horizon K: one
    real 4096-point transform per window (Q + B - 1) and per output block (B), each a 2048-point
    complex FFT (5 H log2 H, H = 2048) plus its split / merge (~10 flops per bin pair), the
    partition MACs (8 flops per complex MAC, B x H x Q), and the band-state pass
    (hz_fb_state.hip: 2 O 4 ceil((128 + O) / 4) / 128 flops per band-sample of the K-sample
    window on the matrix cores, plus the per-tile M^64 carry 2 O^2 / 128 per band and chunk
    position)."""
    import math
    P, H, lgH = 2048, 2048, 11
    Q = K // P
    B = -(-S // P)
    fft = 5.0 * H * lgH + 10.0 * H
    conv = (Q + B - 1) * fft + B * H * Q * 8.0 + B * fft
    state = N * K * (2.0 * O * 4 * math.ceil((128 + O) / 4) / 128) + N * 64 * 2.0 * O * O * (K // 8192)
    return conv, state


def stream_block_flops(K, P=1024):
    """FP64 flops of one streaming block (hz_fb_stream.hip): per column (33) the forward's stage 1
    (2048 real x complex MACs, 4 flops each) and stage 3 (32 x 32 complex MACs after a twiddle, 8
    flops each + 6), the partition MAC (K / P complex MACs per bin, 32 bins), the inverse column
    (as stage 3); the last workgroup's combine (1024 outputs x 31 columns x 4 flops)."""
    col = 2048 * 4 + 32 * (32 * 8 + 6) + (K // P) * 32 * 8 + 32 * (32 * 8 + 6)
    return 33.0 * col + 1024 * 31 * 4.0


def resp_alg_bytes(K, S, N, O=2, Qp=24):
    """Algorithmic HBM bytes of one stationary call (no engine intermediates: the window spectra Z
    and output spectra Y live only between the engine's own kernels).  Returns (dominant kernel,
    whole call):
      * inverse kernel + band-state pass: the output (8 S), the state window's K inputs (8 K, read
        once), the history after the call (8 K), the pass's per-band operand rows (pin E_0, pin E_H
        and the carry / Horner weights: 2432 + 1152 doubles per group of 16 bands at O = 2,
        hz_fb_state.h grp_doubles), the states out (8 N O) and the smoothers (16 N in, 16 N out);
      * the whole call adds the input read by the forward transforms (8 S + 8 K history) and the
        response's partition spectra (Qp x 2049 complex, read by the MAC)."""
    groups = -(-N // (32 // O))
    ops = groups * ((32 // O) * 152 + 2 * 16 * 9 * 4) * 8
    dom = 8 * S + 8 * K + 8 * K + ops + 8 * N * O + 32 * N
    call = dom + 8 * S + 8 * K + Qp * (2 * 2048 + 1) * 8
    return dom, call


def modal_kernels(K, S, N, nexc=1, n_call=None, first=0):
    """Per-kernel (flops, algorithmic bytes) of a stationary call with MODAL band states
    (hz_fb_modal.h), for the three launches, over a share of S output samples starting at `first`
    of a call of n_call samples (the whole call at N = 1; a rank's time share at N > 1).  The bytes
    are SURVEY.md 8(d)'s: the kernel's own inputs and outputs that are NOT engine intermediates --
    the window spectra Z (forward -> MAC), the output spectra Y (MAC -> inverse) and phase 1's A
    (forward -> inverse) live only between the engine's own kernels and are not counted:
      * resp_fwd_kernel: the window transforms (Q + B - 1 real 4096-point) + phase 1 (the fold, 2
        flops per window sample and map, and 2 x 128 x 64 x 64 real x complex MACs) + the
        exceptional direct sums (2 dot products of K in double-double, ~20 flops per term); bytes:
        the distinct input samples read (the share's windows [first - K, first + S) of [history |
        call] and phase 1's window, the call's last K inputs) and the exceptional bands' responses;
      * resp_mac_kernel: B x 2048 x Q complex MACs; bytes: the Q partition spectra H;
      * resp_inv_kernel: the output blocks' inverse transforms + phase 2 (2 x 64 x 128 x 128
        complex MACs + ~60 flops per band); bytes: the output share, the history after the call
        (the call's last K inputs read, written), the per-band parameters (64 B), states (16 B) and
        smoothers (32 B per band).
    Returns {kernel: (flops, bytes)} and, under "call", the whole call's (flops, bytes) with the
    history's K inputs counted once."""
    H, lgH, P = 2048, 11, 2048
    n_call = S if n_call is None else n_call
    Q, B = K // P, -(-S // P)
    fft = 5.0 * H * lgH + 10.0 * H
    row = 16 * (H + 1)
    a_lo, a_hi = first - K, first + S               # the share's windows, in call coordinates
    b_lo, b_hi = n_call - K, n_call                 # phase 1's window
    inp = (a_hi - a_lo) + (b_hi - b_lo) - max(0, min(a_hi, b_hi) - max(a_lo, b_lo))
    fwd_f = (Q + B - 1) * fft + 4.0 * K + 2 * 128 * 64 * 64 * 4 + nexc * 2 * K * 20.0
    fwd_b = 8 * inp + nexc * 8 * (K + 1)
    mac_f = B * H * Q * 8.0
    mac_b = Q * row
    inv_f = B * fft + 2 * 64 * 128 * 128 * 8.0 + 60.0 * N
    inv_b = 8 * S + 8 * K + 8 * K + N * (64 + 16 + 32)
    out = {"resp_fwd_kernel": (fwd_f, fwd_b), "resp_mac_kernel": (mac_f, mac_b), "resp_inv_kernel": (inv_f, inv_b)}
    out["call"] = (fwd_f + mac_f + inv_f, fwd_b + mac_b + inv_b - 8 * K)
    return out


def resp_inv_flops(S):
    """FP64 flops of the inverse transforms of a stationary call's output blocks (as resp_step_flops)."""
    H, lgH = 2048, 11
    return -(-S // 2048) * (5.0 * H * lgH + 10.0 * H)


PMC_FLOP_COUNTERS = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                     "SQ_INSTS_VALU_MFMA_MOPS_F64")


def pmc_pass(counters, kernels, extra=(), per_step=None):
    """One rocprofv3 --pmc pass (kernel trace only, no other tracing) of a short bench run as a
    child process: per kernel (name substring) and counter the mean over its two largest
    dispatches (the per-step launches).  Returns ({kernel: {counter: value}}, None) or
    (None, reason)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="hz_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [exe, "--pmc", *counters, "--kernel-trace", "-d", d, "-o", "pmc", "--output-format", "csv",
           "--", sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "3",
           "--no-cpu-baseline", "--stream-blocks", "0", "--no-traffic", "--side-steps", "0", "--no-per-sample",
           "--no-general-side", *extra]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=300,
                       env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
    except Exception as e:  # noqa: BLE001
        shutil.rmtree(d, ignore_errors=True)
        return None, f"rocprofv3 --pmc {' '.join(counters)} failed: {e}"
    rows = []
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                rows += list(csv.DictReader(open(os.path.join(root, f))))
    shutil.rmtree(d, ignore_errors=True)
    out = {}
    for k in kernels:
        for c in counters:
            per = {}
            for r in rows:
                if r["Counter_Name"] == c and k in r["Kernel_Name"]:
                    per[r.get("Dispatch_Id", len(per))] = per.get(r.get("Dispatch_Id", len(per)), 0.0) + \
                        float(r["Counter_Value"])
            if per_step:   # several launches per step: all dispatches' sum per step
                if per:
                    out.setdefault(k, {})[c] = sum(per.values()) * per_step / len(per)
                continue
            v = sorted(per.values())[-2:]
            if v:
                out.setdefault(k, {})[c] = sum(v) / len(v)
    if not out:
        return None, "no counter rows for " + ", ".join(kernels)
    return out, None


def pmc_traffic(kernels, extra=(), per_step=None):
    """HBM bytes per launch of each kernel from two separate rocprofv3 --pmc passes (FETCH_SIZE,
    WRITE_SIZE; kernel-trace only).  Correction per MI355X_MICROARCH.md 'HBM': FETCH_SIZE counts
    wide coalesced streaming reads at 1/2 of their bytes, so it is doubled; WRITE_SIZE is taken as
    is; both are in KB.  Returns ({kernel: bytes}, detail) or (None, reason)."""
    per = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        res, err = pmc_pass((counter,), kernels, extra, per_step=per_step)
        if res is None:
            return None, err
        for k, cv in res.items():
            per.setdefault(k, {})[counter] = cv.get(counter, 0.0) * 1024.0
    byk = {k: 2.0 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0) for k, v in per.items()}
    return byk, {"per_kernel": per, "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                                              "FETCH x2 (gfx950); bytes per launch"}


def pmc_flops(kernels, extra=()):
    """Executed FP64 flops per launch of each kernel: 64 lanes x (2 FMA + MUL + ADD) F64 VALU
    wave-instructions + 512 per F64 MFMA mop (scripts/flops_pmc.sh), one rocprofv3 --pmc pass."""
    res, err = pmc_pass(PMC_FLOP_COUNTERS, kernels, extra)
    if res is None:
        return None, err
    fl = {k: 64.0 * (2 * c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) +
                     c.get("SQ_INSTS_VALU_ADD_F64", 0)) + 512.0 * c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
          for k, c in res.items()}
    return fl, res


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


def emulated_collectives(Filterbank, fwd, back, device):
    """(--emulate-world P on one GPU) the three host all-reduces of the time split as one process
    sees them at world P: the sum of the band shards' responses is the whole bank's response (a
    whole-bank handle's), the max of the shards' horizons the whole bank's horizon (the protocol's
    0/1 failure flag passes through), the min of the readiness flags this rank's own flag."""
    full = Filterbank(2, N_BANDS, 0.1, 1.0, device=device)
    for n in range(N_BANDS):
        full.coefficients(n, fwd[n], back[n])
    full.boost(np.ones(N_BANDS))
    full.open()
    full.response(8192)
    K_full = int(full.response_info()[0])
    h_full = full.response(K_full)
    full.close()
    return ((lambda hv: h_full[:len(hv)].copy() if len(hv) <= K_full else np.concatenate([h_full, np.zeros(len(hv) - K_full)])),
            (lambda k: max(int(k), K_full) if k > 1 else int(k)),
            (lambda k: int(k)))


def c2_setup_time_split(fb, rank, world, coll) -> bool:
    """Time-split stationary calls (huygens_amd.shard.set_time_shards: the whole bank's response
    on every rank, this rank's share of the output blocks), with disjoint share-only outputs
    (hz_fb_set_time_shard_fill(h, 0)).  coll = (all_reduce_sum, all_reduce_max, all_reduce_min)."""
    from huygens_amd.shard import set_time_shards
    ok = set_time_shards(fb, rank, world, coll[0], coll[1])
    if ok:
        fb.set_time_shard_fill(False)
    return ok


def c2_prime(fb, step, n, tsplit, all_reduce_min, path_response, stop_early=False, armed=None, max_calls=8):
    """Untimed calls until the engine the run settles on, every decision agreed over the ranks:
    time split -- after each call every rank asks whether the next call of n samples would be
    stationary and the handles of ALL ranks are armed in the same call (huygens_amd.shard.
    arm_when_ready, all-reduce MIN); otherwise -- stop once every rank's last call was stationary
    (all-reduce MIN of the flag), or after 3 calls for the per-band runs.  `armed` ([bool]) is set
    when the time split is armed.  Returns the number of priming calls."""
    from huygens_amd.shard import arm_when_ready
    for i in range(max_calls):
        step()
        if tsplit:
            if arm_when_ready(fb, n, all_reduce_min):
                if armed is not None:
                    armed[0] = True
                return i + 1
            continue
        done = fb.last_path() == path_response or (stop_early and i >= 2)
        if int(all_reduce_min(1 if done else 0)) == 1:
            return i + 1
    return max_calls


def general_softclip_figures(Filterbank, device, stream, x, y, S, traffic=True, steps=10):
    """The general engine (hz_filterbank.hip fb_mix_kernel) on the reference demos' own calls:
    F(x, &softclip) with the one-argument softclip (width 0.125, tests/filterbank.cpp:158-171,
    200-215) -- a distortion functor keeps every call off the converged engines.  4096 bands (the
    C2 bank, k_p = 0.1, k_g = 1) and the demo's FFilterbank<double, 864, 2> (k_p = 0.001, k_g = 1,
    tests/filterbank.cpp:191), each on 480,000-sample calls and 1024-sample calls.  frac = the
    reference recurrence's 18 flops per band-sample over the mix kernel's event
    time, against the FP64 peak; PMC executed flops and HBM bytes of fb_mix_kernel from child
    rocprofv3 passes (bench.py --dist softclip)."""
    import torch
    from huygens_amd._lib import HZ_DIST_SOFTCLIP
    out = {}
    B = 1024
    for N, kp, name in ((N_BANDS, 0.1, "c2_4096_bands"), (864, 0.001, "ffilterbank_864_bands")):
        fwd, back = c2_coefficients(N=N)
        fb = Filterbank(2, N, kp, 1.0, device=device)
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        fb.boost(np.ones(N))
        fb.open()
        fb.distortion(HZ_DIST_SOFTCLIP)
        fb.set_stream(stream.cuda_stream)

        def long_call():
            fb.process_device(x.data_ptr(), y.data_ptr(), S)
        for _ in range(2):
            long_call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            long_call()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        fb.profile(True)
        for _ in range(steps):
            long_call()
        torch.cuda.synchronize()
        seg_ms, mix_ms, red_ms, launches = fb.profile_read()
        fb.profile(False)
        mix_avg = mix_ms / max(1, launches) / 1e3
        ref_fl = FLOPS_PER_BAND_SAMPLE * N * S
        rec = {"long_calls": {"ms_per_call": 1e3 * dt, "band_samples_per_s": N * S / dt,
                              "mix_kernel_ms": 1e3 * mix_avg, "reduce_kernel_ms": red_ms / max(1, launches),
                              "frac_18_flops": ref_fl / mix_avg / 1e12 / FP64_PEAK_TFLOPS if mix_avg > 0 else None,
                              "path": {1: "general"}.get(fb.last_path(), str(fb.last_path()))}}
        nb = min(469, S // B)

        def blocks(k):
            for i in range(k):
                fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
        blocks(16)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        blocks(nb)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rec["blocks_1024"] = {"us_per_block": 1e6 * dt / nb, "band_samples_per_s": N * B * nb / dt,
                              "path": {1: "general"}.get(fb.last_path(), str(fb.last_path()))}
        fb.close()
        out[name] = rec
    if traffic:
        tr, _ = pmc_traffic(("fb_mix_kernel", "fb_reduce"), ["--dist", "softclip"])
        fl, _ = pmc_flops(("fb_mix_kernel",), ["--dist", "softclip"])
        mix_ms = out["c2_4096_bands"]["long_calls"]["mix_kernel_ms"]
        out["pmc_c2_4096"] = {
            "fb_mix_kernel_bytes": tr.get("fb_mix_kernel") if tr else None,
            "fb_reduce_bytes": tr.get("fb_reduce") if tr else None,
            "fb_mix_kernel_flops": fl.get("fb_mix_kernel") if fl else None,
            "executed_tflops": (fl["fb_mix_kernel"] / (mix_ms / 1e3) / 1e12) if (fl and mix_ms) else None,
            "executed_frac": (fl["fb_mix_kernel"] / (mix_ms / 1e3) / 1e12 / FP64_PEAK_TFLOPS) if (fl and mix_ms) else None,
            "hbm_frac": (tr["fb_mix_kernel"] / (mix_ms / 1e3) / 1e9 / HBM_PEAK_GBS) if (tr and mix_ms) else None}
    out["note"] = ("F(x, &softclip) per band (filterbank.h:133-139), width 0.125; the distortion keeps the calls on "
                   "the general engine (smoothers and functor per band-sample)")
    return out


def churn_cpp(x):
    """tests/cpp/churn.cpp (the reference's language, C ABI on device buffers): the same churn from a
    C++ caller, against its own converged calls; None when the compiler is unavailable"""
    import shutil
    import subprocess
    import tempfile
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    d = tempfile.mkdtemp(prefix="hz_churn_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        fwd, back = c2_coefficients()
        np.concatenate([np.asarray(fwd)[:, :3], np.asarray(back)[:, :2]], axis=1).astype(np.float64).tofile(
            os.path.join(d, "coef.bin"))
        np.ascontiguousarray(x, dtype=np.float64).tofile(os.path.join(d, "x.bin"))
        lib = os.path.join(ROOT, "huygens_amd", "lib")
        exe = os.path.join(d, "churn")
        subprocess.run([hipcc, "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "cpp", "churn.cpp"), "-o", exe, "-L", lib, "-lhuygens_hip",
                        f"-Wl,-rpath,{lib}"], check=True, capture_output=True, timeout=180)
        r = subprocess.run([exe, d], check=True, capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)[:300]}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def setter_churn_figure(fb, x, y, nb, stream_rate, B=1024, every=4800, nbands=9):
    """1024-sample calls with mix() on `nbands` random bands every `every` samples: device-resident
    calls issued back to back (against `streaming`), then host buffers per call (against
    streaming.end_to_end_host_buffers); the path of every call and the setters applied as
    transients"""
    import torch
    from huygens_amd._lib import HZ_FB_PATH_STREAM
    rng = np.random.default_rng(17)
    N = fb.N

    def setters(i):
        if (i * B) // every != ((i - 1) * B) // every:
            for b, v in zip(rng.choice(N, nbands, replace=False), rng.uniform(0.5, 1.5, nbands)):
                fb.mix(int(b), float(v))
            return 1
        return 0

    def run(k, host=None):
        n_set = streamed = 0
        for i in range(k):
            n_set += setters(i)
            if host is None:
                fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
            else:
                fb.process_host(host[0].data_ptr() + 8 * B * i, host[1].data_ptr() + 8 * B * i, B)
            streamed += fb.last_path() == HZ_FB_PATH_STREAM
        return n_set, streamed

    # untimed: the bank back to streaming first (the figures before may have reset its history):
    # K samples of converged calls, without setters
    warm = -(-fb.response_info()[0] // B) + 8
    for i in range(warm):
        fb.process_device(x.data_ptr() + 8 * B * (i % nb), y.data_ptr() + 8 * B * (i % nb), B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_set, streamed = run(nb)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    hx = torch.empty(nb * B, dtype=torch.float64).pin_memory()
    hy = torch.empty(nb * B, dtype=torch.float64).pin_memory()
    hx.copy_(x[:nb * B].cpu())
    t1 = time.perf_counter()
    h_set, h_streamed = run(nb, (hx, hy))
    dth = time.perf_counter() - t1
    us = 1e6 * dt / nb
    stat_us = 1e6 * N * B / stream_rate
    cpp = churn_cpp(x[:nb * B].cpu().numpy())
    return {"us_per_block": us, "band_samples_per_s": N * B * nb / dt, "blocks": nb, "setters": n_set,
            "cpp_caller": cpp,
            "bands_per_setter": nbands, "setter_every_samples": every, "blocks_streamed": streamed,
            "vs_converged_streaming": us / stat_us,
            "host_buffers": {"us_per_block": 1e6 * dth / nb, "setters": h_set, "blocks_streamed": h_streamed},
            "note": "mix() on 9 random bands every 4800 samples between 1024-sample process() calls; the bank keeps "
                    "streaming with the gain transient as a second convolution (hz_fb_stream.hip); "
                    "vs_converged_streaming = us_per_block over `streaming`'s converged figure"}


def launch_plan(gpus: int, env) -> tuple[str, str | None]:
    """What `bench.py --gpus N` does in this environment (no torch / HIP import before it):
    'run' (world matches), 'relaunch' (N > 1 and no launcher: rerun under torch.distributed.run),
    or 'mismatch' (a launcher's WORLD_SIZE disagrees with --gpus: refuse, exit non-zero)."""
    if gpus < 1:
        return "mismatch", f"--gpus {gpus}: at least one GPU"
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("relaunch" if gpus > 1 else "run"), None
    try:
        world = int(ws)
    except ValueError:
        return "mismatch", f"WORLD_SIZE={ws!r} is not an integer"
    if world != gpus:
        return "mismatch", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
    return "run", None


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def relaunch_cmd(gpus: int, argv, port: int):
    """one process per GPU on this node, rendezvous on 127.0.0.1"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def forward_child(cmd, env=None) -> int:
    """Run `cmd` as a CHILD process (this process never touched the GPU, and nothing is exec'd over
    it), echo its output to stderr as it arrives, and print its JSON result line(s) -- rank 0's
    bench line -- on stdout.  Returns the child's exit status."""
    import subprocess
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    for ln in p.stdout:
        t = ln.strip()
        if t.startswith("{") and '"metric"' in t:
            print(t, flush=True)
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    return p.wait()


def launcher(args) -> int | None:
    """--gpus N: None = run here; otherwise the exit status to return (relaunched or refused)."""
    plan, why = launch_plan(args.gpus, os.environ)
    if plan == "run":
        return None
    if plan == "mismatch":
        sys.stderr.write(f"bench.py: {why}\n")
        return 2
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return forward_child(relaunch_cmd(args.gpus, sys.argv[1:], free_port()), env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 x 0.06 ms: short runs carry a fixed start-up cost in the timed region
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--samples", type=int, default=SAMPLES_PER_STEP)
    ap.add_argument("--stream-blocks", type=int, default=469, help="1024-sample calls for the streaming figure")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-sample", action="store_true", help="skip the per-sample drop-in figure")
    ap.add_argument("--dist", choices=["none", "softclip"], default="none",
                    help="C2 with the reference demos' &softclip on every band (the general engine)")
    ap.add_argument("--no-general-side", action="store_true",
                    help="skip side.general_softclip (the general engine on the reference demos' softclip calls)")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 --pmc child passes")
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--bands-per-wave", type=int, default=0)
    ap.add_argument("--lti", default="", help="LTI engine geometry 'chunk,bands_per_wave,waves' (default engine choice)")
    ap.add_argument("--general", action="store_true", help="force the general engine (no converged fast path)")
    ap.add_argument("--response", type=int, default=-1,
                    help="stationary engine: 0 off (per-band engines only), 1 eager (default), 2 lazy")
    ap.add_argument("--resp-engine", type=int, default=-1,
                    help="(A/B) stationary long calls: 1 column-split, 0 three-kernel path (default)")
    ap.add_argument("--modal", type=int, default=-1,
                    help="(A/B) stationary band states: 1 modal (default where the bank qualifies), 0 matrix-core pass")
    ap.add_argument("--gather", action="store_true",
                    help="N > 1, time-sharded stationary calls: gather the shares on rank 0 inside each step")
    ap.add_argument("--side-steps", type=int, default=50,
                    help="timed steps of the side figures (per-band engine, lazy states, band partition)")
    ap.add_argument("--target-groups", type=int, default=0, help="(tuning) workgroups wanted per launch")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="(1 GPU, diagnostics) run one rank's share of an N-GPU job alone: per-GPU time at N")
    ap.add_argument("--emulate-rank", type=int, default=-1,
                    help="(with --emulate-world P) the rank to run (default P - 1: the shard with the "
                         "exceptional Nyquist band, the heaviest)")
    ap.add_argument("--band-partition", action="store_true",
                    help="N > 1: the value path on band shards + RCCL sum-reduce instead of the time split")
    ap.add_argument("--workload", choices=["c2", "c3", "c3osc", "c4", "c5", "c6", "c7", "c8", "c9"], default="c2",
                    help="c2 = the BASELINE.json metric (default); c3/c4/c5 = the other SURVEY.md 8(d) rows; c6 = Granulator, c7 = Freezer, c8 = heterodyne chain, c9 = per-sample coefficient streams (8(f) rows 1-4)")
    args = ap.parse_args()
    rc = launcher(args)   # --gpus N > 1 without a launcher: N ranks under torch.distributed.run
    if rc is not None:
        return rc
    if os.environ.get("HZ_BENCH_DRY") == "1":   # (tests/test_bench_launcher_cpu.py) the launch alone
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"metric": "dry launch", "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
                              "gpus_arg": args.gpus}), flush=True)
        return 0
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
    from huygens_amd._lib import (HZ_FB_PATH_GENERAL, HZ_FB_PATH_LTI, HZ_FB_PATH_RESPONSE, HZ_FB_PATH_STREAM,
                                  HZ_FB_RESP_EAGER, HZ_FB_RESP_LAZY, HZ_FB_RESP_OFF)
    fwd, back = c2_coefficients()
    # the time split's ranks: the real world at N > 1, or (--emulate-world P, one GPU) rank
    # --emulate-rank of P alone -- its per-rank step time at N = P
    P = world if world > 1 else max(1, args.emulate_world)
    r_split = rank if world > 1 else (args.emulate_rank if args.emulate_rank >= 0 else P - 1)
    if not 0 <= r_split < P:
        raise SystemExit(f"--emulate-rank {r_split} outside [0, {P})")
    b0, cnt = shard_of(r_split, P)
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
        fb.set_path(HZ_FB_PATH_GENERAL)
    if args.response >= 0:
        fb.set_response(args.response)
    if args.resp_engine >= 0:
        fb.tune_response_engine(bool(args.resp_engine))
    if args.modal >= 0:
        fb.tune_modal(bool(args.modal))
    if args.dist == "softclip":   # F(x, &softclip): width 0.125 (tests/filterbank.cpp:168-171)
        from huygens_amd._lib import HZ_DIST_SOFTCLIP
        fb.distortion(HZ_DIST_SOFTCLIP)
    stream = torch.cuda.current_stream(dev)
    fb.set_stream(stream.cuda_stream)

    def ar(v, op):   # all-reduce of one host integer / float over the ranks
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=op)
        return t.item()

    S = args.samples
    rng = np.random.default_rng(1234)
    x = torch.from_numpy(rng.uniform(-1, 1, S).astype(np.float32).astype(np.float64)).to(dev)
    ys = [torch.empty_like(x), torch.empty_like(x)]
    y = ys[0]

    # N > 1 (`value`): the FIXED 10 s call of N = 1 split by TIME over the ranks (STRONG scaling).
    # Once stationary, a call's output depends only on its input and the K inputs before it, so
    # rank r convolves its run of whole 2048-sample output blocks with the WHOLE bank's response
    # (the band shards' responses summed by one all-reduce at setup) from the shared input, and
    # computes its own band shard's states over the call's last K inputs (modal pass).  The shares
    # are disjoint and final (hz_fb_set_time_shard_fill(h, 0)): no data-path collective in the
    # step.  side.gather_to_rank0 adds one RCCL gather of the shares per step (1/N of the output
    # per rank); side.band_partition_* are the band-sharded decompositions with the 3.84 MB RCCL
    # sum-reduce of the partial mixes (src/filterbank.h:130's mixdown, sharded).
    if world > 1:
        def ar_sum(hv):
            t = torch.from_numpy(np.ascontiguousarray(hv)).to(dev)
            dist.all_reduce(t)
            return t.cpu().numpy()

        def ar_max(k):
            return int(ar(k, dist.ReduceOp.MAX))

        def ar_min(k):
            return int(ar(k, dist.ReduceOp.MIN))
        coll = (ar_sum, ar_max, ar_min)
    elif P > 1:
        coll = emulated_collectives(Filterbank, fwd, back, local)
    else:
        coll = None
    tsplit = False
    if coll is not None and not args.general and args.response != 0 and not args.band_partition:
        tsplit = c2_setup_time_split(fb, r_split, P, coll)
    share_first, share_count = (fb.time_shard_info(S)[1:] if tsplit else (0, S))

    works = [None, None]
    nstep = [0]

    def reduce_async(t):
        if isinstance(dist, _HostDist):
            dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
            return None
        return dist.reduce(t, dst=0, op=dist.ReduceOp.SUM, async_op=True)

    def step():
        """one step of the value path: time split (no collective) -- or, when the bank cannot run
        stationary (--general, --response 0, --band-partition), band shards whose partial mixes are
        summed to rank 0 (double-buffered: a buffer is reused after its reduce completed)"""
        k = nstep[0] & 1
        nstep[0] += 1
        if works[k] is not None:
            works[k].wait()
            works[k] = None
        fb.process_device(x.data_ptr(), ys[k].data_ptr(), S)
        if world > 1 and not armed[0]:
            works[k] = reduce_async(ys[k])

    def drain():
        for k in (0, 1):
            if works[k] is not None:
                works[k].wait()
                works[k] = None

    def barrier():
        drain()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    # Priming (untimed, before the W warmup steps): calls until the engine the run settles on --
    # the smoothers converge during the first 10 s call (k_g = 1 s), the stationary engine needs K
    # samples of converged history.  Every decision is agreed over the ranks (all-reduce MIN), so
    # every rank issues the same calls and collectives.
    armed = [False]
    primed = c2_prime(fb, step, S, tsplit, coll[2] if coll else (lambda k: k), HZ_FB_PATH_RESPONSE,
                      stop_early=args.general or args.response == 0 or args.dist != "none", armed=armed)
    value_split = tsplit and armed[0]   # the value path is the time split (its shares only)
    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_enq = time.perf_counter() - t0   # host time to issue the steps (launch-bound if ~ elapsed)
    barrier()
    elapsed = time.perf_counter() - t0
    # the engine's GPU time per step (roofline): a separate pass of the same steps with HIP events
    # on the handle's stream (no event records inside the timed region above)
    fb.profile(True, repeat=8)   # (modal path: each kernel 8x between its events, per-launch times)
    for _ in range(args.steps):
        step()
    barrier()
    seg_ms, mix_ms, red_ms, launches = fb.profile_read()
    path = fb.last_path()
    lti = path == HZ_FB_PATH_LTI
    resp = path == HZ_FB_PATH_RESPONSE
    chunk = fb.lti_chunk()   # the timed steps' chunk (the streaming calls below use a shorter one)
    horizon = fb.response_info()[0]
    modal = bool(resp and fb.modal_info()[3])   # band states by the modal pass (hz_fb_modal.h)
    nexc = max(0, fb.modal_info()[2]) if modal else 0
    fb.profile(False)

    def timed(fn, warm, steps, n_samples):
        """ms per step and band-samples/s (whole job, max over ranks) of `fn` after `warm` calls"""
        for _ in range(warm):
            fn()
        barrier()
        ts = time.perf_counter()
        for _ in range(steps):
            fn()
        barrier()
        dt = time.perf_counter() - ts
        if world > 1:
            dt = ar(dt, dist.ReduceOp.MAX)
        return {"ms_per_step": 1e3 * dt / steps, "value": N_BANDS * n_samples * steps / dt,
                "path": {1: "general", 2: "lti", 3: "response"}.get(fb.last_path(), "?")}

    side = {}
    if tsplit and args.side_steps > 0 and world > 1:
        # the value path + one gather of the shares to rank 0 per step (1/N of the output per rank,
        # fixed-size slots; double-buffered: step i + 2 reuses step i's buffer after its gather)
        from huygens_amd.shard import ShareGather
        gathers = [ShareGather(S, rank, world, ys[k]) for k in (0, 1)]
        gworks = [None, None]

        def step_gather():
            k = nstep[0] & 1
            nstep[0] += 1
            if gworks[k] is not None:
                gworks[k].wait()
                gathers[k].finish(ys[k])
                gworks[k] = None
            fb.process_device(x.data_ptr(), ys[k].data_ptr(), S)
            w = gathers[k].start(ys[k], dist, async_op=not isinstance(dist, _HostDist))
            if w is None:   # (rehearsal: the gather ran synchronously through host copies)
                gathers[k].finish(ys[k])
            gworks[k] = w

        tg = timed(step_gather, 3, args.side_steps, S)
        for k in (0, 1):
            if gworks[k] is not None:
                gworks[k].wait()
                gathers[k].finish(ys[k])
                gworks[k] = None
        tg["note"] = (f"the value path plus one RCCL gather per step of the {world} disjoint time shares to "
                      f"rank 0 ({8 * max(c for _, c in gathers[0].shares)} B per rank), overlapped with the next "
                      "step (double-buffered)")
        side["gather_to_rank0"] = tg
    if tsplit and args.side_steps > 0:
        # the band-partitioned decompositions (north_star's wording; round 5's N > 1 value): every
        # rank runs its band shard's own engine over the whole call and the partial mixes are summed
        # to rank 0 (3.84 MB per step)
        armed[0] = False
        fb.arm_time_shard(False)
        fb.set_bank_response(np.zeros(0))   # back to this shard's own response
        for _ in range(4):
            step()
        bp = timed(step, 3, args.side_steps, S)
        bp["note"] = (f"{cnt} bands per rank through the shard's own stationary engine (its response alone), "
                      "partial mixes summed to rank 0 by an RCCL reduce per step: every rank redoes the "
                      "whole convolution")
        side["band_partition_stationary"] = bp
        tsplit = False
    if resp and args.side_steps > 0:
        fb.set_response(HZ_FB_RESP_OFF)
        side["per_band_engine"] = timed(step, 3, args.side_steps, S)
        if P > 1:
            side["per_band_engine"]["note"] = (f"{N_BANDS} bands over {P} GPUs ({cnt} per GPU), per-band "
                                               "engines, partial mixes reduced to rank 0 (strong scaling)")
        fb.set_response(HZ_FB_RESP_LAZY)
        side["stationary_lazy_states"] = timed(step, 3, args.side_steps, S)
        fb.set_response(HZ_FB_RESP_EAGER if args.response < 0 else args.response)
        if modal and P == 1:   # the same eager states by the matrix-core pass (hz_fb_state.h)
            fb.tune_modal(False)
            side["matrix_core_states"] = timed(step, 3, args.side_steps, S)
            fb.tune_modal(True)
        drain()
    # the engine's GPU time per call: the event sum (stationary path: forward + MAC kernels, then the
    # inverse kernel carrying the band-state pass)
    eng_ms = seg_ms + mix_ms + red_ms
    if world > 1:
        eng_ms_max = ar(eng_ms, dist.ReduceOp.MAX)
        elapsed = ar(elapsed, dist.ReduceOp.MAX)
    else:
        eng_ms_max = eng_ms

    # streaming figure: one process() call per 1024-sample block -- the reference's audio callback
    # (tests/resynthesis.cpp:33-42).  On the stationary bank these calls take the streaming engine
    # (hz_fb_stream.hip: one launch per block); the per-band engine's rate is measured beside it
    stream_rate, stream_detail = None, {}
    if args.stream_blocks > 0:
        B = 1024   # (N > 1: band shards stream their own bands' response; the mixes are reduced per block)
        nb = min(args.stream_blocks, S // B)

        def stream_blocks(n_blocks):
            for i in range(n_blocks):
                fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
                if world > 1:
                    dist.reduce(y[i * B:(i + 1) * B], dst=0, op=dist.ReduceOp.SUM)

        def stream_figure():
            stream_blocks(min(8, nb))   # untimed: the engine's spectra / records are built on first use
            barrier()
            ts = time.perf_counter()
            stream_blocks(nb)
            barrier()
            tst = time.perf_counter() - ts
            if world > 1:
                tst = ar(tst, dist.ReduceOp.MAX)
            s_path_ = fb.last_path()
            # the same blocks with HIP events on the handle's stream: the GPU's share of a block
            fb.profile(True)
            stream_blocks(nb)
            barrier()
            s_seg, s_mix, s_red, s_calls = fb.profile_read()
            s_chunk = fb.lti_chunk()
            fb.profile(False)
            return tst, s_path_, s_chunk, 1e3 * (s_seg + s_mix + s_red) / max(1, s_calls), \
                1e3 * s_mix / max(1, s_calls), 1e3 * s_red / max(1, s_calls)

        def e2e_figure():
            """host buffers (pinned), one synchronous call per block: H2D + engine + D2H"""
            hx = torch.empty(nb * B, dtype=torch.float64).pin_memory()
            hy = torch.empty(nb * B, dtype=torch.float64).pin_memory()
            hx.copy_(x[:nb * B].cpu())
            for i in range(min(8, nb)):
                fb.process_host(hx.data_ptr() + 8 * B * i, hy.data_ptr() + 8 * B * i, B)
            ts = time.perf_counter()
            for i in range(nb):
                fb.process_host(hx.data_ptr() + 8 * B * i, hy.data_ptr() + 8 * B * i, B)
            dt = time.perf_counter() - ts
            return {"us_per_block": 1e6 * dt / nb, "band_samples_per_s": N_BANDS * B * nb / dt, "path": name_of(fb.last_path()),
                    "note": "hz_fb_process on host buffers per 1024-sample call (the reference's callback shape, "
                            "host I/O included): input copied into device-mapped pinned staging, the streaming "
                            "kernel reads and writes it directly, the host waits on per-workgroup completion "
                            "flags, output copied out"}

        def name_of(p):
            return {HZ_FB_PATH_GENERAL: "general", HZ_FB_PATH_LTI: "lti", HZ_FB_PATH_RESPONSE: "response",
                    HZ_FB_PATH_STREAM: "stream"}.get(p, str(p))

        tstream, s_path, s_chunk, gpu_us, mix_us, red_us = stream_figure()
        stream_rate = N_BANDS * B * nb / tstream
        wall_us = 1e6 * N_BANDS * B / stream_rate
        e2e = e2e_figure() if world == 1 else None
        # the per-band engine on the same 1024-sample calls (streaming engine off)
        fb.tune_stream(False)
        pb_t, pb_path, pb_chunk, pb_gpu_us, pb_mix, pb_red = stream_figure()
        fb.tune_stream(True)
        per_band = {"us_per_block": 1e6 * pb_t / nb, "band_samples_per_s": N_BANDS * B * nb / pb_t,
                    "path": name_of(pb_path), "chunk": pb_chunk, "profiled_us_per_block": pb_gpu_us,
                    "profiled_components_us": {"state_or_mix": pb_mix, "reduce": pb_red},
                    "kernels": [f"fb_lti_kernel<2, {pb_chunk}, *>", f"fb_lti_reduce_short_kernel<2, {pb_chunk}>"]
                    if pb_path == HZ_FB_PATH_LTI else None}
        stream_flops = stream_block_flops(horizon)
        stream_detail = {
            "path": name_of(s_path),
            "kernels": (["stream_block_kernel<%d>" % (horizon // 8192)] if s_path == HZ_FB_PATH_STREAM else
                        [f"fb_lti_kernel<2, {s_chunk}, *>", f"fb_lti_reduce_short_kernel<2, {s_chunk}>"]),
            "launches_per_block": 1 if s_path == HZ_FB_PATH_STREAM else 2,
            # event-bracketed (records add their own latency: the sum can exceed the un-instrumented
            # wall time per block)
            "profiled_us_per_block": gpu_us,
            "end_to_end_host_buffers": e2e,
            "per_band_engine": per_band,
            "roofline": {"bound": "latency: %s per block" % ("1 kernel launch" if s_path == HZ_FB_PATH_STREAM
                                                             else "2 dependent kernel launches"),
                         "achieved_tflops": stream_flops / (wall_us * 1e-6) / 1e12 if wall_us > 0 else None,
                         "flops_per_block": stream_flops,
                         "reference_equivalent_tflops": FLOPS_PER_BAND_SAMPLE * N_BANDS * B / (wall_us * 1e-6) / 1e12
                         if wall_us > 0 else None,
                         "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": FLOPS_PER_BAND_SAMPLE * N_BANDS * B / (wall_us * 1e-6) / 1e12 / FP64_PEAK_TFLOPS
                         if wall_us > 0 else None,
                         "note": "frac = the reference recurrence's 18 flops per band-sample over the wall time per "
                                 "block (reference-equivalent); achieved = the streaming engine's own FP64 work "
                                 "(bench.stream_block_flops) over the same time"},
        }

    # setter churn: the reference demos retarget mix() on every MIDI note
    # (tests/filterbank.cpp:217-252) -- here 9 random bands every 4800 samples (100 ms) over the
    # 1024-sample calls; the streaming engine keeps running with a transient term (hz_fb_stream.hip
    # fb_stream_gain_setter).  Last figure on the main handle: its gains change.
    if world == 1 and args.stream_blocks > 0 and stream_rate and args.side_steps > 0:
        side["setter_churn"] = setter_churn_figure(fb, x, y, min(args.stream_blocks, S // 1024), stream_rate)

    # the high-Q variant of C2 (tests/eigen.cpp:26's r = 0.9999): the same
    # recipe at R = 0.9999, whose horizon (~0.4 M samples) is past the streaming head's 2^17 -- the
    # 1024-sample calls add the response tail from per-epoch convolutions on a side stream
    # (hz_fb_stream.hip); parity: tests/test_fullsize_gpu.py::test_c2_high_q_*,
    # tests/test_fb_stream_gpu.py::test_stream_high_q_tail
    if world == 1 and args.side_steps > 0 and args.stream_blocks > 0 and not args.general and args.response != 0:
        fq, bq = c2_coefficients(R=0.9999)
        hq = Filterbank(2, N_BANDS, 0.1, 1.0, device=local)
        for n in range(N_BANDS):
            hq.coefficients(n, fq[n], bq[n])
        hq.boost(np.ones(N_BANDS))
        hq.open()
        hq.set_stream(stream.cuda_stream)
        yq = ys[1]

        def hq_long():
            hq.process_device(x.data_ptr(), yq.data_ptr(), S)

        for _ in range(6):   # priming: smoothers, then K samples of converged history
            hq_long()
            if hq.last_path() == HZ_FB_PATH_RESPONSE:
                break
        long_t = timed(hq_long, 3, min(args.side_steps, 20), S)
        long_t["path"] = {1: "general", 2: "lti", 3: "response"}.get(hq.last_path(), "?")
        hq.profile(True)   # the three launches' event times (forward, MAC, inverse + states)
        for _ in range(5):
            hq_long()
        barrier()
        f_ms, m_ms, i_ms, nl = hq.profile_read()
        hq.profile(False)
        long_t["kernels_ms_per_call"] = {"resp_fwd_kernel": f_ms / max(1, nl), "resp_mac_kernel": m_ms / max(1, nl),
                                         "resp_inv_kernel": i_ms / max(1, nl)}
        long_t["partitions"] = hq.response_info()[0] // 2048
        B = 1024
        nbq = min(args.stream_blocks, S // B)

        def hq_blocks(n_blocks):
            for i in range(n_blocks):
                hq.process_device(x.data_ptr() + 8 * B * i, yq.data_ptr() + 8 * B * i, B)

        hq_blocks(min(32, nbq))   # untimed: ring, head and tail spectra, first epochs
        barrier()
        ts = time.perf_counter()
        hq_blocks(nbq)
        barrier()
        tq = time.perf_counter() - ts
        side["high_q"] = {
            "R": 0.9999, "horizon": hq.response_info()[0],
            "long_calls": long_t,
            "streaming": {"us_per_block": 1e6 * tq / nbq, "band_samples_per_s": N_BANDS * B * nbq / tq,
                          "blocks": nbq, "path": {3: "response", 4: "stream"}.get(hq.last_path(), str(hq.last_path())),
                          "note": "one process() call per 1024-sample block; past the head's 2^17 samples the "
                                  "response tail is convolved per 16384-sample epoch ahead of time on a side "
                                  "stream and added by the block kernel (still one launch per block on the "
                                  "handle's stream)"},
        }
        hq.close()

    if world == 1 and P == 1 and args.side_steps > 0 and not args.no_general_side and args.dist == "none":
        side["general_softclip"] = general_softclip_figures(Filterbank, local, stream, x, ys[1], S,
                                                            traffic=not args.no_traffic and S == SAMPLES_PER_STEP)

    total_band_samples = N_BANDS * S * args.steps
    value = total_band_samples / elapsed
    if rank == 0:
        launch_avg_s = (eng_ms_max / 1e3) / max(1, launches)    # whole engine step, per process() call
        # this GPU's outputs per step: its time share (N > 1 / emulated) or the whole call
        out_samples = share_count if value_split else S
        # band-samples of one call on this GPU: all bands over its share, or its bands over the call
        bs_launch = (N_BANDS if value_split else cnt) * out_samples
        # ---- dominant kernel (roofline): the stationary engine's inverse kernel, which carries the
        # band-state pass (hz_fb_state.h: MFMA, ~96% of its flops) beside the output blocks' inverse
        # transforms; the state kernel of the per-band LTI engine; the mix kernel of the general
        # engine -- its average duration from the HIP events around it on the handle's stream
        mk = modal_kernels(horizon, out_samples, cnt, nexc=nexc, n_call=S,
                           first=share_first if value_split else 0) if modal else None
        if modal:
            # the three launches are each one wave of workgroups (latency-bound, intensity 2-5
            # flop/B, under the 9.8 flop/B ridge): the longest one by the events, against HBM
            per_k = {"resp_fwd_kernel": seg_ms, "resp_mac_kernel": mix_ms, "resp_inv_kernel": red_ms}
            dom = max(per_k, key=per_k.get)
            dom_name = {"resp_fwd_kernel": "resp_fwd_kernel (window transforms + modal phase 1: the fold and "
                                           "64-point DFTs of the band states)",
                        "resp_mac_kernel": "resp_mac_kernel_lds<%d> (partition MACs, operands staged in LDS)" % (horizon // 2048),
                        "resp_inv_kernel": "resp_inv_kernel<0> (inverse transforms of the output blocks + modal "
                                           "phase 2: 128-point DFTs and the band states)"}[dom]
            dom_ms = per_k[dom] / max(1, launches)
            dom_model = mk[dom][0]
        elif resp:
            dom = "resp_inv_kernel"
            dom_name = ("resp_inv_kernel<2> (inverse transforms of the output blocks + the band-state pass: "
                        "zero-start pass over the %d-sample history on the FP64 matrix cores)" % horizon)
            dom_ms = red_ms / max(1, launches)
            dom_model = resp_step_flops(horizon, out_samples, cnt)[1] + resp_inv_flops(out_samples)
        elif lti:
            dom = "fb_lti_kernel<2, %d, 2" % chunk
            dom_name = "fb_lti_kernel<2,%d,STATE> (chunk end states on MFMA + scan)" % chunk
            dom_ms = mix_ms / max(1, launches)
            dom_model = None
        else:
            dom = "fb_mix_kernel"
            dom_name = "fb_mix_kernel<2,NONE,1,MIX>"
            dom_ms = mix_ms / max(1, launches)
            dom_model = 20.0 * cnt * S
        step_kernels = (("fb_lti_kernel", "fb_lti_gemm", "fb_lti_reduce", "fb_lti_seg_carry", "fb_lti_sum",
                         "fb_lti_xrows") if lti
                        else ("resp_fwd_kernel", "resp_mac_kernel", "resp_inv_kernel") if resp
                        else ("fb_mix_kernel", "fb_reduce"))
        extra = (["--lti", args.lti] if args.lti else []) + (["--general"] if args.general else []) + \
                (["--response", str(args.response)] if args.response >= 0 else []) + \
                (["--modal", str(args.modal)] if args.modal >= 0 else [])
        traffic = flops = None
        traffic_detail = flops_detail = "skipped (--no-traffic, N > 1 or a non-default step length)"
        if not args.no_traffic and world == 1 and S == SAMPLES_PER_STEP:
            traffic, traffic_detail = pmc_traffic(step_kernels, extra)
            flops, flops_detail = pmc_flops(step_kernels, extra)
        dom_flops = flops.get(dom) if flops else None
        dom_traffic = traffic.get(dom) if traffic else None
        dom_fl = dom_flops if dom_flops else dom_model
        achieved = dom_fl / (dom_ms / 1e3) / 1e12 if (dom_fl and dom_ms > 0) else None
        # ---- the whole step: every kernel of a process() call over its whole GPU time
        if modal:
            step_model = mk["call"][0]
        elif resp:
            conv_f, state_f = resp_step_flops(horizon, out_samples, cnt)
            step_model = conv_f + state_f
        else:
            step_model = fb_executed_flops(lti, chunk, N=cnt) * cnt * S
        # algorithmic bytes of the whole call: the input and history in, the output and the history
        # out, the partition spectra, the per-band rows (modal: parameters, states, smoothers; the
        # matrix-core pass: its operand rows) -- not the engine's Z / Y / A intermediates
        if modal:
            call_bytes = mk["call"][1]
        elif resp:
            call_bytes = resp_alg_bytes(horizon, out_samples, cnt)[1]
        else:
            call_bytes = 16 * out_samples + 120 * cnt
        step_pmc = sum(flops.values()) if flops else None
        step_fl = step_pmc or step_model
        cpu = None
        if not args.no_cpu_baseline:   # rank 0's host cores, at every N (the other ranks wait)
            cpu = cpu_baseline(fwd, back)
        line = {
            "metric": "band-samples/s (bands x frames/s) for 4096-band Filterbank",
            "value": value,
            "unit": "band-samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "host_issue_ms_per_step": 1e3 * t_enq / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic white noise uniform[-1,1) (float32 -> double), seed 1234, resident in HBM",
            "config": {"workload": "C2 Filterbank<double>(order 2, 4096 bands), resonant band-pass "
                                   "f_i=0.5(i+1)SR/4096 R=0.999, boost 1 + open, k_p=0.1 k_g=1",
                       "samples_per_step": S, "samples_per_gpu": out_samples,
                       "call": f"one process() call of {S} samples per step (== {S // 1024} x 1024-sample "
                               f"blocks in result; the 1024-block streaming rate is `streaming`)",
                       "partition": 2048 if resp else None,
                       "bands": N_BANDS, "bands_per_gpu": cnt,
                       "parallelism": ("single GPU, all bands, no collective" if world == 1 else
                                       f"time split x{world}: rank r outputs its run of whole 2048-sample blocks "
                                       f"of the call ({out_samples} samples on rank 0) for all {N_BANDS} bands from "
                                       f"the shared input with a {horizon}-sample halo (whole-bank response, one "
                                       f"all-reduce at setup) and its own {cnt} bands' states; disjoint shares, "
                                       "no data-path collective" if value_split else
                                       f"bands partitioned x{world} ({cnt} per GPU), partial mixes summed to "
                                       "rank 0 by an RCCL reduce per step (overlapped with the next step's "
                                       "compute, double-buffered)")},
            "rehearsal": (f"{world} ranks on one GPU, collectives over gloo through host copies "
                          "(HZ_BENCH_REHEARSAL=1): the N > 1 code path, not an N-GPU figure")
                         if world > 1 and os.environ.get("HZ_BENCH_REHEARSAL") == "1" else None,
            "decomposition": None if P == 1 else {
                "value": (f"STRONG scaling: the FIXED 10 s call of N = 1 split by time over {P} GPUs; each rank "
                          "convolves its share of the output blocks with the whole bank's response (a stationary "
                          "call's output depends only on its input and the K inputs before it) and keeps its band "
                          "shard's states; shares disjoint and final, no collective in the step" if value_split else
                          f"STRONG scaling: a FIXED 10 s call per step, {N_BANDS} bands partitioned over {P} GPUs, "
                          "each rank's partial mix summed to rank 0 by an RCCL reduce (src/filterbank.h:130's "
                          "mixdown, sharded)"),
                "gather_to_rank0": side.get("gather_to_rank0"),
                "band_partition_stationary": side.get("band_partition_stationary"),
                "latency_floor": ("each rank's step is three dependent launches of one workgroup wave each; at "
                                  "N = 8 a share is 30 output blocks, so a launch is set by its latency, not its "
                                  "work: strong scaling is latency-floored near 3 launch latencies (DESIGN.md 5)"),
            },
            "emulated": ({"world": P, "rank": r_split, "note": (
                f"ONE GPU running rank {r_split} of {P} alone (--emulate-world): value = the whole job's "
                "band-samples over THIS rank's step time, i.e. the N-GPU figure if every rank took as long "
                "(no collective involved)")} if world == 1 and P > 1 else None),
            "engine": "stationary (bank response convolution, eager band states: %s)" % (
                "modal pass, hz_fb_modal.h" if modal else "matrix-core pass, hz_fb_state.h") if resp
                      else "per-band LTI" if lti else "per-band general",
            "roofline": {
                **({"bound": "hbm", "achieved": mk[dom][1] / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else None,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": mk[dom][1] / (dom_ms / 1e3) / 1e9 / HBM_PEAK_GBS if dom_ms > 0 else None,
                    "algorithmic_bytes_source": "bench.modal_kernels (the kernel's own inputs and outputs)",
                    "achieved_tflops": achieved,
                    "kernels_ms_per_call": {"resp_fwd_kernel": seg_ms / max(1, launches),
                                            "resp_mac_kernel": mix_ms / max(1, launches),
                                            "resp_inv_kernel": red_ms / max(1, launches)},
                    "modal_note": "band states by the modal pass (hz_fb_modal.h, DESIGN.md 3.11): the 0.83 GFLOP "
                                  "matrix-core pass is gone; each of the three launches is one wave of workgroups "
                                  "at 2-5 flop/B (FP64 ridge 9.8), so the dominant one is quoted against HBM"}
                   if modal else
                   {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": (achieved / FP64_PEAK_TFLOPS) if achieved else None}),
                "traffic": dom_traffic,
                "kernel": dom_name,
                "kernel_avg_ms": dom_ms,
                "flops_per_launch": dom_fl,
                "flops_source": "pmc (SQ_INSTS_VALU_{FMA,MUL,ADD}_F64, SQ_INSTS_VALU_MFMA_MOPS_F64)" if dom_flops
                                else "model (bench.resp_step_flops)",
                "model_flops_per_launch": dom_model,
                # inverse kernel + state pass: bench.resp_alg_bytes (the output, the state window,
                # the history written, the pass's operand rows, the states and smoothers -- not the
                # Y spectra, an engine intermediate); per-band engines: the block I/O and the band
                # records
                "algorithmic_bytes_per_launch": mk[dom][1] if modal else
                                                resp_alg_bytes(horizon, out_samples, cnt)[0] if resp
                                                else (16 * out_samples + 120 * cnt),
                "traffic_over_algorithmic": (dom_traffic / (mk[dom][1] if modal else
                                                            resp_alg_bytes(horizon, out_samples, cnt)[0]))
                                            if (resp and dom_traffic) else None,
                "peak_note": "FP64 MFMA peak = FP64 vector peak on MI355X (78.6 TFLOP/s); the state pass is "
                             "v_mfma_f64_16x16x4f64 chains (scripts/probe/mfma_f64_probe.hip: 71-78 TFLOP/s)",
                "step": {
                    "kernels": list(step_kernels),
                    "ms_per_call": 1e3 * launch_avg_s,
                    "components_ms_per_call": ({"forward": seg_ms / max(1, launches),
                                                "mac": mix_ms / max(1, launches),
                                                "inverse_and_states": red_ms / max(1, launches)} if resp else
                                               {"segment_prepass": seg_ms / max(1, launches),
                                                "convolution_or_state": mix_ms / max(1, launches),
                                                "states_or_gemm": red_ms / max(1, launches)}),
                    "flops_per_call": step_fl,
                    "flops_source": "pmc" if step_pmc else "model",
                    "model_flops_per_call": step_model,
                    "achieved_tflops": step_fl / launch_avg_s / 1e12 if launch_avg_s > 0 else None,
                    "frac": step_fl / launch_avg_s / 1e12 / FP64_PEAK_TFLOPS if launch_avg_s > 0 else None,
                    "traffic_per_call": sum(traffic.values()) if traffic else None,
                    "algorithmic_bytes_per_call": call_bytes,
                    "traffic_over_algorithmic": (sum(traffic.values()) / call_bytes) if (resp and traffic) else None,
                    "traffic_per_kernel": traffic, "flops_per_kernel": flops,
                    "traffic_detail": traffic_detail if not traffic else traffic_detail.get("method"),
                    "flops_detail": flops_detail if not flops else "pmc",
                    "reference_equivalent_tflops": FLOPS_PER_BAND_SAMPLE * bs_launch / launch_avg_s / 1e12
                                                   if launch_avg_s > 0 else None,
                    "note": ("reference_equivalent = the reference recurrence's 18 flops per band-sample (SURVEY.md "
                             "8(d)) over the step's GPU time; the stationary engine's cost does not grow with the "
                             "bands, so it exceeds the peak"),
                },
            },
            "side": side or None,
            "per_sample": per_sample_rates(dev.index or 0) if (world == 1 and not args.no_per_sample) else None,
            "streaming": {"band_samples_per_s": stream_rate, "block": 1024,
                          "us_per_block": (1e6 * N_BANDS * 1024 / stream_rate) if stream_rate else None,
                          "note": "one process() call per 1024-sample block, device-resident I/O, calls issued "
                                  "back to back (end_to_end_host_buffers: host I/O, synchronous per block)",
                          **stream_detail},
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
    if world > 1 and args.workload not in ("c3", "c3osc", "c4"):
        raise SystemExit("--workload c5..c9 are single-GPU configs (SURVEY.md 8(d)); c3, c3osc and c4 shard")
    shard_runs = {"c3": bench_rows.run_c3, "c3osc": bench_rows.run_c3osc, "c4": bench_rows.run_c4}
    rehearsal = world > 1 and os.environ.get("HZ_BENCH_REHEARSAL") == "1"
    if rehearsal:   # (one-GPU box: every rank on cuda:0, the reduces through host copies over gloo)
        local = 0
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group("gloo")
            bench_rows.COLL = _HostDist(dist)
        else:
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            dist.init_process_group("nccl", device_id=dev)
        body = shard_runs[args.workload](args, torch, dev, rank, world)
        if rehearsal:
            body["rehearsal"] = (f"{world} ranks on one GPU, reduces over gloo through host copies "
                                 "(HZ_BENCH_REHEARSAL=1): the N > 1 code path, not an N-GPU figure")
    elif args.workload in shard_runs and args.emulate_world:
        body = shard_runs[args.workload](args, torch, dev, 0, 1, args.emulate_world)
    else:
        fn = {"c3": bench_rows.run_c3, "c3osc": bench_rows.run_c3osc, "c4": bench_rows.run_c4, "c5": bench_rows.run_c5,
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
    sys.exit(main() or 0)
