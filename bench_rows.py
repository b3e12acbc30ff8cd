"""Secondary bench workloads for `bench.py --workload ...`.

Each returns the same JSON shape as the headline C2 line: value = whole-job throughput in
the config's unit with inputs resident in HBM, `roofline` for the dominant kernel from
HIP-event kernel time on the engine's stream, and a bounded `cpu_baseline` from the
oracle.  Only bench.py's C2 line is the BASELINE.json metric; these are per-row
measurements of the other configs.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
SR = 48000
FP64_PEAK = 78.6      # TFLOP/s
FP32_PEAK = 157.3     # TFLOP/s (vector)
HBM_PEAK = 8000.0     # GB/s


def _tests_path():
    p = os.path.join(ROOT, "tests")
    if p not in sys.path:
        sys.path.insert(0, p)


# the collectives of a multi-rank row: torch.distributed over RCCL, or (HZ_BENCH_REHEARSAL=1,
# several ranks on one GPU) bench._HostDist over gloo; set by bench.run_row
COLL = None


def _coll():
    if COLL is None:
        import torch.distributed as dist
        return dist
    return COLL


def _sync(torch, dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _stream_handle(torch, dev):
    return torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0


def _timed(step, steps, warmup, torch, dev, world=1):
    """Wall time of `steps` steps after `warmup`, barrier + synchronize on both sides; the
    max over ranks when world > 1."""
    dist = _coll() if world > 1 else None
    for _ in range(warmup):
        step()
    _sync(torch, dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _sync(torch, dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


# --------------------------------------------------------------------------- C3
# FP64 flops the Additive engine executes per partial-sample, measured with PMC counters on the
# C3 row (profiles/r2/flops_pmc.txt: add_mix_kernel 1.97e11 flops over 5 steps of 7.86e9
# partial-samples with the two-term sine recurrence in 32-sample chunks; it was 9.1 with the
# per-sample complex rotation)
EXEC_C3 = 5.0

# rocprofv3 --pmc counter sets (one pass each: <= 8 SQ counters)
PMC_VALU = ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_TRANS_F32",
            "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")
PMC_F64_MFMA = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES")


def pmc_counts(kernel, workload, counters):
    """one rocprofv3 --pmc pass over a short run of this row (bench.pmc_pass: kernel trace only, a
    child process): per-launch counts of `kernel` and the flops / lane-ops they imply"""
    import bench
    res, err = bench.pmc_pass(counters, (kernel,), extra=("--workload", workload))
    if res is None:
        return {"error": err}
    c = res.get(kernel, {})
    out = {"counters": c, "counters_per": "launch (mean of the two largest dispatches)"}
    lanes = 64.0
    out["f32_flops"] = lanes * (2 * c.get("SQ_INSTS_VALU_FMA_F32", 0) + c.get("SQ_INSTS_VALU_MUL_F32", 0) +
                                c.get("SQ_INSTS_VALU_ADD_F32", 0))
    out["f64_flops"] = lanes * (2 * c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) +
                                c.get("SQ_INSTS_VALU_ADD_F64", 0)) + 512.0 * c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
    out["trans_ops"] = lanes * (c.get("SQ_INSTS_VALU_TRANS_F32", 0) + c.get("SQ_INSTS_VALU_TRANS_F64", 0))
    if c.get("SQ_BUSY_CYCLES"):
        out["mfma_busy_frac"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / c["SQ_BUSY_CYCLES"]
    return out


def row_evidence(kernel, workload, seconds_per_unit, counters=PMC_VALU, per_step=None, alg_bytes=None):
    """PMC evidence for a row's dominant kernel: HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, separate
    passes) and executed FP32 / FP64 flops and transcendental lane-ops, each over
    `seconds_per_unit` (the kernel's HIP-event time per launch, or per step when `per_step` = the
    launches per step: then the counts are summed over all dispatches and divided by
    dispatches / per_step) against its pipe's peak.  The binding pipe is the largest fraction."""
    import bench
    mode = "launch" if per_step is None else f"step ({per_step} launches)"
    res, err = bench.pmc_pass(counters, (kernel,), extra=("--workload", workload), per_step=per_step)
    if res is None:
        return {"error": err}
    c = res.get(kernel, {})
    tr, terr = bench.pmc_traffic((kernel,), extra=("--workload", workload), per_step=per_step)
    lanes = 64.0
    f32 = lanes * (2 * c.get("SQ_INSTS_VALU_FMA_F32", 0) + c.get("SQ_INSTS_VALU_MUL_F32", 0) +
                   c.get("SQ_INSTS_VALU_ADD_F32", 0))
    f64 = lanes * (2 * c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) +
                   c.get("SQ_INSTS_VALU_ADD_F64", 0)) + 512.0 * c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
    trans = lanes * (c.get("SQ_INSTS_VALU_TRANS_F32", 0) + c.get("SQ_INSTS_VALU_TRANS_F64", 0))
    traffic = (tr or {}).get(kernel)
    out = {"kernel": kernel, "per": mode, "counters": c, "f32_flops": f32, "f64_flops": f64, "trans_ops": trans,
           "traffic_bytes": traffic, "traffic_error": terr if tr is None else None,
           "algorithmic_bytes": alg_bytes, "seconds": seconds_per_unit}
    if seconds_per_unit:
        fr = {"fp32_valu": f32 / seconds_per_unit / 1e12 / FP32_PEAK,
              "fp64_valu": f64 / seconds_per_unit / 1e12 / FP64_PEAK,
              "transcendental": trans / seconds_per_unit / 1e12 / (FP32_PEAK / 8)}
        if traffic:
            fr["hbm"] = traffic / seconds_per_unit / 1e9 / HBM_PEAK
        out.update(tflops_fp64=f64 / seconds_per_unit / 1e12, tflops_fp32=f32 / seconds_per_unit / 1e12,
                   gbs=traffic / seconds_per_unit / 1e9 if traffic else None, fracs=fr,
                   binding_pipe=max(fr, key=fr.get))
        if traffic and alg_bytes:
            out["traffic_over_algorithmic"] = traffic / alg_bytes
    out["note"] = ("counts from rocprofv3 --pmc passes of this row (kernel trace only); seconds from HIP events "
                   "on the engine's stream; the row's rocprofv3 kernel-trace summary (profiles/r5/rows/*_kernel_"
                   "stats*.csv) reproduces the time")
    return out


def pipe_fracs(counts, seconds):
    """each pipe's executed rate over the kernel's time against that pipe's peak"""
    if not counts or "error" in counts or not seconds:
        return counts
    f32 = counts["f32_flops"] / seconds / 1e12
    f64 = counts["f64_flops"] / seconds / 1e12
    tr = counts["trans_ops"] / seconds / 1e12
    fr = {"fp32_valu": f32 / FP32_PEAK, "fp64_valu": f64 / FP64_PEAK, "transcendental": tr / (FP32_PEAK / 8)}
    return dict(counts, seconds_per_launch=seconds, tflops_fp32=f32, tflops_fp64=f64, trans_tops=tr, fracs=fr,
                binding_pipe=max(fr, key=fr.get),
                trans_peak_note="transcendental peak taken as a quarter of the FP32 FMA lane rate: FP32_PEAK / 8 "
                                "lane-ops/s")


def run_c3(args, torch, dev, rank=0, world=1, shard_world=None, probe=None):
    """Additive<double>(&cycle, 64, 256, 0.75, 1.0), all voices via makenote(36+v, 1),
    voices 0-7 released at sample 24,000; one step = 480,000 samples.  With world > 1 (the
    BASELINE config: 8 GPUs) each rank owns a contiguous overtone range (huygens_amd.shard,
    hz_add_create_shard) and the partial mixes are summed to rank 0 by an RCCL reduce.  `probe`
    (tests) is called with the last step's output after the timed steps."""
    from huygens_amd import Additive
    from huygens_amd.shard import shard_of
    V, O, S = 64, 256, args.samples
    sw = shard_world or world   # --emulate-world P: rank 0's shard of P, on one GPU, no reduce
    o0, oc = shard_of(rank, sw, O)
    add = Additive(V, O, 0.75, 1.0, device=dev.index or 0, shard=(o0, oc) if sw > 1 else None)
    for v in range(V):
        add.makenote(36 + v, 1.0)
    add.set_stream(_stream_handle(torch, dev))
    y = torch.empty(S, dtype=torch.float64, device=dev)
    rel = min(24000, S)

    def step():
        add.fill_device(y.data_ptr(), rel)
        for v in range(8):
            add.release(v)
        add.fill_device(y.data_ptr() + 8 * rel, S - rel)
        if world > 1:
            dist.reduce(y, dst=0, op=dist.ReduceOp.SUM)

    dist = _coll() if world > 1 else None
    for _ in range(args.warmup):
        step()
    elapsed = _timed(step, args.steps, 0, torch, dev, world)
    if probe is not None:
        probe(y)
    add.profile(True)   # kernel times: a separate profiled pass (no events in the timed region)
    _timed(step, args.steps, 0, torch, dev)
    ms, launches = add.profile_read()
    add.profile(False)
    units = V * (O if shard_world is None else oc * sw) * S * args.steps
    kern_s = ms / 1e3
    flops = 22.0 * V * oc * S * args.steps   # 22 flops (+ 3 transcendentals) per partial-sample
    achieved = flops / kern_s / 1e12 if kern_s > 0 else None
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        _tests_path()
        from oracle_osc import OracleAdditive
        o = OracleAdditive(V, O, 0.75, 1.0)
        for v in range(V):
            o.makenote(36 + v, 1.0)
        n = 1500
        t0 = time.perf_counter()
        o.fill(n)
        dt = time.perf_counter() - t0
        cpu = {"value": V * O * n / dt, "unit": "partial-samples/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle_osc.c Additive, {V}x{O} partials x {n} samples, 1 thread, {dt:.2f} s"}
    xach = EXEC_C3 * units / kern_s / 1e12 if kern_s > 0 else None
    ev = None
    if not getattr(args, "no_traffic", True) and sw == 1:
        ev = row_evidence("add_mix_kernel", "c3", kern_s / args.steps, per_step=2,
                          alg_bytes=8.0 * S)   # the mix's output
        if ev and "error" not in ev:
            ev["traffic_note"] = ("add_mix_kernel writes one partial mix per overtone group ([G][n], summed by "
                                  "add_reduce_kernel): the excess over the output is those partials, by design; "
                                  "HBM stays near 1.5 % of its peak while FP64 is the binding pipe")
    return {
        "metric": "partial-samples/s for 64-voice x 256-overtone Additive",
        "value": units / elapsed, "unit": "partial-samples/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f64",
        "data": "synthetic: makenote(36+v, 1.0) for 64 voices, voices 0-7 released at sample 24000",
        "config": {"workload": "C3 Additive<double>(&cycle, 64, 256, 0.75, 1.0), physics off",
                   "samples_per_step": S, "voices": V, "overtones": O, "overtones_per_gpu": oc,
                   "parallelism": f"overtones sharded x{world}, RCCL reduce"},
        "n_gpus": world, "scaling": "strong", "emulated_world": shard_world,
        "roofline": {"bound": "valu", "achieved": xach, "peak": FP64_PEAK, "unit": "TFLOP/s",
                     "frac": xach / FP64_PEAK if xach else None,
                     "traffic": (ev or {}).get("traffic_bytes"), "pmc_evidence": ev,
                     "kernel": "add_mix_kernel (+ add_reduce_kernel, add_advance_kernel)",
                     "kernel_avg_ms": ms / max(1, launches), "launches": launches,
                     "kernel_ms_per_step": ms / args.steps, "launches_per_step": launches / max(1, args.steps),
                     "launch_note": "two add_mix launches per step (24,000 then 456,000 samples, the release "
                                    "between): kernel_avg_ms is their mean; a rocprofv3 summary of this row "
                                    "reproduces kernel_ms_per_step as TotalDurationNs / steps",
                     "flops_per_unit": EXEC_C3,
                     "flops_source": "rocprofv3 --pmc SQ_INSTS_VALU_{FMA,MUL,ADD}_F64 on this row "
                                     "(profiles/r2/flops_pmc.txt)",
                     "reference_equivalent": {"flops_per_unit": 22, "achieved": achieved,
                                              "frac": achieved / FP64_PEAK if achieved else None},
                     "note": "achieved = the FP64 work the closed-form engine performs per partial-sample (PMC) "
                             "over the whole launch (mix + reduce + advance); reference_equivalent = the "
                             "algorithmic 22 flops (+ 3 transcendentals) of the reference's per-sample update "
                             "(SURVEY.md 8(d)) over the same time"},
        "cpu_baseline": cpu,
    }


# ------------------------------------------------------------------ C3 (Oscbank variant)
def c3_frequencies(V=64, O=256):
    """The C3 partials' target frequencies as Additive::request sets them (src/additive.h:91-110,
    harm = 1): f_vj = mtof(ftom(f0_v (1 + j))), f0_v = mtof(36 + v) (src/includes.h mtof / ftom)"""
    import math

    def mtof(m):
        return 440.0 * 2.0 ** ((m - 69) / 12)

    def ftom(f):
        return 69 + math.log2(f / 440.0) * 12
    return np.array([mtof(ftom(mtof(36 + v) * (1 + j))) for v in range(V) for j in range(O)])


def run_c3osc(args, torch, dev, rank=0, world=1, shard_world=None, probe=None):
    """C3's secondary variant: Oscbank<double, 16384> with the C3 partials'
    frequencies (c3_frequencies), every partial active (open()), and the complex Mixer mixdown
    (src/oscbank.h:59-90, src/mixer.h:9) over 480,000 samples per step.  world > 1: partials sharded
    (hz_osc_create_shard), the complex mixes (2 x 480,000 doubles) summed to rank 0 by an RCCL reduce."""
    from huygens_amd import Oscbank
    from huygens_amd.shard import shard_of
    N, S = 16384, args.samples
    f = c3_frequencies()
    sw = shard_world or world
    p0, pc = shard_of(rank, sw, N)
    ob = Oscbank(N, device=dev.index or 0, shard=(p0, pc) if sw > 1 else None)
    for i in range(p0, p0 + pc):
        ob.freqmod(i, f[i])
    ob.open()
    ob.set_stream(_stream_handle(torch, dev))
    mix = torch.empty(2 * S, dtype=torch.float64, device=dev)

    def step():
        ob.fill_device(mix.data_ptr(), None, S)
        if world > 1:
            dist.reduce(mix, dst=0, op=dist.ReduceOp.SUM)

    dist = _coll() if world > 1 else None
    for _ in range(args.warmup):
        step()
    elapsed = _timed(step, args.steps, 0, torch, dev, world)
    if probe is not None:
        probe(mix)
    ob.profile(True)
    _timed(step, args.steps, 0, torch, dev)
    ms, launches = ob.profile_read()
    ob.profile(False)
    units = N * S * args.steps if shard_world is None else pc * sw * S * args.steps
    kern_s = ms / 1e3
    ref_fl = 15.0 * pc * S * args.steps   # SURVEY.md 8(d) C3 Oscbank: 15 FP64 flops per partial-sample
    achieved = ref_fl / kern_s / 1e12 if kern_s > 0 else None
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        _tests_path()
        from oracle import OracleOscbank
        o = OracleOscbank(N)
        for i in range(N):
            o.freqmod(i, f[i])
        o.open()
        n = 2000
        t0 = time.perf_counter()
        o.fill(n)
        dt = time.perf_counter() - t0
        cpu = {"value": N * n / dt, "unit": "partial-samples/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle_osc.c Oscbank, {N} partials x {n} samples, 1 thread, {dt:.2f} s"}
    ev = None
    if not getattr(args, "no_traffic", True) and sw == 1:
        ev = row_evidence("osc_mix_kernel", "c3osc", kern_s / max(1, launches), alg_bytes=16.0 * S)
    return {
        "metric": "partial-samples/s for Oscbank<double,16384> + complex mixdown (C3 variant)",
        "value": units / elapsed, "unit": "partial-samples/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f64",
        "data": "synthetic: the C3 partials' frequencies (64 voices x 256 overtones of mtof(36 + v)), all active",
        "config": {"workload": "C3 variant: Oscbank<double,16384> + Mixer, 480,000 samples per step",
                   "samples_per_step": S, "partials": N, "partials_per_gpu": pc,
                   "parallelism": f"partials sharded x{world}, RCCL reduce of the complex mix"},
        "n_gpus": world, "scaling": "strong", "emulated_world": shard_world,
        "roofline": {"bound": "valu", "achieved": achieved, "peak": FP64_PEAK, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK if achieved else None,
                     "traffic": (ev or {}).get("traffic_bytes"), "pmc_evidence": ev,
                     "kernel": "osc_mix_kernel (+ osc_reduce_kernel, osc_advance_kernel)",
                     "kernel_avg_ms": ms / max(1, launches), "launches": launches,
                     "flops_per_unit": 15,
                     "note": "achieved = SURVEY.md 8(d)'s 15 FP64 flops per partial-sample of the reference's "
                             "renormalised phasor recurrence over the whole launch (mix + reduce + advance); the "
                             "engine evaluates z0 w^t in closed form (pmc_evidence: its executed work)"},
        "cpu_baseline": cpu,
    }


# --------------------------------------------------------------------------- C4
def c4_signal(n, seed=3):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / float(SR)
    x = 0.1 * rng.standard_normal(n)
    for k in range(1, 9):
        x += 0.5 * np.sin(2 * np.pi * 220 * k ** 1.5 * t)
    return x


def run_c4(args, torch, dev, rank=0, world=1, shard_world=None, probe=None):
    """StaticSTFT(4096, 4) with its built-in gate over 480,000 samples (C4 (i)); the
    Fourier(gate625) variant (ii) is timed beside it.  Under torchrun (world > 1) every rank
    streams the whole input but computes only its runs of frames (runs of ceil(frames per
    step / world) frames rotate over the ranks: hz_stft_set_frame_shard, SURVEY.md 8(e) STFT
    row) and the partial outputs are summed to rank 0 over RCCL."""
    from huygens_amd import Fourier, StaticSTFT
    from huygens_amd.stft import frames_before
    N, laps, S = 4096, 4, args.samples
    x = torch.from_numpy(c4_signal(S)).to(dev)
    yr = torch.empty_like(x)
    yi = torch.empty_like(x)
    out = {}
    for name, eng in (("static", StaticSTFT(N, laps)), ("gate625", Fourier(2, N, laps))):
        eng.set_stream(_stream_handle(torch, dev))
        sw = shard_world or world   # --emulate-world: rank 0's share of an sw-GPU job, no reduce
        if sw > 1:
            eng.set_frame_shard(rank, sw, -(-frames_before(N, laps, S) // sw))

        def step():
            eng.process_block_device(x.data_ptr(), 0, yr.data_ptr(), yi.data_ptr(), S)
            if world > 1:
                dist = _coll()
                dist.reduce(yr, dst=0, op=dist.ReduceOp.SUM)

        for _ in range(args.warmup):
            step()
        _sync(torch, dev)
        f0 = eng.frames()[0]
        elapsed = _timed(step, args.steps, 0, torch, dev, world)
        if probe is not None and name == "static":
            probe(yr)
        frames = eng.frames()[0] - f0
        # kernel times from a separate profiled pass: each block's frame launch repeated 8x
        # between one event pair (an event pair costs about as much as one ~20 us launch)
        eng.profile(True, repeat=8)
        for _ in range(args.steps):
            step()
        fms, oms, blocks = eng.profile_read()
        eng.profile(False)
        out[name] = (elapsed, fms, oms, blocks, frames)
    elapsed, fms, oms, blocks, frames = out["static"]
    sw = shard_world or world
    flops = 491520.0 * frames / sw   # 2 x 5 N log2 N per frame, this rank's share
    achieved = flops / (fms / 1e3) / 1e12 if fms > 0 else None
    cpu = None
    if not args.no_cpu_baseline and sw == 1:
        _tests_path()
        from oracle_stft import OracleSTFT
        o = OracleSTFT(N, laps, 1, 1)
        n = 96000
        xs = c4_signal(n)
        t0 = time.perf_counter()
        o.process_block(xs)
        dt = time.perf_counter() - t0
        cpu = {"value": o.frames() / dt, "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle_stft.c StaticSTFT(4096,4), {n} samples ({o.frames()} frames), "
                         f"long double radix-2 FFT, 1 thread, {dt:.2f} s"}
    e2, f2, o2, b2, fr2 = out["gate625"]
    traffic, tdetail = None, "not collected (--no-traffic)"
    pmc = None
    # StaticSTFT(4096)'s gate kernel (hz_stft.hip): HZ_STFT_FRAME=half (one frame per workgroup) or pair
    pair = os.environ.get("HZ_STFT_FRAME", "pair") != "half"
    kname = "stft_pair4096_kernel" if pair else "stft_half4096_kernel"
    if not args.no_traffic and sw == 1:
        import bench
        tb, tdetail = bench.pmc_traffic((kname, "stft_ola_seg_kernel"), extra=("--workload", "c4"))
        traffic = tb   # HBM bytes per launch (one frame launch + one overlap-add launch per step)
        pmc = pmc_counts(kname, "c4", PMC_F64_MFMA)
    return {
        "metric": "STFT frames/s, StaticSTFT 4096-pt / 75% overlap spectral gate",
        "value": frames / elapsed, "unit": "frames/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f64",
        "samples_per_s": S * args.steps / elapsed,
        "data": "synthetic: white noise sigma 0.1 + 8 sinusoids 0.5 sin(2 pi 220 k^1.5 t), seed 3",
        "config": {"workload": "C4 StaticSTFT(4096, 4) built-in gate (100, 0.1)", "samples_per_step": S,
                   "frames_per_step": frames // args.steps,
                   "parallelism": f"frames by time range x{world}, RCCL reduce" if world > 1 else "1 GPU"},
        "n_gpus": world, "scaling": "strong", "emulated_world": shard_world,
        "roofline": {"bound": "valu", "achieved": achieved, "peak": FP64_PEAK, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK if achieved else None,
                     "traffic": (traffic or {}).get(kname), "traffic_ola": (traffic or {}).get("stft_ola_seg_kernel"),
                     "traffic_detail": tdetail,
                     "kernel": ("stft_pair4096_kernel<STATIC_GATE> (two real frames per transform: window, "
                                "radix-8 FFT, split + gate + merge, IFFT in LDS)") if pair else
                               ("stft_half4096_kernel<STATIC_GATE> (one real frame per workgroup as a 2048-point "
                                "even/odd transform: window, radix-8/4 FFT, split + gate + merge, IFFT in LDS)"),
                     "kernel_ms_per_step": fms / args.steps, "ola_ms_per_step": oms / args.steps,
                     "flops_per_frame": 491520,
                     "pmc": pmc,
                     "executed_flops_per_launch": (pmc or {}).get("f64_flops"),
                     "mfma_utilisation": (pmc or {}).get("mfma_busy_frac"),
                     "mfma_note": "0 by design: the DFT runs as a radix-8 FFT on the FP64 VALU. An FP64 MFMA DFT "
                                  "(v_mfma_f64_16x16x4f64, 64 x 64 factorisation) does 17x the FFT's flops at the "
                                  "same FP64 rate (FP64 MFMA and VALU share the pipe on MI355X) and measured 2.63x "
                                  "slower (DESIGN.md 4.1)"},
        "variant_fourier_gate625": {"frames_per_s": fr2 / e2, "kernel_ms_per_step": f2 / args.steps,
                                    "ola_ms_per_step": o2 / args.steps},
        "cpu_baseline": cpu,
    }


# --------------------------------------------------------------------------- C5
def c5_model(M=2048, seed=5):
    rng = np.random.default_rng(seed)
    f = np.exp(rng.uniform(np.log(20.0), np.log(16000.0), M))
    a = rng.uniform(1e-4, 5e-2, M)
    d = rng.uniform(0.05, 15.0, M)
    return f, a, d


def run_c5(args, torch, dev):
    """Bowl<float>(2048) fill(buf, 1024) x 469 with trigger() at t = 0, feeding
    Delaybank<float,64>: line k = Delay<float>(3, 2 SR), fwd {(0,1)},
    fb {(10000+37k, .5), (20000+53k, .5)}, lines mixed / 64.  One step = the 469 blocks."""
    from huygens_amd import Bowl, Delaybank
    M, L, B = 2048, 64, 1024
    nb = max(1, args.samples // B)
    f, a, d = c5_model(M)
    bowl = Bowl(M, f, a, d, np.float32)
    bank = Delaybank(L, 3, 2 * SR, np.float32)
    for k in range(L):
        bank.coefficients(k, [(0, 1.0)], [(10000 + 37 * k, 0.5), (20000 + 53 * k, 0.5)])
    stream = torch.cuda.Stream(dev)   # one stream for both handles (the fused call requires it)
    bowl.set_stream(stream.cuda_stream)
    bank.set_stream(stream.cuda_stream)
    buf = torch.empty(nb * B, dtype=torch.float32, device=dev)
    mix = torch.empty(nb * B, dtype=torch.float32, device=dev)

    def step_calls():   # the reference's two calls per block: fill, then process (4 launches)
        bowl.trigger()
        for i in range(nb):
            bowl.fill_device(buf.data_ptr() + 4 * B * i, B)
            bank.process_device(buf.data_ptr() + 4 * B * i, mix.data_ptr() + 4 * B * i, B, False, True)

    def step():   # the same two calls as one launch per block (hz_bowl_fill_delaybank)
        bowl.trigger()
        for i in range(nb):
            bowl.fill_delaybank(bank, buf.data_ptr() + 4 * B * i, mix.data_ptr() + 4 * B * i, B, True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    elapsed = _timed(step, args.steps, 0, torch, dev)   # no event records in the timed region
    elapsed_calls = _timed(step_calls, args.steps, 1, torch, dev)
    # kernel times of the streamed blocks: a separate profiled pass (the fused launch is the bowl's)
    bowl.profile(True)
    bank.profile(True)
    _timed(step, args.steps, 0, torch, dev)
    fms, fl = bowl.profile_read()
    bowl.profile(False)
    bank.profile(False)
    bowl.profile(True)
    bank.profile(True)
    _timed(step_calls, args.steps, 0, torch, dev)
    bms, bl = bowl.profile_read()
    dms, dl = bank.profile_read()
    bowl.profile(False)
    bank.profile(False)

    # whole-signal kernels (one call each), the rates the roofline is quoted on
    n = nb * B
    bowl.profile(True)
    bank.profile(True)
    torch.cuda.synchronize(dev)
    for _ in range(max(1, args.steps)):
        bowl.trigger()
        bowl.fill_device(buf.data_ptr(), n)
        bank.process_device(buf.data_ptr(), mix.data_ptr(), n, False, True)
    torch.cuda.synchronize(dev)
    bms_w, bl_w = bowl.profile_read()
    dms_w, dl_w = bank.profile_read()
    bowl.profile(False)
    bank.profile(False)
    split_ms = {}
    for mode in (1, 2):   # one workgroup per line looping over sub-blocks / a launch per sub-block
        bank.set_split(mode)
        bank.profile(True)
        for _ in range(max(1, args.steps)):
            bank.process_device(buf.data_ptr(), mix.data_ptr(), n, False, True)
        torch.cuda.synchronize(dev)
        ms_, l_ = bank.profile_read()
        bank.profile(False)
        split_ms[str(mode)] = ms_ / max(1, l_)
    bank.set_split(0)
    bowl_rate = M * n * bl_w / (bms_w / 1e3) if bms_w > 0 else None
    dly_rate = L * n * dl_w / (dms_w / 1e3) if dms_w > 0 else None
    achieved = bowl_rate * 8 / 1e12 if bowl_rate else None
    pipes = chain_pipes = chain_traffic = None
    if not args.no_traffic:
        import bench
        kb = bms_w / max(1, bl_w) / 1e3                         # whole-signal bowl_mix_kernel, s
        kc = fms / max(1, fl) / 1e3                              # fused block kernel, s
        pipes = pipe_fracs(pmc_counts("bowl_mix_kernel", "c5", PMC_VALU), kb)
        chain_pipes = pipe_fracs(pmc_counts("bowl_dly_chain_kernel", "c5", PMC_VALU), kc)
        chain_traffic, _ = bench.pmc_traffic(("bowl_dly_chain_kernel",), extra=("--workload", "c5"))
        mix_traffic, _ = bench.pmc_traffic(("bowl_mix_kernel",), extra=("--workload", "c5"))
        if pipes and "error" not in pipes:
            pipes["traffic_bytes"] = (mix_traffic or {}).get("bowl_mix_kernel")
            pipes["algorithmic_bytes"] = 12.0 * M + 8.0 * n   # mode table in, f64 mix out
            if pipes["traffic_bytes"]:
                pipes["gbs"] = pipes["traffic_bytes"] / kb / 1e9
                pipes["fracs"]["hbm"] = pipes["gbs"] / HBM_PEAK
    cpu = None
    if not args.no_cpu_baseline:
        _tests_path()
        from oracle_bowl import OracleBowl
        o = OracleBowl(M, f, a, d, np.float32)
        ns = 4096
        t0 = time.perf_counter()
        o.fill(ns)
        dt = time.perf_counter() - t0
        cpu = {"value": M * ns / dt, "unit": "mode-samples/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle_bowl.c Bowl<float>(2048), {ns} samples, 1 thread, {dt:.2f} s"}
    return {
        "metric": "mode-samples/s for Bowl<float>(2048) streamed in 1024-sample blocks into Delaybank<float,64>",
        "value": M * n * args.steps / elapsed, "unit": "mode-samples/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f32 (phase model) / f64 accumulation",
        "line_samples_per_s": L * n * args.steps / elapsed,
        "data": "synthetic modal model seed 5: f log-uniform [20,16000] Hz, a U[1e-4,5e-2], d U[0.05,15]",
        "config": {"workload": "C5 Bowl<float>(2048) fill x 469 blocks + Delaybank<float,64>(3, 2SR), mix /64",
                   "samples_per_step": n, "block": B, "modes": M, "lines": L},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": FP32_PEAK, "unit": "TFLOP/s",
                     "frac": achieved / FP32_PEAK if achieved else None,
                     "traffic": (pipes or {}).get("traffic_bytes"),
                     "kernel": "bowl_mix_kernel (float phase model)",
                     "kernel_ms_whole_signal": bms_w / max(1, bl_w), "flops_per_unit": 8,
                     "mode_samples_per_s_kernel": bowl_rate,
                     "executed_pipes": pipes,
                     "note": "frac: the model's 8 flops per mode-sample over the FP32 vector peak (SURVEY.md 8(d) "
                             "C5); executed_pipes: PMC-counted FP32 / FP64 flops and transcendental lane-ops of the "
                             "same kernel over its time, each against its own pipe's peak -- the largest fraction "
                             "names the binding pipe"},
        "roofline_delaybank": {"bound": "hbm", "achieved": dly_rate * 20 / 1e9 if dly_rate else None,
                               "peak": HBM_PEAK, "unit": "GB/s",
                               "frac": dly_rate * 20 / 1e9 / HBM_PEAK if dly_rate else None,
                               "kernel": "dly_line_kernel<float>", "kernel_ms_whole_signal": dms_w / max(1, dl_w),
                               "line_samples_per_s_kernel": dly_rate, "bytes_per_unit": 20,
                               "whole_signal_ms_by_split": split_ms},
        "streamed_kernel_ms_per_step": {"bowl": bms / args.steps, "delaybank": dms / args.steps},
        "block": {"us_per_block": 1e6 * elapsed / args.steps / nb, "launches_per_block": 1,
                  "kernel": "bowl_dly_chain_kernel (hz_bowl_fill_delaybank: the block's Bowl samples, "
                            "every line, the ring commit and the mixdown in one launch)",
                  "kernel_us_per_block": 1e3 * fms / max(1, fl),
                  "executed_pipes": chain_pipes,
                  "traffic_per_launch": (chain_traffic or {}).get("bowl_dly_chain_kernel"),
                  "two_calls_per_block": {"us_per_block": 1e6 * elapsed_calls / args.steps / nb,
                                          "launches_per_block": 4,
                                          "value": M * n * args.steps / elapsed_calls,
                                          "kernel_us_per_block": 1e3 * (bms + dms) / args.steps / nb}},
        "cpu_baseline": cpu,
    }


# --------------------------------------------------------------------------- C6
def c6_requests(n, seed=6, every=26):
    """Granary-like grain stream: one request every `every` samples (about what keeps 512
    voices busy at a 275 ms mean grain), sizes U[50,500] ms, speeds U[0.5,2], offsets
    U[0,1] s, gains U[0,1].  Requests with no free voice return -1, as in the reference."""
    from huygens_amd import GRAIN_REQ
    rng = np.random.default_rng(seed)
    at = np.arange(0, n, every)
    r = np.zeros(at.size, dtype=GRAIN_REQ)
    r["at"] = at
    r["offset"] = rng.uniform(0.0, 1.0, at.size)
    r["size"] = rng.uniform(0.05, 0.5, at.size)
    r["speed"] = rng.uniform(0.5, 2.0, at.size)
    r["gain"] = rng.uniform(0.0, 1.0, at.size)
    return r


def run_c6(args, torch, dev):
    """Granulator<double>(&hann, Buffer(3 SR), polyphony 512) over 480,000 samples per step
    with the c6_requests grain stream (tests/granny.cpp loop body per sample)."""
    from huygens_amd import Granulator
    P, S = 512, args.samples
    rng = np.random.default_rng(7)
    x = torch.from_numpy(rng.uniform(-1.0, 1.0, S)).to(dev)
    y = torch.empty_like(x)
    reqs = c6_requests(S)
    g = Granulator(3 * SR, P)
    g.set_stream(torch.cuda.current_stream(dev).cuda_stream)

    def step():
        g.process_device(x.data_ptr(), y.data_ptr(), S, reqs)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    g.profile(True)
    elapsed = _timed(step, args.steps, 0, torch, dev)
    ms, launches, gs = g.profile_read()
    g.profile(False)
    flops = 16.0 * gs   # per grain-sample: 16 FP64 flops + 1 cos + 1 divide
    achieved = flops / (ms / 1e3) / 1e12 if ms > 0 else None
    ev = None
    if not getattr(args, "no_traffic", True) and launches:
        per = max(1, round(launches / args.steps))
        ev = row_evidence("gran_kernel", "c6", ms / 1e3 / args.steps, per_step=per,
                          alg_bytes=16.0 * S + 8.0 * 3 * SR)   # input + output per sample, the 3 s ring once
    cpu = None
    if not args.no_cpu_baseline:
        _tests_path()
        from oracle_gran import OracleGranulator
        o = OracleGranulator(3 * SR, P)
        n = 96000
        rq = c6_requests(n)
        xs = rng.uniform(-1.0, 1.0, n)
        reqs_t = [(int(r["at"]), r["offset"], r["size"], r["speed"], r["gain"], 0.0) for r in rq]
        t0 = time.perf_counter()
        o.process(xs, reqs_t)
        dt = time.perf_counter() - t0
        cpu = {"value": n / dt, "unit": "samples/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle_gran.c Granulator(512), {n} samples of the same grain stream "
                         f"(voices fill up over the sample), 1 thread, {dt:.2f} s"}
    return {
        "metric": "grain-samples/s, Granulator<double>(hann, Buffer(3 SR), polyphony 512)",
        "value": gs / elapsed, "unit": "grain-samples/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f64",
        "samples_per_s": S * args.steps / elapsed,
        "data": "synthetic: uniform[-1,1) input seed 7; c6_requests grain stream seed 6 (one request / 26 samples)",
        "config": {"workload": "C6 Granulator<double>(&hann, Buffer(3*SR), 512) (SURVEY.md 8(f) row 1)",
                   "samples_per_step": S, "requests_per_step": int(reqs.size), "polyphony": P},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": FP64_PEAK, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK if achieved else None,
                     "traffic": (ev or {}).get("traffic_bytes"), "pmc_evidence": ev,
                     "kernel": "gran_kernel", "kernel_ms_per_step": ms / args.steps, "launches": launches,
                     "grain_samples_per_step": gs / args.steps, "flops_per_unit": 16,
                     "note": "16 FP64 flops + cos + divide per grain-sample; transcendental-bound"},
        "cpu_baseline": cpu,
    }


# --------------------------------------------------------------------------- C7
def run_c7(args, torch, dev):
    """Freezer<2048>(8, 1) (tests/freezer.cpp) over 480,000 samples per step: dry for 2 s,
    frozen for 6 s, dry again (freeze() before sample 96,000, unfreeze() before 384,000)."""
    import ctypes
    from huygens_amd import Freezer
    N, laps, S = 2048, 8, args.samples
    t = np.arange(S)
    rng = np.random.default_rng(8)
    x = torch.from_numpy(0.3 * np.sin(2 * np.pi * 440 * t / SR) + 0.05 * rng.standard_normal(S)).to(dev)
    y = torch.empty_like(x)
    ev = [(S // 5, 1), (4 * S // 5, 0)]
    fr = Freezer(N, laps, 1.0)
    fr.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctypes.CDLL(None).srand(1)

    def step():
        fr.process_device(x.data_ptr(), y.data_ptr(), S, ev)

    elapsed = _timed(step, args.steps, args.warmup, torch, dev)
    fr.profile(True)   # the output kernel's launches, HIP events, a separate pass
    _timed(step, args.steps, 0, torch, dev)
    kms, klaunch = fr.profile_read()
    fr.profile(False)
    cpu = None
    if not args.no_cpu_baseline:
        _tests_path()
        from oracle_frz import OracleFreezer
        o = OracleFreezer(N, laps, 1.0)
        n = 48000
        xs = x.cpu().numpy()[:n]
        t0 = time.perf_counter()
        o.process(xs, [(n // 5, 1), (4 * n // 5, 0)])
        dt = time.perf_counter() - t0
        cpu = {"value": n / dt, "unit": "samples/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle_frz.c Freezer<2048>(8, 1), {n} samples (same freeze pattern), "
                         f"long double DFTs, 1 thread, {dt:.2f} s"}
    # GB/s of the dominant kernel: 8 B in + 8 B out per sample over its launches' mean duration
    kern_s = kms / 1e3 / max(1, klaunch)
    achieved = 16.0 * S * args.steps / max(1, klaunch) / kern_s / 1e9 if kern_s > 0 else None
    ev = None
    if not getattr(args, "no_traffic", True) and klaunch:
        per = max(1, round(klaunch / args.steps))
        ev = row_evidence("frz_out_kernel", "c7", kms / 1e3 / args.steps, per_step=per, alg_bytes=16.0 * S)
    return {
        "metric": "samples/s, Freezer<2048>(8, 1) spectral freeze",
        "value": S * args.steps / elapsed, "unit": "samples/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f64",
        "data": "synthetic: 0.3 sin(2 pi 440 t) + 0.05 N(0,1) seed 8; freeze at 2 s, unfreeze at 8 s",
        "config": {"workload": "C7 Freezer<2048>(laps 8, width 1) (SURVEY.md 8(f) row 2)", "samples_per_step": S},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK if achieved else None,
                     "traffic": (ev or {}).get("traffic_bytes"), "pmc_evidence": ev, "kernel": "frz_out_kernel",
                     "kernel_avg_ms": 1e3 * kern_s, "launches_per_step": klaunch / max(1, args.steps),
                     "whole_step_gbs": 16.0 * S * args.steps / elapsed / 1e9,
                     "note": "16 B per sample over the output kernel's HIP-event time; the step also holds "
                             "the freeze-frame FFT passes and the host run/slot-map bookkeeping (whole_step_gbs)"},
        "cpu_baseline": cpu,
    }


# --------------------------------------------------------------------------- C8
C8_CHANNELS = 262144
C8_SAMPLES = 48000


def c8_bank(N, seed=8):
    """harmbank chain parameters (tests/harmbank.cpp: Slidebank order 4, RMSbank SR/20,
    Latchbank(0.0005), Stickbank(1, -0.9)) over N channels with partials spread 40 Hz-8 kHz;
    gain 3 x 96 / N keeps the mix at the 96-channel instrument's level."""
    rng = np.random.default_rng(seed)
    radii = np.zeros(2 * N)
    fa = rng.uniform(40.0, 8000.0, N) * np.where(rng.random(N) < 0.5, -1.0, 1.0)
    radii[0::2] = np.minimum(0.999, np.exp((np.log(0.5) - 4 - 1) / (25 * SR / np.abs(fa))))   # measure()
    return fa, radii, dict(thresh=0.0005, ratio=0.2, width=SR // 20, stick_order=1, stick_rad=-0.9, dry=0.0,
                           gain=3.0 * 96 / N)


def run_c8(args, torch, dev):
    """Heterodyne bank chain (tests/harmbank.cpp:77-101) fused over 262,144 channels; one step
    = 1 s of 48 kHz audio.  The reference's own 96-channel instrument is timed beside it."""
    from huygens_amd import Heterodyne, harmbank
    N = C8_CHANNELS
    S = C8_SAMPLES if args.samples == 480000 else args.samples
    fa, radii, kw = c8_bank(N)
    g = Heterodyne(N, 4, radii, **kw)
    for h in (g,):
        h.freqmod(0, np.arange(N), fa)
        h.freqmod(1, np.arange(N), -2 * fa)
        h.open(0)
        h.open(1)
    rng = np.random.default_rng(8)
    x = torch.from_numpy(0.2 * rng.standard_normal(S)).to(dev)
    y = torch.empty_like(x)
    g.set_stream(torch.cuda.current_stream(dev).cuda_stream)

    def step():
        g.process_device(x.data_ptr(), y.data_ptr(), S)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    g.profile(True)
    elapsed = _timed(step, args.steps, 0, torch, dev)
    ms, launches, cs = g.profile_read()
    g.profile(False)
    # dominant kernel het_chain_kernel<4,1,true>: algorithmic HBM bytes = the RMS ring's read +
    # write, 16 B per channel-sample; FP64 work 108 flops + 5 divides + 1 sqrt
    gbs = 16.0 * cs / (ms / 1e3) / 1e9 if ms > 0 else None
    tflops = 114.0 * cs / (ms / 1e3) / 1e12 if ms > 0 else None
    traffic, tdetail = None, "not collected (--no-traffic)"
    if not args.no_traffic:
        import bench
        tb, tdetail = bench.pmc_traffic(("het_chain_kernel",), extra=("--workload", "c8"))
        traffic = tb
    # the reference's instrument: 96 channels, 1 s of audio (latency-bound: one wave)
    n96, fa96, fs96, r96 = harmbank()
    h96 = Heterodyne(n96, 4, r96, 0.0005, 0.2, SR // 20, 1, -0.9, 0.0, 3.0)
    h96.freqmod(0, np.arange(n96), fa96)
    h96.freqmod(1, np.arange(n96), fs96)
    h96.open(0)
    h96.open(1)
    h96.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    x96 = x[:min(S, SR)]
    y96 = torch.empty_like(x96)
    h96.process_device(x96.data_ptr(), y96.data_ptr(), x96.numel())
    e96 = _timed(lambda: h96.process_device(x96.data_ptr(), y96.data_ptr(), x96.numel()), 3, 0, torch, dev)
    inst = {"channels": n96, "gpu_samples_per_s": 3 * x96.numel() / e96}
    cpu = None
    if not args.no_cpu_baseline:
        _tests_path()
        from oracle_het import OracleHet
        n = 1024
        o = OracleHet(N, 4, radii, kw["thresh"], kw["ratio"], kw["width"], 1, -0.9, 0.0, kw["gain"])
        o.freqmod(0, np.arange(N), fa)
        o.freqmod(1, np.arange(N), -2 * fa)
        o.open(0)
        o.open(1)
        xs = x[:n].cpu().numpy()
        t0 = time.perf_counter()
        o.process(xs)
        dt = time.perf_counter() - t0
        cpu = {"value": N * n / dt, "unit": "channel-samples/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle_het.c, the same {N}-channel chain over {n} samples, 1 thread, "
                         f"{dt:.2f} s"}
        o96 = OracleHet(n96, 4, r96, 0.0005, 0.2, SR // 20, 1, -0.9, 0.0, 3.0)
        o96.freqmod(0, np.arange(n96), fa96)
        o96.freqmod(1, np.arange(n96), fs96)
        o96.open(0)
        o96.open(1)
        xs = x96.cpu().numpy()
        t0 = time.perf_counter()
        o96.process(xs)
        inst["cpu_samples_per_s"] = xs.size / (time.perf_counter() - t0)
    return {
        "metric": "channel-samples/s, heterodyne bank chain (harmbank: Oscbank x2, Modbank, Slidebank(4), "
                  "RMSbank, Latchbank, Stickbank, Mixer)",
        "value": N * S * args.steps / elapsed, "unit": "channel-samples/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f64",
        "samples_per_s": S * args.steps / elapsed,
        "data": "synthetic: N(0, 0.2^2) input seed 8; partials uniform 40 Hz-8 kHz, random sign, seed 8",
        "config": {"workload": "C8 heterodyne chain (tests/harmbank.cpp:77-101) over 262144 channels "
                               "(SURVEY.md 8(f) row 3)", "channels": N, "samples_per_step": S, "order": 4,
                   "rms_width": SR // 20},
        "roofline": {"bound": "valu", "achieved": tflops, "peak": FP64_PEAK, "unit": "TFLOP/s",
                     "frac": tflops / FP64_PEAK if tflops else None, "traffic": traffic,
                     "traffic_detail": tdetail, "kernel": "het_chain_kernel<4,1,true>",
                     "kernel_ms_per_step": ms / args.steps, "launches_per_step": launches / args.steps,
                     "flops_per_unit": 114, "algorithmic_bytes_per_unit": 16,
                     "hbm_achieved_gbs": gbs, "hbm_frac": gbs / HBM_PEAK if gbs else None,
                     "note": "flops count div/sqrt as 1; each expands to ~11 VALU instructions"},
        "instrument_96ch": inst,
        "cpu_baseline": cpu,
    }


# --------------------------------------------------------------------------- C9
C9_BANDS = 16384
C9_SAMPLES = 48000


def run_c9(args, torch, dev):
    """Filterbank(2, N) with per-sample resonant-frequency streams (Subtractive ALLINONE,
    src/subtractive.h:215-228): every band retuned every sample; one step = 1 s of audio.
    The reference's instrument size (7 voices x 7 overtones = 49 bands) is timed beside it, and
    the raw-coefficient stream kind (40 B per band-sample) on a shorter step."""
    from huygens_amd import Filterbank
    from huygens_amd.filterbank import TV_COEFFS, TV_RESONANT
    N = C9_BANDS
    S = C9_SAMPLES if args.samples == 480000 else args.samples
    R = 0.99999
    rng = np.random.default_rng(9)
    base = torch.from_numpy(rng.uniform(60.0, 3000.0, N)).to(dev)
    phase = torch.from_numpy(rng.uniform(0.0, 1.0, N)).to(dev)
    t = torch.arange(S, device=dev, dtype=torch.float64)[:, None]
    freqs = (base[None, :] * (1 + 0.05 * torch.sin(2 * np.pi * (t / 4800.0 + phase[None, :])))).contiguous()
    del t
    x = torch.from_numpy(rng.uniform(-1.0, 1.0, S)).to(dev)
    y = torch.empty_like(x)
    g = Filterbank(2, N, 0.1, 1.0)
    g.boost([0.7 ** (i % 7) for i in range(N)])   # boost(i * overtones + j, decay^j)
    g.open()
    g.set_stream(torch.cuda.current_stream(dev).cuda_stream)

    def step():
        g.process_tv_device(x.data_ptr(), y.data_ptr(), S, TV_RESONANT, freqs.data_ptr(), R)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    g.profile(True)
    elapsed = _timed(step, args.steps, 0, torch, dev)
    seg_ms, mix_ms, red_ms, launches = g.profile_read()
    g.profile(False)
    bs = N * S * args.steps
    tflops = 49.0 * bs / (mix_ms / 1e3) / 1e12 if mix_ms > 0 else None
    gbs = 8.0 * bs / (mix_ms / 1e3) / 1e9 if mix_ms > 0 else None
    traffic, tdetail = None, "not collected (--no-traffic)"
    if not args.no_traffic:
        import bench
        traffic, tdetail = bench.pmc_traffic(("fb_tv_res_kernel",), extra=("--workload", "c9"))
    # raw coefficient streams: [n][5][N] (40 B per band-sample), 4800 samples
    n2 = min(S, 4800)
    st = torch.zeros((n2, 5, N), dtype=torch.float64, device=dev)
    st[:, 0, :] = 1 - R
    st[:, 2, :] = -(1 - R)
    st[:, 3, :] = -2 * R * torch.cos(2 * np.pi * freqs[:n2] / SR)
    st[:, 4, :] = R * R
    g.process_tv_device(x.data_ptr(), y.data_ptr(), n2, TV_COEFFS, st.data_ptr(), 0.0)
    g.profile(True)
    e2 = _timed(lambda: g.process_tv_device(x.data_ptr(), y.data_ptr(), n2, TV_COEFFS, st.data_ptr(), 0.0), 3, 0,
                torch, dev)
    _, m2, _, _ = g.profile_read()
    g.profile(False)
    coeffs = {"band_samples_per_s": 3 * N * n2 / e2, "kernel_ms": m2 / 3,
              "hbm_achieved_gbs": 40.0 * N * n2 / (m2 / 3 / 1e3) / 1e9 if m2 > 0 else None,
              "algorithmic_bytes_per_unit": 40}
    del st
    # the reference's instrument: Subtractive(7, 7, ...) = 49 bands, 1 s of audio
    g49 = Filterbank(2, 49, 0.1, 1.0)
    g49.boost([0.7 ** (i % 7) for i in range(49)])
    g49.open()
    g49.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    f49 = freqs[:, :49].contiguous()
    g49.process_tv_device(x.data_ptr(), y.data_ptr(), S, TV_RESONANT, f49.data_ptr(), R)
    e49 = _timed(lambda: g49.process_tv_device(x.data_ptr(), y.data_ptr(), S, TV_RESONANT, f49.data_ptr(), R), 3, 0,
                 torch, dev)
    inst = {"bands": 49, "gpu_samples_per_s": 3 * S / e49}
    cpu = None
    if not args.no_cpu_baseline:
        _tests_path()
        from oracle import OracleFilterbank
        n = 960
        o = OracleFilterbank(2, N, 0.1, 1.0)
        o.boost([0.7 ** (i % 7) for i in range(N)])
        o.open()
        xs, fs = x[:n].cpu().numpy(), freqs[:n].cpu().numpy()
        t0 = time.perf_counter()
        o.process_tv(xs, TV_RESONANT, fs, R)
        dt = time.perf_counter() - t0
        cpu = {"value": N * n / dt, "unit": "band-samples/s", "cores": 1, "kind": "port",
               "sample": f"oracle/hz_oracle.c orc_fb_process_tv, the same {N}-band resonant streams over {n} "
                         f"samples, 1 thread, {dt:.2f} s"}
        o49 = OracleFilterbank(2, 49, 0.1, 1.0)
        o49.boost([0.7 ** (i % 7) for i in range(49)])
        o49.open()
        m = min(S, 24000)
        f49h = f49[:m].cpu().numpy()
        t0 = time.perf_counter()
        o49.process_tv(x[:m].cpu().numpy(), TV_RESONANT, f49h, R)
        inst["cpu_samples_per_s"] = m / (time.perf_counter() - t0)
    return {
        "metric": "band-samples/s, Filterbank(2, N) retuned every sample (resonant-frequency streams, "
                  "Subtractive ALLINONE)",
        "value": bs / elapsed, "unit": "band-samples/s",
        "ms_per_step": 1e3 * elapsed / args.steps, "dtype": "f64",
        "samples_per_s": S * args.steps / elapsed,
        "data": "synthetic: uniform[-1,1) input seed 9; per-band frequency tracks base uniform 60-3000 Hz, "
                "5 % vibrato at 10 Hz, generated on the device",
        "config": {"workload": "C9 per-sample coefficient streams (SURVEY.md 8(f) row 4)", "bands": N,
                   "samples_per_step": S, "order": 2, "R": R, "kind": "HZ_FB_TV_RESONANT"},
        "roofline": {"bound": "valu", "achieved": tflops, "peak": FP64_PEAK, "unit": "TFLOP/s",
                     "frac": tflops / FP64_PEAK if tflops else None, "traffic": traffic,
                     "traffic_detail": tdetail, "kernel": "fb_tv_res_kernel<NONE> (15 producer waves + 1 recurrence wave per 64 bands)",
                     "kernel_ms_per_step": mix_ms / args.steps, "mix_reduce_ms_per_step": red_ms / args.steps,
                     "launches_per_step": launches / args.steps, "flops_per_unit": 49,
                     "algorithmic_bytes_per_unit": 8, "hbm_achieved_gbs": gbs,
                     "note": "coefficients time-parallel in 15 producer waves, the recurrence sequential "
                             "in one wave per 64 bands (DESIGN.md 4.5); cos, sincos, 4 divides, hypot, sqrt "
                             "counted as 1 flop each"},
        "variant_coeff_stream": coeffs,
        "instrument_49_bands": inst,
        "cpu_baseline": cpu,
    }
