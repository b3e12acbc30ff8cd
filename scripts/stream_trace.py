"""Summarise an HZ_STREAM_TRACE file (hz_fb_stream.hip trace_flush): per launch kind, the span from
the first workgroup's start to the last workgroup's end, and the gaps between consecutive launches
(the last workgroup's end of one to the first workgroup's start of the next), in microseconds."""
import collections
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
rec = 8 + 1024 * 8
n = len(raw) // rec
kinds, spans, starts, ends = [], [], [], []
for i in range(n):
    k, wg = np.frombuffer(raw, dtype=np.int32, count=2, offset=i * rec)
    st = np.frombuffer(raw, dtype=np.uint64, count=1024, offset=i * rec + 8)
    s0, e0 = st[:wg], st[512:512 + wg]
    kinds.append(int(k))
    starts.append(int(s0.min()))
    ends.append(int(e0.max()))
names = {0: "block", 1: "block+transient", 2: "setter", 3: "setter taps"}
print(f"{n} launches")
span = collections.defaultdict(list)
for k, s, e in zip(kinds, starts, ends):
    span[names[k]].append((e - s) / 100.0)
for k, v in span.items():
    print(f"  {k:16s} n={len(v):5d} span mean {np.mean(v):6.2f} median {np.median(v):6.2f} us")
gaps = collections.defaultdict(list)
for i in range(1, n):
    g = (starts[i] - ends[i - 1]) / 100.0
    if g < 1000:   # (between separate passes: host time)
        gaps[(names[kinds[i - 1]], names[kinds[i]])].append(g)
for k, v in gaps.items():
    print(f"  gap {k[0]:16s} -> {k[1]:16s} n={len(v):5d} mean {np.mean(v):6.2f} median {np.median(v):6.2f} us")
# the churn pass: from the first setter to the last launch
f = kinds.index(2) if 2 in kinds else 0
tot = (ends[-1] - starts[f]) / 100.0
nb = sum(1 for k in kinds[f:] if k != 2)
print(f"  from the first setter: {tot:.1f} us over {nb} blocks = {tot / max(1, nb):.2f} us per block")
# setter launches: per role (columns [0, 33), taps [33, 33 + K/256), upkeep), the workgroups' start and
# end after the launch's first start
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 192
roles = collections.defaultdict(lambda: [[], []])
for i in range(n):
    if kinds[i] != 2:
        continue
    k, wg = np.frombuffer(raw, dtype=np.int32, count=2, offset=i * rec)
    st = np.frombuffer(raw, dtype=np.uint64, count=1024, offset=i * rec + 8).astype(np.int64)
    s0 = st[:wg].min()
    for name, lo, hi in (("columns", 0, 33), ("taps", 33, 33 + nt), ("upkeep", 33 + nt, wg)):
        if hi > wg or hi <= lo:
            continue
        roles[name][0].append((st[lo:hi] - s0).mean() / 100.0)
        roles[name][1].append((st[512 + lo:512 + hi] - s0).max() / 100.0)
for name, (a, b) in roles.items():
    print(f"  setter {name:8s} start mean {np.mean(a):6.2f} us, last end {np.mean(b):6.2f} us after the launch's first start")
# column phase marks (trace[768 + 6 c + k], k = 0 before the batch, 1 after its loads and barrier,
# 2 after its compute, 3 after the spectra stores, 4 at the end), after the launch's first start
marks = [[] for _ in range(5)]
for i in range(n):
    if kinds[i] != 2:
        continue
    k, wg = np.frombuffer(raw, dtype=np.int32, count=2, offset=i * rec)
    st = np.frombuffer(raw, dtype=np.uint64, count=1024, offset=i * rec + 8).astype(np.int64)
    s0 = st[:wg].min()
    for m in range(5):
        marks[m].append(np.mean([st[768 + 6 * c + m] - s0 for c in range(33)]) / 100.0)
print("  column marks (us after the launch's first start):", " ".join(f"{m}:{np.mean(v):.2f}" for m, v in enumerate(marks)))
# block launches: per role, the last workgroup end after the launch's first start
OUTWG = int(__import__("os").environ.get("OUTWG", "64"))
brole = {0: (("transform", 0, 33), ("mac", 33, 66), ("out", 66, 66 + OUTWG)),
         1: (("transform", 0, 33), ("mac", 33, 66), ("out", 66, 66 + OUTWG), ("D transform", 66 + OUTWG, 99 + OUTWG), ("D mac", 99 + OUTWG, 132 + OUTWG))}
for kind in (0, 1):
    acc = collections.defaultdict(list)
    for i in range(n):
        if kinds[i] != kind:
            continue
        k, wg = np.frombuffer(raw, dtype=np.int32, count=2, offset=i * rec)
        st = np.frombuffer(raw, dtype=np.uint64, count=1024, offset=i * rec + 8).astype(np.int64)
        s0 = st[:wg].min()
        for name, lo, hi in brole[kind]:
            acc[name].append((st[512 + lo:512 + hi] - s0).max() / 100.0)
    if acc:
        print(f"  {names[kind]} role ends:", " ".join(f"{k} {np.mean(v):.2f}" for k, v in acc.items()))
# output workgroups' phase marks (trace[768 + 4 k + m]: m = 0 after the operand loads and the first
# barrier, 1 after the head / tail partials, 2 after the partial sums), after the launch's first start
for kind in (0, 1):
    mk = [[] for _ in range(3)]
    ends = []
    for i in range(n):
        if kinds[i] != kind:
            continue
        k, wg = np.frombuffer(raw, dtype=np.int32, count=2, offset=i * rec)
        st = np.frombuffer(raw, dtype=np.uint64, count=1024, offset=i * rec + 8).astype(np.int64)
        s0 = st[:wg].min()
        for m in range(3):
            mk[m].append(np.mean([st[768 + 4 * kk + m] - s0 for kk in range(min(OUTWG, 64))]) / 100.0)
        ends.append(np.mean(st[512 + 66:512 + 66 + OUTWG] - s0) / 100.0)
    if ends:
        print(f"  {names[kind]} output marks:", " ".join(f"{m}:{np.mean(v):.2f}" for m, v in enumerate(mk)), f"end {np.mean(ends):.2f}")
